#!/bin/bash
# round 6 (w): SQ issue / wait / LDS counters of the fused LNB (channel-blocked input) and feature_edges
set -o pipefail
export MICRO_ARGS="--size 256 --c8 1"
timeout -k 10 300 bash scripts/pmc_sq.sh lnb lnb_fused16 r06w/lnb || exit 1
export MICRO_ARGS="--size 256"
timeout -k 10 300 bash scripts/pmc_sq.sh feature_edges_c8 feat_edge r06w/fe || exit 1

#!/bin/bash
# Round 5: SQ issue / wait counters of the fused LNB (map1 full, producer-only, consumer-only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in map1 m1d1 m1d2; do
  GRR_LIB=exp/libgrr_$v.so timeout -k 10 300 bash scripts/pmc_sq.sh lnb lnb_fused16 r05e/$v > gpurun_out/r05e_$v.log 2>&1 || { cat gpurun_out/r05e_$v.log | tail; exit 1; }
  tail -3 gpurun_out/r05e_$v.log
done

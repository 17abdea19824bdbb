#!/bin/bash
# step2 with the half level inside (tests + bench), then SQ counters of the LNB head and of step2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_step2h.sh || exit $?
bash scripts/pmc_sq.sh lnb lnb_head16 sq_head16 || exit $?
bash scripts/pmc_sq.sh step2 graph_step2 sq_step2 || exit $?

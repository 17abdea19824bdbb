#!/bin/bash
# Same-box A/B of LNB head-kernel variants (exp/libgrr_*.so): full C=96 block and the replicated first block
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for k in lnb lnb_rep; do
  for sz in ${SIZES:-256 128}; do
    for r in 1 2; do
      for L in "$@"; do
        printf "%-8s %4s %-24s " $k $sz "$(basename $L)"
        GRR_LIB=$L timeout -k 10 120 python scripts/micro.py --kernel $k --size $sz --iters 20 2>&1 | tail -1 || exit $?
      done
    done
  done
done

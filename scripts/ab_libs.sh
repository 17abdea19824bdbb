#!/bin/bash
# Same-box A/B: time one micro kernel under several libgrr builds, two alternating rounds.
#   bash scripts/ab_libs.sh <kernel> exp/libgrr_a.so exp/libgrr_b.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K=$1; shift
for r in 1 2; do
  for L in "$@"; do
    printf "%-28s " "$(basename $L)"
    GRR_LIB=$L timeout -k 10 120 python scripts/micro.py --kernel "$K" --iters 30 2>&1 | tail -1 || exit $?
  done
done

#!/bin/bash
# A/B of two libgrr builds on the same box: micro step kernel, alternating A B A B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=${1:-imagerestoration-development-unrolling_amd/libgrr.so}
B=${2:-exp/libgrr_oldstep.so}
K=${3:-step}
for r in 1 2; do
  for L in "$A" "$B"; do
    echo "== $L"; GRR_LIB=$L timeout -k 10 120 python scripts/micro.py --kernel "$K" --iters 30 2>&1 | tail -1 || exit $?
  done
done

#!/bin/bash
# same-box A/B of libgrr LNB variants (exp/libgrr_<name>.so) on the two-kernel path (GRR_LNB_FUSED=0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in "$@"; do
    for sz in 256 128; do
      echo "variant=$v size=$sz"
      GRR_LNB_FUSED=0 GRR_LIB=exp/libgrr_$v.so timeout -k 10 120 python scripts/micro.py --kernel lnb --iters 10 --size $sz 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done

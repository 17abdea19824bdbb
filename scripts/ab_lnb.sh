#!/bin/bash
# A/B of the LocalNonLinearBlock paths on the GPU box: fused (default) vs head + mix (GRR_LNB_FUSED=0),
# micro shape (64 x 96 x 256^2, hid 256) and half resolution, then the bench breakdown with each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 0; do
  for sz in 256 128; do
    echo "GRR_LNB_FUSED=$v size=$sz"
    GRR_LNB_FUSED=$v timeout -k 10 120 python scripts/micro.py --kernel lnb --iters 10 --size $sz || exit $?
  done
done

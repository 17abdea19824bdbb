#!/bin/bash
# LNB head phase stamps (GRR_FUSED_STAMP builds): staggered vs all-gate-first, C = 96 and the replicated block
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/st
for L in exp/libgrr_stamp.so exp/libgrr_stampns.so; do
  for k in lnb lnb_rep; do
    echo "== $L $k"; GRR_LIB=$L timeout -k 10 120 python scripts/micro.py --kernel $k --iters 5 2>&1 | grep -v amdgpu.ids || exit 1
  done
done 2>&1 | tee gpurun_out/st/stamps.log

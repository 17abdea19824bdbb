#!/bin/bash
# LNB head with the packed (mask, value) depthwise gate vs the previous build (exp/libgrr_prev.so)
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_prev.so; do
    GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel lnb --iters 20 2>&1 | grep "lnb:" | sed "s|^|$(basename $lib) |" || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_psnr.py -x -q --timeout 240 --timeout-method thread -k "local_nonlinear or x3 or msgf or psnr or c3 or replicated" 2>&1 | tail -2

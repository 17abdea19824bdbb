#!/bin/bash
# lnb_rep_kernel v2 (fp16 GEMM2 with running exponent, 4-slot ring): parity + variants (occupancy, GEMM1 pipelining)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04f; mkdir -p $out
export TMPDIR=/tmp
for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_occ4.so exp/libgrr_nopipe4.so; do
  GRR_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -rf -k "replicated or msgf" \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests_$(basename $lib .so).log 2>&1; rc=$?
  echo "$lib $(tail -1 $out/tests_$(basename $lib .so).log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_occ4.so exp/libgrr_nopipe4.so; do for sz in 256 128; do
  echo "r$r $lib $sz $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel lnb_rep --size $sz --split --iters 20 2>&1 | grep lnb_rep_fused)" >> $out/micro.txt || exit 1
done; done; done
cat $out/micro.txt

#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/gemm; mkdir -p $out
export TMPDIR=/tmp
for v in 23 43; do
  GRR_WGRAD_TILE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests_$v.log 2>&1
  rc=$?; tail -2 $out/tests_$v.log; [ $rc -eq 0 ] || exit $rc
  GRR_WGRAD_TILE=$v timeout -k 10 200 python -u scripts/micro_wgrad.py > $out/micro_$v.txt 2>&1; rc=$?; grep wgrad $out/micro_$v.txt; [ $rc -eq 0 ] || exit $rc
done

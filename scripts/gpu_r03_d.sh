#!/bin/bash
# step2 channel groups (F = 6 / 12): step2 + v1.0 model GPU tests; then the bench-shape PMC traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r03d; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_step2.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -rf \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_bench.sh 64 || exit $?

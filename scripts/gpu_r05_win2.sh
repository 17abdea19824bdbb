#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05win2; mkdir -p $out
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_window_grad.py \
  -k "fused_gather or solver_reverse" > $out/tests.log 2>&1; tail -30 $out/tests.log | grep -v "^E  \|tensor" | tail -25

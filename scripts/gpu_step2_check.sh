#!/bin/bash
# step2 GPU tests, then the A/B bench (two-stage launches on / off)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_step2.py -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/step2_tests.log 2>&1 || { tail -30 gpurun_out/step2_tests.log; exit 1; }
tail -2 gpurun_out/step2_tests.log
bash scripts/ab_step2.sh

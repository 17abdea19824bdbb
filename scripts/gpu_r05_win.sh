#!/bin/bash
# window reverse: fused gather parity + A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05win; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_window_grad.py \
  tests/test_gpu_configs.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u scripts/win_gather_ab.py > $out/ab.txt 2>&1 || { tail -20 $out/ab.txt; exit 1; }
cat $out/ab.txt

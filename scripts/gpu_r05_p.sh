#!/bin/bash
# term ring + x-gradient pass: the term / training / determinism suites
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05p}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_term_acc.py \
  tests/test_gpu_term_ring.py tests/test_gpu_term_rows.py tests/test_gpu_deterministic.py tests/test_gpu_training.py \
  tests/test_gpu_grad.py tests/test_gpu_first_pair.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log

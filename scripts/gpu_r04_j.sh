#!/bin/bash
# Round 4: fixed-order reductions in the training reverse -- determinism + gradient suites, then the
# training lines and the term reverse's PMC traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04j; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_deterministic.py tests/test_gpu_term_rows.py tests/test_gpu_grad.py tests/test_gpu_padj2.py \
  tests/test_gpu_streams.py tests/test_gpu_subapi_grad.py tests/test_gpu_dwconv.py tests/test_gpu_glue.py \
  tests/test_gpu_ffn.py tests/test_gpu_ddp.py tests/test_gpu_training.py tests/test_gpu_window.py \
  tests/test_gpu_window_grad.py > $out/tests.log 2>&1
rc=$?; tail -15 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_i.sh

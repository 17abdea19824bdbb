#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/ffnb; mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_window_grad.py tests/test_gpu_grad.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench_window.py --train --batch 4 --no-cpu-baseline --breakdown > $out/train256.json 2> $out/train256.err || { tail $out/train256.err; exit 1; }
head -c 300 $out/train256.json; echo

#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/x3k; mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_parity.py -k "ffn or ffblock or feature or conv or x3" -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/micro_wgrad.py > $out/micro.txt 2>&1; rc=$?; grep conv1x1 $out/micro.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench_window.py --no-cpu-baseline --breakdown > $out/bench_window.json 2> $out/bench_window.err || { tail $out/bench_window.err; exit 1; }
head -c 300 $out/bench_window.json; echo; grep -v amdgpu $out/bench_window.err | head -8

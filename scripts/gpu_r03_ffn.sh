#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/ffn; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_window.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -4 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench_window.py --no-cpu-baseline --breakdown > $out/bench_window.json 2> $out/bench_window.err || { tail $out/bench_window.err; exit 1; }
head -c 600 $out/bench_window.json; echo; grep -v amdgpu $out/bench_window.err | head -30

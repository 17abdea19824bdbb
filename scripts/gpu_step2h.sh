#!/bin/bash
# step2 with stage A's half level inside: the step2 parity tests, the filter parity tests, then the
# bench line (kernel_ms_per_step: system_half should drop to the two single-stage launches)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/s2h; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_step2.py tests/test_gpu_parity.py tests/test_gpu_streams.py -x -q \
  -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
python -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_ms_per_step'])"
timeout -k 10 120 python scripts/micro.py --kernel step2 --iters 20 2>&1 | tail -1

#!/bin/bash
# Round 4 checkpoint (continued): the fixed training test, then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04h; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('kernel_ms_per_step'))"

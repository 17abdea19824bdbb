#!/bin/bash
# round 6 end: full GPU suite, smoke, the default bench line (with the round-6 traffic files), the C4 training line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R06E_OUT:-r06e}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?
tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "
import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['kernel_ms_per_step'])"
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/train_c4.json 2> $out/train_c4.err || { tail $out/train_c4.err; exit 1; }
echo "train_c4 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $out/train_c4.json | tr '\n' ' ')"

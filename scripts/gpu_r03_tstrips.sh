#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/tstrips; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_term_rows.py tests/test_gpu_grad.py tests/test_gpu_training.py tests/test_gpu_step2.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -4 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
head -c 300 $out/c4.json; echo
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline > $out/abstract.json 2> $out/abstract.err || exit 1
head -c 250 $out/abstract.json | grep -o '"ms_per_step": [0-9.]*'

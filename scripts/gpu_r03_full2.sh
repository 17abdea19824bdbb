#!/bin/bash
# Full GPU suite after the step2 strips, then the training lines (msgf, v1.0 at 256^2, C4 at 512^2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/full2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?
tail -8 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline > $out/msgf.json 2> $out/msgf.err || { tail $out/msgf.err; exit 1; }
head -c 300 $out/msgf.json | grep -o '"ms_per_step": [0-9.]*'
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline > $out/abstract.json 2> $out/abstract.err || { tail $out/abstract.err; exit 1; }
head -c 300 $out/abstract.json | grep -o '"ms_per_step": [0-9.]*'
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
head -c 300 $out/c4.json | grep -o '"ms_per_step": [0-9.]*'

#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/s2train; mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 600 python -u -m pytest tests/test_gpu_step2.py tests/test_gpu_grad.py tests/test_gpu_training.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -4 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 8 --warmup 2 --no-cpu-baseline --watchdog 45 > $out/msgf_$r.json 2> $out/msgf_$r.err || exit 1
  head -c 250 $out/msgf_$r.json | grep -o '"ms_per_step": [0-9.]*'
done
GRR_STEP2=0 timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 8 --warmup 2 --no-cpu-baseline > $out/msgf_nostep2.json 2> $out/msgf_nostep2.err || exit 1
printf "no step2: "; head -c 250 $out/msgf_nostep2.json | grep -o '"ms_per_step": [0-9.]*'
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline > $out/abstract.json 2> $out/abstract.err || exit 1
printf "abstract: "; head -c 250 $out/abstract.json | grep -o '"ms_per_step": [0-9.]*'

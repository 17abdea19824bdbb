#!/bin/bash
# half-level reverse on a second stream (GRR_LEVEL_STREAMS): equivalence tests, then A/B on the msgf
# and v1.0 training steps (same box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/levels; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_grad.py tests/test_gpu_training.py tests/test_gpu_step2.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for ls in 0 1; do
    GRR_LEVEL_STREAMS=$ls timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 5 --warmup 2 --no-cpu-baseline > $out/msgf_${ls}_$r.json 2> $out/msgf_${ls}_$r.err || { tail $out/msgf_${ls}_$r.err; exit 1; }
    GRR_LEVEL_STREAMS=$ls timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline > $out/abs_${ls}_$r.json 2> $out/abs_${ls}_$r.err || { tail $out/abs_${ls}_$r.err; exit 1; }
    echo "levels=$ls run $r: msgf $(grep -o '"ms_per_step": [0-9.]*' $out/msgf_${ls}_$r.json) abstract $(grep -o '"ms_per_step": [0-9.]*' $out/abs_${ls}_$r.json)"
  done
done

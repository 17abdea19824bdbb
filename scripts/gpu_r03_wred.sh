#!/bin/bash
# wgrad's chunk reduction as 64-output x 16-wave workgroups: wgrad tests, then msgf / v1.0 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/wred; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_ffn.py tests/test_gpu_grad.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
GRR_FEATURE_STREAMS_TRAIN=0 timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 4 --warmup 2 --no-cpu-baseline --breakdown > $out/msgf_1s.json 2> $out/msgf_1s.err || { tail $out/msgf_1s.err; exit 1; }
grep -E "wgrad" $out/msgf_1s.err
for r in 1 2; do
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 5 --warmup 2 --no-cpu-baseline > $out/msgf_$r.json 2> $out/msgf_$r.err || { tail $out/msgf_$r.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $out/msgf_$r.json
done
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline > $out/abstract.json 2> $out/abstract.err || { tail $out/abstract.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $out/abstract.json

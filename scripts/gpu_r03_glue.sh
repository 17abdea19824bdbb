#!/bin/bash
# vectorised glue kernels of the training reverse: unit tests, gradient tests, msgf training step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/glue; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_glue.py tests/test_gpu_grad.py tests/test_gpu_training.py tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -4 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 5 --warmup 2 --no-cpu-baseline --breakdown > $out/msgf_$r.json 2> $out/msgf_$r.err || { tail $out/msgf_$r.err; exit 1; }
grep -E "bwd_lincomb|bwd_graph_dot|unpool2" $out/msgf_$r.err; head -c 300 $out/msgf_$r.json | grep -o '"ms_per_step": [0-9.]*'
done

#!/bin/bash
# saved D x_k (SAVE_POOLED): parity tests, then same-box training A/B (v1.0 256^2 x8, C4 512^2 x32)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05s; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_step2.py \
  tests/test_gpu_grad.py tests/test_gpu_training.py tests/test_compile_training.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for rep in 1 2; do
for sp in 0 1; do
GRR_SAVE_POOLED=$sp timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/abs_$sp.$rep.json 2> $out/abs_$sp.$rep.err || { tail $out/abs_$sp.$rep.err; exit 1; }
echo "abs sp=$sp rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $out/abs_$sp.$rep.json | tr '\n' ' ')"
done
done
for sp in 0 1; do
GRR_SAVE_POOLED=$sp timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/c4_$sp.json 2> $out/c4_$sp.err || { tail $out/c4_$sp.err; exit 1; }
echo "c4 sp=$sp $(grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*\|"pool2": [0-9.]*' $out/c4_$sp.json | tr '\n' ' ')"
done

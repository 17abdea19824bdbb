#!/bin/bash
# glue-pooled gu (GLUE_POOL): parity tests, same-box training A/B, then the C4 term-shape sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05t; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_term_acc.py \
  tests/test_gpu_step2.py tests/test_gpu_grad.py tests/test_gpu_training.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for rep in 1 2; do
for gp in 0 1; do
GRR_GLUE_POOL=$gp timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/abs_$gp.$rep.json 2> $out/abs_$gp.$rep.err || { tail $out/abs_$gp.$rep.err; exit 1; }
echo "abs gp=$gp rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"pool2": [0-9.]*\|"bwd_cg_glue": [0-9.]*' $out/abs_$gp.$rep.json | tr '\n' ' ')"
done
done
for gp in 0 1; do
GRR_GLUE_POOL=$gp timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/c4_$gp.json 2> $out/c4_$gp.err || { tail $out/c4_$gp.err; exit 1; }
echo "c4 gp=$gp $(grep -o '"ms_per_step": [0-9.]*\|"pool2": [0-9.]*\|"bwd_cg_glue": [0-9.]*' $out/c4_$gp.json | tr '\n' ' ')"
done
timeout -k 10 400 python -u scripts/term_sweep.py > $out/term_sweep.txt 2>&1 || { tail $out/term_sweep.txt; exit 1; }
cat $out/term_sweep.txt

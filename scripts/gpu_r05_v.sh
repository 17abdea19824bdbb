#!/bin/bash
# wgrad tile plans: parity, per-shape A/B, training A/B (v1.0 256^2 x8, C4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05v; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_wgrad.py \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 python -u scripts/wgrad_ab.py > $out/wgrad_ab.txt 2>&1 || { tail -20 $out/wgrad_ab.txt; exit 1; }
cat $out/wgrad_ab.txt
for rep in 1 2; do
for wt in 0 1; do
GRR_WGRAD_TILES=$wt timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/abs_$wt.$rep.json 2> $out/abs_$wt.$rep.err || { tail $out/abs_$wt.$rep.err; exit 1; }
echo "abs wt=$wt rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"wgrad": [0-9.]*' $out/abs_$wt.$rep.json | tr '\n' ' ')"
done
done
for wt in 0 1; do
GRR_WGRAD_TILES=$wt timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/c4_$wt.json 2> $out/c4_$wt.err || { tail $out/c4_$wt.err; exit 1; }
echo "c4 wt=$wt $(grep -o '"ms_per_step": [0-9.]*\|"wgrad": [0-9.]*' $out/c4_$wt.json | tr '\n' ' ')"
done

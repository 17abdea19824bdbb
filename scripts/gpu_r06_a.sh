#!/bin/bash
# round 6 (a): full GPU suite, bench, fused-LNB start-phase stagger A/B (micro + bench)
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
for sz in 256 128; do
  for st in 0,3 16,3 16,2 8,5 32,2; do
    timeout -k 10 120 python scripts/micro.py --kernel lnb --size $sz --iters 20 --stagger $st > $O/micro_${sz}_${st}.txt 2>&1 || exit 1
    echo "$sz $st $(grep -h lnb $O/micro_${sz}_${st}.txt | tail -1)"
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --lnb-stagger 16,3 > $O/bench_st16_3.json 2> $O/bench_st.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/bench2.json 2>> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --lnb-stagger 16,2 > $O/bench_st16_2.json 2>> $O/bench_st.err || exit 1
for f in $O/bench*.json; do python -c "
import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['kernel_ms_per_step'].get('lnb_fused'))"; done

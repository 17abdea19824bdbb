#!/bin/bash
# round 6 (h): feature_edges with hardware rcp / sqrt / exp2 -- parity, per launch, knock-outs, bench
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_feature_edges.py tests/test_gpu_compile.py -x -q --timeout 120 --timeout-method thread > $O/fe.log 2>&1 || { tail -40 $O/fe.log; exit 1; }
tail -1 $O/fe.log
for sz in 256 128; do
  for kern in conv_edges feature_edges_c8; do
    timeout -k 10 120 python scripts/micro.py --kernel $kern --size $sz --iters 20 > $O/m_${kern}_$sz.txt 2>&1 || exit 1
    echo "$sz $kern: $(grep -h 'mean=' $O/m_${kern}_$sz.txt | tr '\n' ' ')"
  done
done
for v in fed1 fed4 fed5; do
  GRR_LIB=exp/libgrr_$v.so timeout -k 10 120 python scripts/micro.py --kernel feature_edges_c8 --size 256 --iters 20 > $O/m_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'mean=' $O/m_$v.txt | tr '\n' ' ')"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "
import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"

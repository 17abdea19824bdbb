#!/bin/bash
# round 6 (v): feature_edges loader with main rows two ahead (FE_AHEAD2) -- parity, per launch A/B
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
GRR_LIB=exp/libgrr_a2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_feature_edges.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for rep in 1 2; do
for sz in 256 128; do
  for v in base a2; do
    lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
    GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel feature_edges_c8 --size $sz --iters 20 > $O/m_${v}_$sz.txt 2>&1 || exit 1
    echo "$sz $v: $(grep -h 'mean=' $O/m_${v}_$sz.txt | tr '\n' ' ')"
  done
done
done

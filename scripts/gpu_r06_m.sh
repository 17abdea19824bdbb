#!/bin/bash
# round 6 (m): feature_edges candidate (GRR_LIB exp) -- parity, per launch A/B
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
GRR_LIB=exp/libgrr_fe3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_feature_edges.py -x -q --timeout 120 --timeout-method thread > $O/fe.log 2>&1 || { tail -40 $O/fe.log; exit 1; }
tail -1 $O/fe.log
for sz in 256 128; do
  for v in fe2 fe3; do
    lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
    for kern in feature_edges_c8; do
      GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel $kern --size $sz --iters 20 > $O/m_${v}_${kern}_$sz.txt 2>&1 || exit 1
      echo "$sz $v $kern: $(grep -h 'mean=' $O/m_${v}_${kern}_$sz.txt | tr '\n' ' ')"
    done
  done
done

#!/bin/bash
# round 6 (g): feature_edges per launch vs the two-pass path, and timing-only knock-out builds
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
for sz in 256 128; do
  for kern in conv_edges feature_edges feature_edges_c8; do
    timeout -k 10 120 python scripts/micro.py --kernel $kern --size $sz --iters 20 > $O/m_${kern}_$sz.txt 2>&1 || exit 1
    echo "$sz $kern: $(grep -h 'mean=' $O/m_${kern}_$sz.txt | tr '\n' ' ')"
  done
done
for v in fed1 fed2 fed4 fed8 fed15; do
  GRR_LIB=exp/libgrr_$v.so timeout -k 10 120 python scripts/micro.py --kernel feature_edges_c8 --size 256 --iters 20 > $O/m_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'mean=' $O/m_$v.txt | tr '\n' ' ')"
done

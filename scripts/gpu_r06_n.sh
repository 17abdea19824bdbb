#!/bin/bash
# round 6 (n): feature_edges knock-outs (timing only): 4 no loads, 2 no edges, 8 no conv, 1 no stores
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
for v in fs1 fd4 fd2 fd8 fd1; do
  GRR_LIB=exp/libgrr_$v.so timeout -k 10 120 python scripts/micro.py --kernel feature_edges_c8 --size 256 --iters 20 > $O/m_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'mean=' $O/m_$v.txt | tr '\n' ' ')"
done

#!/bin/bash
# round 6 (k): feature_edges knock-outs (timing only): no stores / no loads / neither
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
for v in base fed1 fed4 fed5; do
  lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
  GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel feature_edges_c8 --size 256 --iters 20 > $O/m_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'mean=' $O/m_$v.txt | tr '\n' ' ')"
done

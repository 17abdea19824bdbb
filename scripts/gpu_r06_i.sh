#!/bin/bash
# round 6 (i): feature_edges -- are the stores slow because the 29-column strips write partial cache lines?
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
for v in base fed16 fed20; do
  lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
  GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel feature_edges_c8 --size 256 --iters 20 > $O/m_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'mean=' $O/m_$v.txt | tr '\n' ' ')"
done

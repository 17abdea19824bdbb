#!/bin/bash
# round 6 (p): fused LNB consumer knock-outs (timing only): 4 gate LDS reads, 8 exp/rcp, 12 both, 1 consumer
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
for v in base fd4 fd8 fd12 fd1; do
  lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
  GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel lnb --size 256 --iters 20 --c8 1 > $O/m_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'mean=' $O/m_$v.txt | tr '\n' ' ')"
done

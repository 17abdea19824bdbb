#!/bin/bash
# round 6 (r): fused LNB phase stamps after the duo layout
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
GRR_LIB=exp/libgrr_stamp.so timeout -k 10 120 python scripts/micro.py --kernel lnb --size 256 --iters 5 --c8 1 --stamps > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt | tail -12

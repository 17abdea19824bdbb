#!/bin/bash
# round 6 (c): fused LNB prologue diagnosis -- phase stamps with the start-phase stagger, and with a quarter of the
# prologue loads (timing only)
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
for cfg in "stamppro 0,3" "stamppro 16,3" "stamppro 32,4" "stampq 0,3"; do
  set -- $cfg
  GRR_LIB=exp/libgrr_$1.so timeout -k 10 120 python scripts/micro.py --kernel lnb --size 256 --iters 5 --stamps --stagger $2 > $O/stamps_$1_$2.txt 2>&1 || exit 1
  echo "$1 $2"; grep "stamps\|lnb_fused" $O/stamps_$1_$2.txt
done

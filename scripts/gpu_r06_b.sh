#!/bin/bash
# round 6 (b): fused LNB -- all prologue loads up front (GRR_FUSED_PRO_ALL) vs base; phase stamps of both
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
GRR_LIB=exp/libgrr_proall.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lnb or nonlinear" --timeout 120 --timeout-method thread > $O/parity_proall.log 2>&1 || { tail -30 $O/parity_proall.log; exit 1; }
tail -1 $O/parity_proall.log
for rep in 1 2; do
for v in base proall; do
  lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
  for sz in 256 128; do
    GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel lnb --size $sz --iters 20 > $O/micro_${v}_${sz}_$rep.txt 2>&1 || exit 1
    echo "$v $sz $(grep -h lnb_fused $O/micro_${v}_${sz}_$rep.txt | tail -1)"
  done
done
done
for v in stamp stamppro; do
  GRR_LIB=exp/libgrr_$v.so timeout -k 10 120 python scripts/micro.py --kernel lnb --size 256 --iters 5 --stamps > $O/stamps_$v.txt 2>&1 || exit 1
  echo "$v"; grep stamps $O/stamps_$v.txt
done

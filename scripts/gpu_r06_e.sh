#!/bin/bash
# round 6 (e): consumer gate two pairs ahead (GRR_GATE_AHEAD=2) vs one, per layout; parity of the variant
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
GRR_LIB=exp/libgrr_g2.so timeout -k 10 200 python -u -m pytest tests/test_gpu_lnb_c8.py tests/test_gpu_parity.py -x -q -k "lnb or nonlinear or c8" --timeout 120 --timeout-method thread > $O/parity_g2.log 2>&1 || { tail -30 $O/parity_g2.log; exit 1; }
tail -1 $O/parity_g2.log
for rep in 1 2; do
for v in base g2; do
  lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
  for c8 in 0 1; do
    GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel lnb --size 256 --iters 20 --c8 $c8 > $O/micro_${v}_${c8}_$rep.txt 2>&1 || exit 1
    echo "$v c8=$c8 $(grep -h lnb_fused $O/micro_${v}_${c8}_$rep.txt | tail -1)"
  done
done
done

#!/bin/bash
# round 6 (u): the gate + depthwise reverse's one-strip ring instance at W = 512 (V = 8, two DMAs per ring row)
# -- parity of the candidate (all gate / ring tests), per launch A/B at the C4 shapes
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
GRR_LIB=exp/libgrr_v8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dwconv.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for rep in 1 2; do
for hid in 96 192; do
  for v in base v8; do
    lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
    GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel gate_dw3_bwd --size 512 --batch 32 --graphs 1 --fts $hid --iters 10 > $O/m_${v}_$hid.txt 2>&1 || exit 1
    echo "hid $hid $v: $(grep -h 'mean=' $O/m_${v}_$hid.txt | tr '\n' ' ')"
  done
done
done

#!/bin/bash
# round 6 (q): LNB-touching GPU tests on the in-tree library + per-launch timing
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lnb_c8.py tests/test_gpu_grad.py tests/test_gpu_compile.py tests/test_gpu_feature_edges.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for sz in 256 128; do
  timeout -k 10 120 python scripts/micro.py --kernel lnb --size $sz --iters 20 --c8 1 > $O/m_$sz.txt 2>&1 || exit 1
  echo "$sz: $(grep -h 'mean=' $O/m_$sz.txt | tr '\n' ' ')"
done
for sz in 256 128; do
  timeout -k 10 120 python scripts/micro.py --kernel feature_edges_c8 --size $sz --iters 20 > $O/fe_$sz.txt 2>&1 || exit 1
  echo "$sz: $(grep -h 'mean=' $O/fe_$sz.txt | tr '\n' ' ')"
done

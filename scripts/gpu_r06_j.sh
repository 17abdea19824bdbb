#!/bin/bash
# round 6 (j): feature_edges on 32-aligned strips with halo columns -- parity, per launch, bench
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_feature_edges.py tests/test_gpu_compile.py tests/test_gpu_lnb_c8.py -x -q --timeout 120 --timeout-method thread > $O/fe.log 2>&1 || { tail -40 $O/fe.log; exit 1; }
tail -1 $O/fe.log
for sz in 256 128; do
  for kern in conv_edges feature_edges_c8 feature_edges; do
    timeout -k 10 120 python scripts/micro.py --kernel $kern --size $sz --iters 20 > $O/m_${kern}_$sz.txt 2>&1 || exit 1
    echo "$sz $kern: $(grep -h 'mean=' $O/m_${kern}_$sz.txt | tr '\n' ' ')"
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "
import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"

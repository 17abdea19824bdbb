#!/bin/bash
# round 6 (f): fused feature conv + edge weights -- parity, then the bench
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_feature_edges.py tests/test_gpu_lnb_c8.py -x -q --timeout 120 --timeout-method thread > $O/fe.log 2>&1 || { tail -40 $O/fe.log; exit 1; }
tail -1 $O/fe.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "
import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['kernel_ms_per_step'],d['psnr'] if 'psnr' in d else '')"

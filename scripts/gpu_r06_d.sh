#!/bin/bash
# round 6 (d): channel-blocked LNB chains -- parity (new tests + LNB / model parity), micro per layout, bench
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lnb_c8.py tests/test_gpu_parity.py tests/test_gpu_psnr.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sz in 256 128; do
  for l in 0 1 2 3; do
    timeout -k 10 120 python scripts/micro.py --kernel lnb --size $sz --iters 20 --c8 $l > $O/micro_${sz}_$l.txt 2>&1 || exit 1
    echo "$sz c8=$l $(grep -h lnb_fused $O/micro_${sz}_$l.txt | tail -1)"
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "
import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"

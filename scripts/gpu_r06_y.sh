#!/bin/bash
# round 6 (y): step2 / first pair half-level weight reads as single ds_read_b64 (GRR_S2_B64)
set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
GRR_LIB=exp/libgrr_s2b.so timeout -k 10 400 python -u -m pytest tests/test_gpu_step2.py tests/test_gpu_first_pair.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for rep in 1 2; do
  for v in base s2b; do
    lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
    GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel step2 --size 256 --iters 20 > $O/m_${v}.txt 2>&1 || exit 1
    echo "$v: $(grep -h 'mean=' $O/m_${v}.txt | tr '\n' ' ')"
  done
done
for v in base s2b; do
  lib=imagerestoration-development-unrolling_amd/libgrr.so; [ $v = base ] || lib=exp/libgrr_$v.so
  GRR_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python -c "
import json;d=json.load(open('$O/bench_$v.json'));k=d['kernel_ms_per_step'];print('$v', d['value'],d['ms_per_step'],'step2',k['system_step2'],'first',k['system_first_pair'])"
done

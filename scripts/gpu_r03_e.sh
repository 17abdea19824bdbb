#!/bin/bash
# head16 gate/GEMM1 interleave: parity tests on the default build (interleaved), step2 channel groups,
# micro lnb + bench A/B (exp/libgrr_hi0 = partner-wave schedule, hi1 = interleaved), then PMC traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r03e; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step2.py tests/test_gpu_configs.py \
  tests/test_gpu_streams.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_libs.sh lnb exp/libgrr_hi0.so exp/libgrr_hi1.so || exit $?
for r in 1 2; do
  for v in hi0 hi1; do
    GRR_LIB=exp/libgrr_$v.so timeout -k 10 300 python -u bench.py --steps 20 --no-secondary > $out/b_${v}_$r.json 2> $out/b_${v}_$r.err || exit $?
    python -c "
import json; d=json.load(open('$out/b_${v}_$r.json')); k=d['kernel_ms_per_step']
print('$v run $r', d['value'], d['ms_per_step'], 'head', k['lnb_head'], 'mix', k['lnb_mix'], 'step2', k['system_step2'])"
  done
done
bash scripts/pmc_bench.sh 64 || exit $?

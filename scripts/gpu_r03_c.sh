#!/bin/bash
# step2 load distance A/B (exp/libgrr_a1.so vs a2), the step2 tests on the default build, and the
# HBM traffic of the default step2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r03c; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_step2.py -x -q -rf --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_libs.sh step2 exp/libgrr_a1.so exp/libgrr_a2.so || exit $?
for r in 1 2; do
  for v in a1 a2; do
    GRR_LIB=exp/libgrr_$v.so timeout -k 10 300 python -u bench.py --steps 20 > $out/b_${v}_$r.json 2> $out/b_${v}_$r.err || exit $?
    python -c "
import json; d=json.load(open('$out/b_${v}_$r.json')); k=d['kernel_ms_per_step']
print('$v run $r', d['value'], d['ms_per_step'], 'step2', k['system_step2'], 'frac', d['roofline']['frac'])"
  done
done
bash scripts/pmc_step2.sh > $out/pmc.log 2>&1 || { tail -5 $out/pmc.log; exit 1; }
tail -3 $out/pmc.log

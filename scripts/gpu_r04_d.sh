#!/bin/bash
# Fused replicated-block LNB (lnb_rep_kernel): parity tests, micro timing, same-box bench A/B against
# head16 + mix (GRR_LNB_REP=0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04d; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_psnr.py tests/test_gpu_streams.py -q -x -rf \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1; rc=$?; tail -4 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 0; do for sz in 256 128; do
  echo "REP=$rep $sz $(GRR_LNB_REP=$rep timeout -k 10 120 python -u scripts/micro.py --kernel lnb_rep --size $sz --split --iters 20 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> $out/micro.txt || exit 1
done; done
cat $out/micro.txt
for r in 1 2; do for rep in 1 0; do
  GRR_LNB_REP=$rep timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $out/bench_rep${rep}_$r.json 2> $out/bench_rep${rep}_$r.err || { tail -5 $out/bench_rep${rep}_$r.err; exit 1; }
  python -c "import json;d=json.loads(open('$out/bench_rep${rep}_$r.json').read().strip().splitlines()[-1]);print('REP=$rep', d['value'], d['ms_per_step'], d.get('kernel_ms_per_step'))"
done; done

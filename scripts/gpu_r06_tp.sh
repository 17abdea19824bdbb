#!/bin/bash
# round 6: term policy (GLR on 4-column lanes at W > 256, the ring for prox at one-column lanes): term / grad tests,
# the C4-shape sweep under both policies, C4 training alternating policy 0 / 1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06tp; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_term_ring.py tests/test_gpu_term_acc.py tests/test_gpu_term_rows.py \
  tests/test_gpu_grad.py tests/test_gpu_deterministic.py tests/test_gpu_training.py -x -q -rf --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || exit $rc
for p in 0 1; do
  GRR_TERM_POLICY=$p timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 > $out/sweep_p$p.txt 2>&1 || { tail $out/sweep_p$p.txt; exit 1; }
  tail -1 $out/sweep_p$p.txt
done
for p in 0 1 0 1; do
  GRR_TERM_POLICY=$p timeout -k 10 300 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 \
    --no-cpu-baseline > $out/train_c4_p$p.json 2> $out/train_c4_p$p.err || { tail $out/train_c4_p$p.err; exit 1; }
  python -c "
import json;d=json.load(open('$out/train_c4_p$p.json'));r=d['roofline'];print('policy $p', d['ms_per_step'], 'term frac', r['frac'], 'term ms/step', d['kernel_ms_per_step']['bwd_term_fused'])"
done

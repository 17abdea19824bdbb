#!/bin/bash
# round 6: term reverse segment rule (new default 2048 waves / 128 rows vs the round-5 8192 / whole planes):
# term tests, 256^2 sweep, C4 and v1.0 training alternating old / new
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06seg; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_term_ring.py tests/test_gpu_term_acc.py tests/test_gpu_term_rows.py \
  tests/test_gpu_grad.py tests/test_gpu_deterministic.py tests/test_gpu_training.py -x -q -rf --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?
tail -2 $out/tests.log
[ $rc -eq 0 ] || exit $rc
OLD="GRR_TERM_MIN_WAVES=8192 GRR_TERM_MAX_SEG=100000"
for v in old new; do
  e=""; [ $v = old ] && e=$OLD
  env $e timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 --size 256 --batch 8 > $out/sweep256_$v.txt 2>&1 || { tail $out/sweep256_$v.txt; exit 1; }
  echo "256 sweep $v: $(tail -1 $out/sweep256_$v.txt)"
done
for v in old new old new; do
  e=""; [ $v = old ] && e=$OLD
  env $e timeout -k 10 300 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 \
    --no-cpu-baseline > $out/train_c4_$v.json 2> $out/train_c4_$v.err || { tail $out/train_c4_$v.err; exit 1; }
  env $e timeout -k 10 300 python -u bench_train.py --model abstract --no-cpu-baseline > $out/train_v1_$v.json 2> $out/train_v1_$v.err || { tail $out/train_v1_$v.err; exit 1; }
  python -c "
import json
for m in ('c4','v1'):
    d=json.load(open('$out/train_'+m+'_$v.json'));r=d['roofline'];print('$v', m, d['ms_per_step'], 'term frac', r['frac'], 'term ms/step', d['kernel_ms_per_step']['bwd_term_fused'])"
done

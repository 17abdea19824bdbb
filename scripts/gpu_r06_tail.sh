#!/bin/bash
# round 6: term reverse tail launch — ring/acc/rows/grad tests, then C4 training with the tail off / on / off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06tail; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_term_ring.py tests/test_gpu_term_acc.py tests/test_gpu_term_rows.py \
  tests/test_gpu_grad.py tests/test_gpu_deterministic.py -x -q -rf --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $out/tests.log 2>&1
rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || exit $rc
for t in 0 1 0 1; do
  GRR_TERM_TAIL=$t timeout -k 10 300 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 \
    --no-cpu-baseline > $out/train_c4_tail$t.json 2> $out/train_c4_tail$t.err || { tail $out/train_c4_tail$t.err; exit 1; }
  echo "tail=$t $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $out/train_c4_tail$t.json | tr '\n' ' ')"
  python -c "
import json;d=json.load(open('$out/train_c4_tail$t.json'));r=d['roofline'];print('term frac', r['frac'], 'mean_launch_ms', r['mean_launch_ms'], 'term ms/step', d['kernel_ms_per_step']['bwd_term_fused'])"
done

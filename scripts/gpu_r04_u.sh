#!/bin/bash
# Round 4: the x-gradient pass inside the term reverse (grr_bwd_term_fused_acc, solver_grad.TERM_ACC):
# parity against the two-pass path and the gradient / determinism suites, then the training lines with
# --term-acc 1 / 0 alternated (same build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04u; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_term_acc.py tests/test_gpu_term_rows.py tests/test_gpu_deterministic.py tests/test_gpu_training.py \
  tests/test_gpu_streams.py tests/test_gpu_grad.py > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for acc in 1 0; do
  for mb in "msgf 16 256" "abstract 8 256"; do
    set -- $mb; m=$1; tag=${m}_$3_acc${acc}_$r
    timeout -k 10 300 python -u bench_train.py --model $m --batch $2 --size $3 --steps 6 --warmup 2 --no-cpu-baseline \
      --term-acc $acc > $out/train_$tag.json 2> $out/train_$tag.err || { tail -5 $out/train_$tag.err; exit 1; }
    python -c "import json;d=json.loads(open('$out/train_$tag.json').read().strip().splitlines()[-1]);k=d['kernel_ms_per_step'];print('$tag', d['value'], d['ms_per_step'], 'term', k.get('bwd_term_fused'), 'stencil', k.get('bwd_stencil'))"
  done
done; done
timeout -k 10 500 python -u bench_train.py --model abstract --batch 32 --size 512 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/c4_acc1.json 2> $out/c4_acc1.err || { tail -5 $out/c4_acc1.err; exit 1; }
echo "c4 acc1 $(grep -o '"ms_per_step": [0-9.]*' $out/c4_acc1.json)"

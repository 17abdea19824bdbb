#!/bin/bash
# Round 4: the LNB skip term inside the norm reverse (solver_grad.LN_SKIP_FUSED): tests, then
# the training lines with --ln-skip 1 / 0 alternated (same build), C4 both ways
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04aa; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_term_acc.py tests/test_gpu_deterministic.py tests/test_gpu_training.py tests/test_gpu_streams.py \
  tests/test_gpu_grad.py tests/test_gpu_ddp.py > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for fo in 1 0; do
  for mb in "msgf 16 256" "abstract 8 256"; do
    set -- $mb; m=$1; tag=${m}_$3_lnskip${fo}_$r
    timeout -k 10 300 python -u bench_train.py --model $m --batch $2 --size $3 --steps 6 --warmup 2 --no-cpu-baseline \
      --ln-skip $fo > $out/train_$tag.json 2> $out/train_$tag.err || { tail -5 $out/train_$tag.err; exit 1; }
    python -c "import json;d=json.loads(open('$out/train_$tag.json').read().strip().splitlines()[-1]);k=d['kernel_ms_per_step'];print('$tag', d['value'], d['ms_per_step'], 'normbwd', k.get('lnb_norm_bwd'), 'dot', k.get('bwd_graph_dot'), 'lincomb', k.get('bwd_lincomb'))"
  done
done; done
for fo in 1 0; do
  timeout -k 10 500 python -u bench_train.py --model abstract --batch 32 --size 512 --steps 3 --warmup 1 --no-cpu-baseline \
    --ln-skip $fo > $out/c4_lnskip$fo.json 2> $out/c4_lnskip$fo.err || { tail -5 $out/c4_lnskip$fo.err; exit 1; }
  echo "c4 lnskip$fo $(grep -o '"ms_per_step": [0-9.]*' $out/c4_lnskip$fo.json)"
done

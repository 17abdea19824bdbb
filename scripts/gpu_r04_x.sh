#!/bin/bash
# Round 4: grr_pool2 on 2 x 4 float4 blocks (in-tree build) vs the per-output kernel (exp/libgrr_pool0.so):
# tests, the pool kernel per call (training lines' kernel_ms_per_step), the training lines alternated
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04x; mkdir -p $out
export TMPDIR=/tmp
L=imagerestoration-development-unrolling_amd/libgrr.so
timeout -k 10 600 python -u -m pytest -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_term_acc.py tests/test_gpu_step2.py tests/test_gpu_psnr.py tests/test_gpu_parity.py \
  tests/test_gpu_deterministic.py tests/test_gpu_streams.py tests/test_gpu_grad.py > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for lib in $L exp/libgrr_pool0.so; do
  n=$(basename $lib .so)
  for mb in "msgf 16 256" "abstract 8 256"; do
    set -- $mb; m=$1; tag=${m}_$3_${n}_$r
    GRR_LIB=$lib timeout -k 10 300 python -u bench_train.py --model $m --batch $2 --size $3 --steps 6 --warmup 2 \
      --no-cpu-baseline > $out/train_$tag.json 2> $out/train_$tag.err || { tail -5 $out/train_$tag.err; exit 1; }
    python -c "import json;d=json.loads(open('$out/train_$tag.json').read().strip().splitlines()[-1]);k=d['kernel_ms_per_step'];print('$tag', d['value'], d['ms_per_step'], 'pool2', k.get('pool2'))"
  done
done; done
for lib in $L exp/libgrr_pool0.so; do
  n=$(basename $lib .so)
  GRR_LIB=$lib timeout -k 10 500 python -u bench_train.py --model abstract --batch 32 --size 512 --steps 3 --warmup 1 \
    --no-cpu-baseline > $out/c4_$n.json 2> $out/c4_$n.err || { tail -5 $out/c4_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$out/c4_$n.json').read().strip().splitlines()[-1]);k=d['kernel_ms_per_step'];print('c4 $n', d['value'], d['ms_per_step'], 'pool2', k.get('pool2'))"
done

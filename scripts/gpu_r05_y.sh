#!/bin/bash
# x3k GEMM (buffer-loaded x, opaque ring DMA, branch-free chunk body): parity, per-shape A/B against
# exp/libgrr_x3base.so (the same tree with the previous feature_ops), training A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05y; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_deterministic.py \
  tests/test_gpu_wgrad.py tests/test_gpu_training.py tests/test_gpu_grad.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for mk in "48 192" "48 96" "96 48" "96 384" "96 192" "192 48" "3 96" "129 33"; do
  set -- $mk
  sz=512; [ "$1 $2" = "96 384" ] && sz=256; [ "$1 $2" = "96 192" ] && sz=256
  for lib in base new; do
    L=""; [ $lib = base ] && L=exp/libgrr_x3base.so
    GRR_LIB=${L:-imagerestoration-development-unrolling_amd/libgrr.so} timeout -k 10 120 python -u scripts/micro.py --kernel conv_mk --cin $1 --cout $2 --batch 32 --size $sz --graphs 8 --fts 3 --iters 10 \
      > $out/t_$1_$2_$lib.txt 2>&1 || { tail $out/t_$1_$2_$lib.txt; exit 1; }
    echo "cin $1 cout $2 ${sz}^2 $lib: $(grep 'conv1x1 ' $out/t_$1_$2_$lib.txt | tr -s ' ' | cut -d' ' -f4-6)"
  done
done
for rep in 1 2; do
for lib in base new; do
L=imagerestoration-development-unrolling_amd/libgrr.so; [ $lib = base ] && L=exp/libgrr_x3base.so
GRR_LIB=$L timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/abs_$lib.$rep.json 2> $out/abs_$lib.$rep.err || { tail $out/abs_$lib.$rep.err; exit 1; }
echo "abs $lib rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"conv1x1": [0-9.]*' $out/abs_$lib.$rep.json | tr '\n' ' ')"
done
done
for lib in base new; do
L=imagerestoration-development-unrolling_amd/libgrr.so; [ $lib = base ] && L=exp/libgrr_x3base.so
GRR_LIB=$L timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/c4_$lib.json 2> $out/c4_$lib.err || { tail $out/c4_$lib.err; exit 1; }
echo "c4 $lib $(grep -o '"ms_per_step": [0-9.]*\|"conv1x1": [0-9.]*' $out/c4_$lib.json | tr '\n' ' ')"
done

#!/bin/bash
# LNB gate + depthwise reverse at V = 2 past one strip (W > 256, aligned ring chunks): parity of the
# candidate exp/libgrr_g2.so, reverse micro A/B and C4 training A/B against the in-tree library (V = 4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05g2; mkdir -p $out
export TMPDIR=/tmp
GRR_LIB=exp/libgrr_g2.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_dwconv.py \
  tests/test_gpu_deterministic.py tests/test_gpu_training.py tests/test_gpu_grad.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
for lib in base new; do
  L=exp/libgrr_g2.so; [ $lib = base ] && L=imagerestoration-development-unrolling_amd/libgrr.so
  GRR_LIB=$L timeout -k 10 120 python -u scripts/micro.py --kernel gate_dw3_bwd --fts 96 --graphs 1 --batch 32 --size 512 --iters 10 \
    > $out/g_$lib.$rep.txt 2>&1 || { tail $out/g_$lib.$rep.txt; exit 1; }
  echo "rep $rep hid 96 512^2 $lib: $(grep 'lnb_gate_dw3_bwd' $out/g_$lib.$rep.txt | tr -s ' ' | cut -d' ' -f2-6)"
done
done
for lib in base new; do
L=exp/libgrr_g2.so; [ $lib = base ] && L=imagerestoration-development-unrolling_amd/libgrr.so
GRR_LIB=$L timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/c4_$lib.json 2> $out/c4_$lib.err || { tail $out/c4_$lib.err; exit 1; }
echo "c4 $lib $(grep -o '"ms_per_step": [0-9.]*' $out/c4_$lib.json | tr '\n' ' ')"
done

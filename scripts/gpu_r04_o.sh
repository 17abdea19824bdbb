#!/bin/bash
# Round 4: LNB depthwise row kernels at W > 256 on 2-column lanes (GRR_DW3_WIDE_V=2, exp/libgrr_dw2.so; 1-column lanes fail the fused gate reverse, whose reach is two columns)
# vs 4-column lanes: parity tests with each variant, the gate + depthwise reverse at the C4 level-1 shape,
# the C4 training line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04o; mkdir -p $out
export TMPDIR=/tmp
for v in dw2; do
  GRR_LIB=exp/libgrr_$v.so timeout -k 10 300 python -u -m pytest -q -rf --timeout 200 --timeout-method thread \
    -p no:cacheprovider tests/test_gpu_dwconv.py tests/test_gpu_deterministic.py > $out/tests_$v.log 2>&1
  rc=$?; tail -2 $out/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
L=imagerestoration-development-unrolling_amd/libgrr.so
: > $out/micro.txt
for lib in $L exp/libgrr_dw2.so; do
  echo "$(basename $lib) gate_dw3_bwd B32 hid96 S512 $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel gate_dw3_bwd \
    --batch 32 --fts 96 --size 512 --iters 10 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> $out/micro.txt || exit 1
done
cat $out/micro.txt
export MIOPEN_FIND_MODE=FAST   # the same convolution solutions for every variant, no per-box search
for lib in $L exp/libgrr_dw2.so; do
  n=$(basename $lib .so)
  GRR_LIB=$lib timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 \
    --no-cpu-baseline > $out/c4_$n.json 2> $out/c4_$n.err || { tail $out/c4_$n.err; exit 1; }
  echo "$n C4 $(grep -o '"ms_per_step": [0-9.]*' $out/c4_$n.json)"
done

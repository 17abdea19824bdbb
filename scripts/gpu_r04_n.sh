#!/bin/bash
# Round 4: wide term-reverse strips on 2-column lanes (GRR_TERM_WIDE_V=2, exp/libgrr_wv2.so) vs 4-column
# lanes (default): parity tests with the variant, per-shape timings at W = 512, the C4 training line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04n; mkdir -p $out
export TMPDIR=/tmp
GRR_LIB=exp/libgrr_wv2.so timeout -k 10 300 python -u -m pytest -q -rf --timeout 200 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_term_rows.py tests/test_gpu_deterministic.py > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
L=imagerestoration-development-unrolling_amd/libgrr.so
: > $out/micro.txt
for lib in $L exp/libgrr_wv2.so; do
  for spec in "32 8 6 512 0" "32 8 6 512 1" "32 8 6 512 2" "8 16 6 512 0"; do
    set -- $spec
    echo "$(basename $lib) B$1 G$2 F$3 S$4 mode$5 $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel term \
      --batch $1 --graphs $2 --fts $3 --size $4 --mode $5 --iters 10 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> $out/micro.txt || exit 1
  done
done
sed 's/term: bwd_term_fused   //' $out/micro.txt
for lib in exp/libgrr_wv2.so $L; do
  n=$(basename $lib .so)
  GRR_LIB=$lib timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 \
    --no-cpu-baseline > $out/c4_$n.json 2> $out/c4_$n.err || { tail $out/c4_$n.err; exit 1; }
  echo "$n C4 $(grep -o '"ms_per_step": [0-9.]*' $out/c4_$n.json)"
done

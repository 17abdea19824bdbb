#!/bin/bash
# Round 4: the gw-row LDS-DMA ring restricted to the instances where gpu_r04_q.sh measured it faster (MODE 0/1,
# strips or W <= 128): parity + determinism tests, the term reverse at W = 128 / 256 / 512, the training lines
# (msgf, abstract, C4) against exp/libgrr_gwdma0.so, twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04r; mkdir -p $out
export TMPDIR=/tmp
L=imagerestoration-development-unrolling_amd/libgrr.so
timeout -k 10 400 python -u -m pytest -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_term_rows.py tests/test_gpu_deterministic.py tests/test_gpu_training.py > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
: > $out/micro.txt
for spec in "16 32 3 128" "32 8 6 512" "32 16 6 256"; do
  set -- $spec
  for mode in 0 1; do
    for lib in $L exp/libgrr_gwdma0.so $L exp/libgrr_gwdma0.so; do
      echo "$(basename $lib .so) B$1 G$2 F$3 S$4 mode$mode $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel term \
        --batch $1 --graphs $2 --fts $3 --size $4 --mode $mode --iters 10 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> $out/micro.txt || exit 1
    done
  done
done
cat $out/micro.txt
for r in 1 2; do for lib in $L exp/libgrr_gwdma0.so; do
  n=$(basename $lib .so)
  for mb in "msgf 16 256" "abstract 8 256" "abstract 32 512"; do
    set -- $mb; m=$1; tag=${m}_$3
    st=6; [ $3 = 512 ] && st=3
    GRR_LIB=$lib timeout -k 10 400 python -u bench_train.py --model $m --batch $2 --size $3 --steps $st --warmup 1 --no-cpu-baseline \
      > $out/train_${tag}_${n}_$r.json 2> $out/train_${tag}_$n.err || { tail -5 $out/train_${tag}_$n.err; exit 1; }
    echo "$n $tag $(grep -o '"value": [0-9.]*' $out/train_${tag}_${n}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $out/train_${tag}_${n}_$r.json)"
  done
done; done

#!/bin/bash
# Round 4: term reverse row kernel reading gw rows through a one-row-ahead LDS-DMA ring (GRR_TERM_GW_DMA=1,
# the in-tree build) vs the global read after the barrier (exp/libgrr_gwdma0.so): parity + determinism tests
# with the new build (the ring in the GGLR / signed-graph instances, MODE 0 / 1), the term reverse at the training shapes, the msgf / abstract training lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04q; mkdir -p $out
export TMPDIR=/tmp
L=imagerestoration-development-unrolling_amd/libgrr.so
timeout -k 10 400 python -u -m pytest -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_term_rows.py tests/test_gpu_deterministic.py > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
: > $out/micro.txt
for spec in "16 32 3 256" "16 32 3 128" "32 8 6 512" "32 16 6 256" "32 16 12 128" "32 32 12 64"; do
  set -- $spec
  for mode in 0 1 2; do
    for lib in $L exp/libgrr_gwdma0.so $L exp/libgrr_gwdma0.so; do
      echo "$(basename $lib .so) B$1 G$2 F$3 S$4 mode$mode $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel term \
        --batch $1 --graphs $2 --fts $3 --size $4 --mode $mode --iters 10 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> $out/micro.txt || exit 1
    done
  done
done
cat $out/micro.txt
for lib in $L exp/libgrr_gwdma0.so; do
  n=$(basename $lib .so)
  for mb in "msgf 16" "abstract 8"; do
    set -- $mb; m=$1
    GRR_LIB=$lib timeout -k 10 300 python -u bench_train.py --model $m --batch $2 --steps 6 --warmup 2 --no-cpu-baseline \
      > $out/train_${m}_$n.json 2> $out/train_${m}_$n.err || { tail -5 $out/train_${m}_$n.err; exit 1; }
    echo "$n $m $(grep -o '"value": [0-9.]*' $out/train_${m}_$n.json) $(grep -o '"ms_per_step": [0-9.]*' $out/train_${m}_$n.json)"
  done
done

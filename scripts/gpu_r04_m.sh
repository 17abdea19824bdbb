#!/bin/bash
# Round 4: (1) GPU tests touched by the reverse changes (fixed-order finish pass, early gw reads, kept
# LNB gate); (2) same-box A/B of the early gw read in the term reverse (GRR_TERM_EARLY_GW 2 / 1 / 0)
# per shape and on the training lines; (3) kept-gate A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04m; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_deterministic.py tests/test_gpu_term_rows.py tests/test_gpu_streams.py tests/test_gpu_grad.py \
  tests/test_gpu_padj2.py tests/test_gpu_ddp.py tests/test_gpu_window_grad.py > $out/tests.log 2>&1
rc=$?; tail -4 $out/tests.log; [ $rc -eq 0 ] || exit $rc
L=imagerestoration-development-unrolling_amd/libgrr.so
: > $out/micro.txt
for lib in $L exp/libgrr_ke1.so exp/libgrr_ke0.so; do
  for spec in "16 32 3 256 0" "16 32 3 256 2" "32 8 6 512 0" "32 8 6 512 2" "32 8 6 256 0" "32 16 6 256 0" "32 16 12 128 0"; do
    set -- $spec
    echo "$(basename $lib) B$1 G$2 F$3 S$4 mode$5 $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel term \
      --batch $1 --graphs $2 --fts $3 --size $4 --mode $5 --iters 10 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> $out/micro.txt || exit 1
  done
done
sed 's/term: bwd_term_fused   //' $out/micro.txt
for lib in $L exp/libgrr_ke0.so; do
  n=$(basename $lib .so)
  GRR_LIB=$lib timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline \
    > $out/msgf_$n.json 2> $out/msgf_$n.err || { tail $out/msgf_$n.err; exit 1; }
  GRR_LIB=$lib timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
    > $out/abstract_$n.json 2> $out/abstract_$n.err || { tail $out/abstract_$n.err; exit 1; }
  echo "$n msgf $(grep -o '"ms_per_step": [0-9.]*' $out/msgf_$n.json) abstract $(grep -o '"ms_per_step": [0-9.]*' $out/abstract_$n.json)"
done
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline --keep-gate 0 \
  > $out/msgf_nokeep.json 2> $out/msgf_nokeep.err || { tail $out/msgf_nokeep.err; exit 1; }
echo "no keep-gate msgf $(grep -o '"ms_per_step": [0-9.]*' $out/msgf_nokeep.json)"

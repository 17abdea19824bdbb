#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: one rocprofv3 pass each) of the training step's dominant reverse
# kernel (the operator-term reverse, kind bwd_term_fused = term_row_kernel) at bench_train.py's default
# workloads, written where bench_train.py's roofline.traffic looks for it:
# gpurun_out/pmct/traffic_bwd_term_fused_<model>.json (workload-tagged; copied to profiles/r04/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
OUT=gpurun_out/pmct; mkdir -p $OUT
for spec in "msgf:16" "abstract:8"; do
  model=${spec%%:*}; B=${spec#*:}
  CMD="python bench_train.py --model $model --batch $B --size 256 --steps 2 --warmup 1 --no-cpu-baseline"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "term_row_kernel" --output-format csv \
      -d $OUT/$model/$ctr -o run -- $CMD > $OUT/${model}_$ctr.log 2>&1 || { echo "$model $ctr pass failed"; tail -5 $OUT/${model}_$ctr.log; exit 1; }
  done
  python scripts/collect_traffic.py $OUT/$model/FETCH_SIZE $OUT/$model/WRITE_SIZE --kernel "term_row_kernel" \
    --out $OUT/traffic_bwd_term_fused_$model.json --batch $B --size 256 || exit 1
done

#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: one rocprofv3 pass each) of the training reverse's term kernel at the
# C4 workload (v1.0, 32 x 512^2): gpurun_out/pmct/traffic_bwd_term_fused_abstract_b32_s512.json, which
# bench_train.py's roofline.traffic reads for that exact shape (copied to profiles/r04/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
OUT=gpurun_out/pmct; mkdir -p $OUT
CMD="python bench_train.py --model abstract --batch 32 --size 512 --steps 1 --warmup 1 --no-cpu-baseline"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-include-regex "term_row_kernel" --output-format csv \
    -d $OUT/c4/$ctr -o run -- $CMD > $OUT/c4_$ctr.log 2>&1 || { echo "c4 $ctr pass failed"; tail -5 $OUT/c4_$ctr.log; exit 1; }
done
python scripts/collect_traffic.py $OUT/c4/FETCH_SIZE $OUT/c4/WRITE_SIZE --kernel "term_row_kernel" \
  --out $OUT/traffic_bwd_term_fused_abstract_b32_s512.json --batch 32 --size 512

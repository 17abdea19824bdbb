#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: one rocprofv3 pass each) of the bench's own launches at the
# bench batch, for the kernels bench.py reports a roofline for, plus the kernel-trace summary of
# the same command.  Writes gpurun_out/pmcb/traffic_*.json (copied to profiles/ by the session script)
# (workload-tagged: bench.py ignores a summary taken at another batch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
OUT=gpurun_out/pmcb; mkdir -p $OUT
B=${1:-64}
CMD="python bench.py --steps 2 --warmup 1 --batch $B --no-cpu-baseline --no-secondary"
RX="graph_step2|lnb_head16|lnb_mix|lnb_rep_kernel|lnb_fused16|graph_row_kernel|feat_edge_kernel"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" --output-format csv -d $OUT/$ctr -o run -- \
    $CMD > $OUT/$ctr.log 2>&1 || { echo "$ctr pass failed"; tail -5 $OUT/$ctr.log; exit 1; }
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $CMD \
  > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -5 $OUT/trace.log; exit 1; }
for spec in "graph_step2_kernel<false, false, false>:profiles/traffic_system_step2.json" \
            "graph_step2_kernel<false, false, true>:profiles/r06/traffic_system_first_pair.json" \
            "lnb_fused16_kernel:profiles/r06/traffic_lnb_fused.json" "lnb_rep_kernel:profiles/r06/traffic_lnb_rep.json" \
            "feat_edge_kernel:profiles/r06/traffic_feature_edges.json"; do
  python scripts/collect_traffic.py $OUT/FETCH_SIZE $OUT/WRITE_SIZE --kernel "${spec%%:*}" --out "$OUT/$(basename ${spec#*:})" \
    --batch $B --size 256 || exit 1
done
cp $OUT/trace/run_kernel_stats.csv $OUT/bench_kernel_stats.csv
head -12 $OUT/bench_kernel_stats.csv | cut -c1-160

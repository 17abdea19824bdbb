#!/bin/bash
# lnb_rep_kernel after the epilogue / prologue changes: parity, micro, SQ counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04e; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -rf -k "replicated or nonlinear or msgf" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for sz in 256 128; do
  echo "$sz $(timeout -k 10 120 python -u scripts/micro.py --kernel lnb_rep --size $sz --split --iters 20 2>&1 | grep lnb_rep_fused)" >> $out/micro.txt || exit 1
done
cat $out/micro.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
  --kernel-include-regex "lnb_rep_kernel" --output-format csv -d $out/sq -o run -- python scripts/micro.py --kernel lnb_rep --size 256 --split --iters 5 > $out/sq.log 2>&1 || { tail -5 $out/sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES \
  --kernel-include-regex "lnb_rep_kernel" --output-format csv -d $out/sq2 -o run -- python scripts/micro.py --kernel lnb_rep --size 256 --split --iters 5 > $out/sq2.log 2>&1 || { tail -5 $out/sq2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python scripts/micro.py --kernel lnb_rep --size 256 --split --iters 5 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
python - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/r04e/sq", "gpurun_out/r04e/sq2"):
    tot = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(d, dict(tot))
PY
head -5 $out/trace/run_kernel_stats.csv | cut -c1-150

#!/bin/bash
# LNB head diagnostics (timing-only variants, wrong results): gate without g stores / without LDS window
# reads / without exp+rcp, against the default build; SQ counters of the replicated (gate-only) head
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04b; mkdir -p $out
export TMPDIR=/tmp
for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_nostore.so exp/libgrr_nolds.so exp/libgrr_noexp.so; do
  for k in lnb_rep lnb; do
    echo "$lib $k" >> $out/micro.txt
    GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel $k --size 256 --split --iters 20 2>&1 | grep lnb_head >> $out/micro.txt || exit 1
  done
done
cat $out/micro.txt
for k in lnb_rep lnb; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS \
    --kernel-include-regex "lnb_head16" --output-format csv -d $out/sq_$k -o run -- python scripts/micro.py --kernel $k --size 256 --split --iters 5 > $out/sq_$k.log 2>&1 || { tail -5 $out/sq_$k.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM \
    --kernel-include-regex "lnb_head16" --output-format csv -d $out/sq2_$k -o run -- python scripts/micro.py --kernel $k --size 256 --split --iters 5 > $out/sq2_$k.log 2>&1 || { tail -5 $out/sq2_$k.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/r04b/sq*_lnb*")):
    tot = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(d, dict(tot))
PY

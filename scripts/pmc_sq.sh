#!/bin/bash
# Issue / wait / LDS counters of one kernel (two SQ passes of <= 8 counters) over scripts/micro.py
#   bash scripts/pmc_sq.sh <micro kernel> <kernel-name regex> <out dir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
MK=$1; RX=$2; OUT=gpurun_out/$3; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM"
n=1
for P in "$P1" "$P2"; do
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d $OUT/p$n -o run -- \
    python scripts/micro.py --kernel $MK --iters 3 ${MICRO_ARGS:-} > $OUT/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $OUT/p$n.log; exit 1; }
  n=$((n+1))
done
python - "$OUT" <<'PY'
import csv, glob, collections, sys, json
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.Counter()
for f in glob.glob(f'{out}/p*/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        acc[row['Kernel_Name'][:60]][row['Counter_Name']] += float(row['Counter_Value'])
res = {k: dict(d) for k, d in acc.items()}
json.dump(res, open(f'{out}/sq_counters.json', 'w'), indent=1)
for k, d in res.items():
    print(k); print('  ', {c: f'{v:.4g}' for c, v in sorted(d.items())})
PY

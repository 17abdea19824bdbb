#!/bin/bash
# Matrix / vector co-issue counters of the LNB head kernel (scripts/micro.py --kernel lnb)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmclnb
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS \
  --kernel-include-regex "lnb_head" --output-format csv -d gpurun_out/pmclnb/sq -o run -- \
  python scripts/micro.py --kernel lnb --iters 3 > gpurun_out/pmclnb/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmclnb/trace -o run -- \
  python scripts/micro.py --kernel lnb --iters 5 > gpurun_out/pmclnb/trace.log 2>&1 || exit 1
python - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmclnb/sq/**/*counter_collection.csv', recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for row in csv.DictReader(open(f[0])):
    k = row['Kernel_Name'][:40]
    acc[k][row['Counter_Name']] += float(row['Counter_Value'])
for k, d in acc.items():
    print(k, {c: v for c, v in d.items()})
t = glob.glob('gpurun_out/pmclnb/trace/**/*kernel_stats.csv', recursive=True)
for row in csv.DictReader(open(t[0])):
    if 'lnb' in row['Name']: print(row['Name'][:50], row['Calls'], row['AverageNs'])
PY

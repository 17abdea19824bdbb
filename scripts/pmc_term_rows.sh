#!/bin/bash
# SQ issue / stall counters of the term-row reverse kernel inside one msgf training step
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmctr
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU \
  --kernel-include-regex "term_row|step2|lnb_head" --output-format csv -d gpurun_out/pmctr/sq -o run -- \
  python bench_train.py --model msgf --batch 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmctr/sq.log 2>&1 || exit 1
python - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmctr/sq/**/*counter_collection.csv', recursive=True)
print(f)
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for row in csv.DictReader(open(f[0])):
    k = row['Kernel_Name'].split('(')[0][-60:]
    acc[k][row['Counter_Name']] += float(row['Counter_Value'])
for k, d in acc.items():
    w = d.get('SQ_WAVE_CYCLES', 1)
    print(k, {c: round(v / w, 3) for c, v in d.items() if c != 'SQ_WAVE_CYCLES'}, 'wave_cycles', w)
PY

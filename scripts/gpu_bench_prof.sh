#!/bin/bash
# PMC traffic of the step2 kernel, the default bench line, and the rocprofv3 kernel summary of a bench run
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/bp
bash scripts/pmc_step2.sh || exit 1
cp gpurun_out/pmc2/traffic_system_step2.json profiles/traffic_system_step2.json
timeout -k 10 400 python bench.py > gpurun_out/bp/bench.json 2> gpurun_out/bp/bench.err || { tail -20 gpurun_out/bp/bench.err; exit 1; }
tail -c 2500 gpurun_out/bp/bench.json
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bp/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/bp/trace_bench.json 2> gpurun_out/bp/trace_bench.err || exit 1
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/bp/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:8]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), "ms avg", r["Percentage"])
PY

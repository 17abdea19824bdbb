#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/ffnprof; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 -u bench_window.py --no-cpu-baseline --steps 2 --warmup 1 > $out/b.json 2> $out/b.err || { tail $out/b.err; exit 1; }
f=$(find $out/prof -name '*kernel_stats.csv' | head -1); cp $f $out/kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/ffnprof/kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:8.3f} ms  {r['Name'][:110]}")
PY

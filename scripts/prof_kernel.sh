#!/bin/bash
# rocprofv3 kernel trace + stats of one micro-benchmarked kernel: bash scripts/prof_kernel.sh <kernel> [iters] [size]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K=${1:-lnb}; IT=${2:-10}; SZ=${3:-256}
OUT=gpurun_out/prof_$K
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python scripts/micro.py --kernel "$K" --iters "$IT" --size "$SZ" > "$OUT/trace.log" 2>&1 || exit $?
tail -n 2 "$OUT/trace.log"
python - "$OUT" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY

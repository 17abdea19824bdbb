#!/bin/bash
# Same-box A/B under a rocprofv3 kernel trace: per-kernel mean for each libgrr build.
#   bash scripts/ab_prof.sh <micro-kernel> <kernel-name-substring> exp/libgrr_a.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
K=$1; PAT=$2; shift 2
for r in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)_$r
    GRR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$n -o run -- \
      python scripts/micro.py --kernel "$K" --iters 20 > gpurun_out/ab/$n.log 2>&1 || exit $?
    python - "$n" "$PAT" gpurun_out/ab/$n/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[3])):
    if sys.argv[2] in r["Name"]:
        print(f"{sys.argv[1]:24s} {float(r['AverageNs'])/1e6:8.3f} ms  {r['Name'][:70]}")
PY
  done
done

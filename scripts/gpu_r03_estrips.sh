#!/bin/bash
# edge-weight reverse in column strips (W > 256): row-kernel parity, then the C4 step (v1.0, 32 x 512^2)
# with a kernel summary
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/estrips; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_term_rows.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -4 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
head -c 300 $out/c4.json; echo
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python -u bench_train.py --model abstract --size 512 --batch 32 --steps 2 --warmup 1 --no-cpu-baseline > $out/c4p.json 2> $out/c4p.err || { tail $out/c4p.err; exit 1; }
f=$(find $out/prof -name '*kernel_stats.csv' | head -n 1); cp "$f" $out/kernel_stats.csv
python - $out/kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print("%10.2f ms %6d %9.3f ms  %s" % (float(r["TotalDurationNs"]) / 1e6, int(r["Calls"]), float(r["AverageNs"]) / 1e6, r["Name"][:110]))
PY

#!/bin/bash
# fused LNB: non-temporal epilogue stores / skip re-read (keep the weight fragments in L2): bench + PMC A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05nt; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "lnb or x3" \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for lib in base nt; do
  L=imagerestoration-development-unrolling_amd/libgrr.so; [ $lib = base ] && L=exp/libgrr_base.so
  GRR_LIB=$L timeout -k 10 300 python -u bench.py > $out/b_$lib.$rep.json 2> $out/b_$lib.$rep.err || { tail $out/b_$lib.$rep.err; exit 1; }
  echo "bench $lib: $(grep -o '"value": [0-9.]*, "unit": "MPix/s"\|"lnb_fused": [0-9.]*' $out/b_$lib.$rep.json | head -2 | tr '\n' ' ')"
done
done
for lib in base nt; do
  L=imagerestoration-development-unrolling_amd/libgrr.so; [ $lib = base ] && L=exp/libgrr_base.so
  GRR_LIB=$L timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-include-regex lnb_fused16 --output-format csv -d $out/pmc_$lib -o run -- python scripts/micro.py --kernel lnb --iters 3 > $out/pmc_$lib.log 2>&1 || { tail -5 $out/pmc_$lib.log; exit 1; }
  python - $out/pmc_$lib <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
print(sys.argv[1], {k: round(sum(v) / len(v) / 1024 / 1024, 3) for k, v in acc.items()}, 'GiB-ish (KiB/1024^2 mean per dispatch)')
PY
done

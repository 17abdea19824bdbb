#!/bin/bash
# step2 with / without non-temporal streams: time (micro) and PMC read bytes
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/nt
for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_nont.so; do
  tag=$(basename $lib .so)
  for r in 1 2; do
    GRR_LIB=$lib timeout -k 10 120 python scripts/micro.py --kernel step2 --iters 20 2>&1 | grep step2: | sed "s/^/$tag /" || exit 1
  done
  GRR_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/nt/$tag -o run -- python scripts/micro.py --kernel step2 --iters 3 > gpurun_out/nt/$tag.log 2>&1 || exit 1
  python - gpurun_out/nt/$tag <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE" and "step2" in r["Kernel_Name"]]
print(sys.argv[1], "read GB per launch (2 x FETCH_SIZE):", round(2 * 1024 * sum(v) / len(v) / 1e9, 3))
PY
done

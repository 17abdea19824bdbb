#!/bin/bash
# Round 4: the C4 and v1.0 256^2 training lines three times in a row on one box (MIOpen find-db filled by
# the first run) with the package's MIOPEN_DEBUG_DISABLE_FIND_DB default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04t; mkdir -p $out
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 400 python -u bench_train.py --model abstract --batch 32 --size 512 --steps 3 --warmup 1 --no-cpu-baseline \
    > $out/c4_$r.json 2> $out/c4_$r.err || { tail -5 $out/c4_$r.err; exit 1; }
  echo "c4 run $r $(grep -o '"ms_per_step": [0-9.]*' $out/c4_$r.json)"
  timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 6 --warmup 2 --no-cpu-baseline \
    > $out/abs_$r.json 2> $out/abs_$r.err || { tail -5 $out/abs_$r.err; exit 1; }
  echo "abstract 256 run $r $(grep -o '"ms_per_step": [0-9.]*' $out/abs_$r.json)"
done
ls ~/.config/miopen 2>&1

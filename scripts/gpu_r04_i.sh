#!/bin/bash
# Round 4: training lines at the current build (msgf 16 x 256^2, v1.0 8 x 256^2 and C4 32 x 512^2,
# kernel breakdowns), then the term reverse's PMC traffic for bench_train.py's roofline.traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04j; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --breakdown --no-cpu-baseline \
  > $out/msgf.json 2> $out/msgf.err || { tail $out/msgf.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $out/msgf.json
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --breakdown --no-cpu-baseline \
  > $out/abstract.json 2> $out/abstract.err || { tail $out/abstract.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $out/abstract.json
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --breakdown \
  --no-cpu-baseline > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $out/c4.json
timeout -k 10 500 bash scripts/pmc_train.sh > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
tail -5 $out/pmc.log
ls gpurun_out/pmct/

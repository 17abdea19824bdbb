#!/bin/bash
# Round 4: the C4 training line (v1.0, 32 x 512^2) on a fresh box and again with MIOpen's user find-db warm
# from the first run (gpu_r04_r.sh measured 1.03 s then 2.7 s per step): kernel stats of both runs, then a run
# with the find-db disabled
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04s; mkdir -p $out
scr=/tmp/r04s; mkdir -p $scr
export TMPDIR=/tmp
for run in 1 2; do
  timeout -s KILL 500 rocprofv3 --kernel-trace --stats -d $scr/kt$run -o run -- python -u bench_train.py --model abstract \
    --batch 32 --size 512 --steps 2 --warmup 1 --no-cpu-baseline > $out/c4_$run.json 2> $out/c4_$run.err \
    || { tail -5 $out/c4_$run.err; exit 1; }
  echo "run $run $(grep -o '"ms_per_step": [0-9.]*' $out/c4_$run.json)"
  find $scr/kt$run -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats_$run.csv \;
done
cp ~/.config/miopen/*.ufdb.txt $out/ufdb.txt
MIOPEN_DEBUG_DISABLE_FIND_DB=1 timeout -k 10 400 python -u bench_train.py --model abstract --batch 32 --size 512 --steps 3 \
  --warmup 1 --no-cpu-baseline > $out/c4_nofdb.json 2> $out/c4_nofdb.err || { tail -5 $out/c4_nofdb.err; exit 1; }
echo "nofdb $(grep -o '"ms_per_step": [0-9.]*' $out/c4_nofdb.json)"

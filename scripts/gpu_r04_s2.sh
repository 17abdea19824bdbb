#!/bin/bash
# Round 4: C4 with MIOpen's find-db warm: kernel stats of the slow run (after a plain run filled the db),
# then the line with torch.backends.cudnn.benchmark (MIOpen Find) on the warm db
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04s; mkdir -p $out
scr=/tmp/r04s; mkdir -p $scr
export TMPDIR=/tmp
C4="bench_train.py --model abstract --batch 32 --size 512 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 python -u $C4 --steps 2 > $out/w_1.json 2> $out/w_1.err || { tail -5 $out/w_1.err; exit 1; }
echo "fresh $(grep -o '"ms_per_step": [0-9.]*' $out/w_1.json)"
timeout -s KILL 500 rocprofv3 --kernel-trace --stats --output-format csv -d $scr/kt -o run -- python -u $C4 --steps 2 \
  > $out/w_2.json 2> $out/w_2.err || { tail -5 $out/w_2.err; exit 1; }
echo "warm db, profiled $(grep -o '"ms_per_step": [0-9.]*' $out/w_2.json)"
find $scr/kt -name "*stats.csv" | while read f; do cp $f $out/warm_$(basename $f); done
timeout -k 10 400 python -u $C4 --steps 3 --conv-benchmark > $out/w_bm.json 2> $out/w_bm.err || { tail -5 $out/w_bm.err; exit 1; }
echo "warm db, cudnn.benchmark $(grep -o '"ms_per_step": [0-9.]*' $out/w_bm.json)"
timeout -k 10 400 python -u $C4 --steps 3 --conv-benchmark > $out/w_bm2.json 2> $out/w_bm2.err || { tail -5 $out/w_bm2.err; exit 1; }
echo "warm db, cudnn.benchmark again $(grep -o '"ms_per_step": [0-9.]*' $out/w_bm2.json)"
ls $out

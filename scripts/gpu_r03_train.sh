#!/bin/bash
# Training: ten msgf benches with the side stream on (stall stress, faulthandler watchdog), the v1.0
# model at 8 x 256^2, and the C4 shape (v1.0, 32 x 512^2 per GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/train; mkdir -p $out
export TMPDIR=/tmp
for r in 1 2 3 4 5 6 7 8 9 10; do
  GRR_FEATURE_STREAMS_TRAIN=1 timeout -k 10 150 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 \
    --no-cpu-baseline --watchdog 45 > $out/t_on_$r.json 2> $out/t_on_$r.err
  rc=$?; printf "streams on run %s rc=%s: " $r $rc; head -c 300 $out/t_on_$r.json | grep -o '"ms_per_step": [0-9.]*'; echo
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --breakdown \
  > $out/abstract.json 2> $out/abstract.err || { tail $out/abstract.err; exit 1; }
head -c 400 $out/abstract.json; echo
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
head -c 400 $out/c4.json; echo

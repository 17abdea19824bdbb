#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/wgrad2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/micro_wgrad.py > $out/micro.txt 2>&1; rc=$?; cat $out/micro.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
GRR_TIMER_SHAPES=1 timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 4 --warmup 2 \
  --no-cpu-baseline --breakdown > $out/train.json 2> $out/train.err || { tail $out/train.err; exit 1; }
grep -E "conv1x1|wgrad" $out/train.err | head -40

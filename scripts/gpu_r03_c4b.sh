#!/bin/bash
# C4 shape and v1.0 at 256^2 with the level streams; msgf per-shape GEMM breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/c4b; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $out/c4.json
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline > $out/abstract.json 2> $out/abstract.err || { tail $out/abstract.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $out/abstract.json
GRR_TIMER_SHAPES=1 timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 4 --warmup 2 --no-cpu-baseline --breakdown > $out/msgf_shapes.json 2> $out/msgf_shapes.err || { tail $out/msgf_shapes.err; exit 1; }
grep -E "conv1x1|wgrad" $out/msgf_shapes.err

#!/bin/bash
# Training benches (C4 family) on one GPU: msgf at 16x256^2 and the v1.0 model, with roofline + CPU baseline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench_train.py --model msgf --batch 16 --steps 5 --warmup 2 --breakdown \
  > gpurun_out/bench_train_msgf.json 2> gpurun_out/bench_train_msgf.err || exit 1
timeout -k 10 300 python bench_train.py --model abstract --batch 8 --steps 3 --warmup 1 --breakdown \
  > gpurun_out/bench_train_abstract.json 2> gpurun_out/bench_train_abstract.err || exit 1
tail -c 3000 gpurun_out/bench_train_msgf.json

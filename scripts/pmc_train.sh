#!/bin/bash
# HBM traffic (PMC) of the dominant training reverse kernel (term_row_kernel = grr_bwd_term_fused's row
# form) in one msgf / v1.0 training step at the bench_train shapes: one rocprofv3 pass per counter
# (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2), then per-launch bytes with the gfx950 read correction
# (scripts/collect_traffic.py) into profiles/r03/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmctrain; mkdir -p $out profiles/r03
for m in msgf abstract; do
  b=16; [ $m = abstract ] && b=8
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "term_row_kernel" --output-format csv \
      -d $out/${m}_$c -o run -- python bench_train.py --model $m --batch $b --steps 1 --warmup 1 --no-cpu-baseline \
      > $out/${m}_$c.log 2>&1 || { tail -5 $out/${m}_$c.log; exit 1; }
  done
  python scripts/collect_traffic.py $out/${m}_FETCH_SIZE $out/${m}_WRITE_SIZE --kernel term_row_kernel \
    --out profiles/r03/traffic_bwd_term_fused_$m.json --batch $b --size 256 || exit 1
done

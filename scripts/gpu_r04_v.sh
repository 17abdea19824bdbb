#!/bin/bash
# Round 4: grr_bwd_term_fused_acc (acc 1) vs the term pass + stencil x-gradient pass (acc 2) per mode at the
# training shapes (msgf B16 G32 F3 256 / 128; v1.0 levels at C4 and 8 x 256^2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04v; mkdir -p $out
export TMPDIR=/tmp
: > $out/micro.txt
for spec in "16 32 3 256" "16 32 3 128" "8 8 6 256" "8 16 6 128" "8 16 12 64" "32 8 6 512"; do
  set -- $spec
  for mode in 0 1 2; do
    for acc in 1 2; do
      echo "B$1 G$2 F$3 S$4 mode$mode acc$acc $(timeout -k 10 120 python -u scripts/micro.py --kernel term --batch $1 \
        --graphs $2 --fts $3 --size $4 --mode $mode --acc $acc --iters 10 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> $out/micro.txt || exit 1
    done
  done
done
cat $out/micro.txt

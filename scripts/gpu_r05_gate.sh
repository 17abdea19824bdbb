#!/bin/bash
# LNB gate + depthwise reverse at the C4 shapes (hid x size), ring vs register kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05gate; mkdir -p $out
for hs in "96 512" "192 256" "384 128" "768 64"; do
  set -- $hs
  timeout -k 10 120 python -u scripts/micro.py --kernel gate_dw3_bwd --fts $1 --graphs 1 --batch 32 --size $2 --iters 10 > $out/g_$1.txt 2>&1 || { tail $out/g_$1.txt; exit 1; }
  echo "hid $1 ${2}^2: $(grep 'lnb_gate_dw3_bwd' $out/g_$1.txt | tr -s ' ' | cut -d' ' -f2-6)"
done

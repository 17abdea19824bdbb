#!/bin/bash
# GEMM / wgrad shapes of one C4 and one v1.0 training step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05u; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_shapes.py > $out/c4.txt 2>&1 || { tail -30 $out/c4.txt; exit 1; }
cat $out/c4.txt
timeout -k 10 300 python -u scripts/gemm_shapes.py --size 256 --batch 8 > $out/abs.txt 2>&1 || { tail -30 $out/abs.txt; exit 1; }
cat $out/abs.txt

#!/bin/bash
# Time the LNB tail ablation builds (exp/libgrr_exp{0..3}.so: 0 product, 1 no gate math,
# 2 no MFMA, 3 no in-loop DMA) with a rocprofv3 kernel trace each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for n in 0 4 6 7; do
  GRR_LIB=exp/libgrr_exp$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/abl$n -o run -- python scripts/micro.py --kernel lnb --iters 10 > gpurun_out/abl$n.log 2>&1 || exit $?
  echo "exp$n: $(grep lnb_tail gpurun_out/abl$n/run_kernel_stats.csv | cut -d, -f1-4)"
done

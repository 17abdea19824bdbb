#!/bin/bash
# Round 5: fused LNB knockout timings (diagnostic builds, wrong results): which role sets the pace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05d}; mkdir -p $out
export TMPDIR=/tmp
for lib in exp/libgrr_map1.so exp/libgrr_m1d1.so exp/libgrr_m1d2.so exp/libgrr_m1d3.so exp/libgrr_m0d2.so imagerestoration-development-unrolling_amd/libgrr.so; do for sz in 256; do
  echo "$(basename $lib) $sz: $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel lnb --size $sz --iters 20 2>&1 | grep lnb_ | tr '\n' ' ')" >> $out/micro.txt || exit 1
done; done
cat $out/micro.txt

#!/bin/bash
# Round 5: fused LNB consumer priority A/B (same box, alternating)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05f}; mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do for v in base prio1 prio2; do for sz in 256 128; do
  echo "r$r $v $sz: $(GRR_LIB=exp/libgrr_$v.so timeout -k 10 120 python -u scripts/micro.py --kernel lnb --size $sz --iters 20 2>&1 | grep lnb_ | tr '\n' ' ')" >> $out/micro.txt || exit 1
done; done; done
cat $out/micro.txt

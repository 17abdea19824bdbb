#!/bin/bash
# Round 5: fused LNB per-phase s_memtime stamps (diagnostic build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05g}; mkdir -p $out
export TMPDIR=/tmp
for v in stamp stampd2; do for sz in 256 128; do
  echo "== $v $sz" >> $out/stamps.txt
  GRR_LIB=exp/libgrr_$v.so timeout -k 10 120 python -u scripts/micro.py --kernel lnb --size $sz --iters 5 --stamps >> $out/stamps.txt 2>&1 || exit 1
done; done
cat $out/stamps.txt

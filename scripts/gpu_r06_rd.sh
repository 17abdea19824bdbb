#!/bin/bash
# round 6: term ring depth 4 / 5 / 6 at the C4 shapes (sweep only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06rd; mkdir -p $out
export TMPDIR=/tmp
for d in 4 5 6 4; do
  GRR_TERM_RING_D=$d timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 --levels L0f,L0h,L1f,L2h,L3f > $out/sweep_d$d.txt 2>&1 || { tail $out/sweep_d$d.txt; exit 1; }
  echo "depth $d"; grep -v amdgpu $out/sweep_d$d.txt | cut -c1-90
done

#!/bin/bash
# round 6: term reverse segment split (minimum waves per launch 8192 / 16384 / 32768 / 4096) at the C4 shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06mw; mkdir -p $out
export TMPDIR=/tmp
for mw in 8192 16384 32768 4096 8192; do
  GRR_TERM_MIN_WAVES=$mw timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 > $out/sweep_mw$mw.txt 2>&1 || { tail $out/sweep_mw$mw.txt; exit 1; }
  echo "min waves $mw: $(tail -1 $out/sweep_mw$mw.txt)"
done

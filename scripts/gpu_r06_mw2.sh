#!/bin/bash
# round 6: term reverse segment split, second pass: (min waves, max segment rows) pairs at the C4 shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06mw2; mkdir -p $out
export TMPDIR=/tmp
for cfg in ${CFGS:-8192:100000 4096:128}; do
  mw=${cfg%%:*}; ms=${cfg#*:}
  GRR_TERM_MIN_WAVES=$mw GRR_TERM_MAX_SEG=$ms timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 > $out/sweep_${mw}_$ms.txt 2>&1 || { tail $out/sweep_${mw}_$ms.txt; exit 1; }
  echo "min waves $mw max seg $ms: $(tail -1 $out/sweep_${mw}_$ms.txt)"
done

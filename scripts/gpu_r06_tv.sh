#!/bin/bash
# round 6: term reverse A/B — tail on/off, 4-column lanes at W = 512 for GLR / prox, ring at narrow widths
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06tv; mkdir -p $out
export TMPDIR=/tmp
for env in "GRR_TERM_WIDE_V=4" "GRR_TERM_RING_NARROW=1"; do
  # (GRR_TERM_WIDE_V=4: the x-gradient pass no longer fits the ring's LDS at W = 512 F = 6, so the acc file's
  # shape expectations do not hold; the ring file only)
  files="tests/test_gpu_term_ring.py"; [ "${env%%=*}" = GRR_TERM_RING_NARROW ] && files="$files tests/test_gpu_term_acc.py"
  env $env timeout -k 10 300 python -u -m pytest $files -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests_${env%%=*}.log 2>&1 || { tail -30 $out/tests_${env%%=*}.log; exit 1; }
  echo "$env $(tail -1 $out/tests_${env%%=*}.log)"
done
timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 --tail 0,1 > $out/sweep_default.txt 2>&1 || { tail $out/sweep_default.txt; exit 1; }
cat $out/sweep_default.txt
GRR_TERM_WIDE_V=4 timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 --tail 0,1 --levels L0f --modes 0,2 > $out/sweep_widev4.txt 2>&1 || { tail $out/sweep_widev4.txt; exit 1; }
cat $out/sweep_widev4.txt
GRR_TERM_RING_NARROW=1 timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 --levels L2h,L3f,L3h > $out/sweep_narrow.txt 2>&1 || { tail $out/sweep_narrow.txt; exit 1; }
cat $out/sweep_narrow.txt

#!/bin/bash
# term ring: depth A/B for the pair term and a kernel trace of one shape
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05k}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_term_ring.py > $out/tests_ring.log 2>&1 || { tail -30 $out/tests_ring.log; exit 1; }
tail -2 $out/tests_ring.log
for d in 0 4 5; do
  echo "== depth $d"
  GRR_TERM_RING_D=$d timeout -k 10 200 python -u scripts/term_ring_ab.py --shapes all --iters 10 > $out/ab_d$d.txt 2>&1 || { tail -20 $out/ab_d$d.txt; exit 1; }
  grep mode $out/ab_d$d.txt
done

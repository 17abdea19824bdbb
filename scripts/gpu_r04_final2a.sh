#!/bin/bash
# Round-4 end evidence, part 1: the full GPU suite and smoke() on the final build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R04_OUT:-r04final2}; mkdir -p $out
export TMPDIR=/tmp
MIOPEN_FIND_MODE=FAST timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 \
  || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log

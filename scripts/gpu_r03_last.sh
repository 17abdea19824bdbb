#!/bin/bash
# last check of the session: full GPU suite and smoke() on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/last; mkdir -p $out
export TMPDIR=/tmp
MIOPEN_FIND_MODE=FAST timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -2 $out/smoke.log

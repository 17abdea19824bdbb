#!/bin/bash
# the whole GPU suite (one process) + smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05all}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log

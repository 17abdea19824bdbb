#!/bin/bash
# Full GPU parity suite (all failures listed), then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/full; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?
tail -12 $out/gpu_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 1200 $out/bench.json
exit $rc

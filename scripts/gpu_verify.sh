#!/bin/bash
# Full GPU parity suite, then the default bench line (state check after a rebuild)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/verify
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/verify/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/verify/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/verify/bench.json 2> gpurun_out/verify/bench.err || { tail -20 gpurun_out/verify/bench.err; exit 1; }
tail -c 1500 gpurun_out/verify/bench.json

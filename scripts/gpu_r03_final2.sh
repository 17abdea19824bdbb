#!/bin/bash
# End-of-session evidence: full GPU suite (MIOpen FAST find for the test run only), PMC HBM traffic of
# the roofline kernels at the bench batch with the rocprofv3 kernel summary, the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/final2; mkdir -p $out
export TMPDIR=/tmp
MIOPEN_FIND_MODE=FAST timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_bench.sh 64 > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
tail -14 $out/pmc.log
cp gpurun_out/pmcb/traffic_system_step2.json profiles/traffic_system_step2.json

cp gpurun_out/pmcb/bench_kernel_stats.csv $out/
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 3000 $out/bench.json

#!/bin/bash
# End-of-round evidence: full GPU suite, the default bench line (CPU baseline, secondary workload),
# PMC HBM traffic of the roofline kernels at the bench batch and the rocprofv3 kernel summary
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/final; mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_bench.sh 64 > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
tail -14 $out/pmc.log
cp gpurun_out/pmcb/traffic_system_step2.json profiles/traffic_system_step2.json
cp gpurun_out/pmcb/traffic_lnb_head16.json gpurun_out/pmcb/traffic_lnb_mix.json profiles/r03/
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 3000 $out/bench.json

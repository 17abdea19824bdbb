#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "nonlinear or x3 or msgf or c3 or patch_independent or replicated or abstract or psnr or compile" > gpurun_out/lnb_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/ab_lnb.sh > gpurun_out/ab_lnb.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --breakdown --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1

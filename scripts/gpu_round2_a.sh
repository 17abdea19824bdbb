#!/bin/bash
# round-2 GPU call: full GPU test suite, then train the PSNR weights fixture
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --durations=15 --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "gpu_tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u scripts/train_psnr_fixture.py --iters ${ITERS:-3000} --batch 8 --workers 12 > gpurun_out/train_fixture.log 2>&1
rc=$?
echo "train rc=$rc"
exit $rc

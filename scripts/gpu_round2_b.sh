#!/bin/bash
# round-2 GPU call: train the PSNR weights fixture, then its parity tests and the bench on it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/train_psnr_fixture.py --iters ${ITERS:-4000} --batch 8 --workers 12 > gpurun_out/train_fixture.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_psnr.py -q -rf -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/psnr_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --breakdown > gpurun_out/bench.log 2>&1

#!/bin/bash
# round-2 GPU call: PSNR + C5 tests on the trained fixture, then LNB PMC counters (micro shape)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_psnr.py "tests/test_gpu_configs.py::test_c5_tiled_2048_vs_whole_image_and_oracle" -q -rf -s --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/psnr_c5_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
mkdir -p gpurun_out/pmc_lnb
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_lnb/a -o run -- python scripts/micro.py --kernel lnb --iters 3 > gpurun_out/pmc_lnb/a.log 2>&1
echo "pmc a rc=$?"

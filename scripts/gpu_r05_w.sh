#!/bin/bash
# conv1x1 at the v1.0 first-level shapes (C4): timing + SQ counters of the two GEMM kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05w; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_wgrad.py \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for mk in "192 48" "48 192" "48 96" "96 48" "96 192"; do
  set -- $mk
  timeout -k 10 120 python -u scripts/micro.py --kernel conv_mk --cin $1 --cout $2 --batch 32 --size 512 --graphs 8 --fts 3 --iters 10 \
    > $out/t_$1_$2.txt 2>&1 || { tail $out/t_$1_$2.txt; exit 1; }
  echo "cin $1 cout $2: $(grep -v amdgpu.ids $out/t_$1_$2.txt | tail -2 | tr '\n' ' ')"
done
MICRO_ARGS="--cin 192 --cout 48 --batch 32 --size 512 --graphs 8 --fts 3" timeout -k 10 300 bash scripts/pmc_sq.sh conv_mk gemm_x3k r05w/sq_192_48 > $out/sq_192_48.txt 2>&1 || { tail $out/sq_192_48.txt; exit 1; }
cat $out/sq_192_48.txt
MICRO_ARGS="--cin 48 --cout 192 --batch 32 --size 512 --graphs 8 --fts 3" timeout -k 10 300 bash scripts/pmc_sq.sh conv_mk gemm_x3_kernel r05w/sq_48_192 > $out/sq_48_192.txt 2>&1 || { tail $out/sq_48_192.txt; exit 1; }
cat $out/sq_48_192.txt

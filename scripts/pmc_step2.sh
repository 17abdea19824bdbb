#!/bin/bash
# HBM traffic of grr_system_step2 alone (scripts/micro.py --kernel step2): one rocprofv3 pass per
# counter, plus the kernel-trace summary of the same command
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc2
timeout -k 10 120 python scripts/micro.py --kernel step2 --iters 10 > gpurun_out/pmc2/micro.log 2>&1 || exit 1
cat gpurun_out/pmc2/micro.log | grep -v amdgpu.ids
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc2/$ctr -o run -- python scripts/micro.py --kernel step2 --iters 3 > gpurun_out/pmc2/$ctr.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc2/trace -o run -- python scripts/micro.py --kernel step2 --iters 10 > gpurun_out/pmc2/trace.log 2>&1 || exit 1
python scripts/collect_traffic.py gpurun_out/pmc2/FETCH_SIZE gpurun_out/pmc2/WRITE_SIZE --kernel graph_step2_kernel --out gpurun_out/pmc2/traffic_system_step2.json

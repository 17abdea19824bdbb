#!/bin/bash
# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, one pass each) of the LNB head and mix kernels at the micro shape
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmclnb
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmclnb/$ctr -o run -- python scripts/micro.py --kernel lnb --iters 3 > gpurun_out/pmclnb/$ctr.log 2>&1 || exit 1
done
python scripts/collect_traffic.py gpurun_out/pmclnb/FETCH_SIZE gpurun_out/pmclnb/WRITE_SIZE --kernel "lnb_head_kernel<3, 4>" --out gpurun_out/pmclnb/traffic_lnb_head.json || exit 1
python scripts/collect_traffic.py gpurun_out/pmclnb/FETCH_SIZE gpurun_out/pmclnb/WRITE_SIZE --kernel "lnb_mix_kernel<3, true>" --out gpurun_out/pmclnb/traffic_lnb_mix.json || exit 1
cat gpurun_out/pmclnb/traffic_lnb_head.json; echo; cat gpurun_out/pmclnb/traffic_lnb_mix.json

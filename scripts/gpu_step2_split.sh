#!/bin/bash
# step2 split-wave build: step2 + filter parity tests, then same-box A/B of the step2 kernel and the bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s2; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "step2 or msgf or c3 or psnr or filter or configs" > gpurun_out/s2/tests.log 2>&1 || { tail -40 gpurun_out/s2/tests.log; exit 1; }
tail -1 gpurun_out/s2/tests.log
bash scripts/ab_libs.sh step2 exp/libgrr_s0.so exp/libgrr_s1.so 2>&1 | tee gpurun_out/s2/ab_step2.log || exit 1
for L in exp/libgrr_s0.so exp/libgrr_s1.so; do GRR_LIB=$L timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-secondary > gpurun_out/s2/bench_$(basename $L .so).json 2> gpurun_out/s2/bench_$(basename $L .so).err || exit 1; head -c 260 gpurun_out/s2/bench_$(basename $L .so).json; echo; done

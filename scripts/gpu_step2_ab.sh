#!/bin/bash
# step2 variants: tests on the candidate (CAND), then same-box A/B of the kernel and the bench line
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s2; export TMPDIR=/tmp
GRR_LIB=exp/libgrr_${CAND}.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "step2 or msgf or c3 or psnr or configs" > gpurun_out/s2/tests_$CAND.log 2>&1 || { tail -40 gpurun_out/s2/tests_$CAND.log; exit 1; }
tail -1 gpurun_out/s2/tests_$CAND.log
bash scripts/ab_libs.sh step2 $LIBS 2>&1 | tee gpurun_out/s2/ab_step2.log || exit 1
for L in $LIBS; do GRR_LIB=$L timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-secondary > gpurun_out/s2/bench_$(basename $L .so).json 2> gpurun_out/s2/bench_$(basename $L .so).err || exit 1; head -c 200 gpurun_out/s2/bench_$(basename $L .so).json | cut -c 100-200; echo; done

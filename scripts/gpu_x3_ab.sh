#!/bin/bash
# split-bf16 1x1 conv: workgroup width A/B (4 vs 8 waves), accuracy tests on the candidate, bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/x3; export TMPDIR=/tmp
GRR_LIB=exp/libgrr_${CAND:-w8}.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "x3 or conv or msgf or c3 or psnr or nonlinear or abstract" > gpurun_out/x3/tests.log 2>&1 || { tail -30 gpurun_out/x3/tests.log; exit 1; }
tail -1 gpurun_out/x3/tests.log
bash scripts/ab_libs.sh conv1x1 $LIBS 2>&1 | tee gpurun_out/x3/ab.log || exit 1
for L in $NAMES; do GRR_LIB=exp/libgrr_$L.so timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-secondary > gpurun_out/x3/b_$L.json 2> gpurun_out/x3/b_$L.err || exit 1; printf "%s " $L; grep -o '"ms_per_step": [0-9.]*' gpurun_out/x3/b_$L.json; done

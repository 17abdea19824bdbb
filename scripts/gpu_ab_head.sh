#!/bin/bash
# LNB head variants: LNB GPU tests per correct variant, then same-box A/B (micro lnb / lnb_rep)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab
for v in ${TESTED:-trim trimprio}; do GRR_LIB=exp/libgrr_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "nonlinear or replicated or lnb or psnr" > gpurun_out/ab/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/ab/tests_$v.log; exit 1; }; tail -1 gpurun_out/ab/tests_$v.log; done
bash scripts/ab_head.sh ${LIBS:-exp/libgrr_base.so exp/libgrr_trim.so} 2>&1 | tee gpurun_out/ab/ab_head.log

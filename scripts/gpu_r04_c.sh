#!/bin/bash
# LNB head gate variants (same box): default, column-pair lanes, DPP side columns, both; parity of each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04c; mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_colpair.so exp/libgrr_dpp.so exp/libgrr_cpdpp.so; do
  for k in lnb_rep lnb; do for sz in 256 128; do
    echo "r$r $lib $k $sz $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel $k --size $sz --split --iters 20 2>&1 | grep lnb_head)" >> $out/micro.txt || exit 1
  done; done
done
done
cat $out/micro.txt
for lib in exp/libgrr_colpair.so exp/libgrr_dpp.so exp/libgrr_cpdpp.so; do
  GRR_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "nonlinear or x3 or msgf or abstract" \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests_$(basename $lib .so).log 2>&1; rc=$?
  echo "$lib $(tail -1 $out/tests_$(basename $lib .so).log)"; [ $rc -eq 0 ] || exit $rc
done

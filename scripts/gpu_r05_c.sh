#!/bin/bash
# Round 5: persistent fused LNB (two consumer mappings) -- parity, then micro A/B against head + mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05c}; mkdir -p $out
export TMPDIR=/tmp
for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_map1.so; do
  GRR_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "fused_lnb or local_nonlinear_block or x3_gemm_is_fp32" > $out/t_$(basename $lib).log 2>&1
  st=$?; echo "$lib: $(tail -1 $out/t_$(basename $lib).log)"; [ $st -eq 0 ] || { grep -B5 -A40 "Error\|FAILED\|assert" $out/t_$(basename $lib).log | head -80; exit 1; }
done
for r in 1 2; do for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_map1.so; do for sz in 256 128; do
  echo "r$r $(basename $lib) $sz: $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel lnb --size $sz --iters 20 2>&1 | grep lnb_ | tr '\n' ' ')" >> $out/micro.txt || exit 1
done; done; done
for sz in 256 128; do
  echo "head+mix $sz: $(timeout -k 10 120 python -u scripts/micro.py --kernel lnb --size $sz --lnb-fused 0 --split --iters 20 2>&1 | grep lnb_ | tr '\n' ' ')" >> $out/micro.txt || exit 1
done
cat $out/micro.txt

#!/bin/bash
# Round 5: fused LNB -- epilogue in one load round, prologue loads at once; parity, A/B, stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05h}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "fused_lnb or local_nonlinear_block or x3_gemm_is_fp32" > $out/t.log 2>&1
st=$?; tail -1 $out/t.log; [ $st -eq 0 ] || { grep -B5 -A40 "Error\|FAILED\|assert" $out/t.log | head -80; exit 1; }
for r in 1 2; do for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_proser.so exp/libgrr_ahead2.so; do for sz in 256 128; do
  echo "r$r $(basename $lib) $sz: $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel lnb --size $sz --iters 20 2>&1 | grep lnb_ | tr '\n' ' ')" >> $out/micro.txt || exit 1
done; done; done
cat $out/micro.txt
GRR_LIB=exp/libgrr_stamp.so timeout -k 10 120 python -u scripts/micro.py --kernel lnb --size 256 --iters 5 --stamps 2>&1 | grep stamps

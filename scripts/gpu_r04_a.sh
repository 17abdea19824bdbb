#!/bin/bash
# Round 4, first box: the tests this round added or changed (compile without codegen, 2-rank HIP DDP,
# stream guard, wgrad workspace cap, C5 tiling without the all-reduce, the LNB gate), LNB head / mix
# micro timings, then the bench line and a C5 line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04a; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_compile.py tests/test_gpu_ddp.py tests/test_gpu_stream_guard.py \
  tests/test_gpu_wgrad.py tests/test_gpu_tiling.py tests/test_gpu_configs.py tests/test_gpu_psnr.py \
  "tests/test_gpu_parity.py" -x -q -rf --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -15 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for nw in 8 16; do for k in lnb lnb_rep; do for sz in 256 128; do
  echo "NW=$nw $k $sz" >> $out/micro_lnb.txt
  GRR_HEAD16_NW=$nw timeout -k 10 120 python -u scripts/micro.py --kernel $k --size $sz --split --iters 20 >> $out/micro_lnb.txt 2>&1 || exit 1
done; done; done
cat $out/micro_lnb.txt
GRR_HEAD16_NW=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "nonlinear or x3 or psnr or abstract or msgf" \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests_nw16.log 2>&1; rc=$?; tail -3 $out/tests_nw16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --breakdown > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 1500 $out/bench.json
timeout -k 10 300 python -u bench_tiled.py --images 2 --steps 3 > $out/tiled.json 2> $out/tiled.err || { tail -20 $out/tiled.err; exit 1; }
cat $out/tiled.json

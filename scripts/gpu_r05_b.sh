#!/bin/bash
# Round 5: the fused C <= 96 LocalNonLinearBlock (lnb_fused16_kernel) -- its parity tests, micro A/B
# against head + mix at the bench shapes, then the whole GPU suite and the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05b}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "fused_lnb or local_nonlinear_block or x3_gemm_is_fp32" > $out/t_fused.log 2>&1
st=$?; tail -3 $out/t_fused.log; [ $st -eq 0 ] || { grep -B5 -A40 "Error\|FAILED\|assert" $out/t_fused.log | head -120; exit 1; }
for sz in 256 128; do for f in 1 0; do
  echo "size $sz fused $f: $(timeout -k 10 120 python -u scripts/micro.py --kernel lnb --size $sz --lnb-fused $f --split --iters 20 2>&1 | grep lnb_ | tr '\n' ' ')" >> $out/micro.txt || exit 1
done; done
cat $out/micro.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1
st=$?; tail -3 $out/tests.log; [ $st -eq 0 ] || { grep -B5 -A30 "Error\|FAILED\|assert" $out/tests.log | head -80; exit 1; }
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 2500 $out/bench.json
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline \
  > $out/train_msgf.json 2> $out/train_msgf.err || { tail $out/train_msgf.err; exit 1; }
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/train_abstract.json 2> $out/train_abstract.err || { tail $out/train_abstract.err; exit 1; }
for f in train_msgf train_abstract; do echo "$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $out/$f.json | tr '\n' ' ')"; done

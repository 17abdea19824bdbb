#!/bin/bash
# Round 5: the term reverse's LDS-ring row kernel -- parity against the register kernel, determinism,
# A/B per training shape, then the three training lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05j}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_term_ring.py \
  > $out/tests_ring.log 2>&1 || { tail -30 $out/tests_ring.log; exit 1; }
tail -3 $out/tests_ring.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_term_rows.py \
  tests/test_gpu_deterministic.py tests/test_gpu_term_acc.py > $out/tests_rows.log 2>&1 || { tail -30 $out/tests_rows.log; exit 1; }
tail -3 $out/tests_rows.log
timeout -k 10 400 python -u scripts/term_ring_ab.py > $out/ab.txt 2>&1 || { tail -20 $out/ab.txt; exit 1; }
cat $out/ab.txt
if [ "${R05_TRAIN:-1}" = 1 ]; then
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline \
  > $out/train_msgf.json 2> $out/train_msgf.err || { tail $out/train_msgf.err; exit 1; }
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/train_abstract.json 2> $out/train_abstract.err || { tail $out/train_abstract.err; exit 1; }
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/train_c4.json 2> $out/train_c4.err || { tail $out/train_c4.err; exit 1; }
for f in train_msgf train_abstract train_c4; do echo "$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $out/$f.json | tr '\n' ' ')"; done
fi

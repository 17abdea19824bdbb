#!/bin/bash
# term ring default (depth 4): term-reverse tests, training gradients, then the three training lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05l}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_term_ring.py \
  tests/test_gpu_term_rows.py tests/test_gpu_deterministic.py tests/test_gpu_term_acc.py tests/test_gpu_training.py \
  tests/test_gpu_grad.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline \
  > $out/train_msgf.json 2> $out/train_msgf.err || { tail $out/train_msgf.err; exit 1; }
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/train_abstract.json 2> $out/train_abstract.err || { tail $out/train_abstract.err; exit 1; }
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/train_c4.json 2> $out/train_c4.err || { tail $out/train_c4.err; exit 1; }
for f in train_msgf train_abstract train_c4; do echo "$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $out/$f.json | tr '\n' ' ')"; done
python - $out <<'PY'
import json, sys
for n in ("train_msgf", "train_abstract", "train_c4"):
    d = json.load(open(f"{sys.argv[1]}/{n}.json"))
    k = d.get("kernel_ms_per_step", {})
    print(n, {x: k[x] for x in ("bwd_term_fused", "bwd_cg_glue", "bwd_stencil", "wgrad", "conv1x1", "lnb_gate_dw3_bwd") if x in k})
PY

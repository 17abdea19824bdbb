#!/bin/bash
# fp16 two-term LNB head (lnb_head16_kernel) vs the split-bf16 head (GRR_LNB_HEAD=bf16): LNB parity
# tests, micro timings (C = 96 block at 256^2 and 128^2, replicated first block), bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/h16; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; grep FAILED $out/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in f16 bf16; do
  for k in "lnb --size 256" "lnb --size 128" "lnb_rep --size 256"; do
    printf "%s %s: " $v "$k"
    GRR_LNB_HEAD=$v timeout -k 10 120 python scripts/micro.py --kernel $k --iters 10 2>&1 | tail -1 || exit 1
  done
done
for r in 1 2; do for v in f16 bf16; do
  GRR_LNB_HEAD=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-secondary > $out/b_${v}_$r.json 2> $out/b_${v}_$r.err || { tail -20 $out/b_${v}_$r.err; exit 1; }
  printf "%s run %s: " $v $r; python -c "import json,sys; d=json.load(open('$out/b_${v}_$r.json')); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step']['lnb'])"
done; done

#!/bin/bash
# round 6: term policy at the 256^2 training shapes (v1.0 8 x 256^2, msgf 16 x 256^2): sweep + training A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06tp2; mkdir -p $out
export TMPDIR=/tmp
for p in 0 1; do
  GRR_TERM_POLICY=$p timeout -k 10 300 python -u scripts/term_sweep.py --rows 2 --size 256 --batch 8 > $out/sweep256_p$p.txt 2>&1 || { tail $out/sweep256_p$p.txt; exit 1; }
  tail -1 $out/sweep256_p$p.txt
done
for p in 0 1 0 1; do
  for m in abstract msgf; do
    b=8; [ $m = msgf ] && b=16
    GRR_TERM_POLICY=$p timeout -k 10 300 python -u bench_train.py --model $m --batch $b --no-cpu-baseline \
      > $out/train_${m}_p$p.json 2> $out/train_${m}_p$p.err || { tail $out/train_${m}_p$p.err; exit 1; }
    python -c "
import json;d=json.load(open('$out/train_${m}_p$p.json'));print('policy $p $m', d['ms_per_step'], d['value'], 'term ms/step', d['kernel_ms_per_step']['bwd_term_fused'])"
  done
done

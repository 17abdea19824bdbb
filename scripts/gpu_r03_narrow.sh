#!/bin/bash
# A/B: the strip pass on the v1.0 model's narrower levels (W = 128 / 64) vs one launch per stage
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/narrow; mkdir -p $out
export TMPDIR=/tmp
for mw in 257 128 64 257; do
  GRR_STEP2_MIN_W=$mw timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/b_$mw.json 2> $out/b_$mw.err || { tail $out/b_$mw.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('$out/b_$mw.json')); s=d['secondary_workload']; print($mw, {k: s[k] for k in s if k in ('value','ms_per_step')}, {k:v for k,v in s.get('kernel_ms_per_step',{}).items() if 'system' in k})"
done

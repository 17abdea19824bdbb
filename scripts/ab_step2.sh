#!/bin/bash
# A/B of two-stage launches (grr_system_step2) vs one launch per stage in the headline bench
set -o pipefail
mkdir -p gpurun_out
for v in 1 0 1 0; do
  GRR_STEP2=$v timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --breakdown \
    > gpurun_out/ab_step2_$v.json 2> gpurun_out/ab_step2_$v.err || exit 1
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_step2_{v}.json").read().strip().splitlines()[-1])
k = d["kernel_ms_per_step"]
print(f"STEP2={v} value={d['value']} ms/step={d['ms_per_step']} step={k.get('system_step')} step2={k.get('system_step2')} half={k.get('system_half')} lnb={k.get('lnb')}")
PY
  grep -E "system_step|system_half" gpurun_out/ab_step2_$v.err
done

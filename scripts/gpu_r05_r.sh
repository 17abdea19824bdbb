#!/bin/bash
# fused LNB with packed depthwise FMAs: LNB parity tests, micro timing, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05r}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "lnb or fused or local_nonlinear or x3" \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for i in 1 2; do
timeout -k 10 120 python -u scripts/micro.py --kernel lnb --batch 64 --size 256 --graphs 32 --fts 3 --hid 256 --iters 20 >> $out/micro.txt 2>&1 || { tail $out/micro.txt; exit 1; }
done
cat $out/micro.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python - $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline_secondary"]["lnb_fused"]["frac"], d["psnr"]["delta_db"] if "psnr" in d else None)
print(json.dumps(d["kernel_ms_per_step"]))
PY

#!/bin/bash
# first-pair pass: parity tests, step2 / filter tests, micro timing, bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05m}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_first_pair.py \
  > $out/tests_fp.log 2>&1 || { tail -40 $out/tests_fp.log; exit 1; }
tail -2 $out/tests_fp.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_step2.py \
  tests/test_gpu_term_ring.py tests/test_gpu_term_rows.py tests/test_gpu_term_acc.py tests/test_gpu_deterministic.py \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05m/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["psnr"])
print(json.dumps(d["kernel_ms_per_step"]))
PY

#!/bin/bash
# two-stage solver pass in column strips (W != 256): parity, wide-image bench vs one launch per
# stage, and the headline bench (the W = 256 instance must not move)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/s2strips; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_step2.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -6 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_wide.py --size 336x496 --batch 16 --compare-step2 > $out/wide_336x496.json 2> $out/wide.err || { tail $out/wide.err; exit 1; }
timeout -k 10 300 python -u bench_wide.py --size 512x512 --batch 16 --compare-step2 > $out/wide_512.json 2>> $out/wide.err || { tail $out/wide.err; exit 1; }
python - $out <<'PY'
import json, sys
for f in ("wide_336x496.json", "wide_512.json"):
    for l in open(sys.argv[1] + "/" + f):
        d = json.loads(l)
        if "value" in d:
            print(f, d["graph_kernels"][:30], d["value"], d["ms_per_step"], {k: v for k, v in d["kernel_ms"].items() if "system" in k})
        else:
            print(f, d)
PY
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
head -c 400 $out/bench.json; echo

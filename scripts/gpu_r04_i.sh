#!/bin/bash
# LNB + projection (grr_lnb_forward_proj): parity and model tests, bench A/B (GRR_LNB_PROJ)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04i; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_psnr.py tests/test_gpu_streams.py tests/test_gpu_compile.py \
  tests/test_gpu_tiling.py tests/test_gpu_configs.py tests/test_gpu_step2.py -q -x -rf --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for pj in 1 0; do
  GRR_LNB_PROJ=$pj timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $out/bench_p${pj}_$r.json 2> $out/bench_p${pj}_$r.err || { tail -5 $out/bench_p${pj}_$r.err; exit 1; }
  python -c "import json;d=json.loads(open('$out/bench_p${pj}_$r.json').read().strip().splitlines()[-1]);print('PROJ=$pj', d['value'], d['ms_per_step'], d.get('kernel_ms_per_step'))"
done; done

#!/bin/bash
# Round 4: edge weights with hardware reciprocal / exp (GRR_EDGE_FASTDIV=1, exp/libgrr_fastdiv.so) vs the
# IEEE divisions: the edge-weight parity tests with the variant, the kernel at the bench shape, the bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04p; mkdir -p $out
export TMPDIR=/tmp
GRR_LIB=exp/libgrr_fastdiv.so timeout -k 10 300 python -u -m pytest -q -rf --timeout 200 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_psnr.py > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
L=imagerestoration-development-unrolling_amd/libgrr.so
for r in 1 2; do for lib in $L exp/libgrr_fastdiv.so; do
  echo "$(basename $lib) $(GRR_LIB=$lib timeout -k 10 120 python -u scripts/micro.py --kernel edge --iters 20 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
done; done | tee $out/micro.txt
for lib in $L exp/libgrr_fastdiv.so; do
  n=$(basename $lib .so)
  GRR_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $out/bench_$n.json 2> $out/bench_$n.err \
    || { tail -5 $out/bench_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]);print('$n', d['value'], d['ms_per_step'], d['kernel_ms_per_step'].get('edge_weights'))"
done

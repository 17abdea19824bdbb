#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/strips; mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 600 python -u -m pytest tests/test_gpu_dwconv.py tests/test_gpu_grad.py tests/test_gpu_ffn.py tests/test_gpu_configs.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
head -c 300 $out/c4.json; echo
timeout -k 10 700 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline --breakdown > $out/c4b.json 2> $out/c4b.err || { tail $out/c4b.err; exit 1; }
grep -v "amdgpu\|MIOpen\|Warning" $out/c4b.err | head -14

#!/bin/bash
# Round 3 first box run: full GPU suite, default bench line, and the --gpus 2 launcher rehearsal
# (two gloo ranks sharing the one GPU: bench.py spawns them itself)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r03a; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 600 $out/bench.json; echo
GRR_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --no-secondary --no-cpu-baseline > $out/bench_gloo2.json 2> $out/bench_gloo2.err || { tail -20 $out/bench_gloo2.err; exit 1; }
head -c 400 $out/bench_gloo2.json; echo; grep -o '"ranks": {[^}]*}' $out/bench_gloo2.json

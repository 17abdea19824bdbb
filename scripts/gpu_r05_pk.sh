#!/bin/bash
# packed-pair operator pipes in the pair kernel (GRR_S2_PK): parity, micro and bench A/B against
# exp/libgrr_pk0.so (the same tree built with GRR_S2_PK=0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05pk; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_step2.py \
  tests/test_gpu_first_pair.py tests/test_gpu_parity.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
for lib in pk0 pk1; do
  L=imagerestoration-development-unrolling_amd/libgrr.so; [ $lib = pk0 ] && L=exp/libgrr_pk0.so
  GRR_LIB=$L timeout -k 10 120 python -u scripts/micro.py --kernel step2 --iters 20 > $out/m_$lib.$rep.txt 2>&1 || { tail $out/m_$lib.$rep.txt; exit 1; }
  echo "micro step2 $lib: $(grep 'system_step2' $out/m_$lib.$rep.txt | tr -s ' ' | cut -d' ' -f3-6)"
  GRR_LIB=$L timeout -k 10 300 python -u bench.py > $out/b_$lib.$rep.json 2> $out/b_$lib.$rep.err || { tail $out/b_$lib.$rep.err; exit 1; }
  echo "bench $lib: $(grep -o '"value": [0-9.]*, "unit": "MPix/s"\|"system_step2": [0-9.]*\|"system_first_pair": [0-9.]*\|"frac": [0-9.]*' $out/b_$lib.$rep.json | head -4 | tr '\n' ' ')"
done
done

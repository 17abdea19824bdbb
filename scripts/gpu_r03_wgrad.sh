#!/bin/bash
# grr_wgrad replaces the library weight-gradient GEMMs: its tests, the full GPU suite, then the
# training side stream stress (three msgf training benches with GRR_FEATURE_STREAMS_TRAIN=1, one without)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/wgrad; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py -q -rf --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $out/wgrad_tests.log 2>&1
rc=$?; tail -3 $out/wgrad_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -8 $out/gpu_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for r in 1 2 3; do
  GRR_FEATURE_STREAMS_TRAIN=1 timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 8 --warmup 2 \
    --no-cpu-baseline --watchdog 45 > $out/t_on_$r.json 2> $out/t_on_$r.err
  rc=$?; printf "streams on run %s rc=%s: " $r $rc; head -c 300 $out/t_on_$r.json | grep -o '"ms_per_step": [0-9.]*'; echo
  [ $rc -eq 0 ] || exit $rc
done
GRR_FEATURE_STREAMS_TRAIN=0 timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 8 --warmup 2 \
  --no-cpu-baseline > $out/t_off.json 2> $out/t_off.err || exit 1
printf "streams off: "; head -c 300 $out/t_off.json | grep -o '"ms_per_step": [0-9.]*'

#!/bin/bash
# window-graph pair weights: window GPU tests, then bench_window A/B (raw vs pair, same box)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/win; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_window_grad.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/win/tests.log 2>&1 || { tail -40 gpurun_out/win/tests.log; exit 1; }
tail -1 gpurun_out/win/tests.log
for r in 1; do for v in 0 1; do GRR_WIN_PAIR=$v timeout -k 10 300 python -u bench_window.py --train --batch 4 --steps 3 --warmup 1 --breakdown --no-cpu-baseline > gpurun_out/win/b_${v}_$r.json 2> gpurun_out/win/b_${v}_$r.err || { tail -20 gpurun_out/win/b_${v}_$r.err; exit 1; }; printf "pair=%s " $v; grep -E "win_solver|win_pair" gpurun_out/win/b_${v}_$r.err | tr '\n' ' '; grep -o '"ms_per_step": [0-9.]*'  gpurun_out/win/b_${v}_$r.json; done; done

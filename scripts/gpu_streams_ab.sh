#!/bin/bash
# side-stream half-resolution feature branch: parity tests, then same-box bench A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/streams; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "msgf or c3 or psnr or compile or tiling or configs or replicated or golden or abstract or mixture" > gpurun_out/streams/tests.log 2>&1 || { tail -40 gpurun_out/streams/tests.log; exit 1; }
tail -1 gpurun_out/streams/tests.log
for r in 1 2; do for v in 0 1; do GRR_FEATURE_STREAMS=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-secondary > gpurun_out/streams/b_${v}_$r.json 2> gpurun_out/streams/b_${v}_$r.err || { tail -20 gpurun_out/streams/b_${v}_$r.err; exit 1; }; printf "streams=%s " $v; head -c 330 gpurun_out/streams/b_${v}_$r.json | grep -o '"value": [0-9.]*, "unit": "MPix/s", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*'; done; done

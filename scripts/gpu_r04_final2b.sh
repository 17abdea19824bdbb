#!/bin/bash
# Round-4 end evidence, part 2: PMC HBM traffic + rocprofv3 kernel summary of the bench's launches, the
# default bench line, PMC traffic of the training reverse's term kernel, the training lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R04_OUT:-r04final2}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 800 bash scripts/pmc_bench.sh 64 > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
tail -14 $out/pmc.log
cp gpurun_out/pmcb/traffic_*.json gpurun_out/pmcb/bench_kernel_stats.csv $out/
mkdir -p profiles/r04   # this box's tree: the lines below read the fresh summaries (committed afterwards)
cp gpurun_out/pmcb/traffic_system_step2.json profiles/
cp gpurun_out/pmcb/traffic_lnb_*.json profiles/r04/
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 1500 $out/bench.json
timeout -k 10 700 bash scripts/pmc_train.sh > $out/pmct.log 2>&1 || { tail -20 $out/pmct.log; exit 1; }
cp gpurun_out/pmct/traffic_bwd_term_fused_*.json $out/
cp gpurun_out/pmct/traffic_bwd_term_fused_*.json profiles/r04/
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline \
  > $out/train_msgf.json 2> $out/train_msgf.err || { tail $out/train_msgf.err; exit 1; }
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/train_abstract.json 2> $out/train_abstract.err || { tail $out/train_abstract.err; exit 1; }
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/train_c4.json 2> $out/train_c4.err || { tail $out/train_c4.err; exit 1; }
for f in train_msgf train_abstract train_c4; do echo "$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $out/$f.json | tr '\n' ' ')"; done

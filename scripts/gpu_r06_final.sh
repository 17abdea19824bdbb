#!/bin/bash
# Round 6 evidence: PMC traffic + rocprofv3 summary of the bench, the bench line, the three training lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R06_OUT:-r06f}; mkdir -p $out profiles/r06
export TMPDIR=/tmp
timeout -k 10 800 bash scripts/pmc_bench.sh 64 > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
tail -14 $out/pmc.log
cp gpurun_out/pmcb/traffic_*.json gpurun_out/pmcb/bench_kernel_stats.csv $out/
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 1500 $out/bench.json
if [ "${R06_TRAIN:-1}" = 1 ]; then
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline \
  > $out/train_msgf.json 2> $out/train_msgf.err || { tail $out/train_msgf.err; exit 1; }
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/train_abstract.json 2> $out/train_abstract.err || { tail $out/train_abstract.err; exit 1; }
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/train_c4.json 2> $out/train_c4.err || { tail $out/train_c4.err; exit 1; }
for f in train_msgf train_abstract train_c4; do echo "$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $out/$f.json | tr '\n' ' ')"; done
fi

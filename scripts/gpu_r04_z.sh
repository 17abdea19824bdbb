#!/bin/bash
# Round 4: PMC traffic of the term reverse at the C4 workload, then the C4 training line reading it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R04_OUT:-r04final3}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 bash scripts/pmc_train_c4.sh > $out/pmct_c4.log 2>&1 || { tail -20 $out/pmct_c4.log; exit 1; }
cp gpurun_out/pmct/traffic_bwd_term_fused_abstract_b32_s512.json $out/
mkdir -p profiles/r04 && cp gpurun_out/pmct/traffic_bwd_term_fused_abstract_b32_s512.json profiles/r04/
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/train_c4_pmc.json 2> $out/train_c4_pmc.err || { tail $out/train_c4_pmc.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"traffic": [0-9.e+]*' $out/train_c4_pmc.json | tr '\n' ' '

#!/bin/bash
# SQ counters of the pair kernel (bench shape) and of the LNB gate reverse (C4 level 0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05z; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 bash scripts/pmc_sq.sh step2 graph_step2 r05z/sq_step2 > $out/sq_step2.txt 2>&1 || { tail $out/sq_step2.txt; exit 1; }
cat $out/sq_step2.txt
MICRO_ARGS="--fts 96 --batch 32 --size 512" timeout -k 10 300 bash scripts/pmc_sq.sh gate_dw3_bwd dw3_gate r05z/sq_gate > $out/sq_gate.txt 2>&1 || { tail $out/sq_gate.txt; exit 1; }
cat $out/sq_gate.txt
for hs in "96 512" "192 256" "384 128" "768 64"; do
  set -- $hs
  timeout -k 10 120 python -u scripts/micro.py --kernel gate_dw3_bwd --fts $1 --batch 32 --size $2 --iters 10 > $out/gate_$1.txt 2>&1 || { tail $out/gate_$1.txt; exit 1; }
  echo "hid $1 ${2}^2: $(grep -v amdgpu.ids $out/gate_$1.txt | tail -1)"
done

#!/bin/bash
# PMC counter passes for one micro-benchmarked kernel (separate rocprofv3 runs, no tracing
# domains combined with --pmc).  Usage: bash scripts/pmc_session.sh <kernel> [iters]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K=${1:-step}
IT=${2:-10}
OUT=gpurun_out/pmc_$K
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <tag> <counters...>
  local tag=$1; shift
  echo "=== pass $tag: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$tag" -o run -- \
    python scripts/micro.py --kernel "$K" --iters "$IT" > "$OUT/$tag.log" 2>&1
  local rc=$?
  tail -n 3 "$OUT/$tag.log"
  if [ $rc -ne 0 ]; then echo "pass $tag failed rc=$rc"; exit $rc; fi
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python scripts/micro.py --kernel "$K" --iters "$IT" > "$OUT/trace.log" 2>&1 || exit $?
tail -n 2 "$OUT/trace.log"
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
run sq2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
run tcc TCC_HIT_sum TCC_MISS_sum
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE
echo "pmc done"

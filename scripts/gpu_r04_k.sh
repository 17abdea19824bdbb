#!/bin/bash
# Term reverse (grr_bwd_term_fused) at the training shapes: msgf (B16 G32 F3) and the v1.0 levels at
# the C4 shape (B32; G8 F6 512^2 .. G32 F12 32^2), three modes; SQ counters of the widest v1.0 case
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04k; mkdir -p $out
export TMPDIR=/tmp
: > $out/micro.txt
for spec in "16 32 3 256" "16 32 3 128" "32 8 6 512" "32 8 6 256" "32 16 6 256" "32 16 6 128" "32 16 12 128" \
            "32 16 12 64" "32 32 12 64" "32 32 12 32"; do
  set -- $spec
  for mode in 0 1 2; do
    echo "B$1 G$2 F$3 S$4 mode$mode $(timeout -k 10 120 python -u scripts/micro.py --kernel term --batch $1 --graphs $2 \
      --fts $3 --size $4 --mode $mode --iters 10 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> $out/micro.txt || exit 1
  done
done
cat $out/micro.txt
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"; do
  tag=$(echo $ctr | cut -c1-12 | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex "term_row_kernel" --output-format csv -d $out/sq_$tag -o run -- \
    python scripts/micro.py --kernel term --batch 32 --graphs 8 --fts 6 --size 512 --mode 0 --iters 3 > $out/sq_$tag.log 2>&1 \
    || { echo "pmc $tag failed"; tail -5 $out/sq_$tag.log; exit 1; }
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python scripts/micro.py --kernel term --batch 32 \
  --graphs 8 --fts 6 --size 512 --mode 0 --iters 3 > $out/kt.log 2>&1 || { tail -5 $out/kt.log; exit 1; }
find $out/kt -name "*stats*" | head

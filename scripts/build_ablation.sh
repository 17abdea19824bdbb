#!/bin/bash
# Build exp/libgrr_exp{0..3}.so: the LNB tail with GRR_TAIL_EXP = 0 (product), 1 (no gate
# math), 2 (no MFMA), 3 (no in-loop DMA), 4 (no gate, no MFMA), 5 (4 + no in-loop DMA), 6 (4 with channel-blocked h addressing, timing only), 7 (0 with it).  Timed on the GPU by scripts/tail_ablation.sh.
set -eu
cd "$(dirname "$0")/.."
mkdir -p exp
H=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include"
S=imagerestoration-development-unrolling_amd/csrc
$H $F -c $S/graph_ops.hip -o exp/g.o
for n in 0 4 6 7; do
  $H $F -DGRR_TAIL_EXP=$n -c $S/feature_ops.hip -o exp/f$n.o
  $H --offload-arch=gfx950 -shared -fPIC -o exp/libgrr_exp$n.so exp/g.o exp/f$n.o
done
rm -f exp/*.o

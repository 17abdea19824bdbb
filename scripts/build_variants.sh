#!/bin/bash
# Build libgrr variants into exp/ for same-box A/B timing:
#   bash scripts/build_variants.sh NAME "-DMACRO=V ..." [NAME "-D..."]...
set -eu
cd "$(dirname "$0")/.."
mkdir -p exp
H=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include"
S=imagerestoration-development-unrolling_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  $H $F $defs -c $S/graph_ops.hip -o exp/g_$name.o &
  $H $F $defs -c $S/feature_ops.hip -o exp/f_$name.o &
  $H $F -fno-slp-vectorize $defs -c $S/lnb_ops.hip -o exp/l_$name.o &
  wait
  $H --offload-arch=gfx950 -shared -fPIC -o exp/libgrr_$name.so exp/g_$name.o exp/f_$name.o exp/l_$name.o
  rm -f exp/g_$name.o exp/f_$name.o exp/l_$name.o
done

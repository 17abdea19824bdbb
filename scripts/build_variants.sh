#!/bin/bash
# Build libgrr variants into exp/ for same-box A/B timing:
#   bash scripts/build_variants.sh NAME "-DMACRO=V ..." [NAME "-D..."]...
set -eu
cd "$(dirname "$0")/.."
mkdir -p exp
H=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include"
S=imagerestoration-development-unrolling_amd/csrc
SRCS="graph_ops feature_ops wgrad_ops lnb_ops graph_bwd lnb_bwd window_ops window_bwd subapi_ops subapi_bwd feature_edge"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  objs=""
  for src in $SRCS; do
    extra=""; { [ "$src" = lnb_ops ] || [ "$src" = graph_ops ]; } && extra=-fno-slp-vectorize
    $H $F $extra $defs -c $S/$src.hip -o exp/${src}_$name.o &
    objs="$objs exp/${src}_$name.o"
  done
  wait
  $H --offload-arch=gfx950 -shared -fPIC -o exp/libgrr_$name.so $objs
  rm -f $objs
done

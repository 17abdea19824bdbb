#!/bin/bash
# Same-box A/B of the default libgrr.so against exp/libgrr_$1.so on bench.py (2 rounds):
#   bash scripts/ab_lib.sh VARIANT [extra bench.py args]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab_$1
v=$1; shift
for r in 1 2; do
  for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_$v.so; do
    tag=$(basename $lib .so)
    GRR_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --breakdown "$@" \
      > gpurun_out/ab_$v/$tag.json 2> gpurun_out/ab_$v/$tag.err || exit 1
    echo "$tag $(python -c "import json;d=json.loads(open('gpurun_out/ab_$v/$tag.json').read().strip().splitlines()[-1]);k=d['kernel_ms_per_step'];print(d['value'], d['ms_per_step'], {x: k[x] for x in ('lnb','conv1x1','system_step2','edge_weights') if x in k})")"
  done
done

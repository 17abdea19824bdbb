#!/bin/bash
# term-row kernel at 3 waves/SIMD (default build) vs unconstrained registers (exp/libgrr_wpe1.so)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abtr
for r in 1 2; do
  for lib in imagerestoration-development-unrolling_amd/libgrr.so exp/libgrr_wpe1.so; do
    tag=$(basename $lib .so)
    GRR_LIB=$lib timeout -k 10 200 python bench_train.py --model msgf --batch 16 --steps 4 --warmup 2 --no-cpu-baseline --breakdown \
      > gpurun_out/abtr/$tag.json 2> gpurun_out/abtr/$tag.err || exit 1
    echo "$tag $(grep -E 'bwd_term_fused' gpurun_out/abtr/$tag.err) $(python -c "import json;d=json.loads(open('gpurun_out/abtr/$tag.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done

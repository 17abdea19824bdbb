#!/bin/bash
# term-row reverse: gw rows prefetched (GRR_TERM_GWP=2) vs read at the RMW (0), at 3 (default) or 2
# (b8: 512-thread bound, no spills) waves per SIMD; msgf training step, same box, two rounds
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abgwp
export TMPDIR=/tmp
for r in 1 2; do
  for tag in gwp0 gwp2 gwp0b8 gwp2b8; do
    GRR_LIB=exp/libgrr_$tag.so timeout -k 10 200 python bench_train.py --model msgf --batch 16 --steps 4 --warmup 2 --no-cpu-baseline --breakdown \
      > gpurun_out/abgwp/${tag}_$r.json 2> gpurun_out/abgwp/${tag}_$r.err || { tail gpurun_out/abgwp/${tag}_$r.err; exit 1; }
    echo "$tag $(grep -E 'bwd_term_fused' gpurun_out/abgwp/${tag}_$r.err | head -1) $(python -c "import json;d=json.loads(open('gpurun_out/abgwp/${tag}_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done

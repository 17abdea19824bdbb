#!/bin/bash
# round 6: depthwise / gate row kernels' segment rule A/B inside the C4 training step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06dseg; mkdir -p $out
export TMPDIR=/tmp
for cfg in ${CFGS:-4096:100000 4096:128 2048:128 4096:100000 4096:128 2048:128}; do
  mw=${cfg%%:*}; ms=${cfg#*:}
  GRR_DW3_MIN_WAVES=$mw GRR_DW3_MAX_SEG=$ms timeout -k 10 300 python -u bench_train.py --model abstract --size 512 --batch 32 \
    --steps 3 --warmup 1 --no-cpu-baseline > $out/train_c4_${mw}_$ms.json 2> $out/train_c4_${mw}_$ms.err || { tail $out/train_c4_${mw}_$ms.err; exit 1; }
  python -c "
import json;d=json.load(open('$out/train_c4_${mw}_$ms.json'));k=d['kernel_ms_per_step'];print('$mw $ms', d['ms_per_step'], 'gate_dw3_bwd', k['lnb_gate_dw3_bwd'], 'dw3_gate', k['lnb_dw3_gate'], 'term', k['bwd_term_fused'])"
done

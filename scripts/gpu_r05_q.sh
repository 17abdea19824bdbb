#!/bin/bash
# LNB gate + depthwise reverse through a per-wave LDS ring: tests, micro A/B, training lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05q}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dwconv.py \
  tests/test_gpu_deterministic.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u - > $out/ab.txt 2>&1 <<'PY' || { tail -20 $out/ab.txt; exit 1; }
import torch, irdu_amd
irdu_amd.load_native()
from irdu_amd import kernels as K
dev = torch.device("cuda", 0)
for (b, hid, h, w) in [(32, 96, 512, 512), (32, 192, 256, 256), (16, 256, 256, 256), (32, 384, 128, 128), (8, 192, 256, 256), (32, 768, 64, 64)]:
    hh = torch.randn(b, 2 * hid, h, w, device=dev); gq = torch.randn(b, hid, h, w, device=dev)
    wd = torch.randn(2 * hid, 9, device=dev); sc = torch.tensor([0.7], device=dev)
    gw = torch.zeros(2 * hid, 9, device=dev); gd = torch.zeros(1, device=dev)
    nb = 4 * (hh.numel() * 2 + gq.numel())
    res = {0: [], 1: []}
    for _ in range(2):
        for ring in (0, 1):
            K.set_lnb_bwd_ring(bool(ring))
            for _ in range(2): K.lnb_gate_dw3_bwd(None, gq, sc, hh, wd, gw, gd)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): K.lnb_gate_dw3_bwd(None, gq, sc, hh, wd, gw, gd)
            e1.record(); torch.cuda.synchronize()
            res[ring].append(e0.elapsed_time(e1) / 10)
    r0, r1 = min(res[0]), min(res[1])
    print(f"B{b} hid{hid} {h}x{w}: reg {r0:.4f} ms ({nb/r0/1e6:.0f} GB/s) ring {r1:.4f} ms ({nb/r1/1e6:.0f} GB/s) x{r0/r1:.3f}", flush=True)
    del hh, gq
K.set_lnb_bwd_ring(True)
PY
cat $out/ab.txt
if [ "${R05_TRAIN:-1}" = 1 ]; then
timeout -k 10 200 python -u bench_train.py --model msgf --batch 16 --steps 6 --warmup 2 --no-cpu-baseline \
  > $out/train_msgf.json 2> $out/train_msgf.err || { tail $out/train_msgf.err; exit 1; }
timeout -k 10 300 python -u bench_train.py --model abstract --batch 8 --steps 5 --warmup 2 --no-cpu-baseline \
  > $out/train_abstract.json 2> $out/train_abstract.err || { tail $out/train_abstract.err; exit 1; }
timeout -k 10 600 python -u bench_train.py --model abstract --size 512 --batch 32 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/train_c4.json 2> $out/train_c4.err || { tail $out/train_c4.err; exit 1; }
for f in train_msgf train_abstract train_c4; do echo "$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $out/$f.json | tr '\n' ' ')"; done
fi

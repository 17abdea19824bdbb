"""Build libgrr.so (the HIP kernels + C ABI) in-tree for gfx950 with hipcc.

    python imagerestoration-development-unrolling_amd/build_native.py [--force] [--verbose]

The shared library lands next to this file so it travels with the repo snapshot to
the GPU box (it is git-ignored, not gpurun-ignored).  Rebuilds only when a source
or header is newer than the library.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgrr.so")
SOURCES = ["graph_ops.hip", "feature_ops.hip", "lnb_ops.hip", "graph_bwd.hip", "lnb_bwd.hip", "window_ops.hip", "window_bwd.hip", "subapi_ops.hip", "subapi_bwd.hip", "wgrad_ops.hip", "feature_edge.hip"]
HEADERS = [os.path.join(CSRC, "grr_common.h"), os.path.join(ROOT, "include", "grr.h")]
ARCH = "gfx950"
# lnb_ops, graph_ops: no SLP packing of independent f32 FMAs into v_pk_fma_f32 (the packing
# needs register-pair moves that cost more than it saves, MI355X_MICROARCH.md; graph_step2_kernel:
# 1149 -> 1055 VALU instructions per iteration)
EXTRA_FLAGS = {"lnb_ops.hip": ["-fno-slp-vectorize"], "graph_ops.hip": ["-fno-slp-vectorize"]}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libgrr.so)")


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + HEADERS
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    objs, cmds = [], []
    for src in SOURCES:
        obj = os.path.join(CSRC, src.replace(".hip", ".o"))
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-Wno-unused-variable", "-I", os.path.join(ROOT, "include"), "-c",
               os.path.join(CSRC, src), "-o", obj] + EXTRA_FLAGS.get(src, [])
        if verbose:
            cmd.insert(2, "-Rpass-analysis=kernel-resource-usage")
            print(" ".join(cmd), flush=True)
        cmds.append(cmd)
        objs.append(obj)
    # one hipcc per source, in parallel (MAX_JOBS caps it, as on the GPU box)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 16))
    with ThreadPoolExecutor(jobs) as pool:
        for r in pool.map(lambda c: subprocess.run(c), cmds):
            if r.returncode != 0:
                raise subprocess.CalledProcessError(r.returncode, r.args)
    tmp = LIB + ".tmp"
    subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs, check=True)
    os.replace(tmp, LIB)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()
    print(build(force=args.force, verbose=args.verbose))
    sys.exit(0)

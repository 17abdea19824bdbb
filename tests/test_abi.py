"""CPU-only checks of the C ABI and the drop-in module surface (no kernel launches)."""
import os
import re

import numpy as np
import pytest
import torch

import irdu_amd
from irdu_amd import _native
from tests.golden_io import load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "grr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(grr_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_header_symbol():
    lib = _native.load()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), f"libgrr.so does not export {s}"
    assert set(syms) == set(_native.SIGNATURES), "ctypes signature table out of sync with include/grr.h"
    assert lib.grr_version() >= 1
    assert lib.grr_lnb_workspace_bytes(2, 96, 256, 64, 64) > 0
    # the fused C <= 96 block needs its chunk images only, far below the gated tensor's 2*256*64*64 floats
    assert 0 < lib.grr_lnb_fused_workspace_bytes(96, 256) < 4 * 2 * 256 * 64 * 64
    assert lib.grr_lnb_fused_workspace_bytes(128, 256) == 0


def test_python_mirrors_of_native_shape_queries():
    """kernels.feature_edges_ok / lnb_c8_ok are plain Python (traceable by Dynamo); they must agree with the
    library's own queries."""
    from irdu_amd import _native
    from irdu_amd import kernels as K
    lib = _native.load()
    for c, g, f, h, w in [(96, 32, 3, 256, 256), (96, 32, 3, 128, 128), (15, 5, 3, 9, 29), (96, 16, 6, 64, 64),
                          (99, 33, 3, 8, 8), (48, 16, 3, 1, 1), (12, 4, 3, 8192, 8192), (6, 2, 3, 3, 5)]:
        assert K.feature_edges_ok(c, g, f, h, w) == bool(lib.grr_feature_edges_supported(c, g, f, h, w)), (c, g, f)
    for c, hid in [(96, 256), (97, 256), (2, 1), (1, 4), (64, 128)]:
        assert K.lnb_c8_ok(c, hid, 64, 64) == bool(lib.grr_lnb_fused(c, hid)), (c, hid)


def test_invalid_args_report_status_without_gpu():
    lib = _native.load()
    st = lib.grr_pool2(None, None, 1, 1, 4, 4, None)
    assert st == 1  # GRR_ERR_INVALID_ARG, validated before any launch
    assert b"bad args" in lib.grr_last_error()
    with pytest.raises(_native.GrrError):
        _native.call("grr_neighbor_table", None, 4, 4, None)


def test_odd_shape_rejected_like_the_reference():
    lib = _native.load()
    # grr_pool2 with odd H: the reference's view() after the 2x2 conv fails too (REF:665)
    st = lib.grr_pool2(ctypes_ptr(), ctypes_ptr(), 1, 1, 5, 4, None)
    assert st == 2


def ctypes_ptr():
    return 0x1000  # never dereferenced: validation fails first


def test_cpu_tensors_fail_loudly():
    m = irdu_amd.GLRFast(3, 2, M_diag_init=1.0)
    with pytest.raises(RuntimeError, match="GPU"):
        m.extract_edge_weights(torch.randn(1, 2, 3, 8, 8))


def _keys_from_golden(name):
    d = load_golden(name)
    return [k[2:] for k in d.files if k.startswith("p/")], d


def test_state_dict_keys_match_reference_mixture():
    keys, d = _keys_from_golden("mixture_v1.npz")
    g = int(d["meta/n_graphs"])
    m = irdu_amd.MixtureGTVGLR(g, 12 // g, 0.5, 0.1, torch.tensor([[0.001], [0.0001]]),
                               torch.tensor([[0.0001], [0.0001]]), torch.tensor([[0.0001], [0.0001]]))
    sd = m.state_dict()
    assert list(sd.keys()) == keys
    m.load_state_dict({k: torch.from_numpy(d["p/" + k]) for k in keys})
    for k in keys:
        assert tuple(sd[k].shape) == d["p/" + k].shape


def test_state_dict_keys_match_reference_abstract_and_msgf():
    keys, d = _keys_from_golden("abstract_v1.npz")
    cfg = {k[5:]: d[k] for k in d.files if k.startswith("meta/") and k != "meta/n_state_keys"}
    m = irdu_amd.AbtractMultiScaleGraphFilter(
        n_channels_in=3, n_channels_out=3, dims=cfg["dims"].tolist(), hidden_dims=cfg["hidden_dims"].tolist(),
        nsubnets=cfg["nsubnets"].tolist(), ngraphs=cfg["ngraphs"].tolist(), num_blocks=cfg["num_blocks"].tolist(),
        num_blocks_out=int(cfg["num_blocks_out"]))
    assert list(m.state_dict().keys()) == keys
    m.load_state_dict({k: torch.from_numpy(d["p/" + k]) for k in keys}, strict=True)

    keys, d = _keys_from_golden("msgf_v13.npz")
    m = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=int(d["meta/n_graphs"]))
    assert list(m.state_dict().keys()) == keys


def test_stage_count_parameter_shapes():
    m = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=32, n_cgd_iters=10)
    assert tuple(m.localfilter.alphaCGD.shape) == (10, 32)
    assert tuple(m.localfilter.betaCGD.shape) == (10, 32)
    # non-persistent constants follow .to() but stay out of the state_dict
    assert "localfilter.scaling_kernel01" not in m.state_dict()
    assert m.localfilter.GLRmodule00.edge_delta.dtype == torch.int32
    assert np.array_equal(m.localfilter.GLRmodule00.edge_delta.numpy(), [[-1, 0], [0, -1], [0, 1], [1, 0]])


def test_import_leaves_the_environment_unchanged():
    """Importing the package sets no process-wide variable (MIOpen's find-db default belongs to the
    training entry points: irdu_amd.miopen_training_defaults, training.main, bench_train.py)."""
    import subprocess
    import sys
    code = ("import os, sys; sys.path.insert(0, %r); before = dict(os.environ); import irdu_amd; "
            "after = dict(os.environ); d = {k for k in set(before) | set(after) if before.get(k) != after.get(k)}; "
            "print(sorted(d)); sys.exit(1 if d else 0)") % ROOT
    env = {k: v for k, v in os.environ.items() if not k.startswith("MIOPEN_")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run([sys.executable, "-c", "import os, sys; sys.path.insert(0, %r); import irdu_amd; "
                        "irdu_amd.miopen_training_defaults(); print(os.environ['MIOPEN_DEBUG_DISABLE_FIND_DB'])" % ROOT],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "1", r.stdout + r.stderr


def test_scratch_allocator_is_registered_and_empty_without_gpu():
    lib = _native.load()
    assert lib.grr_scratch_bytes() == 0
    assert lib.grr_release_scratch() == 0
    assert lib.grr_set_scratch_allocator(None, 0x1000, None) == 1   # one function without the other


def test_wgrad_tile_plan_without_gpu():
    """grr_wgrad's host plan (no launch): the per-shape tile makes the v1.0 first level's 192 x 48 gradient
    one output tile per pixel chunk instead of two, so it plans twice the chunks (and workspace) of the
    128 x 96 tile at the same wave budget; a 512 x 96 output keeps the 128 x 96 tile either way."""
    lib = _native.load()
    try:
        lib.grr_wgrad_set_tiles(0)
        base_small = lib.grr_wgrad_workspace_bytes(32, 192, 48, 512 * 512)
        base_wide = lib.grr_wgrad_workspace_bytes(16, 512, 96, 256 * 256)
        lib.grr_wgrad_set_tiles(1)
        tiled_small = lib.grr_wgrad_workspace_bytes(32, 192, 48, 512 * 512)
        tiled_wide = lib.grr_wgrad_workspace_bytes(16, 512, 96, 256 * 256)
    finally:
        lib.grr_wgrad_set_tiles(1)
    assert tiled_small > base_small > 0
    assert tiled_wide == base_wide > 0


def test_dw3_ring_dma_geometry_replay():
    """The gate + depthwise reverse ring kernel's DMAs stay inside their ring row and image row at every width
    it takes (W % 4 == 0), including round 5's faulting case W = 32 (V = 1) and the C4 width 512 (strips)."""
    from irdu_amd import _native
    lib = _native.load()
    for w in list(range(4, 1028, 4)) + [32, 100, 256, 300, 512, 744]:
        if w % 4 == 0:
            assert lib.grr_dw3_ring_check(w) == 0, (w, lib.grr_last_error())
    assert lib.grr_dw3_ring_check(30) != 0          # W % 4 != 0 is not a ring shape

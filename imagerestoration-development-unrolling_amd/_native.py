"""ctypes binding of libgrr.so (include/grr.h).

The product path has exactly one implementation: the HIP kernels in this library.
If the library is missing or cannot be loaded, every op raises NativeUnavailable —
there is no CPU or eager-PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_int, c_int64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GRR_LIB", os.path.join(HERE, "libgrr.so"))


class NativeUnavailable(RuntimeError):
    """libgrr.so could not be loaded (build it with build_native.py)."""


class GrrError(RuntimeError):
    """A libgrr.so call returned a non-OK grr_status."""

    def __init__(self, fn: str, status: int, msg: str):
        super().__init__(f"{fn} failed (status {status}): {msg}")
        self.status = status


STATUS_NAMES = {0: "GRR_OK", 1: "GRR_ERR_INVALID_ARG", 2: "GRR_ERR_SHAPE", 3: "GRR_ERR_UNSUPPORTED", 4: "GRR_ERR_HIP"}


class Stencil(ctypes.Structure):
    """grr_stencil: the four [C] stencil parameter vectors of one GLR/GTV module."""
    _fields_ = [("p01", c_void_p), ("p02a", c_void_p), ("p02b", c_void_p), ("p03", c_void_p)]


P = c_void_p
I = c_int
L = c_int64
Fl = ctypes.c_float

# name -> argtypes (restype is grr_status == int unless listed in _RESTYPES)
SIGNATURES = {
    "grr_version": [],
    "grr_last_error": [],
    "grr_set_kernel_variant": [I],
    "grr_lnb_set_phases": [I],
    "grr_lnb_rep_fused": [I, I, I, I],
    "grr_set_scratch_allocator": [P, P, P],
    "grr_release_scratch": [],
    "grr_scratch_bytes": [],
    "grr_neighbor_table": [P, I, I, P],
    "grr_stream_copy": [P, P, L, P],
    "grr_edge_weights": [P, L, P, P, P, I, I, I, I, I, P],
    "grr_gtv_pair_weights": [P, P, I, I, I, I, P],
    "grr_edge_weights_block": [P, L, I, P, I, P, P, P, P, I, I, I, I, I, P],
    "grr_pool2": [P, P, I, I, I, I, P],
    "grr_system_half": [P, P, P, Stencil, Stencil, P, P, P, I, I, I, I, I, P],
    "grr_gtv_rhs_half": [P, P, Stencil, I, P, P, I, I, I, I, I, P],
    "grr_gtv_rhs_full": [P, P, P, Stencil, I, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_gtv_rhs_full_rep": [P, I, P, I, P, Stencil, I, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_system_step": [P, P, P, P, P, P, Stencil, Stencil, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_system_step2": [P, P, P, P, P, P, Stencil, Stencil, P, P, P, P, Stencil, Stencil, P, P, P, P, P, P, P, P,
                         P, P, P, I, I, I, I, I, P],
    "grr_system_first_pair": [P, P, P, I, P, P, P, Stencil, Stencil, P, P, P, P, P, P, Stencil, Stencil, P, P, P, P, P,
                              P, P, P, P, I, I, I, I, I, P],
    "grr_system_step2_train": [P, P, P, P, P, P, Stencil, Stencil, P, P, P, P, Stencil, Stencil, P, P, P, P, P, P,
                               P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_glr_stage": [P, P, P, P, Stencil, P, P, P, P, P, I, I, I, I, I, P],
    "grr_conv1x1": [P, P, P, I, I, I, L, P],
    "grr_conv1x1_workspace_bytes": [I, I],
    "grr_conv1x1_ws": [P, P, P, P, I, I, I, L, P],
    "grr_conv2x2s2": [P, P, P, I, I, I, I, I, P],
    "grr_ffn_workspace_bytes": [I, I, I, I, I],
    "grr_ffn_forward": [P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_wgrad_workspace_bytes": [I, I, I, L],
    "grr_wgrad_set_tiles": [I],
    "grr_wgrad": [P, P, P, P, I, I, I, L, P],
    "grr_lnb_workspace_bytes": [I, I, I, I, I],
    "grr_lnb_forward": [P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_lnb_forward_keep": [P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_lnb_forward_c8": [P, P, P, P, P, P, P, P, I, I, I, I, I, I, P],
    "grr_c8_convert": [P, P, I, I, I, I, I, P],
    "grr_feature_edges_supported": [I, I, I, I, I],
    "grr_feature_edges_workspace_bytes": [I],
    "grr_feature_edges": [P, I, P, P, P, P, P, P, P, I, I, I, I, I, I, P],
    "grr_lnb_fused": [I, I],
    "grr_lnb_fused_workspace_bytes": [I, I],
    "grr_lnb_set_fused": [I],
    "grr_dw3_ring_check": [I],
    "grr_repeat_graphs": [P, P, I, I, I, L, P],
    "grr_lnb_forward_rep": [P, I, I, P, P, P, P, P, P, P, P, I, I, I, I, P],
    # GLRFast / GTVFast sub-API
    "grr_neighbor_gather": [P, P, I, I, I, I, P],
    "grr_normalize_features": [P, P, P, I, I, I, I, I, P],
    "grr_stats_conv": [P, Stencil, I, P, I, I, I, I, I, P],
    "grr_glr_op_l_norm": [P, P, P, I, I, I, I, I, P],
    "grr_gtv_op_c": [P, P, Stencil, P, I, I, I, I, I, P],
    "grr_gtv_op_c_transpose": [P, P, Stencil, P, P, I, I, I, I, I, P],
    "grr_neighbor_gather_bwd": [P, P, I, I, I, I, P],
    "grr_normalize_features_bwd": [P, P, P, P, P, I, I, I, I, I, P],
    "grr_stats_conv_bwd": [P, Stencil, I, P, P, P, I, I, I, I, I, P],
    "grr_glr_op_l_norm_bwd": [P, P, P, P, P, I, I, I, I, I, P],
    "grr_gtv_op_c_bwd": [P, P, Stencil, P, P, P, P, P, I, I, I, I, I, P],
    "grr_gtv_op_c_transpose_bwd": [P, P, Stencil, P, P, P, P, P, P, I, I, I, I, I, P],
    # reverse pass
    "grr_bwd_stencil": [P, P, I, P, I, P, I, I, I, I, I, P],
    "grr_bwd_tapgrad": [P, P, I, P, P, I, I, I, I, I, P],
    "grr_bwd_padj2": [P, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_bwd_glr": [P, P, P, P, Fl, P, P, P, P, I, I, I, I, I, P],
    "grr_bwd_pair": [P, P, P, P, Fl, P, P, P, P, I, I, I, I, I, P],
    "grr_bwd_prox": [P, P, P, P, P, Fl, P, P, P, P, P, I, I, I, I, I, P],
    "grr_bwd_set_term_rows": [I],
    "grr_bwd_set_term_tail": [I],
    "grr_bwd_set_term_acc_max_w": [I],
    "grr_lnb_set_bwd_ring": [I],
    "grr_bwd_term_fused": [I, P, P, P, P, P, P, Fl, P, P, P, P, P, I, I, I, I, I, P],
    "grr_bwd_term_acc_supported": [I, I, I, I],
    "grr_bwd_term_fused_acc": [I, P, P, P, P, P, P, Fl, P, P, P, P, P, I, I, I, I, I, P],
    "grr_bwd_pair_weights": [P, P, P, I, I, I, I, P],
    "grr_bwd_edge_weights": [P, L, P, P, P, P, L, P, I, I, I, I, I, P],
    "grr_bwd_graph_dot": [P, P, Fl, P, I, I, I, I, I, P],
    "grr_bwd_lincomb": [P, P, P, P, P, I, I, I, I, I, I, P],
    "grr_bwd_cg_glue": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_bwd_cg_glue_pool": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_bwd_unpool2_acc": [P, P, I, I, I, I, P],
    "grr_conv2x2s2_bwd_data": [P, P, P, I, I, I, I, I, P],
    "grr_interleave2x2": [P, P, I, I, I, I, P],
    "grr_lnb_norm": [P, P, P, P, I, I, L, P],
    "grr_lnb_norm_bwd": [P, P, P, P, P, P, I, I, L, P],
    "grr_lnb_norm_bwd_skip": [P, P, P, P, P, P, P, P, P, I, I, L, P],
    "grr_dwconv3": [P, P, P, I, I, I, I, P],
    "grr_dwconv3_bwd": [P, P, P, P, P, I, I, I, I, P],
    "grr_lnb_gate": [P, P, P, P, I, I, L, P],
    "grr_lnb_gate_bwd_scaled": [P, P, P, P, P, I, I, L, P],
    "grr_lnb_gate_dw3_bwd": [P, P, P, P, P, P, P, P, I, I, I, I, P],
    "grr_lnb_dw3_gate": [P, P, P, I, I, I, I, P],
    "grr_ffn_dw3_gate": [P, P, P, I, I, I, I, P],
    "grr_ffn_gate_dw3_bwd": [P, P, P, P, P, P, P, I, I, I, I, P],
    # window graphs (REF7 / REF1)
    "grr_win_edge_weights": [P, L, P, P, I, P, P, I, I, I, I, I, P],
    "grr_win_solver": [I, P, I, P, P, P, P, P, P, P, P, P, P, P, P, I, P, P, I, I, I, I, I, P],
    "grr_win_mix": [P, P, P, P, I, I, I, I, I, P],
    "grr_win_pair_weights": [P, P, I, P, I, I, I, I, P],
    "grr_win_bwd_stencil": [P, P, I, P, I, P, I, I, I, I, I, P],
    "grr_win_bwd_tapgrad": [P, P, I, P, P, I, I, I, I, I, P],
    "grr_win_bwd_glr": [P, P, P, P, I, P, Fl, P, P, P, P, P, I, I, I, I, I, P],
    "grr_win_bwd_gtv": [P, P, P, P, I, I, P, P, Fl, P, P, P, P, P, P, I, I, I, I, I, P],
    "grr_win_bwd_gather": [P, P, P, I, P, P, I, I, I, I, I, P],
    "grr_win_bwd_gather_fused": [P, P, P, P, I, I, I, P, P, P, P, I, I, I, I, I, P],
    "grr_win_bwd_edge_weights": [P, L, P, P, P, P, I, P, L, P, I, I, I, I, I, P],
    "grr_win_bwd_mix": [P, P, P, P, P, I, I, I, I, I, P],
}
_RESTYPES = {"grr_version": c_int, "grr_last_error": ctypes.c_char_p, "grr_lnb_workspace_bytes": c_int64,
             "grr_conv1x1_workspace_bytes": c_int64, "grr_wgrad_workspace_bytes": c_int64,
             "grr_ffn_workspace_bytes": c_int64, "grr_scratch_bytes": c_int64,
             "grr_lnb_fused_workspace_bytes": c_int64, "grr_feature_edges_workspace_bytes": c_int64}

_lib = None


def load() -> ctypes.CDLL:
    """Load libgrr.so once and bind every symbol of include/grr.h."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable(
            f"{LIB_PATH} not found: build it with `python imagerestoration-development-unrolling_amd/build_native.py`")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the host
        raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, c_int)
    _register_scratch_allocator(lib)
    _lib = lib
    return lib


# The training reverse's reduction scratch (grr_set_scratch_allocator): PyTorch's caching allocator, on
# the stream the library asks for, so the scratch is ordinary PyTorch memory (torch.cuda.memory_allocated
# counts it, empty_cache can return it once grr_release_scratch gave it back).  The callbacks run only
# when a stream's scratch first appears or grows (a handful of times per process).
_SCRATCH_ALLOC_FN = ctypes.CFUNCTYPE(c_void_p, ctypes.c_uint64, c_int, c_void_p, c_void_p)
_SCRATCH_FREE_FN = ctypes.CFUNCTYPE(None, c_void_p, c_int, c_void_p, c_void_p)


def _scratch_alloc(nbytes, device, stream, _ctx):
    try:
        import torch
        return int(torch.cuda.caching_allocator_alloc(int(nbytes), device, int(stream or 0)))
    except Exception:      # noqa: BLE001 -- the library reports the failed allocation as GRR_ERR_HIP
        return None


def _scratch_free(ptr, _device, _stream, _ctx):
    try:
        import torch
        torch.cuda.caching_allocator_delete(int(ptr))
    except Exception:      # noqa: BLE001
        pass


_scratch_cbs = (_SCRATCH_ALLOC_FN(_scratch_alloc), _SCRATCH_FREE_FN(_scratch_free))   # kept alive


def _register_scratch_allocator(lib) -> None:
    st = lib.grr_set_scratch_allocator(ctypes.cast(_scratch_cbs[0], c_void_p), ctypes.cast(_scratch_cbs[1], c_void_p),
                                       None)
    if st != 0:   # pragma: no cover
        raise NativeUnavailable(f"grr_set_scratch_allocator failed: {lib.grr_last_error()!r}")


def release_scratch() -> None:
    """Give the reverse's reduction scratch back to PyTorch's cache (synchronises the device first)."""
    import torch
    torch.cuda.synchronize()
    call("grr_release_scratch")


def call(name: str, *args) -> None:
    """Call a status-returning entry point; raise GrrError on failure."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != 0:
        msg = lib.grr_last_error()
        raise GrrError(name, st, (msg or b"").decode(errors="replace"))

"""Debug guard for the internal-stream invariant: only libgrr kernels (and trivial ATen work) run on
the side and level streams.

Why: the feature branch (graph_filter._side_stream, inference and training) and the solver reverse's
half level (solver_grad._level_side) run on internal HIP streams beside the caller's.  A library kernel
whose workgroups wait on other workgroups of the same launch (hipBLASLt stream-K GEMMs, some MIOpen
convolutions) assumes all of them become resident; two of them on two streams, or one beside our
one-workgroup-per-CU kernels, can wait on each other forever ("Side-stream stall").
libgrr kernels never wait across workgroups, so the streams are safe as long as nothing else lands on
them.  Nothing in the Python code enforces that by construction -- a future torch op on those streams
would silently bring the hazard back -- so this mode checks it.

``with stream_guard(): ...`` (or ``GRR_STREAM_GUARD=1``, which wraps ``training.Trainer.step``)
installs a TorchDispatchMode.  The mode stays active in autograd's backward (its thread-local state
travels with the graph task), so the reverse is checked too.  While an internal stream is the current
stream, an ATen op must be

* a view or metadata op, an allocation, fill, zero or copy,
* a pointwise op (``torch.Tag.pointwise``) or a plain reduction (``torch.Tag.reduction``), or
* an ``irdu::`` custom op (the opaque HIP nodes under torch.compile);

anything else (mm / addmm / bmm / convolution / MIOpen / hipBLASLt ...) raises
:class:`StreamInvariantError` naming the op and the stream.  The libgrr launches themselves go through
ctypes, not the dispatcher, so the mode never sees them.
"""
from __future__ import annotations

import contextlib
import os

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ENV = os.environ.get("GRR_STREAM_GUARD", "0") == "1"

_TRIVIAL = {
    "empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided", "zeros", "zeros_like",
    "new_zeros", "ones", "ones_like", "new_ones", "full", "full_like", "new_full", "scalar_tensor",
    "fill", "fill_", "zero", "zero_", "copy", "copy_", "clone", "_to_copy", "lift_fresh", "lift_fresh_copy",
    "detach", "alias", "view", "_unsafe_view", "reshape", "as_strided", "slice", "select", "unsqueeze",
    "squeeze", "permute", "expand", "t", "transpose", "unbind", "split", "split_with_sizes", "chunk",
    "narrow", "contiguous", "record_stream", "set_", "resize_", "_local_scalar_dense", "cat", "stack",
    "flip", "_pin_memory", "is_pinned", "index_select", "masked_fill", "masked_fill_",
}


class StreamInvariantError(RuntimeError):
    pass


def internal_streams():
    """CUDA stream handles of the internal side / level streams created so far."""
    from . import graph_filter, solver_grad
    return {s.cuda_stream for s in (*graph_filter._SIDE_STREAMS.values(), *solver_grad._LEVEL_SIDE.values())}


def allowed(func) -> bool:
    if func.namespace == "irdu":
        return True
    name = func._schema.name.split("::")[-1]
    if name in _TRIVIAL or func.is_view:
        return True
    tags = func.tags
    return torch.Tag.pointwise in tags or torch.Tag.reduction in tags


class StreamGuardMode(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.checked = 0        # ops seen on an internal stream (the tests assert the guard looked)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            cur = torch.cuda.current_stream().cuda_stream
            if cur in internal_streams():
                self.checked += 1
                if not allowed(func):
                    raise StreamInvariantError(
                        f"irdu_amd: {func} ran on an internal side/level stream (0x{cur:x}); only libgrr kernels "
                        f"and trivial ATen ops may run there (stream_guard.py)")
        return func(*args, **kwargs)


@contextlib.contextmanager
def stream_guard():
    """Check the internal-stream invariant for everything run inside (forward and backward)."""
    mode = StreamGuardMode()
    with mode:
        yield mode


def maybe_guard():
    """``stream_guard()`` when GRR_STREAM_GUARD=1, else a no-op context."""
    return stream_guard() if ENV else contextlib.nullcontext()

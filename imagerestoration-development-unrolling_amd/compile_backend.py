"""``model.compile()`` without code generation (no Triton).

The reference compiles its model and trains the compiled module
(scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:130, :186-207).  nn.Module.compile defaults
to Inductor, which code-generates Triton kernels for every ATen op it can fuse -- here the stock
encoder / decoder ops and the losses around the HIP graph filter (replicate pad, cat, MSE / L1).
The build uses no Triton, so every drop-in module derives from :class:`HipModule`, whose
``compile()`` maps the default (Inductor) backend to ``irdu_hip``:

* Dynamo captures the Python-level graph as usual (the HIP ops appear as opaque ``irdu::`` custom
  ops, ops.py / train_ops.py);
* AOTAutograd builds the joint forward / backward graphs and partitions them;
* the compiled forward and backward graphs run their nodes as they are -- the ``irdu::`` nodes on
  libgrr.so, the stock ops on their ATen (MIOpen / hipBLASLt / PyTorch-ROCm) kernels.  Nothing is
  generated, so ``torch._inductor.metrics.generated_kernel_count`` stays 0.

Any other backend passed explicitly (``"cudagraphs"``, ``"aot_eager"``, a callable) is honoured
unchanged; ``backend="inductor"`` is mapped as well, since a Triton backend is not part of the build.
"""
from __future__ import annotations

import torch
import torch.nn as nn

BACKEND = "irdu_hip"
_INDUCTOR_ONLY = ("mode", "options")
_registered = False


def _boxed_nop(gm: torch.fx.GraphModule, example_inputs):
    from functorch.compile import make_boxed_func
    return make_boxed_func(gm.forward)


def register() -> str:
    """Register the ``irdu_hip`` Dynamo backend (idempotent); returns its name."""
    global _registered
    if not _registered:
        from torch._dynamo.backends.common import aot_autograd
        from torch._dynamo.backends.registry import register_backend
        register_backend(name=BACKEND, compiler_fn=aot_autograd(
            fw_compiler=_boxed_nop, bw_compiler=_boxed_nop, inference_compiler=_boxed_nop,
            keep_inference_input_mutations=True))
        _registered = True
    return BACKEND


def resolve(kwargs: dict) -> dict:
    """torch.compile keyword arguments with the Inductor default replaced by ``irdu_hip``."""
    kwargs = dict(kwargs)
    backend = kwargs.get("backend", "inductor")
    if backend is None or backend == "inductor":
        kwargs["backend"] = register()
        for k in _INDUCTOR_ONLY:       # Inductor tuning knobs have no meaning without Inductor
            kwargs.pop(k, None)
    return kwargs


class HipModule(nn.Module):
    """nn.Module whose ``compile()`` never selects Inductor (see the module docstring)."""

    def compile(self, *args, **kwargs):
        return super().compile(*args, **resolve(kwargs))


def compile(model, **kwargs):
    """``torch.compile(model, ...)`` with the same backend mapping as ``HipModule.compile``."""
    return torch.compile(model, **resolve(kwargs))

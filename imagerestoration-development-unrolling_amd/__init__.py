"""irdu_amd — MI355X-native engine for the GGTV/GGLR unrolled graph-filter path of
tamthuc1995/ImageRestoration-Development-Unrolling.

Import as ``irdu_amd`` (the root-level ``irdu_amd.py`` loader maps this hyphenated
directory to that package name).  The public surface mirrors the reference's
module ``deep_multiscale_GGLR_GGTV_v1x0`` so callers can swap the import:

    import irdu_amd as model_structure
    model = model_structure.AbtractMultiScaleGraphFilter(...).cuda()

Importing changes no process-wide setting.  A drop-in training script with its own loop calls
``irdu_amd.miopen_training_defaults()`` before its first convolution (MIOpen's find-db otherwise costs
seconds of host time per step on the v1.0 model's stock convolutions after a box's first run,
DESIGN.md §4.r4); the first training-mode forward of AbtractMultiScaleGraphFilter warns once when
MIOPEN_DEBUG_DISABLE_FIND_DB is unset.
"""
from ._native import GrrError, NativeUnavailable, load as load_native  # noqa: F401
from .graph_filter import (  # noqa: F401
    AbtractMultiScaleGraphFilter,
    CustomLayerNorm,
    Downsampling,
    GLRFast,
    GTVFast,
    LocalGatedLinearBlock,
    LocalLowpassFilteringBlock,
    LocalNonLinearBlock,
    MixtureGTVGLR,
    MultiScaleGraphFilter,
    ReginalPixelEmbeding,
    Upsampling,
)
from . import kernels  # noqa: F401
from . import glr_v10 as v10  # noqa: F401  (GLR-only drop-ins of lib/model_GLR_GTV_deep_v10.py)
from .glr_v10 import GLRImageFilter, MixtureGLR, MultiScaleGLRImageFilter, MultiScaleMixtureGLR  # noqa: F401
from . import window_graph  # noqa: F401  (window-graph MixtureGTV of lib/model_GLR_GTV_deep_v7.py)
from . import window_graph_v1  # noqa: F401  (multiblock window denoiser of lib/model_GLR_GTV_deep_v1.py)

from .training import miopen_training_defaults  # noqa: F401

__version__ = "0.1.0"

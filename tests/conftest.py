import os
import sys

# The v1.0 encoder/decoder's plain convolutions run on MIOpen; its exhaustive first-call "find"
# at the C4 shapes (32 x 512^2, up to 384 channels, forward + both backward passes) takes minutes.
# The fast find mode picks an algorithm without benchmarking them all (set before MIOpen loads).
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
# the training entry points' process-wide MIOpen setting (irdu_amd.miopen_training_defaults): the test
# session is such an entry point (GPU training tests run the v1.0 model's stock convolutions)
os.environ.setdefault("MIOPEN_DEBUG_DISABLE_FIND_DB", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")

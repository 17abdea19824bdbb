"""Drop-in v1.0 AbtractMultiScaleGraphFilter (trained dims, S=10) forward only, for rocprofv3 kernel
stats: which kernels the end-to-end model spends its time in (HIP vs stock PyTorch-ROCm)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import D_CFG, STAGES, synthetic_patches  # noqa: E402


def main():
    import irdu_amd
    irdu_amd.load_native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(2204)
    m = irdu_amd.AbtractMultiScaleGraphFilter(3, 3, n_cgd_iters=STAGES, **D_CFG).to(dev).eval()
    _, noisy = synthetic_patches(16, seed=7)
    noisy = noisy.to(dev)
    import time
    with torch.no_grad():
        for _ in range(3):
            m(noisy)
        torch.cuda.synchronize()
        time.sleep(0.5)   # marks the steady-state region in the kernel trace (gap > 0.3 s)
        for _ in range(2):
            m(noisy)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()

"""Experiment: the 64-patch bench batch as K chunks on K HIP streams (MFMA-bound feature CNN of
one chunk overlapping the HBM-bound solver of another) vs one stream."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import build_model, synthetic_patches  # noqa: E402


def main():
    import irdu_amd
    irdu_amd.load_native()
    dev = torch.device("cuda", 0)
    m = build_model(dev)
    _, noisy = synthetic_patches(64, seed=1)
    noisy = noisy.to(dev)
    for k in (1, 2, 4):
        streams = [torch.cuda.Stream(dev) for _ in range(k)]
        chunks = noisy.chunk(k)

        def run():
            main_s = torch.cuda.current_stream(dev)
            outs = []
            for s, c in zip(streams, chunks):
                s.wait_stream(main_s)
                with torch.cuda.stream(s), torch.no_grad():
                    outs.append(m(c))
            for s in streams:
                main_s.wait_stream(s)
            return outs

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        print(f"streams={k}: {dt * 1e3:.2f} ms/step  {64 * 256 * 256 / dt / 1e6:.1f} MPix/s", flush=True)


if __name__ == "__main__":
    main()

"""Time the oracle restatement against the reference itself on the same CPU, same weights and
inputs ("record the restatement/oracle time ratio at the same shapes, ≈ 1").

Build container only (imports the read-only reference; never runs on the GPU box):
    python scripts/calibrate_oracle.py [--ref /root/reference] [--size 128] [--graphs 32] [--runs 3]
Prints one JSON line.  The reference's MultiScaleGraphFilter hard-codes 3 unrolled stages, so
the ratio is measured at S = 3 (the S = 10 bench path repeats the same stage op sequence).
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--graphs", type=int, default=32)
    ap.add_argument("--runs", type=int, default=3)
    args = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(args.ref, "exploration", "model_multiscale_mixture_GLR", "lib"))
    import model_GLR_GTV_deep_v13_no_latent as v13  # noqa: E402
    from oracle import graph_oracle as O
    torch.set_num_threads(os.cpu_count())
    torch.manual_seed(2204)
    ref = v13.MultiScaleGraphFilter(n_channels_in=3, n_channels_out=3, ngraphs=args.graphs).eval()
    state = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    x = torch.rand(args.batch, 3, args.size, args.size)

    def timed(fn):
        with torch.no_grad():
            fn()
            ts = []
            for _ in range(args.runs):
                t0 = time.perf_counter()
                out = fn()
                ts.append(time.perf_counter() - t0)
        return statistics.median(ts), out

    t_ref, y_ref = timed(lambda: ref(x))
    t_orc, y_orc = timed(lambda: O.multiscale_graph_filter(x, state, args.graphs, n_stages=3))
    rel = float((y_orc.double() - y_ref.double()).abs().max() / y_ref.double().abs().max())
    print(json.dumps({"shape": [args.batch, 3, args.size, args.size], "graphs": args.graphs, "stages": 3,
                      "threads": torch.get_num_threads(), "reference_s": round(t_ref, 3),
                      "oracle_s": round(t_orc, 3), "ratio_oracle_over_reference": round(t_orc / t_ref, 3),
                      "rel_err": rel, "runs": args.runs}))


if __name__ == "__main__":
    main()

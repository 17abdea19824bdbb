"""Train the bench's image filter briefly so PSNR parity is measured on weights that denoise.

    python scripts/train_psnr_fixture.py [--iters 3000] [--batch 8] [--size 256] [--out tests/golden/...]

Model: bench.build_model (MultiScaleGraphFilter G=32 F=3 S=10, v13 feature CNN, reference init,
1x1 output = per-colour graph mean).  Data: the synthetic sigma=25 patch pairs of the training
engine (training.SyntheticNoisyPatches, 256x256 RGB).  Loop: the reference's v2 script on the
HIP forward + reverse (L1 loss, Adam lr 4e-4, scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py
:146-207).  Writes the state_dict as safetensors (a weights-only fixture) and prints the PSNR
of the noisy input and of the filter on held-out patches every --eval-every iterations.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--lr", type=float, default=4e-4)
    ap.add_argument("--eval-every", type=int, default=250)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--copy-to", default=os.path.join(ROOT, "gpurun_out", "msgf_trained_g32_s10.safetensors"))
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "msgf_trained_g32_s10.safetensors"))
    args = ap.parse_args()
    import irdu_amd
    from irdu_amd import training as T
    from bench import build_model
    from safetensors.torch import save_file
    irdu_amd.load_native()
    dev = torch.device("cuda", 0)
    model = build_model(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=args.lr, eps=1e-8)
    ds = T.SyntheticNoisyPatches(lambda_noise=25.0, patch_size=args.size, max_num_patchs=args.iters * args.batch,
                                 n_channels=3, seed=31)
    loader = torch.utils.data.DataLoader(ds, batch_size=args.batch, num_workers=args.workers, drop_last=True,
                                         persistent_workers=args.workers > 0)
    held = T.SyntheticNoisyPatches(lambda_noise=25.0, patch_size=args.size, max_num_patchs=8, n_channels=3,
                                   seed=4242)
    hn, hc = (torch.stack(t).permute(0, 3, 1, 2).contiguous().to(dev) for t in zip(*[held[i] for i in range(8)]))

    def psnr(x, c):
        r = torch.round(x.clamp(0, 1).double() * 255.0)
        t = torch.round(c.double() * 255.0)
        mse = ((r - t) ** 2).flatten(1).mean(1)
        return float((20 * torch.log10(255.0 / torch.sqrt(mse))).mean())

    t0 = time.time()
    it = 0
    log = []
    for noisy, clean in loader:
        noisy = noisy.to(dev, non_blocking=True).permute(0, 3, 1, 2).contiguous()
        clean = clean.to(dev, non_blocking=True).permute(0, 3, 1, 2).contiguous()
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.l1_loss(model(noisy), clean)
        loss.backward()
        opt.step()
        it += 1
        if it % args.eval_every == 0 or it == args.iters:
            model.eval()
            with torch.no_grad():
                p_out = psnr(model(hn), hc)
            model.train()
            rec = {"iter": it, "loss": round(float(loss.detach()), 6), "psnr_noisy": round(psnr(hn, hc), 3),
                   "psnr_out": round(p_out, 3), "elapsed_s": round(time.time() - t0, 1)}
            log.append(rec)
            print(json.dumps(rec), flush=True)
        if it >= args.iters:
            break
    state = {k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()}
    save_file(state, args.out, metadata={"model": "MultiScaleGraphFilter", "ngraphs": "32", "n_cgd_iters": "10",
                                         "iters": str(it), "batch": str(args.batch), "size": str(args.size),
                                         "final_psnr_out": str(log[-1]["psnr_out"] if log else "")})
    if args.copy_to:
        os.makedirs(os.path.dirname(args.copy_to), exist_ok=True)
        import shutil
        shutil.copyfile(args.out, args.copy_to)
    print(json.dumps({"saved": args.out, "iters": it, "seconds": round(time.time() - t0, 1)}))


if __name__ == "__main__":
    main()

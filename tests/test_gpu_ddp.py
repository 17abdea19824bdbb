"""Data-parallel training on the HIP path (§8e, config C4's step): two ranks on the one GPU (gloo process
group on CUDA tensors -- the reducer's stream handling is the same as under RCCL), each running
``training.Trainer.step`` of a MultiScaleGraphFilter on its half of the batch with the training side
stream (feature branch) and the level stream (solver reverse) on.  The averaged gradients the
``OverlappedGradReducer`` writes back must equal one process's full-batch gradients (scripts_v2/
run_abtract_lightformer_GGTV_GGLR_sigma25.py:186-207 is the single-process loop this shards).

The gradients of the half-resolution branch are accumulated on the side stream while the main branch's
land on the main stream; both sit in one bucket, so the bucket's flatten has to wait for both streams
(sharding.py, OverlappedGradReducer._launch)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, H, W, G, S = 4, 64, 64, 8, 4


def _model():
    import irdu_amd
    from tests.test_gpu_parity import perturb_mixture
    torch.manual_seed(31)
    m = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=G, n_cgd_iters=S)
    perturb_mixture(m.localfilter, 41)
    return m


def _batch():
    g = torch.Generator().manual_seed(7)
    clean = torch.rand(B, H, W, 3, generator=g)
    return clean + torch.randn(B, H, W, 3, generator=g) * (25.0 / 255.0), clean


def _grads_after_step(tr, noisy, clean):
    tr.step(noisy, clean)
    return {k: p.grad.detach().cpu().numpy() for k, p in tr.model.named_parameters()}


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import irdu_amd
        from irdu_amd import graph_filter, solver_grad, training
        irdu_amd.load_native()
        assert graph_filter.FEATURE_STREAMS_TRAIN and solver_grad.LEVEL_STREAMS
        tr = training.Trainer(_model(), {"lr": 1e-6}, torch.device("cuda:0"))
        # one bucket holds every parameter: main- and side-stream gradients are flattened together
        assert len(tr.reducer.buckets) == 1
        noisy, clean = _batch()
        per = B // world
        sl = slice(rank * per, (rank + 1) * per)
        grads = [_grads_after_step(tr, noisy[sl], clean[sl])]
        # the weights step 1 starts from (the parent's full-batch reference starts step 1 from them too)
        after0 = {k: v.detach().cpu().numpy() for k, v in tr.model.state_dict().items()}
        grads.append(_grads_after_step(tr, noisy[sl].flip(1), clean[sl].flip(1)))   # a second step
        q.put((rank, (grads, after0), tr.reducer.launched_in_backward))
    except BaseException as e:   # report instead of leaving the parent waiting on the queue
        q.put((rank, repr(e), -1))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_hip_training_step_equals_full_batch():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = {r: (g, n) for r, g, n in (q.get(timeout=240) for _ in procs)}
        res = {r: (g if isinstance(g, str) else g[0], n, None if isinstance(g, str) else g[1])
               for r, (g, n) in res.items()}
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in (0, 1):
        assert not isinstance(res[r][0], str), res[r][0]
        assert res[r][1] >= 1, ("no bucket was reduced inside backward", r)
    for k in res[0][2]:
        assert np.array_equal(res[0][2][k], res[1][2][k]), k     # the replicas stay identical
    for p in procs:
        assert p.exitcode == 0

    import irdu_amd
    from irdu_amd import training
    irdu_amd.load_native()
    tr = training.Trainer(_model(), {"lr": 1e-6}, torch.device("cuda:0"))
    noisy, clean = _batch()
    ref = [_grads_after_step(tr, noisy, clean)]
    # step 1 from the ranks' post-step-0 weights: the full-batch reference and the two ranks then start
    # from identical weights, so the bound measures the reducer, not Adam's first ~lr sign(g) update
    # amplifying the different rounding of two half-batch sums into different weights
    tr.model.load_state_dict({k: torch.from_numpy(v) for k, v in res[0][2].items()})
    ref.append(_grads_after_step(tr, noisy.flip(1), clean.flip(1)))
    for step in (0, 1):
        for k, want in ref[step].items():
            scale = max(float(np.abs(want).max()), 1e-30)
            for r in (0, 1):
                got = res[r][0][step][k]
                err = float(np.abs(got - want).max()) / scale
                # the two half-batch sums + all-reduce round differently from one full-batch sum
                assert err <= (1e-4 if step == 0 else 2e-4), (step, k, r, err)
            assert np.array_equal(res[0][0][step][k], res[1][0][step][k]), (step, k)

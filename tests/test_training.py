"""Host logic of the training engine (irdu_amd/training.py) on CPU: YAML surface, datasets,
ResumeableSampler semantics (environ/data/data_sampler.py:6-31), the reference's LR schedule
(scripts_v2/...sigma25.py:153-171), checkpoint/resume, and the data-parallel step over gloo.
The graph filter itself needs the GPU (tests/test_gpu_training.py); here a small stock
PyTorch model stands in, since the engine is model-agnostic."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from irdu_amd import training as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class TinyModel(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Conv2d(3, 4, 3, padding=1, bias=False)
        self.b = torch.nn.Conv2d(4, 3, 1, bias=False)

    def encode(self, x):
        return (self.a(x),)

    def decode(self, lat):
        return self.b(lat[0])

    def forward(self, x):
        return self.decode(self.encode(x))


def test_example_yaml_parses_with_reference_keys():
    conf = T.parse_options(os.path.join(ROOT, "experiment_conf", "example.yaml"))
    for key in ("name", "manual_seed", "path", "datasets"):
        assert key in conf
    ds = conf["datasets"]["train"]
    # config C1 as BASELINE.json states it: single-scale GLR, 1 stage, 64x64 gray, sigma 25, batch 1
    assert ds["type"] in T.DATASETS and ds["dataloader_args"]["batch_size"] == 1
    assert ds["dataset_args"]["patch_size"] == 64 and ds["dataset_args"]["lambda_noise"] == 25.0
    assert ds["dataset_args"]["n_channels"] == 1
    assert conf["model"]["type"] == "GLRImageFilter" and conf["model"]["args"]["n_cgd_iters"] == 1
    small = T.parse(os.path.join(ROOT, "experiment_conf", "example_v1x0_small.yaml"))
    assert small["datasets"]["train"]["dataloader_args"]["batch_size"] == 4
    c4 = T.parse(os.path.join(ROOT, "experiment_conf", "c4_train.yaml"))
    assert c4["model"]["args"]["n_cgd_iters"] == 10 and c4["datasets"]["train"]["dataset_args"]["patch_size"] == 512


def test_synthetic_dataset_deterministic_and_noise_law():
    ds = T.SyntheticNoisyPatches(lambda_noise=25.0, patch_size=32, max_num_patchs=8)
    n0, c0 = ds[3]
    n1, c1 = ds[3]
    assert torch.equal(n0, n1) and torch.equal(c0, c1)
    assert n0.shape == (32, 32, 3) and c0.min() >= 0 and c0.max() <= 1
    assert torch.allclose(c0 * 255, torch.round(c0 * 255), atol=1e-4)      # uint8 grid
    noise = (n0 - c0).flatten()
    assert abs(float(noise.std()) - 25.0 / 255.0) < 0.15 * 25.0 / 255.0


def test_multiblocks_yaml_noise_mix_and_schedule():
    """experiment_conf/multiblocks_v7.yaml: the multiblocks script's noise mix
    (lib/dataloader.py:165-169, one sigma per patch) and Adam + MultiStepLR(0.5)."""
    conf = T.parse_options(os.path.join(ROOT, "experiment_conf", "multiblocks_v7.yaml"))
    args = dict(conf["datasets"]["train"]["dataset_args"], patch_size=16, max_num_patchs=400)
    ds = T.SyntheticNoisyPatches(**args)
    sig = np.array([float((ds[i][0] - ds[i][1]).std()) * 255.0 for i in range(400)])
    levels = np.array([1.0, 10.0, 15.0, 20.0, 25.0])
    picked = levels[np.abs(sig[:, None] - levels[None]).argmin(1)]
    assert abs(float((picked == 25.0).mean()) - 0.6) < 0.1
    assert set(np.unique(picked)) <= set(levels)
    opt, sched = T.build_optimizer(TinyModel(), dict(conf["train"], milestones=[2, 4]))
    lrs = []
    for _ in range(6):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sched.step()
    assert lrs == pytest.approx([4e-4, 4e-4, 2e-4, 2e-4, 1e-4, 1e-4])


def test_resumeable_sampler_resumes_and_shards():
    ds = T.SyntheticNoisyPatches(patch_size=16, max_num_patchs=10)
    s = T.ResumeableSampler(ds)
    assert list(s) == list(range(10))
    s = T.ResumeableSampler(ds)
    s.set_epoch_and_current_sample(0, 3)
    assert list(s) == list(range(4, 10))                 # resumes after sample 3
    parts = [list(T.ResumeableSampler(ds, batch_size=2, rank=r, world_size=2)) for r in range(2)]
    # the epoch is cut to whole global batches (10 -> 8 samples): both ranks take 2 full steps
    assert parts[0] == [0, 1, 4, 5] and parts[1] == [2, 3, 6, 7]
    assert T.ResumeableSampler(ds, batch_size=2, rank=0, world_size=2).steps_per_epoch() == 2
    assert T.ResumeableSampler(ds, batch_size=4).steps_per_epoch() == 3      # partial last batch (1 rank)
    assert T.ResumeableSampler(ds, batch_size=4).steps_per_epoch(drop_last=True) == 2   # loader drops it
    assert T.ResumeableSampler(ds, batch_size=16).steps_per_epoch(drop_last=True) == 0


def test_run_with_drop_last_counts_whole_batches(tmp_path, monkeypatch):
    """dataloader_args.drop_last: the epoch length is floor(n / batch) (2 steps of 4 of 10 samples), so
    resume offsets and epoch boundaries follow the loader; a dataset smaller than one batch raises."""
    conf = _tiny_conf(tmp_path, 5)
    conf["datasets"]["train"]["dataloader_args"]["drop_last"] = True
    tr = _run_tiny(monkeypatch, conf)
    assert tr.i == 5
    small = _tiny_conf(tmp_path / "s", 3, bs=4, n=3)
    small["datasets"]["train"]["dataloader_args"]["drop_last"] = True
    with pytest.raises(ValueError, match="holds no batch"):
        _run_tiny(monkeypatch, small)


def test_lr_schedule_matches_reference_formula():
    m = TinyModel()
    opt, sched = T.build_optimizer(m, {"milestones": [3, 6], "cosine_from": 8, "cosine_T_max": 10,
                                       "cosine_base_lr": 5e-5, "eta_min": 1e-6})
    lrs = []
    for _ in range(12):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sched.step()
    g = math.sqrt(math.sqrt(0.5))
    assert lrs[0] == pytest.approx(4e-4) and lrs[3] == pytest.approx(4e-4 * g) and lrs[6] == pytest.approx(4e-4 * g * g)
    # after the switch: cosine from the reset base lr 5e-5 towards 1e-6
    for k in range(8, 12):
        t = k - 8
        assert lrs[k] == pytest.approx(1e-6 + (5e-5 - 1e-6) * (1 + math.cos(math.pi * t / 10)) / 2, rel=1e-6)


def test_checkpoint_roundtrip_and_resume(tmp_path):
    torch.manual_seed(0)
    tr = T.Trainer(TinyModel(), {"milestones": [2]}, torch.device("cpu"))
    ds = T.SyntheticNoisyPatches(patch_size=16, max_num_patchs=8, lambda_noise=25.0)
    batch = [torch.stack(x) for x in zip(*[ds[i] for i in range(4)])]
    losses = [tr.step(*batch) for _ in range(3)]
    assert all(np.isfinite(losses))
    path = tmp_path / "ck.pt"
    torch.save(tr.state_dict(), path)
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"i", "model", "optimizer", "lr_scheduler"} and ck["i"] == 3
    tr2 = T.Trainer(TinyModel(), {"milestones": [2]}, torch.device("cpu"))
    tr2.load_state_dict(ck)
    torch.manual_seed(5)          # the latent-perturbation loss draws noise
    a = tr.step(*batch)
    torch.manual_seed(5)
    b = tr2.step(*batch)
    assert a == pytest.approx(b, rel=1e-6)
    assert tr2.optimizer.param_groups[0]["lr"] == pytest.approx(tr.optimizer.param_groups[0]["lr"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        tr = T.Trainer(TinyModel(), {"loss03_weight": 0.0}, torch.device("cpu"))
        ds = T.SyntheticNoisyPatches(patch_size=16, max_num_patchs=8)
        idx = [i for i in T.ResumeableSampler(ds, batch_size=2, rank=rank, world_size=world)][:2]
        batch = [torch.stack(x) for x in zip(*[ds[i] for i in idx])]
        tr.step(*batch)
        q.put((rank, {k: v.detach().numpy() for k, v in tr.model.state_dict().items()}))
    finally:
        dist.destroy_process_group()


def test_data_parallel_step_equals_full_batch_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    tr = T.Trainer(TinyModel(), {"loss03_weight": 0.0}, torch.device("cpu"))
    ds = T.SyntheticNoisyPatches(patch_size=16, max_num_patchs=8)
    batch = [torch.stack(x) for x in zip(*[ds[i] for i in range(4)])]
    tr.step(*batch)
    for k, v in tr.model.state_dict().items():
        for r in (0, 1):
            assert np.allclose(res[r][k], v.numpy(), rtol=1e-5, atol=1e-7), (k, r)


def _tiny_conf(root, total, bs=4, n=10):
    return {"name": "tiny", "manual_seed": 1, "path": {"root_dir": str(root)},
            "datasets": {"train": {"type": "SyntheticNoisyPatches",
                                   "dataset_args": {"patch_size": 16, "max_num_patchs": n, "lambda_noise": 25.0},
                                   "dataloader_args": {"batch_size": bs}}},
            "train": {"total_iters": total, "checkpoint_every": 1000, "verbose_every": 1000,
                      "loss03_weight": 0.0, "milestones": [100]}}


def _run_tiny(monkeypatch, conf, seed=0):
    def build(_conf):
        torch.manual_seed(seed)
        return TinyModel()
    monkeypatch.setattr(T, "build_model", build)
    return T.run(conf, device=torch.device("cpu"))


def test_run_trains_past_one_epoch_and_saves_final(tmp_path, monkeypatch):
    """total_iters beyond one epoch (3 steps of 4, 4, 2 samples) keeps training over epochs and the
    final state is checkpointed even when it is not a multiple of checkpoint_every."""
    tr = _run_tiny(monkeypatch, _tiny_conf(tmp_path, 7))
    assert tr.i == 7
    files = sorted(os.listdir(T.checkpoint_dir(_tiny_conf(tmp_path, 7))))
    assert files == ["checkpoint_iter00000007.pt"]


def test_resume_continues_the_same_sample_order(tmp_path, monkeypatch):
    """Interrupted at iteration 4 (inside epoch 1) and resumed to 7 == one uninterrupted run to 7."""
    full = _run_tiny(monkeypatch, _tiny_conf(tmp_path / "a", 7))
    _run_tiny(monkeypatch, _tiny_conf(tmp_path / "b", 4))
    resumed = _run_tiny(monkeypatch, _tiny_conf(tmp_path / "b", 7), seed=123)   # weights come from the ckpt
    assert resumed.i == 7
    for (k, v), (k2, v2) in zip(full.model.state_dict().items(), resumed.model.state_dict().items()):
        assert k == k2 and torch.allclose(v, v2, rtol=1e-6, atol=1e-8), k


def _run_worker(rank, world, port, root, q):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        T.build_model = lambda _c: (torch.manual_seed(rank), TinyModel())[1]   # replicas start different
        tr = T.run(_tiny_conf(root, 5, bs=2, n=10), device=torch.device("cpu"))
        q.put((rank, tr.i, {k: v.detach().numpy() for k, v in tr.model.state_dict().items()}))
    finally:
        dist.destroy_process_group()


def _resume_worker(rank, world, port, roots, q):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        T.build_model = lambda _c: (torch.manual_seed(rank), TinyModel())[1]
        tr = T.run(_tiny_conf(roots[rank], 7, bs=2, n=10), device=torch.device("cpu"))
        q.put((rank, tr.i, {k: v.detach().numpy() for k, v in tr.model.state_dict().items()}))
    finally:
        dist.destroy_process_group()


def test_data_parallel_resume_follows_rank0_checkpoint(tmp_path, monkeypatch):
    """Only rank 0's checkpoint folder holds a checkpoint (iteration 4): both ranks resume from rank
    0's file (broadcast choice), run to 7 in lock step and end with identical weights."""
    _run_tiny(monkeypatch, _tiny_conf(tmp_path / "r0", 4, bs=2, n=10))
    roots = [str(tmp_path / "r0"), str(tmp_path / "r1")]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_resume_worker, args=(r, 2, port, roots, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (i, sd) for r, i, sd in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0] == 7
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k


def test_data_parallel_run_over_epochs_stays_in_sync(tmp_path):
    """2 gloo ranks, 10 samples, batch 2 per rank: each epoch is cut to 2 whole global batches, the
    run crosses two epoch boundaries without a rank blocking in the all-reduce, and the replicas
    (built from different seeds) are broadcast from rank 0 and stay identical."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (i, sd) for r, i, sd in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0] == 5
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k


class _ShapeTiny(TinyModel):
    """TinyModel that records the spatial size of every training forward (the curriculum's stage)."""
    seen: list = []

    def forward(self, x):
        if self.training:
            _ShapeTiny.seen.append((x.shape[0], x.shape[2]))
        return super().forward(x)


def _stage(ps, bs, n):
    return {"type": "SyntheticNoisyPatches", "dataset_args": {"patch_size": ps, "max_num_patchs": n,
                                                              "lambda_noise": 25.0},
            "dataloader_args": {"batch_size": bs}}


def _chain_conf(root, total, stages, verbose=1000):
    return {"name": "chain", "manual_seed": 1, "path": {"root_dir": str(root)},
            "datasets": {"train": stages},
            "train": {"total_iters": total, "checkpoint_every": 1000, "verbose_every": verbose,
                      "loss03_weight": 0.0, "milestones": [100]}}


def test_curriculum_stages_chain_per_epoch_and_resume(tmp_path, monkeypatch):
    """datasets.train as a list: the v2 script's curriculum (itertools.chain of its loaders, :185).  An
    epoch runs stage 0 (16^2 x 4, 2 steps) then stage 1 (24^2 x 2, 3 steps); training past one epoch
    starts the chain again; a run interrupted inside stage 1 and resumed equals the uninterrupted run."""
    stages = [_stage(16, 4, 8), _stage(24, 2, 6)]

    def build(_conf):
        torch.manual_seed(0)
        return _ShapeTiny()
    monkeypatch.setattr(T, "build_model", build)
    _ShapeTiny.seen = []
    full = T.run(_chain_conf(tmp_path / "a", 12, stages), device=torch.device("cpu"))
    assert full.i == 12
    assert _ShapeTiny.seen == ([(4, 16)] * 2 + [(2, 24)] * 3) * 2 + [(4, 16)] * 2
    T.run(_chain_conf(tmp_path / "b", 3, stages), device=torch.device("cpu"))     # stops inside stage 1
    _ShapeTiny.seen = []
    resumed = T.run(_chain_conf(tmp_path / "b", 12, stages), device=torch.device("cpu"))
    assert resumed.i == 12 and _ShapeTiny.seen == [(2, 24)] * 2 + ([(4, 16)] * 2 + [(2, 24)] * 3) + [(4, 16)] * 2
    for (k, v), (k2, v2) in zip(full.model.state_dict().items(), resumed.model.state_dict().items()):
        assert k == k2 and torch.allclose(v, v2, rtol=1e-6, atol=1e-8), k
    short = _stage(24, 8, 6)
    short["dataloader_args"]["drop_last"] = True
    with pytest.raises(ValueError, match="stage 1: .* holds no batch"):
        T.run(_chain_conf(tmp_path / "c", 2, [_stage(16, 4, 8), short]), device=torch.device("cpu"))


def test_train_metrics_window_matches_reference_formula(tmp_path, monkeypatch):
    """Training-time PSNR / MSE (:212-223): per step MSE of the clipped output against the clipped
    clean patch (float64), PSNR = 10 log10(1 / MSE), logged as the running mean of the last <= 100 steps."""
    monkeypatch.setattr(T, "build_model", lambda _c: (torch.manual_seed(0), TinyModel())[1])
    tr = T.run(_chain_conf(tmp_path, 4, [_stage(16, 4, 8)], verbose=2), device=torch.device("cpu"))
    assert [i for i, _, _ in tr.train_history] == [2, 4]
    # recompute steps 1..4 with the reference's numpy formula from a replay of the same run
    torch.manual_seed(0)
    ref = T.Trainer(TinyModel(), _chain_conf(tmp_path, 4, [])["train"], torch.device("cpu"))
    ds = T.SyntheticNoisyPatches(patch_size=16, max_num_patchs=8, lambda_noise=25.0)
    ds.random_permute(seed=2024)
    psnrs, mses = [], []
    for step in range(4):
        idx = [(4 * step + j) % 8 for j in range(4)]
        if step == 2:
            ds.random_permute(seed=2025)
        noisy, clean = [torch.stack(x) for x in zip(*[ds[i] for i in idx])]
        ref.model.eval()
        with torch.no_grad():
            out = ref.model(noisy.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
        ref.step(noisy, clean)
        a = np.clip(clean.numpy(), 0, 1).astype(np.float64)
        b = np.clip(out.numpy(), 0, 1).astype(np.float64)
        mse = np.square(a - b).mean()
        mses.append(mse)
        psnrs.append(10 * np.log10(1 / mse))
    assert tr.train_history[-1][1] == pytest.approx(np.mean(psnrs), rel=1e-6)
    assert tr.train_history[-1][2] == pytest.approx(np.mean(mses), rel=1e-6)
    assert tr.train_history[0][1] == pytest.approx(np.mean(psnrs[:2]), rel=1e-6)


def _chain_worker(rank, world, port, root, q):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        T.build_model = lambda _c: (torch.manual_seed(0), _ShapeTiny())[1]
        _ShapeTiny.seen = []
        tr = T.run(_chain_conf(root, 7, [_stage(16, 2, 8), _stage(24, 1, 6)], verbose=7),
                   device=torch.device("cpu"))
        q.put((rank, tr.i, list(_ShapeTiny.seen), tr.train_history,
               {k: v.detach().numpy() for k, v in tr.model.state_dict().items()}))
    finally:
        dist.destroy_process_group()


def test_data_parallel_curriculum_splits_each_stage_batch(tmp_path, monkeypatch):
    """Curriculum under data parallelism (gloo, 2 ranks): a stage's batch_size is per rank, so its global
    batch is batch_size x world (stage 1, 24^2 x 1 per rank: global batch 2) and every rank runs the same
    steps per stage (2 + 3 per epoch), in one all-reduce sequence.  The result equals one process
    training on the global batches (16^2 x 4, then 24^2 x 2), and so do the training PSNR / MSE."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chain_worker, args=(r, 2, port, str(tmp_path / f"r{r}"), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert res[r][0] == 7
        assert res[r][1] == [(2, 16)] * 2 + [(1, 24)] * 3 + [(2, 16)] * 2
    monkeypatch.setattr(T, "build_model", lambda _c: (torch.manual_seed(0), TinyModel())[1])
    one = T.run(_chain_conf(tmp_path / "one", 7, [_stage(16, 4, 8), _stage(24, 2, 6)], verbose=7),
                device=torch.device("cpu"))
    for k, v in one.model.state_dict().items():
        for r in (0, 1):
            assert np.allclose(res[r][3][k], v.numpy(), rtol=1e-5, atol=1e-7), (k, r)
    for r in (0, 1):
        assert res[r][2][-1][1] == pytest.approx(one.train_history[-1][1], rel=1e-9)
        assert res[r][2][-1][2] == pytest.approx(one.train_history[-1][2], rel=1e-9)


def test_v2_curriculum_yaml_states_the_reference_stages():
    conf = T.parse(os.path.join(ROOT, "experiment_conf", "v2_curriculum.yaml"))
    stages = T.train_stage_confs(conf)
    got = [(s["dataset_args"]["patch_size"], s["dataloader_args"]["batch_size"], s["dataset_args"]["max_num_patchs"])
           for s in stages]
    assert got == [(128, 4, 800000), (192, 3, 600000), (256, 2, 400000), (384, 1, 200000)]
    assert conf["model"]["type"] == "AbtractMultiScaleGraphFilter"


class _PadProbe(torch.nn.Module):
    """Identity that records the shapes it sees (the validation recipe pads to multiples of 16)."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.ones(()))
        self.seen = []

    def forward(self, x):
        self.seen.append(tuple(x.shape))
        return x * self.w


def _reference_val_psnr(images, sigma=25.0, seed=2204):
    """scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:240-288 for an identity model, restated
    in numpy: noise from one RandomState stream, pad / crop (a no-op for identity), clamp, ubyte, PSNR."""
    rs = np.random.RandomState(seed=seed)
    out = []
    for img in images:
        img_true = np.asarray(img, dtype=np.float32)
        noisy = img_true.copy()
        noisy += rs.normal(0, sigma / 255.0, img_true.shape)
        restored = np.clip(noisy, 0, 1).astype(np.float32)
        restored = np.clip(np.rint(np.multiply(restored, 255, dtype=np.float32)), 0, 255).astype(np.uint8).astype(np.float32)
        mse = np.square(np.rint(img_true.astype(np.float64) * 255).astype(np.float32) - restored).mean()
        out.append(20 * np.log10(255.0 / np.sqrt(mse)))
    return float(np.mean(out))


def test_img_as_ubyte_rounds_the_float32_product():
    """skimage's img_as_ubyte (the reference's :279) multiplies a float32 image by 255 in float32, then
    rint (half to even): at the float32 value nearest (k + 0.5) / 255 the float32 product is exactly
    k + 0.5 and goes to the even neighbour, where a float64 product (just above k + 0.5) would round up."""
    ks = np.arange(0, 255)
    ties = ((ks + 0.5) / 255.0).astype(np.float32)
    f32 = np.multiply(ties, np.float32(255.0), dtype=np.float32)
    f64 = ties.astype(np.float64) * 255.0
    exact = f32 == ks + 0.5                                         # exact ties in float32 ...
    straddle = exact & (f64 > ks + 0.5) & (ks % 2 == 0)             # ... whose float64 product lies above
    assert straddle.sum() >= 30, straddle.sum()
    got = T._img_as_ubyte(ties)
    assert np.array_equal(got[straddle], ks[straddle].astype(np.uint8))          # half to even: down to k
    assert np.array_equal(np.rint(f64[straddle]), ks[straddle] + 1.0)             # float64 would give k + 1
    assert np.array_equal(got, np.clip(np.rint(f32), 0, 255).astype(np.uint8))
    assert np.array_equal(T._img_as_ubyte(np.array([0.0, 1.0, 0.2], np.float32)), np.array([0, 255, 51], np.uint8))


def test_validation_recipe_pads_crops_and_scores():
    imgs = T.SyntheticTestImages(n_images=3, height=100, width=140)
    m = _PadProbe()
    psnr = T.validate(m, imgs, sigma=25.0, device=torch.device("cpu"))
    assert m.seen == [(1, 3, 112, 144)] * 3                   # reflect-padded to x16, cropped back
    assert psnr == pytest.approx(_reference_val_psnr([imgs[i] for i in range(3)]), rel=1e-6)
    assert 19.0 < psnr < 23.0                                   # noisy input at sigma 25: ~20 dB
    aligned = T.SyntheticTestImages(n_images=1, height=64, width=80)
    m2 = _PadProbe()
    T.validate(m2, aligned, device=torch.device("cpu"))
    assert m2.seen == [(1, 3, 64, 80)]                          # sides already x16 are not padded


def test_run_validates_every_val_every(tmp_path, monkeypatch):
    conf = _tiny_conf(tmp_path, 4)
    conf["train"]["val_every"] = 2
    conf["datasets"]["val"] = {"type": "SyntheticTestImages", "sigma": 25.0,
                               "dataset_args": {"n_images": 2, "height": 40, "width": 36}}
    tr = _run_tiny(monkeypatch, conf)
    assert [i for i, _ in tr.val_history] == [2, 4]
    assert all(np.isfinite(p) for _, p in tr.val_history)


def _val_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        m = TinyModel()
        q.put((rank, T.validate(m, T.SyntheticTestImages(n_images=5, height=36, width=52),
                                device=torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


def test_validation_sharded_over_ranks_equals_one_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_val_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    one = T.validate(TinyModel(), T.SyntheticTestImages(n_images=5, height=36, width=52), device=torch.device("cpu"))
    assert res[0] == pytest.approx(one, rel=1e-12) and res[1] == pytest.approx(one, rel=1e-12)


def test_run_train_plumbing_without_gpu(tmp_path):
    """Config C1 as BASELINE.md states it (PyTorch-CPU plumbing, no GPU): on a host without a GPU,
    run_train.py does what the reference's run_train.py:38-121 does -- latest-checkpoint discovery,
    experiment folders, the config logged to log_files/run_train_<name>.log, dataset + resumable sampler
    + dataloader -- and returns without building a model."""
    import yaml as _yaml
    from irdu_amd import training as T
    conf = _yaml.safe_load(open(os.path.join(ROOT, "experiment_conf", "example.yaml")))
    conf["path"]["root_dir"] = str(tmp_path)
    conf["datasets"]["train"]["dataset_args"]["max_num_patchs"] = 8
    path = tmp_path / "c1.yaml"
    path.write_text(_yaml.safe_dump(conf))
    assert T.main(["-yaml_path", str(path), "-plumbing_only"]) is None
    exp = tmp_path / "experiments" / conf["name"]
    assert (exp / "learning_checkpoints").is_dir()
    log = (exp / "log_files" / f"run_train_{conf['name']}.log").read_text()
    assert "environ_conf=" in log and "train dataset: 8 samples" in log
    parts = T.plumbing(T.parse_options(str(path)))
    noisy, clean = next(iter(parts["dataloader"]))
    assert noisy.shape == clean.shape and parts["latest_checkpoint_path"] is None

"""Training engine: the reference's run_train.py / experiment_conf YAML surface on the HIP path.

Mirrors (reference paths):
  run_train.py:20-121                      parse_options, checkpoint discovery, logger, dataset/dataloader
  environ/utils/custom_parser.py:23-30     YAML -> dict
  environ/data/__init__.py:29-69           create_dataset (by ``type``), create_dataloader
  environ/data/data_sampler.py:6-31        ResumeableSampler (resume inside an epoch)
  environ/data/images_pair_restoration_dataset.py:15-116
                                           AddictiveGaussianNoiseImagePair (patch grid, permute, noise)
  exploration/model_multiscale_mixture_GLR/scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py
    :120-151  model / losses (L1 + 0.1 MSE(enc-dec) + 0.5 MSE(latent-perturbed decode))
    :153-171  Adam(4e-4, eps 1e-8), MultiStepLR(gamma = 0.5**0.25) -> CosineAnnealingLR (SequentialLR)
    :186-224  training step, checkpoint dict {'i', 'model', 'optimizer', 'lr_scheduler'}
    :235-288  periodic validation: reflect-pad to x16, crop, clamp, img_as_ubyte, mean PSNR (validate)

The reference's run_train.py stops after building the dataloader; the YAML here adds
``model:`` and ``train:`` sections so the same entry point runs the training loop of the
v2 scripts.  Multi-GPU: one process per GPU (torchrun); every rank trains on its own
slice of each global batch and gradients are averaged with bucketed RCCL all-reduces
(sharding.OverlappedGradReducer, launched from backward hooks so they overlap the
reverse sweep) — the only collective of the path.

Datasets: no image data ships with the reference, so ``SyntheticNoisyPatches`` (seeded
procedural clean patches, the same noise law) is the default; the CSV/PNG dataset type
is kept for real data.  Samples are (noisy, clean) HWC float32 like the reference's.
"""
from __future__ import annotations

import argparse
import json
import logging
import math
import os
import random
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import yaml
from torch.utils.data import Dataset, Sampler

from . import sharding, stream_guard

LOG = logging.getLogger("irdu_amd.train")


def miopen_training_defaults() -> None:
    """Process-wide MIOpen setting for the training entry points (run_train.py / training.main,
    bench_train.py), never applied on import: MIOPEN_DEBUG_DISABLE_FIND_DB=1 unless the environment
    already sets it.  The stock convolutions outside the graph path (the v1.0 model's embedding,
    down/up-sampling and channel combines) run on MIOpen; with MIOpen's user find-db filled by an earlier
    process its immediate mode spends host time per call -- the C4 training step (v1.0, 32 x 512^2) went
    1.03 s (fresh box) -> 2.7-4.0 s on every later run, GPU kernel time unchanged at 1.09 s; with the
    find-db off every run stays at 1.02-1.03 s (profiles/r04/miopen/).  MIOpen reads the
    variable at its first convolution, so call this before any convolution runs in the process."""
    os.environ.setdefault("MIOPEN_DEBUG_DISABLE_FIND_DB", "1")


# ---------------------------------------------------------------------------
# options (run_train.py:20-36, custom_parser.py:23-30, small_utils.py:12-18)
# ---------------------------------------------------------------------------
def parse(yaml_file_path: str) -> dict:
    with open(yaml_file_path) as f:
        return yaml.safe_load(f)


def set_random_seed(seed: int = 2204) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def parse_options(yaml_path: str) -> dict:
    conf = parse(yaml_path)
    if conf.get("manual_seed") is None:
        conf["manual_seed"] = random.randint(1, 10000)
    set_random_seed(conf["manual_seed"])
    return conf


# ---------------------------------------------------------------------------
# data (environ/data/*)
# ---------------------------------------------------------------------------
def _noisy(patch: np.ndarray, rs: np.random.RandomState, dist_mode: str, lambda_noise) -> np.ndarray:
    """images_pair_restoration_dataset.py:101-110: additive Gaussian noise, sigma = lambda/255;
    vary_addictive_noise (model_multiscale_mixture_GLR/lib/dataloader.py:165-169): lambda_noise =
    [levels, probabilities], one level drawn per patch."""
    if dist_mode == "addictive_noise":
        noise = rs.normal(loc=0.0, scale=lambda_noise / 255.0, size=patch.shape)
    elif dist_mode == "vary_addictive_noise":
        level = rs.choice(lambda_noise[0], p=lambda_noise[1])
        noise = rs.normal(loc=0.0, scale=level / 255.0, size=patch.shape)
    elif dist_mode == "addictive_noise_scale":
        noise = rs.normal(loc=0.0, scale=1.0, size=patch.shape) * (lambda_noise / 255.0)
    else:
        raise ValueError(f"unknown dist_mode {dist_mode!r}")
    return patch + noise.astype(np.float32)


class AddictiveGaussianNoiseImagePair(Dataset):
    """CSV-indexed image patches + noise (images_pair_restoration_dataset.py:15-116).
    csv columns: index, path, height, width (as the reference's *_info.csv)."""

    def __init__(self, csv_path, dist_mode="", lambda_noise=None, patch_size=64, patch_overlap_size=32,
                 max_num_patchs=100000, root_folder="", logger_name=None, device_str="cpu", n_channels=3):
        import pandas as pd
        self.img_infos = pd.read_csv(csv_path, index_col="index")
        self.patch_size, self.patch_overlap_size = patch_size, patch_overlap_size
        self.root_folder, self.lambda_noise, self.dist_mode = root_folder, lambda_noise, dist_mode
        self.n_channels = n_channels
        rows = []
        step = patch_size - patch_overlap_size
        for i in range(self.img_infos.shape[0]):
            info = self.img_infos.iloc[i]
            path = os.path.join(root_folder, info["path"])
            for r in np.arange(0, info["height"] - patch_size, step):
                for c in np.arange(0, info["width"] - patch_size, step):
                    rows.append((int(r), int(c), path))
        self.patchs_data_all = rows
        self.max_num_patchs = min(max_num_patchs, len(rows))
        self.random_permute(seed=2204)

    def random_permute(self, seed=2204):
        self.random_state = np.random.RandomState(seed=seed)
        ind = self.random_state.permutation(self.max_num_patchs)
        self.patchs_data = [self.patchs_data_all[i] for i in ind]

    def __len__(self):
        return len(self.patchs_data)

    def __getitem__(self, idx):
        from PIL import Image
        row, col, path = self.patchs_data[idx]
        img = np.array(Image.open(path))
        patch = img[row:row + self.patch_size, col:col + self.patch_size, :]
        h, w = (patch.shape[0] // 16) * 16, (patch.shape[1] // 16) * 16
        patch = patch[:h, :w].astype(np.float32) / 255.0
        dist = _noisy(patch, self.random_state, self.dist_mode, self.lambda_noise)
        return torch.from_numpy(dist), torch.from_numpy(patch)


def synthetic_clean_patch(rs: np.random.RandomState, h: int, w: int, c: int) -> np.ndarray:
    """Piecewise-smooth clean patch on the uint8 grid (sinusoid background + rectangles), HWC."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    out = np.empty((h, w, c), np.float32)
    for ch in range(c):
        fy, fx, ph = rs.uniform(0.5, 4.0), rs.uniform(0.5, 4.0), rs.uniform(0, 6.28)
        img = 0.5 + 0.3 * np.sin(2 * np.pi * fy * yy / h + ph) * np.cos(2 * np.pi * fx * xx / w)
        for _ in range(3):
            r0, c0 = rs.randint(0, max(1, h - h // 4)), rs.randint(0, max(1, w - w // 4))
            img[r0:r0 + rs.randint(4, max(5, h // 3)), c0:c0 + rs.randint(4, max(5, w // 3))] += rs.uniform(-0.3, 0.3)
        out[..., ch] = img
    return (np.round(np.clip(out, 0, 1) * 255.0) / 255.0).astype(np.float32)


class SyntheticNoisyPatches(Dataset):
    """Deterministic synthetic (noisy, clean) patch pairs: sample i is a function of (seed, i)."""

    def __init__(self, dist_mode="addictive_noise_scale", lambda_noise=25.0, patch_size=64, max_num_patchs=1000,
                 n_channels=3, seed=2204, **_ignored):
        self.dist_mode, self.lambda_noise = dist_mode, lambda_noise
        self.patch_size, self.n_channels, self.seed = patch_size, n_channels, seed
        self.max_num_patchs = max_num_patchs
        self.random_permute(seed=2204)

    def random_permute(self, seed=2204):
        self.order = np.random.RandomState(seed).permutation(self.max_num_patchs)

    def __len__(self):
        return self.max_num_patchs

    def __getitem__(self, idx):
        rs = np.random.RandomState((self.seed * 1000003 + int(self.order[idx])) % (2 ** 32))
        clean = synthetic_clean_patch(rs, self.patch_size, self.patch_size, self.n_channels)
        return torch.from_numpy(_noisy(clean, rs, self.dist_mode, self.lambda_noise)), torch.from_numpy(clean)


DATASETS = {c.__name__: c for c in (AddictiveGaussianNoiseImagePair, SyntheticNoisyPatches)}


# ---------------------------------------------------------------------------
# periodic validation (scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:235-288)
# ---------------------------------------------------------------------------
class TestImagesCSV:
    """Whole clean test images listed in a csv (column ``path``, as the reference's
    dataset/CBSD68_testing_data_info.csv), HWC float32 in [0, 1] on the uint8 grid (:250-258)."""

    def __init__(self, csv_path, root_folder="", **_ignored):
        import pandas as pd
        self.paths = [os.path.join(root_folder, p) for p in pd.read_csv(csv_path, index_col="index")["path"].tolist()]

    def __len__(self):
        return len(self.paths)

    def __getitem__(self, idx):
        from PIL import Image
        return np.array(Image.open(self.paths[idx])).astype(np.float32) / 255.0


class SyntheticTestImages:
    """Deterministic synthetic clean test images (no image data ships with the reference); the default
    sizes are not multiples of 16, so the reflect padding of the recipe is exercised."""

    def __init__(self, n_images=4, height=100, width=140, n_channels=3, seed=68, **_ignored):
        self.n, self.h, self.w, self.c, self.seed = n_images, height, width, n_channels, seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        return synthetic_clean_patch(np.random.RandomState(self.seed * 7919 + idx), self.h, self.w, self.c)


VAL_DATASETS = {c.__name__: c for c in (TestImagesCSV, SyntheticTestImages)}


def _img_as_ubyte(x: np.ndarray) -> np.ndarray:
    """skimage.util.img_as_ubyte of a float32 image in [0, 1] (the reference's :279): skimage's
    float -> uint8 ``_convert`` multiplies in the smallest float type of at least the input's size that
    holds the output (float32 here: ``np.multiply(x, 255, dtype=float32)``), rounds half to even
    (``np.rint``), clips to [0, 255] and casts.  The float32 product matters at ties: a value whose
    float64 product lies just below k + 0.5 can round to k + 0.5 in float32 and go to the even k."""
    y = np.multiply(np.asarray(x, dtype=np.float32), np.float32(255.0), dtype=np.float32)
    np.rint(y, out=y)
    np.clip(y, 0, 255, out=y)
    return y.astype(np.uint8)


@torch.no_grad()
def validate(model: nn.Module, images, sigma: float = 25.0, factor: int = 16, seed: int = 2204,
             device=None) -> float:
    """The reference's test loop (:235-288): per image, add N(0, sigma/255) noise from one
    RandomState(seed) stream, reflect-pad the bottom / right to a multiple of ``factor`` (only a side
    that is not already one), filter, crop, clamp to [0, 1], quantise with img_as_ubyte, MSE against
    the clean image x 255, PSNR = 20 log10(255 / sqrt(MSE)); returns the mean PSNR over the images.

    Several ranks: each filters a contiguous share of the images -- the noise draws follow the global
    image order, as one rank would make them -- and the PSNR sum and count are all-reduced."""
    rank, world = sharding.world()
    was_training = model.training
    model.eval()
    if device is None:
        device = next(model.parameters()).device
    rs = np.random.RandomState(seed=seed)
    s, e = sharding.shard_range(len(images), rank, world)
    psnrs = []
    for i in range(len(images)):
        img_true = np.asarray(images[i], dtype=np.float32)
        noisy_raw = img_true.copy()
        noisy_raw += rs.normal(0, sigma / 255.0, img_true.shape)     # float32 += float64 draws (:258)
        if not s <= i < e:
            continue
        noisy = torch.from_numpy(noisy_raw).permute(2, 0, 1).unsqueeze(0)
        h, w = noisy.shape[2], noisy.shape[3]
        H, W = ((h + factor) // factor) * factor, ((w + factor) // factor) * factor
        padh = H - h if h % factor != 0 else 0
        padw = W - w if w % factor != 0 else 0
        noisy = nn.functional.pad(noisy, (0, padw, 0, padh), "reflect")
        restored = model(noisy.to(device).contiguous())[:, :, :h, :w]
        restored = torch.clamp(restored, 0, 1).cpu().permute(0, 2, 3, 1).squeeze(0).numpy()
        restored = _img_as_ubyte(restored).astype(np.float32)
        img_true_255 = np.rint(img_true.astype(np.float64) * 255.0).astype(np.float32)   # the uint8 image (:253)
        mse = np.square(img_true_255 - restored).mean()                                  # float32, as :273
        psnrs.append(float(20 * np.log10(np.float32(255.0) / np.sqrt(mse))))
    acc = torch.tensor([float(np.sum(psnrs)), float(len(psnrs))], dtype=torch.float64)
    if world > 1:
        if torch.distributed.get_backend() == "nccl":
            acc = acc.to(device)
        torch.distributed.all_reduce(acc)
    if was_training:
        model.train()
    return float(acc[0] / acc[1])


def create_val_dataset(conf: dict):
    """``datasets.val`` of the YAML ({type, dataset_args, sigma, factor}), or None."""
    vconf = conf.get("datasets", {}).get("val")
    if not vconf:
        return None, {}
    cls = VAL_DATASETS.get(vconf["type"])
    if cls is None:
        raise ValueError(f"Validation dataset {vconf['type']} is not found.")
    return cls(**vconf.get("dataset_args", {})), {"sigma": float(vconf.get("sigma", 25.0)),
                                                   "factor": int(vconf.get("factor", 16))}


class ResumeableSampler(Sampler):
    """Deterministic in-order sampling that resumes after ``current_sample`` (data_sampler.py:6-31).
    With world_size > 1 each rank yields its own contiguous slice of every global batch, and the
    epoch is cut to whole global batches (the tail of num_samples % (batch_size * world_size) is
    dropped) so every rank runs the same number of full steps — a rank with one more batch would
    block forever in the gradient all-reduce."""

    def __init__(self, dataset, batch_size: int = 1, rank: int = 0, world_size: int = 1):
        self.dataset = dataset
        self.epoch = 0
        self.current_sample = -1
        self.batch_size, self.rank, self.world_size = batch_size, rank, world_size
        n = len(dataset)
        self.num_samples = n if world_size == 1 else n - n % (batch_size * world_size)

    def _mine(self, i: int) -> bool:
        if self.world_size == 1:
            return True
        gb = self.batch_size * self.world_size
        return (i % gb) // self.batch_size == self.rank

    def __iter__(self) -> Iterator[int]:
        for sample_i in range(self.num_samples):
            if sample_i > self.current_sample:
                self.current_sample += 1
                if self._mine(sample_i):
                    yield sample_i

    def __len__(self):
        return self.num_samples // self.world_size

    def set_epoch_and_current_sample(self, current_epoch, current_sample):
        self.epoch = self.current_epoch = current_epoch
        self.current_sample = current_sample
        self.dataset.random_permute(seed=2024 + current_epoch)

    def steps_per_epoch(self, drop_last: bool = False) -> int:
        """Optimisation steps one epoch holds: a partial last batch counts unless the loader drops
        it (dataloader_args.drop_last); with world_size > 1 there is none (whole global batches)."""
        local = self.num_samples // self.world_size
        return local // self.batch_size if drop_last else -(-local // self.batch_size)


def create_dataset(dataset_conf: dict, environ_conf: dict):
    cls = DATASETS.get(dataset_conf["type"])
    if cls is None:
        raise ValueError(f"Dataset {dataset_conf['type']} is not found.")
    return cls(**dataset_conf["dataset_args"])


def create_dataloader(dataset, sampler, dataset_conf: dict, environ_conf: dict):
    args = dict(dataset_conf["dataloader_args"])
    return torch.utils.data.DataLoader(dataset=dataset, sampler=sampler, **args)


class TrainStage:
    """One loader of the training curriculum: dataset + resumable sampler + dataloader, and the
    optimisation steps it holds per epoch."""

    def __init__(self, index: int, ds_conf: dict, environ_conf: dict, rank: int, world: int):
        self.index = index
        self.dataset = create_dataset(ds_conf, environ_conf)
        self.batch_size = int(ds_conf["dataloader_args"].get("batch_size", 1))
        self.drop_last = bool(ds_conf["dataloader_args"].get("drop_last", False))
        self.sampler = ResumeableSampler(self.dataset, self.batch_size, rank, world)
        self.loader = create_dataloader(self.dataset, self.sampler, ds_conf, environ_conf)
        self.steps = self.sampler.steps_per_epoch(self.drop_last)
        if self.steps <= 0:
            raise ValueError(f"training stage {index}: dataset of {len(self.dataset)} samples holds no batch of "
                             f"{self.batch_size} x {world} ranks")


def train_stage_confs(conf: dict) -> List[dict]:
    """``datasets.train`` as a list of stage configurations: one dict (one loader), or a list of them --
    the v2 script's curriculum, four loaders chained per epoch (128^2 x 4, 192^2 x 3, 256^2 x 2,
    384^2 x 1; scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:50-115, :185)."""
    tr = conf["datasets"]["train"]
    return list(tr) if isinstance(tr, (list, tuple)) else [tr]


def build_train_stages(conf: dict, rank: int = 0, world: int = 1) -> List[TrainStage]:
    """The stages of an epoch, in order.  Data-parallel policy: a stage's ``batch_size`` is per rank (its
    global batch is batch_size x world) and each stage's epoch is cut to whole global batches, so every
    rank runs the same number of steps in every stage and all ranks stay in one all-reduce sequence --
    the 384^2 x 1 stage on 8 GPUs is a global batch of 8, one patch per rank."""
    return [TrainStage(k, dc, conf, rank, world) for k, dc in enumerate(train_stage_confs(conf))]


# ---------------------------------------------------------------------------
# model / optimiser / schedule (v2 script :120-171)
# ---------------------------------------------------------------------------
def build_model(model_conf: dict) -> nn.Module:
    import irdu_amd
    kind = model_conf.get("type", "AbtractMultiScaleGraphFilter")
    from irdu_amd import window_graph, window_graph_v1
    cls = {"AbtractMultiScaleGraphFilter": irdu_amd.AbtractMultiScaleGraphFilter,
           "MultiScaleGraphFilter": irdu_amd.MultiScaleGraphFilter,
           "GLRImageFilter": irdu_amd.GLRImageFilter,
           "MultiScaleGLRImageFilter": irdu_amd.MultiScaleGLRImageFilter,
           # window-graph denoisers of the multiblocks scripts (REF7 v7 / REF1 v1)
           "MultiScaleSequenceDenoiser": window_graph.MultiScaleSequenceDenoiser,
           "MultiScaleSequenceDenoiserV1": window_graph_v1.MultiScaleSequenceDenoiser}.get(kind)
    if cls is None:
        raise ValueError(f"model type {kind!r} has no training path")
    return cls(**model_conf.get("args", {}))


def build_optimizer(model: nn.Module, tconf: dict):
    """Adam + MultiStepLR(gamma=sqrt(sqrt(0.5))) -> CosineAnnealingLR (base lr 5e-5) via SequentialLR;
    ``lr_schedule: multistep`` is the multiblocks scripts' Adam + MultiStepLR(milestones, lr_gamma)
    (run_lightformer_GGTV_GGLR_multiblocks.py:166-174)."""
    from torch.optim.lr_scheduler import CosineAnnealingLR, MultiStepLR, SequentialLR
    opt = torch.optim.Adam(model.parameters(), lr=tconf.get("lr", 4e-4), eps=tconf.get("eps", 1e-8))
    if tconf.get("lr_schedule", "v2") == "multistep":
        return opt, MultiStepLR(opt, milestones=list(tconf.get("milestones", [200000, 500000, 650000])),
                                gamma=float(tconf.get("lr_gamma", 0.5)))
    switch = tconf.get("cosine_from", 600000)
    s1 = MultiStepLR(opt, milestones=list(tconf.get("milestones", range(50000, 600001, 50000))),
                     gamma=float(np.sqrt(np.sqrt(0.5))))
    s2 = CosineAnnealingLR(opt, T_max=tconf.get("cosine_T_max", 701000), eta_min=tconf.get("eta_min", 1e-6))
    s2.base_lrs = [tconf.get("cosine_base_lr", 5e-5) for _ in opt.param_groups]
    return opt, SequentialLR(opt, schedulers=[s1, s2], milestones=[switch])


class Trainer:
    """One optimisation step = the v2 script's loop body (:186-207) + the DDP gradient average."""

    def __init__(self, model: nn.Module, tconf: dict, device):
        self.model, self.device = model.to(device), device
        self.optimizer, self.lr_scheduler = build_optimizer(self.model, tconf)
        self.w_encdec = float(tconf.get("loss02_weight", 0.1))
        self.w_perturb = float(tconf.get("loss03_weight", 0.5))
        self.latent_noise = float(tconf.get("latent_noise", 0.05))
        self.bucket_mb = float(tconf.get("allreduce_bucket_mb", 32.0))
        # all-reduces overlapped with the reverse sweep (post-accumulate-grad hooks); inert on one rank
        self.reducer = sharding.OverlappedGradReducer(self.model.parameters(), bucket_mb=self.bucket_mb)
        self.i = 0
        self.val_history: List[Tuple[int, float]] = []     # (iteration, mean test PSNR)
        # training-time PSNR / MSE (:212-223): per step the batch's squared-error sum (float64, on the
        # device, no host sync) and its element count; summarised by train_metrics()
        self.track_metrics = bool(tconf.get("train_metrics", True))
        self._sse: List[torch.Tensor] = []
        self._n: List[int] = []
        self.train_history: List[Tuple[int, float, float]] = []   # (iteration, mean PSNR, mean MSE)

    def loss(self, noisy: torch.Tensor, clean: torch.Tensor, _out: Optional[list] = None) -> torch.Tensor:
        m = self.model
        out = m(noisy)
        if _out is not None:
            _out.append(out)
        loss = nn.functional.l1_loss(out, clean)
        if hasattr(m, "encode") and (self.w_encdec or self.w_perturb):
            latent = m.encode(clean)
            rec = m.decode(latent)
            disturbed = m.decode(tuple(t + torch.normal(0.0, self.latent_noise, size=t.shape, device=t.device)
                                       for t in latent))
            loss = loss + self.w_encdec * nn.functional.mse_loss(rec, clean)
            loss = loss + self.w_perturb * nn.functional.mse_loss(rec, disturbed)
        return loss

    def step(self, noisy_hwc: torch.Tensor, clean_hwc: torch.Tensor) -> float:
        """noisy/clean: [B,H,W,C] batches as the dataset yields them (permuted like :191-193)."""
        self.model.train()
        self.optimizer.zero_grad(set_to_none=True)
        self.reducer.prepare()
        noisy = noisy_hwc.to(self.device, non_blocking=True).permute(0, 3, 1, 2).contiguous()
        clean = clean_hwc.to(self.device, non_blocking=True).permute(0, 3, 1, 2).contiguous()
        outs: list = []
        with stream_guard.maybe_guard():       # GRR_STREAM_GUARD=1: check the internal-stream invariant
            loss = self.loss(noisy, clean, outs)
            loss.backward()
        self.reducer.finish()
        self.optimizer.step()
        self.lr_scheduler.step()
        if self.track_metrics:
            # :212-214: both images clipped to [0, 1], squared error in float64 (summed here, divided at
            # summary time, so several ranks' shares add up to the global batch's MSE)
            with torch.no_grad():
                d = outs[0].detach().clamp(0.0, 1.0).double() - clean.clamp(0.0, 1.0).double()
                self._sse.append(torch.sum(d * d))
            self._n.append(d.numel())
            del self._sse[:-100], self._n[:-100]
        self.i += 1
        return float(loss.detach())

    def train_metrics(self) -> Tuple[float, float]:
        """Mean PSNR and mean MSE over the last <= 100 steps (the reference's running window, :221-223):
        step k's MSE = its squared-error sum / element count over the global batch (summed over ranks,
        one all-reduce of the window), PSNR_k = 10 log10(1 / MSE_k).  Every rank must call it at the same
        iteration (it is collective when world > 1)."""
        if not self._sse:
            return float("nan"), float("nan")
        acc = torch.stack([torch.stack(self._sse), torch.tensor(self._n, dtype=torch.float64,
                                                                 device=self._sse[0].device)])
        rank, world = sharding.world()
        if world > 1:
            torch.distributed.all_reduce(acc)
        mse = (acc[0] / acc[1]).cpu().numpy()
        return float(np.mean(10.0 * np.log10(1.0 / mse))), float(np.mean(mse))

    def state_dict(self) -> dict:
        return {"i": self.i, "model": self.model.state_dict(), "optimizer": self.optimizer.state_dict(),
                "lr_scheduler": self.lr_scheduler.state_dict()}

    def load_state_dict(self, ckpt: dict) -> None:
        self.model.load_state_dict(ckpt["model"])
        self.optimizer.load_state_dict(ckpt["optimizer"])
        self.lr_scheduler.load_state_dict(ckpt["lr_scheduler"])
        self.i = int(ckpt["i"])


def checkpoint_dir(conf: dict) -> str:
    return os.path.join(conf["path"]["root_dir"], "experiments", conf["name"], "learning_checkpoints")


def latest_checkpoint(conf: dict) -> Optional[str]:
    """run_train.py:42-55: the last file of the sorted checkpoint folder."""
    d = checkpoint_dir(conf)
    files = sorted(os.listdir(d)) if os.path.isdir(d) else []
    return os.path.join(d, files[-1]) if files else None


def run(conf: dict, device=None, max_iters: Optional[int] = None) -> Trainer:
    """Build everything from the YAML dict, resume from the latest checkpoint, train."""
    rank, world = sharding.world()
    if device is None:
        device = torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', 0))}") if torch.cuda.is_available() \
            else torch.device("cpu")
    tconf = conf.get("train", {})
    stages = build_train_stages(conf, rank, world)
    trainer = Trainer(build_model(conf.get("model", {})), tconf, device)
    ckpt_path = conf["path"].get("latest_checkpoint_path") or latest_checkpoint(conf)
    if world > 1:
        # every rank resumes rank 0's choice of checkpoint (ranks never pick their own latest file:
        # without a shared view they could resume at different iterations and block forever in the
        # gradient all-reduce)
        choice = [ckpt_path]
        torch.distributed.broadcast_object_list(choice, src=0)
        ckpt_path = choice[0]
    spe = sum(st.steps for st in stages)
    if ckpt_path:
        trainer.load_state_dict(torch.load(ckpt_path, map_location=device, weights_only=True))
        LOG.info("resumed from %s at iteration %d", ckpt_path, trainer.i)
    if world > 1:
        its = [None] * world
        torch.distributed.all_gather_object(its, trainer.i)
        if len(set(its)) != 1:
            raise RuntimeError(f"ranks resumed at different iterations {its} from {ckpt_path!r}")
    # replicas start identical whatever each rank's seed was (data-parallel averaging never
    # reconciles diverged weights); rank 0's weights are the ones checkpointed
    sharding.broadcast_module(trainer.model)
    os.makedirs(checkpoint_dir(conf), exist_ok=True)
    total = max_iters if max_iters is not None else int(tconf.get("total_iters", spe))
    every = int(tconf.get("checkpoint_every", 5000))
    verbose = int(tconf.get("verbose_every", 100))
    val_set, val_args = create_val_dataset(conf)
    val_every = int(tconf.get("val_every", 0)) if val_set is not None else 0   # the reference's VERBOSE_RATE

    def save():
        if rank == 0:
            torch.save(trainer.state_dict(), os.path.join(checkpoint_dir(conf), f"checkpoint_iter{trainer.i:08d}.pt"))

    # epoch e visits every stage's dataset permuted with seed 2024 + e (data_sampler.py:28-31), for a
    # fresh run and a resumed one alike, so resuming at iteration i continues exactly the order the
    # uninterrupted run would have seen (the reference permutes a fresh run with 2204 instead,
    # images_pair_restoration_dataset.py:41, which makes its resume skip a different order).  An epoch
    # runs the stages in order (the reference's itertools.chain of its loaders, :185); iteration i of
    # the epoch lies in the first stage whose cumulative step count exceeds it.
    epoch, done_in_epoch = divmod(trainer.i, spe)
    start_i, saved_at = trainer.i, None
    while trainer.i < total:
        for st in stages:
            if trainer.i >= total:
                break
            if done_in_epoch >= st.steps:
                done_in_epoch -= st.steps
                continue
            st.sampler.set_epoch_and_current_sample(epoch, done_in_epoch * st.batch_size * world - 1)
            stepped = False
            for noisy, clean in st.loader:
                if trainer.i >= total:
                    break
                loss = trainer.step(noisy, clean)
                stepped = True
                if trainer.i % verbose == 0:
                    psnr_tr, mse_tr = trainer.train_metrics() if trainer.track_metrics else (float("nan"),) * 2
                    trainer.train_history.append((trainer.i, psnr_tr, mse_tr))
                    if rank == 0:
                        LOG.info("iter=%d loss=%.6f lr=%.3e psnr=%.4f mse=%.6e", trainer.i, loss,
                                 trainer.optimizer.param_groups[0]["lr"], psnr_tr, mse_tr)
                if trainer.i % every == 0:
                    save()
                    saved_at = trainer.i
                if val_every and trainer.i % val_every == 0:
                    psnr = validate(trainer.model, val_set, device=device, **val_args)
                    trainer.val_history.append((trainer.i, psnr))
                    if rank == 0:
                        LOG.info("FINISH VAL EPOCH %d - iter=%d - psnr_testing=%.4f", epoch, trainer.i, psnr)
            if not stepped and trainer.i < total:
                raise RuntimeError(f"epoch {epoch} stage {st.index} yielded no batch (dataset {len(st.dataset)}, "
                                   f"batch {st.batch_size}, {world} ranks, drop_last {st.drop_last})")
            done_in_epoch = 0
        epoch, done_in_epoch = epoch + 1, 0
    if trainer.i > start_i and saved_at != trainer.i:     # the final state is always on disk
        save()
    return trainer


def log_files_dir(conf: dict) -> str:
    return os.path.join(conf["path"]["root_dir"], "experiments", conf["name"], "log_files")


def plumbing(conf: dict) -> dict:
    """The reference's run_train.py main (:38-121) as it stands, for config C1 on a host without a GPU:
    find the latest checkpoint of the experiment (only its path: nothing is unpickled), create the
    checkpoint and log-file folders of a fresh run, log the configuration to
    experiments/<name>/log_files/run_train_<name>.log, and build the training dataset, the resumable
    sampler and the dataloader.  Like the reference it builds no model; returns the pieces."""
    ckpt = latest_checkpoint(conf)
    if ckpt:
        conf["path"]["latest_checkpoint_path"] = ckpt
    else:
        os.makedirs(checkpoint_dir(conf), exist_ok=True)
        conf["path"]["checkpoints_folder"] = checkpoint_dir(conf)
        os.makedirs(log_files_dir(conf), exist_ok=True)
        conf["path"]["log_files_folder"] = log_files_dir(conf)
    logger = logging.getLogger(conf["name"])
    logger.setLevel(logging.INFO)
    log_dir = conf["path"].get("log_files_folder") or log_files_dir(conf)
    os.makedirs(log_dir, exist_ok=True)
    fh = logging.FileHandler(os.path.join(log_dir, f"run_train_{conf['name']}.log"))
    fh.setFormatter(logging.Formatter("%(asctime)s %(levelname)s: %(message)s"))
    logger.addHandler(fh)
    try:
        logger.info("environ_conf=%s", json.dumps(conf, indent=1, default=str))
        stages = build_train_stages(conf)
        for st in stages:
            logger.info("train dataset: %d samples", len(st.dataset))
    finally:
        logger.removeHandler(fh)
        fh.close()
    st = stages[0]
    return {"latest_checkpoint_path": ckpt, "dataset": st.dataset, "sampler": st.sampler, "dataloader": st.loader,
            "stages": stages}


def main(argv: Optional[Sequence[str]] = None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-yaml_path", type=str, required=True, help="Path to option YAML file.")
    ap.add_argument("-max_iters", type=int, default=None)
    ap.add_argument("-plumbing_only", action="store_true",
                    help="the reference run_train.py's steps only (no model); the default without a GPU")
    args = ap.parse_args(argv)
    miopen_training_defaults()
    conf = parse_options(args.yaml_path)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s: %(message)s")
    if args.plumbing_only or not torch.cuda.is_available():
        # config C1 (PyTorch-CPU plumbing): the reference's script stops before any model;
        # the HIP model itself needs an MI355X
        parts = plumbing(conf)
        LOG.info("plumbing only (%s): %d training samples, latest checkpoint %s",
                 "no GPU" if not torch.cuda.is_available() else "-plumbing_only", len(parts["dataset"]),
                 parts["latest_checkpoint_path"])
        return None
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1 and not torch.distributed.is_initialized():
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if torch.cuda.is_available():
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        torch.distributed.init_process_group(backend)
    run(conf, max_iters=args.max_iters)

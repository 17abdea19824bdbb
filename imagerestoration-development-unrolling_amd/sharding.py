"""Multi-GPU execution: one process per GPU over torch.distributed (RCCL on MI355X).

Inference: patches / images are independent through the whole path
(no cross-batch op anywhere in REF:707-811), so a global batch is split into
contiguous per-rank shards and each rank filters its shard with no collective in the
data path.  Only scalar metrics (summed squared errors for PSNR) are reduced.

Training (config C4): data parallel — each rank runs forward/backward on its shard
and gradients are averaged with bucketed all-reduces (flattened fp32 buckets, sized
for xGMI ring efficiency rather than per-parameter calls).
"""
from __future__ import annotations

import math
from typing import Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    """(rank, world_size); (0, 1) when torch.distributed is not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, stop) of n units for this rank (first n % world ranks get one more)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world {world_size}")
    base, extra = divmod(n, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_batch(batch: torch.Tensor, rank: Optional[int] = None, world_size: Optional[int] = None) -> torch.Tensor:
    """This rank's slice of a global batch (dim 0)."""
    if rank is None or world_size is None:
        rank, world_size = world()
    s, e = shard_range(batch.shape[0], rank, world_size)
    return batch[s:e]


@torch.no_grad()
def sharded_filter(model, global_batch: torch.Tensor, device=None, micro_batch: Optional[int] = None) -> torch.Tensor:
    """Run ``model`` on this rank's shard of ``global_batch`` (no collective). Returns the local outputs."""
    local = shard_batch(global_batch)
    if device is not None:
        local = local.to(device, non_blocking=True)
    if micro_batch is None or micro_batch >= local.shape[0]:
        return model(local)
    return torch.cat([model(local[i:i + micro_batch]) for i in range(0, local.shape[0], micro_batch)])


def global_psnr_ubyte(restored_local: torch.Tensor, clean_local: torch.Tensor) -> float:
    """Dataset PSNR over all ranks on uint8-quantised images (reference eval recipe,
    scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:276-286): mean of per-image
    PSNRs, reduced with one all_reduce of (sum of PSNRs, count)."""
    r = torch.round(restored_local.detach().clamp(0, 1).double() * 255.0)
    t = torch.round(clean_local.detach().double() * 255.0)
    mse = ((r - t) ** 2).flatten(1).mean(1)
    psnr = 20.0 * torch.log10(255.0 / torch.sqrt(mse))
    acc = torch.stack([psnr.sum(), torch.tensor(float(psnr.numel()), dtype=torch.float64, device=psnr.device)])
    if world()[1] > 1:
        dist.all_reduce(acc)
    return float(acc[0] / acc[1])


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Copy rank src's parameters and buffers to every rank (one flattened broadcast per dtype)."""
    if world()[1] == 1:
        return
    tensors = [t for t in list(module.parameters()) + list(module.buffers()) if t.numel()]
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for ts in by_dtype.values():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.broadcast(flat, src, group=group)
        off = 0
        for t in ts:
            t.copy_(flat[off:off + t.numel()].view_as(t))
            off += t.numel()


def _buckets(params: Sequence[torch.Tensor], bucket_bytes: int) -> List[List[torch.Tensor]]:
    out, cur, size = [], [], 0
    for p in params:
        nb = p.numel() * p.element_size()
        if cur and size + nb > bucket_bytes:
            out.append(cur)
            cur, size = [], 0
        cur.append(p)
        size += nb
    if cur:
        out.append(cur)
    return out


def allreduce_gradients(params: Iterable[torch.nn.Parameter], bucket_mb: float = 32.0,
                        group=None) -> int:
    """Average .grad over ranks with flattened-bucket all-reduces; returns the bucket count.

    Parameters without a gradient contribute zeros (every rank must see the same
    parameter list in the same order).  One all_reduce per bucket: for the v1.0
    model (13.3 M params, 53 MB fp32) two 32 MB buckets.
    """
    rank, ws = world()
    plist = [p for p in params if p.requires_grad]
    if ws == 1 or not plist:
        return 0
    for p in plist:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    buckets = _buckets(plist, int(bucket_mb * 2 ** 20))
    for bucket in buckets:
        flat = torch.cat([p.grad.reshape(-1) for p in bucket])
        dist.all_reduce(flat, group=group)
        _unflatten_mean(flat, bucket, ws)
    return len(buckets)


def _unflatten_mean(flat: torch.Tensor, bucket: Sequence[torch.Tensor], ws: int) -> None:
    flat.div_(ws)
    off = 0
    for p in bucket:
        n = p.numel()
        p.grad.copy_(flat[off:off + n].view_as(p.grad))
        off += n


class OverlappedGradReducer:
    """Gradient average whose all-reduces run while the backward pass is still producing
    gradients (the DDP reducer's schedule, written for this path).

    Parameters are bucketed in REVERSE registration order -- the order the reverse sweep
    finishes them: the solver's scalars and edge stencils (whose gradients the one-Function
    HIP solver reverse returns first) before the feature CNN's weights.  A
    post-accumulate-grad hook counts each parameter in; when a bucket is complete it is
    flattened and handed to an asynchronous all_reduce (RCCL runs it on its own stream,
    ordered after the producing kernels), so the collective overlaps the CNN's reverse.
    Buckets launch strictly in index order on every rank (a bucket that completes early
    waits for its predecessors), so ranks issue identical collective sequences.
    ``finish()`` launches what backward never reached (parameters without a gradient this
    step contribute zeros), waits, and writes the averages back into ``.grad``.
    ``prepare()`` starts a step: it drains anything a step left behind (an exception between
    backward and ``finish()``) and resets the bucket state, so a stale step can never leak into
    the next one's averages; a second backward inside one step raises instead of reducing twice.

    Streams (GPU gradients): the reverse runs on several HIP streams (the feature branch's side
    stream, the solver's level stream), and autograd runs a parameter's accumulation -- and its
    post-accumulate hook -- on the stream that produced the gradient.  The hook therefore records
    an event on its current stream, and a bucket is flattened and reduced on the reducer's own
    stream after waiting on the events of every parameter in it: the flatten can never read a
    gradient another stream is still writing.  ``finish()`` orders the caller's stream after the
    reductions before the averages are written back.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_mb: float = 32.0, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.ws = world()[1]
        self.buckets = _buckets(self.params[::-1], int(bucket_mb * 2 ** 20))
        self._bucket_of = {id(p): i for i, bk in enumerate(self.buckets) for p in bk}
        self._hooks = []
        if self.ws > 1:
            self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self.launched_in_backward = 0
        self._streams = {}
        self._reset()

    def _reset(self):
        self._pending = [len(bk) for bk in self.buckets]
        self._next = 0
        self._work = [None] * len(self.buckets)
        self._flat = [None] * len(self.buckets)
        self._ready = {}            # id(param) -> event recorded on the stream that accumulated its grad

    def _stream(self, dev: torch.device):
        if dev not in self._streams:
            self._streams[dev] = torch.cuda.Stream(device=dev)
        return self._streams[dev]

    def prepare(self) -> None:
        """Begin a step (call before loss.backward())."""
        for w in self._work:
            if w is not None:
                w.wait()
        self._reset()

    def _on_grad(self, p):
        i = self._bucket_of[id(p)]
        if p.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(p.device))
            self._ready[id(p)] = ev
        self._pending[i] -= 1
        if self._pending[i] < 0:
            raise RuntimeError("OverlappedGradReducer: a parameter's gradient arrived twice in one step "
                               "(a second backward without finish(); call prepare() at the start of each step)")
        while self._next < len(self.buckets) and self._pending[self._next] <= 0:
            self._launch(self._next)
            self.launched_in_backward += 1

    def _launch(self, i: int):
        bk = self.buckets[i]
        if not bk[0].is_cuda:
            for p in bk:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            self._flat[i] = torch.cat([p.grad.reshape(-1) for p in bk])
        else:
            # flatten + reduce on the reducer's stream, after every producing stream's accumulation
            red = self._stream(bk[0].device)
            red.wait_stream(torch.cuda.current_stream(bk[0].device))    # zero-filled grads, earlier work
            for p in bk:
                ev = self._ready.get(id(p))
                if ev is not None:
                    red.wait_event(ev)
            with torch.cuda.stream(red):
                for p in bk:
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
                    else:
                        p.grad.record_stream(red)
                self._flat[i] = torch.cat([p.grad.reshape(-1) for p in bk])
                self._work[i] = dist.all_reduce(self._flat[i], group=self.group, async_op=True)
            self._next = i + 1
            return
        self._work[i] = dist.all_reduce(self._flat[i], group=self.group, async_op=True)
        self._next = i + 1

    def finish(self) -> int:
        """Complete this step's average; returns the bucket count (0 on one rank)."""
        if self.ws == 1 or not self.buckets:
            return 0
        while self._next < len(self.buckets):
            self._launch(self._next)
        for i, bk in enumerate(self.buckets):
            self._work[i].wait()
            if bk[0].is_cuda:
                cur = torch.cuda.current_stream(bk[0].device)
                cur.wait_stream(self._stream(bk[0].device))
                self._flat[i].record_stream(cur)
            _unflatten_mean(self._flat[i], bk, self.ws)
        n = len(self.buckets)
        self._reset()
        return n

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

"""Multi-rank plumbing shared by bench.py, bench_train.py and bench_tiled.py.

``python bench.py --gpus N`` must measure N ranks whether the driver starts it under
``torch.distributed.run`` (WORLD_SIZE etc. already in the environment) or as a plain process.
In the plain case ``join_or_spawn`` turns the process into a launcher: it starts N children of
the same script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, waits for
them and exits with the first non-zero child status.  The launcher never touches the GPU (it
only counts devices, which does not initialise HIP on this image), so no process that owns a
GPU context ever execs or forks.

One process per GPU: a rank count above the visible device count is refused unless
GRR_BENCH_BACKEND=gloo, the explicit rehearsal mode in which ranks share the GPUs round-robin.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from typing import List, Optional, Tuple


class LaunchError(SystemExit):
    pass


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def backend() -> str:
    return os.environ.get("GRR_BENCH_BACKEND", "nccl")


def visible_devices() -> int:
    import torch
    return torch.cuda.device_count()


def join_or_spawn(gpus: int, argv: Optional[List[str]] = None, script: Optional[str] = None,
                  dry_run: bool = False) -> Tuple[int, int, int]:
    """Return (world, rank, local_rank) of this process, spawning the ranks first when needed.

    * WORLD_SIZE in the environment (torchrun): it must equal ``gpus``.
    * no WORLD_SIZE and gpus > 1: spawn ``gpus`` children of ``script`` with ``argv`` and exit
      with their status (this call does not return in the launcher).
    * no WORLD_SIZE and gpus == 1: single process.
    """
    if gpus < 1:
        raise LaunchError(f"--gpus must be >= 1 (got {gpus})")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        world = int(env_world)
        if world != gpus:
            raise LaunchError(f"WORLD_SIZE={world} but --gpus {gpus}: launch one rank per requested GPU")
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
        _check_devices(world, dry_run)
        return world, rank, local
    if gpus == 1:
        return 1, 0, 0
    _check_devices(gpus, dry_run)
    script = script or os.path.abspath(sys.argv[0])
    argv = list(sys.argv[1:] if argv is None else argv)
    port = _free_port()
    procs = []
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + argv, env=env))
    raise SystemExit(_wait_all(procs))


def _wait_all(procs, poll_s: float = 0.2, grace_s: float = 10.0) -> int:
    """Wait for every rank; when one exits non-zero, stop the others (they would block in the
    process group's rendezvous or a collective) and return that first failing status, as torchrun does."""
    import time
    first_bad = None
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad and first_bad is None:
            first_bad = bad[0]
            print(f"benchlib: a rank exited with {first_bad}; stopping the others (exit codes {rcs})",
                  file=sys.stderr)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = time.monotonic() + grace_s
            for p in procs:
                try:
                    p.wait(timeout=max(0.0, deadline - time.monotonic()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return first_bad
        if all(rc is not None for rc in rcs):
            return 0
        time.sleep(poll_s)


def _check_devices(world: int, dry_run: bool) -> None:
    if dry_run or world == 1:
        return
    ndev = visible_devices()
    if backend() == "gloo":
        if ndev < 1:
            raise LaunchError("GRR_BENCH_BACKEND=gloo rehearsal still needs one visible GPU")
        return
    if ndev < world:
        raise LaunchError(f"{world} ranks requested but only {ndev} GPU(s) visible (one process per GPU; "
                          "GRR_BENCH_BACKEND=gloo rehearses several ranks on one GPU)")


def dry_run_report(world: int, rank: int, local: int) -> None:
    """--dry-run: each rank reports itself without HIP.  For world > 1 the ranks still join a gloo
    process group on the CPU and count each other with the same ones all-reduce ``ranks_seen`` runs
    on the real backend, so the launcher test checks the fields an N > 1 bench line carries."""
    rep = {"dry_run": True, "rank": rank, "local_rank": local, "world": world,
           "master": f"{os.environ.get('MASTER_ADDR', '')}:{os.environ.get('MASTER_PORT', '')}"}
    if world > 1:
        import torch
        torch.distributed.init_process_group("gloo")
        try:
            rep["ranks_seen"] = ranks_seen(world, torch.device("cpu"))
            rep["backend"] = torch.distributed.get_backend()
        finally:
            torch.distributed.destroy_process_group()
    print(json.dumps(rep), flush=True)


def init(world: int, local: int):
    """Select this rank's device and, for world > 1, join the process group.  Returns the device."""
    import torch
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    if world > 1:
        torch.cuda.set_device(dev)
        if backend() == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend())
    return dev


def ranks_seen(world: int, dev) -> int:
    """Ranks that took part in one all-reduce of ones over the process group (== world when every
    rank joined the group the timing is reduced over).  On the nccl backend the tensor lives on the
    rank's GPU, so the count has crossed RCCL.  1 without a process group."""
    import torch
    if world == 1:
        return 1
    on = dev if torch.distributed.get_backend() == "nccl" else "cpu"
    t = torch.ones(1, dtype=torch.int64, device=on)
    torch.distributed.all_reduce(t)
    return int(t.item())


def check_ranks(world: int, dev) -> dict:
    """The fields every N > 1 bench line carries: ranks_seen (== N, else the run fails) and the
    process group's backend."""
    import torch
    seen = ranks_seen(world, dev)
    if seen != world:
        raise LaunchError(f"ranks_seen={seen} != world {world}: a rank is missing from the process group")
    return {"ranks_seen": seen, "backend": torch.distributed.get_backend() if world > 1 else "none"}


def barrier(world: int, dev) -> None:
    import torch
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)


def max_over_ranks(value: float, world: int, dev) -> float:
    """Max of a per-rank float (the timed region's wall time) over all ranks."""
    import torch
    if world == 1:
        return float(value)
    on = dev if backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=on)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def gather_floats(values, world: int, dev):
    """All ranks' lists of floats (rank order), for per-rank reporting."""
    import torch
    if world == 1:
        return [list(values)]
    on = dev if backend() == "nccl" else "cpu"
    t = torch.tensor(list(values), dtype=torch.float64, device=on)
    out = [torch.empty_like(t) for _ in range(world)]
    torch.distributed.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def finish(world: int) -> None:
    import torch
    if world > 1:
        torch.distributed.destroy_process_group()

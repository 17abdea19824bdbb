"""bench.py / bench_train.py / bench_tiled.py --gpus N: the N ranks exist whether the script is
started under torchrun or plainly (benchlib.join_or_spawn).  CPU-only: --dry-run ranks report
their rank and world without loading HIP."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "GRR_BENCH_BACKEND")}
    env.update(kw)
    return env


def _run(script, args, env):
    return subprocess.run([sys.executable, os.path.join(ROOT, script)] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=180)


@pytest.mark.parametrize("script", ["bench.py", "bench_train.py", "bench_tiled.py"])
def test_plain_start_spawns_n_ranks(script):
    r = _run(script, ["--gpus", "2", "--dry-run"], _env())
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["local_rank"] == d["rank"] for d in lines)
    assert len({d["master"] for d in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")
    # the fields an N > 1 bench line carries: every rank counted by the ones all-reduce, and the backend
    assert all(d["ranks_seen"] == 2 and d["backend"] == "gloo" for d in lines)


def test_single_gpu_dry_run_does_not_spawn():
    r = _run("bench.py", ["--dry-run"], _env())
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines == [{"dry_run": True, "rank": 0, "local_rank": 0, "world": 1, "master": ":"}]


def test_torchrun_world_must_match_gpus():
    r = _run("bench.py", ["--gpus", "4", "--dry-run"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_torchrun_rank_reports_itself():
    # both ranks under torchrun's environment (started by hand here): each reports itself and the group
    port = _free_port()
    env = dict(WORLD_SIZE="2", LOCAL_WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                              cwd=ROOT, env=_env(RANK=str(r), LOCAL_RANK=str(r), **env), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in (0, 1)]
    outs = [p.communicate(timeout=180) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1] for o in outs]
    d = json.loads(outs[1][0].strip().splitlines()[-1])
    assert (d["rank"], d["world"], d["master"]) == (1, 2, f"127.0.0.1:{port}")
    assert d["ranks_seen"] == 2 and d["backend"] == "gloo"


def test_check_ranks_single_process():
    import benchlib
    assert benchlib.check_ranks(1, None) == {"ranks_seen": 1, "backend": "none"}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_more_ranks_than_gpus_is_refused():
    # no GPU in this container: 2 RCCL ranks cannot each own a device -> refused before spawning
    r = _run("bench.py", ["--gpus", "2"], _env())
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr


def test_child_failure_propagates(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import benchlib\n"
        "w, r, l = benchlib.join_or_spawn(2, dry_run=True)\n"
        "sys.exit(3 if r == 1 else 0)\n")
    r = subprocess.run([sys.executable, str(script)], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 3
    assert "a rank exited with 3" in r.stderr


def test_failed_rank_stops_a_blocked_rank(tmp_path):
    """Rank 1 dies while rank 0 stays blocked (as in a rendezvous or collective): the launcher stops
    rank 0 and returns rank 1's status instead of waiting forever."""
    import time
    script = tmp_path / "child.py"
    script.write_text(
        "import os, sys, time\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import benchlib\n"
        "w, r, l = benchlib.join_or_spawn(2, dry_run=True)\n"
        "if r == 1:\n"
        "    sys.exit(5)\n"
        "time.sleep(600)\n")
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(script)], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 5
    assert time.monotonic() - t0 < 60

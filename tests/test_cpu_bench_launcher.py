"""bench.py --gpus N drives N ranks itself: started without a torch.distributed
launcher it spawns torch.distributed.run with N ranks (before any GPU call) and exits with its status;
under a launcher WORLD_SIZE must equal --gpus.  Exercised with --plumbing-check: the ranks bring up
the bench's gloo control plane, gather (rank, local rank, world) and rank 0 prints them -- no GPU call."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_gpus_2_starts_two_ranks():
    r = _run(["--gpus", "2", "--plumbing-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == 2
    assert sorted(tuple(x) for x in lines[0]["plumbing"]) == [(0, 0, 2), (1, 1, 2)]


def test_bench_refuses_world_size_mismatch():
    r = _run(["--gpus", "4", "--plumbing-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
    r = _run(["--plumbing-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})  # --gpus defaults to 1
    assert r.returncode == 2


def test_bench_gpus_1_runs_in_process():
    """--gpus 1 (the default) launches nothing: the plumbing check returns at once in this process."""
    r = _run(["--gpus", "1", "--plumbing-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "torch.distributed.run" not in r.stderr
    assert r.stdout.strip() == ""


def test_resolve_world():
    sys.path.insert(0, ROOT)
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.resolve_world(1, {}) == (1, 0, 0)
    assert b.resolve_world(8, {}) == ("launch", 8)
    assert b.resolve_world(4, {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}) == (4, 3, 3)
    assert b.resolve_world(4, {"WORLD_SIZE": "8"}) == 2
    assert b.resolve_world(0, {}) == 2

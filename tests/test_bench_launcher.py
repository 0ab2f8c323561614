"""bench.py's multi-rank launcher on CPU: `--gpus 2` without WORLD_SIZE
starts torch.distributed.run with two ranks as a child process (nothing
touches a GPU first), every rank joins the process group (gloo here), rank 0
checks the world size against --gpus and prints one line carrying n_gpus and
both ranks' timings.  --selftest swaps the codec step for a CPU stand-in."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env)


def test_gpus2_spawns_two_ranks():
    r = _run(["--selftest", "--gpus", "2", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["warmup"] == 1
    assert d["config"]["world_size"] == 2 and d["config"]["backend"] == "gloo"
    assert [p["rank"] for p in d["per_rank"]] == [0, 1]
    assert d["selftest"] is True


def test_gpus1_runs_in_process():
    r = _run(["--selftest", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and len(d["per_rank"]) == 1


def test_world_size_must_match_gpus():
    r = _run(["--selftest", "--gpus", "2"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)

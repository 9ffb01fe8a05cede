"""CPU test of bench.py's launcher: `bench.py --gpus N` without WORLD_SIZE starts N
ranks (torch.distributed.run as a child process) and each rank sees world == N."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_two_launches_two_ranks():
    lines = run("--gpus", "2", "--dry-run", "--master-port", "29613")
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["dry_run"] for d in lines)
    assert sorted(d["local_rank"] for d in lines) == [0, 1]
    # the sharded construct / score ranks run concurrent shard streams (advisor round 3)
    assert all(d["hw_queues"] >= 16 for d in lines)


def test_gpus_one_runs_in_process():
    lines = run("--gpus", "1", "--dry-run")
    assert [{k: d[k] for k in ("dry_run", "rank", "world", "local_rank")} for d in lines] == \
        [{"dry_run": True, "rank": 0, "world": 1, "local_rank": 0}]


def test_torchrun_without_gpus_flag_takes_world_from_env():
    """`torchrun --nproc-per-node=2 bench.py` (no --gpus): world comes from WORLD_SIZE."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.pop("GPU_MAX_HW_QUEUES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port=29617", os.path.join(ROOT, "bench.py"), "--dry-run"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["hw_queues"] >= 16 for d in lines)


def test_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)

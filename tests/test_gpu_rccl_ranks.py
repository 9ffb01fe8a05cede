"""Multi-process GPU test of the RCCL transport (advisor round 1).

Two ranks, one process per GPU, launched with torch.distributed.run as a child
process: the sharded score (linear and affine, all three kinds) and the sharded
affine construct must equal the single-GPU path bit for bit (tools/rccl_ranks.py).
RCCL refuses two ranks on one device, so the test needs >= 2 GPUs and skips on
the 1-GPU box; in-process virtual ranks cover the same plans there
(test_gpu_shard*.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_gpus() < 2, reason="RCCL needs one device per rank (Duplicate GPU detected on one device)")
def test_rccl_two_ranks_match_single_gpu():
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29537", os.path.join(ROOT, "tools", "rccl_ranks.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ALL_MATCH" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]

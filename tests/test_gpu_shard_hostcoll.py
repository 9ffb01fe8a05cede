"""The one-rank-per-process branch of the sharded construct (rank >= 0) on ONE GPU
(advisor round 5): N processes share device 0, each runs anyseq_shard_construct_hostcoll
-- the device plan gives the other ranks' halves no groups, the level columns, transposed
bottom rows and best cells are zeroed and reduced, each rank walks only its final blocks
and the strings merge by a byte-wise MAX -- with the reductions as gloo all-reduces on host
copies instead of ncclAllReduce (RCCL refuses two ranks on one device).  Every case must
equal the single-GPU construct bit for bit, device-planned and host-built levels
(tools/hostcoll_ranks.py); world 4 also runs the configs[2] fixture."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_hostcoll_ranks_match_single_gpu(world):
    env = dict(os.environ, HOSTCOLL_FIXTURE="1" if world == 4 else "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(29550 + world),
           os.path.join(ROOT, "tools", "hostcoll_ranks.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100 + 30 * world)
    assert r.returncode == 0 and "ALL_MATCH" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]

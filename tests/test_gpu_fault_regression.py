"""Regression for the round-1/2 intermittent GPU memory fault.

The fault appeared only in full-suite processes (many calls of different shapes in
one process, several streams), inside affine fills at single-group Hirschberg
levels.  The audited mechanisms and their fixes:
  * the launch descriptors staged in pinned memory are read by fill_prep_kernel and
    rewritten by the host for every launch: the staging is now COHERENT host memory
    (never served from a GPU cache line of an earlier launch), and a fill group
    checks a digest of EVERY descriptor word (not only an index/epoch magic);
  * device / pinned buffers that grow are retired, not freed, until the device is
    idle (work queued on a transport or caller stream may still reference them);
  * a caller's stream waits for the engine's stream explicitly;
  * no upload reads pageable host memory.

This test runs that shape in ONE child process with the pointer audit on
(ANYSEQ_CHECK_PTRS=1: every descriptor pointer and extent must lie inside a live
allocation): buffers that grow call after call (the per-level rowpool grows at deep
levels), local sharded scores on 4 concurrent streams, the device API on a caller
stream, and the affine construct at single-group levels -- every result compared
with the oracle.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import random, sys
sys.path.insert(0, ROOT)
import torch
import anyseq_amd as A
from oracle import oracle as O
O.build()
rng = random.Random(77)
def rnd(n): return bytes(rng.choice(b"ACGT") for _ in range(n))
def mut(x, p=0.1):
    return bytes(c if rng.random() > p else rng.choice(b"ACGT") for c in x)
dev = torch.device("cuda", 0)
st = torch.cuda.Stream()
checks = 0
for rnd_i in range(3):
    for n, m in [(300, 700), (1200, 1500), (2600, 2300), (700, 4200), (3100, 260)]:
        base = rnd(max(n, m))
        q, s = mut(base[:n]), mut(base[:m])
        for kind in ("global", "semiglobal", "local"):
            sc = (2, -1, -2, -1)
            g = A.construct(kind, q, s, *sc)
            o = O.affine_construct(kind, q, s, *sc)
            assert g == o, ("construct", kind, n, m)
            checks += 1
        # four local shards on concurrent streams (transport threads), then the engine again
        assert A.shard_score_local("semiglobal", q, s, 4, 2, -1, -2, -1) == O.affine_score("semiglobal", q, s, 2, -1, -2, -1)
        checks += 1
        # the device API on a caller stream, inputs and outputs in HBM
        dq = torch.frombuffer(bytearray(q), dtype=torch.uint8).to(dev)
        ds = torch.frombuffer(bytearray(s), dtype=torch.uint8).to(dev)
        aq = torch.empty(n + m, dtype=torch.uint8, device=dev)
        as_ = torch.empty(n + m, dtype=torch.uint8, device=dev)
        with torch.cuda.stream(st):
            v = A.construct_device("local", dq.data_ptr(), n, ds.data_ptr(), m, aq.data_ptr(), as_.data_ptr(),
                                   stream=st.cuda_stream, match=2, mismatch=-1, gap_open=-2, gap_extend=-1)
        st.synchronize()
        o = O.affine_construct("local", q, s, 2, -1, -2, -1)
        assert v == o[0] and aq.cpu().numpy().tobytes() == o[1] and as_.cpu().numpy().tobytes() == o[2]
        checks += 1
        assert A.score("local", q, s) == O.score("local", q, s)
        checks += 1
print("ok", checks, flush=True)
"""


def test_interleaved_calls_pointer_audit():
    env = dict(os.environ, ANYSEQ_CHECK_PTRS="1", GPU_MAX_HW_QUEUES="24")
    r = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip().startswith("ok"), r.stdout[-2000:]

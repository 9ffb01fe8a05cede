"""anyseq_amd.sharded — column-block sharded score, one process per GPU over RCCL.

SURVEY.md §8(e) / DESIGN.md §6.  Rank g owns subject columns
``shard_plan.block(g, world, m)``; the boundary columns travel between
neighbouring ranks with RCCL ncclSend/ncclRecv over xGMI inside
libanyseq.so (anyseq_shard.cpp) while the fills run; the per-rank split
candidates are reduced with one MAX all-reduce.  Linear and affine gaps (the
affine boundary column carries (H, E) plus F of the last row).  torch.distributed (any backend,
``gloo`` is enough) only broadcasts the RCCL unique ids.
"""
from __future__ import annotations

import ctypes

from . import HOST_ALLREDUCE_FN, AnySeqError, _b, _err, _kind, _lib, _scoring, main_random_pair
from . import shard_plan

_ID_BYTES = 128


def init(dist, rank: int, world: int) -> None:
    """Create the RCCL communicators of this rank (collective over the process group)."""
    payload = [None]
    if rank == 0:
        ids = ctypes.create_string_buffer(_ID_BYTES * shard_plan.NCOMMS)
        if _lib.anyseq_shard_unique_ids(ids, shard_plan.NCOMMS) != 0:
            raise AnySeqError(_err())
        payload = [ids.raw]
    dist.broadcast_object_list(payload, src=0)
    if _lib.anyseq_shard_init(rank, world, payload[0], shard_plan.NCOMMS) != 0:
        raise AnySeqError(_err())


def load(query, subject, rank: int, world: int) -> None:
    """Make this rank's inputs resident: the whole query and its subject block."""
    q, s = _b(query), _b(subject)
    c0, w = shard_plan.block(rank, world, len(s))
    blk = s[c0:c0 + w]
    if _lib.anyseq_shard_load(q, len(q), blk, w, c0, len(s)) != 0:
        raise AnySeqError(_err())


def score(kind, match=2, mismatch=-1, gap_open=0, gap_extend=-1) -> int:
    """One sharded fill over the loaded inputs; every rank gets the full score."""
    out = ctypes.c_int64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_shard_score(_kind(kind), ctypes.byref(sc), ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value


def construct(kind, query, subject, match=2, mismatch=-1, gap_open=-2, gap_extend=-1):
    """Sharded affine construct over the initialised ranks (every rank passes the whole
    pair and gets the same (score, alQuery, alSubject)): half fills and final blocks dealt
    round-robin, level columns all-reduced over RCCL."""
    q, s = _b(query), _b(subject)
    L = len(q) + len(s)
    aq = ctypes.create_string_buffer(max(L, 1))
    as_ = ctypes.create_string_buffer(max(L, 1))
    out = ctypes.c_int64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_shard_construct(_kind(kind), ctypes.byref(sc), q, len(q), s, len(s), aq, as_,
                                   ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value, aq.raw[:L], as_.raw[:L]


def construct_hostcoll(dist, rank: int, world: int, kind, query, subject, match=2, mismatch=-1, gap_open=-2,
                       gap_extend=-1):
    """The one-rank-per-process sharded construct (rank >= 0: this process fills only its
    own halves and final blocks) with the level reductions over `dist` (torch.distributed,
    gloo is enough) on host copies instead of RCCL (anyseq_shard_construct_hostcoll).
    Several ranks may share one device: the 1-GPU test of the plan RCCL runs per GPU."""
    import numpy as np
    import torch

    def reduce(buf, count, dtype, op, _user):
        try:
            n = int(count)
            if dtype == 0:
                a = np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ctypes.c_int32)), shape=(n,))
                t = torch.from_numpy(a.copy())
            else:
                a = np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8)), shape=(n,))
                t = torch.from_numpy(a.astype(np.int32))
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX)
            a[:] = t.numpy().astype(a.dtype)
            return 0
        except Exception:   # (a C callback must not raise)
            return 1

    cb = HOST_ALLREDUCE_FN(reduce)
    q, s = _b(query), _b(subject)
    L = len(q) + len(s)
    aq = ctypes.create_string_buffer(max(L, 1))
    as_ = ctypes.create_string_buffer(max(L, 1))
    out = ctypes.c_int64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_shard_construct_hostcoll(_kind(kind), ctypes.byref(sc), q, len(q), s, len(s), int(rank),
                                            int(world), cb, None, aq, as_, ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value, aq.raw[:L], as_.raw[:L]


def finalize() -> None:
    _lib.anyseq_shard_finalize()


def make_weak_step(dist, rank: int, world: int, kind: str, rows: int = 65536, cols_per_rank: int = 65536,
                   gap_open: int = 0):
    """bench.py's weak-scaling workload: `rows` x (cols_per_rank * world) cells, each
    rank owning one block of cols_per_rank columns (main.cpp generator inputs);
    gap_open != 0 runs the affine fill (+2/-1, open gap_open, extend -1)."""
    L = cols_per_rank * world
    q, s = main_random_pair(max(L, rows), max(L, rows))
    q, s = q[:rows], s[:L]
    init(dist, rank, world)
    load(q, s, rank, world)

    def step():
        return score(kind, gap_open=gap_open, gap_extend=-1)

    par = f"column blocks x{world} (RCCL boundary columns over xGMI)"
    return step, rows, cols_per_rank, par


def make_strong_step(dist, rank: int, world: int, query, subject, kind: str, gap_open: int = 0):
    """bench.py --config 4: ONE fixed matrix (strong scaling), rank g owning subject
    block g of `world`; the inputs must be identical on every rank."""
    init(dist, rank, world)
    load(query, subject, rank, world)

    def step():
        return score(kind, gap_open=gap_open, gap_extend=-1)

    par = f"column blocks x{world} (RCCL boundary columns over xGMI)"
    return step, len(_b(query)), len(_b(subject)), par

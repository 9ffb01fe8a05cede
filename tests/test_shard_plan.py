"""CPU test of the column-block sharded decomposition.

world_size-2 (and 3) ``gloo`` process groups run anyseq_amd/shard_plan.py's plan
with a small pure-Python stand-in for each shard's fill (test infrastructure
only): the top front sends its last column to rank g+1, the reversed bottom front
to rank g-1, each rank combines its split columns, and a MAX all-reduce gives the
score, which must equal the oracle's.  The GPU path (anyseq_shard.cpp) implements
the same plan; tests/test_gpu_shard.py checks it on the device.
"""
import os
import random
import socket

import pytest

from anyseq_amd import shard_plan as SP

KINDS = {"global": 0, "semiglobal": 1, "local": 2}


def _fill(kind, rows, cols, left, match=2, mismatch=-1, gap=-1):
    """H of one shard front in its own frame; left = received column (shifted) or None."""
    h, w = len(rows), len(cols)
    init = (lambda i: (i + 1) * gap) if kind == 0 else (lambda i: 0)
    prev = [0] + [init(c) for c in range(w)]          # row -1: corner 0, then the scheme border
    H = []
    for r in range(h):
        cur = [left[r] if left is not None else init(r)] + [0] * w
        for c in range(w):
            v = prev[c] + (match if rows[r] == cols[c] else mismatch)
            v = max(v, cur[c] + gap, prev[c + 1] + gap)
            if kind == 2:
                v = max(v, 0)
            cur[c + 1] = v
        H.append(cur[1:])
        prev = cur
    return H


def _worker(rank, world, port, cases, results):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    for kind_name, q, s in cases:
        kind = KINDS[kind_name]
        n, m = len(q), len(s)
        c0, w = SP.block(rank, world, m)
        h1, h2 = SP.fronts(n)
        gap = -1
        blk = s[c0:c0 + w]
        # top front: receive from rank-1, send to rank+1
        lt = None
        if rank > 0:
            t = torch.zeros(h1, dtype=torch.int64)
            dist.recv(t, src=rank - 1)
            lt = [int(x) + SP.left_shift_top(kind, rank, world, m, gap) for x in t]
        Ht = _fill(kind, q[:h1], blk, lt)
        if rank < world - 1:
            dist.send(torch.tensor([row[w - 1] for row in Ht], dtype=torch.int64), dst=rank + 1)
        # bottom front (reversed): receive from rank+1, send to rank-1
        lb = None
        if rank < world - 1:
            t = torch.zeros(h2, dtype=torch.int64)
            dist.recv(t, src=rank + 1)
            lb = [int(x) + SP.left_shift_bottom(kind, rank, world, m, gap) for x in t]
        Hb = _fill(kind, q[::-1][:h2], blk[::-1], lb)
        if rank > 0:
            dist.send(torch.tensor([row[w - 1] for row in Hb], dtype=torch.int64), dst=rank - 1)
        init = (lambda i: (i + 1) * gap) if kind == 0 else (lambda i: 0)
        adj = SP.combine_adjust(kind, rank, world, m, gap)
        best = 0 if kind == 1 else -2147483647
        for j in SP.split_columns(rank, world, w):
            F = Ht[h1 - 1][j] if j >= 0 else (lt[h1 - 1] if lt is not None else init(h1 - 1))
            jb = w - 2 - j
            B = Hb[h2 - 1][jb] if jb >= 0 else (lb[h2 - 1] if lb is not None else init(h2 - 1))
            best = max(best, F + B + adj)
        if kind == 1:
            if rank == world - 1:
                best = max([best] + [row[w - 1] for row in Ht])
            if rank == 0:
                best = max([best] + [row[w - 1] for row in Hb])
        if kind == 2:
            best = max([best] + [max(r) for r in Ht] + [max(r) for r in Hb])
        t = torch.tensor([best], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out.append(int(t.item()))
    if rank == 0:
        results.put(out)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_plan_matches_oracle(oracle, world):
    import torch.multiprocessing as mp
    rng = random.Random(31 + world)
    cases = []
    for kind in KINDS:
        for n, m in [(2, 7), (9, 13), (40, 33), (57, 90)]:
            q = bytes(rng.choice(b"ACGT") for _ in range(n))
            s = bytes(rng.choice(b"ACGT") for _ in range(m))
            cases.append((kind, q, s))
    ctx = mp.get_context("spawn")
    results = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, results)) for r in range(world)]
    for p in procs:
        p.start()
    got = results.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [oracle.score(k, q, s) for k, q, s in cases]
    assert got == want


def test_plan_partition_and_chunks():
    for m, N in [(10, 3), (65536 * 8, 8), (7, 7)]:
        blocks = [SP.block(g, N, m) for g in range(N)]
        assert blocks[0][0] == 0 and sum(w for _, w in blocks) == m
        assert all(blocks[g][0] + blocks[g][1] == blocks[g + 1][0] for g in range(N - 1))
    assert SP.chunk_rows_for(65536) == 1024 and SP.chunk_rows_for(4_641_652) == 16384
    assert len(SP.chunks(4_641_652)) == 284   # genome-length front: ~280 sends, not ~4500
    ch = SP.chunks(2500, 1024)
    assert ch == [(0, 1024, 16), (1024, 2048, 32), (2048, 2500, 40)]


# ----------------------------------------------- sharded construct plan (§6.2) --
def _construct_worker(rank, world, port, layouts, results):
    """Each rank fills only the rows of its halves (deterministic stand-in values) and
    writes only its blocks' string positions; SUM / MAX all-reduces must rebuild the
    arrays every rank joins on, and the merged strings."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    for n, parts, blocks in layouts:
        LH = torch.zeros(n, dtype=torch.int64)
        RH = torch.zeros(n, dtype=torch.int64)
        owned = []
        for k, p, side, off, ln in SP.level_halves(parts):
            if SP.half_owner(k, world) != rank:
                continue
            owned.append(k)
            col = LH if side == "left" else RH
            for r in range(off, off + ln):
                col[r] = (r * 7 + 1) if side == "left" else -(r * 3 + 2)
        dist.all_reduce(LH, op=dist.ReduceOp.SUM)
        dist.all_reduce(RH, op=dist.ReduceOp.SUM)
        L = sum(h for _, h in blocks) + 128 * len(blocks)
        al = torch.full((L,), ord(" "), dtype=torch.uint8)
        pos = 0
        for b, (oi, h) in enumerate(blocks):
            if SP.block_owner(b, world) == rank:
                for i in range(0, h + 128, 2):   # a diagonal-ish walk: every other position
                    al[pos + i] = ord("ACGT_"[(b + i) % 5])
            pos += h + 128
        t = al.to(torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        owned_t = torch.tensor([len(owned)], dtype=torch.int64)
        dist.all_reduce(owned_t, op=dist.ReduceOp.SUM)
        out.append((LH.tolist(), RH.tolist(), bytes(t.to(torch.uint8).tolist()), int(owned_t.item())))
    if rank == 0:
        results.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_construct_plan(world):
    import torch.multiprocessing as mp
    rng = random.Random(77 + world)
    layouts = []
    for _ in range(4):
        n = rng.randint(5, 300)
        cuts = sorted(rng.randint(0, n) for _ in range(rng.randint(1, 6)))
        bounds = [0] + cuts + [n]
        parts = [None if rng.random() < 0.2 else (a, b - a) for a, b in zip(bounds, bounds[1:])]
        blocks = [(a, b - a) for a, b in zip(bounds, bounds[1:])]
        layouts.append((n, parts, blocks))
    ctx = mp.get_context("spawn")
    results = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_construct_worker, args=(r, world, port, layouts, results)) for r in range(world)]
    for p in procs:
        p.start()
    got = results.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for (n, parts, blocks), (LH, RH, al, nowned) in zip(layouts, got):
        halves = SP.level_halves(parts)
        assert nowned == len(halves)   # every half filled by exactly one rank
        wantL, wantR = [0] * n, [0] * n
        for _, _, side, off, ln in halves:
            for r in range(off, off + ln):
                if side == "left":
                    wantL[r] = r * 7 + 1
                else:
                    wantR[r] = -(r * 3 + 2)
        assert LH == wantL and RH == wantR
        want = bytearray(b" " * len(al))
        pos = 0
        for b, (oi, h) in enumerate(blocks):
            for i in range(0, h + 128, 2):
                want[pos + i] = ord("ACGT_"[(b + i) % 5])
            pos += h + 128
        assert al == bytes(want)



# ------------------------------------ column-blocked construct level 1 (§6.2) --
def _level1_worker(rank, world, port, cases, results):
    """Rank g fills its block of query columns of both transposed level-1 halves
    (pure-Python stand-in fill, linear scores), ships the boundary columns like the
    score plan, writes its bottom rows into zeroed LH / RH at level1_segments, shifted by
    level1_frame; a SUM all-reduce must give the columns of the whole halves."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    gap = -1
    for kind_name, q, s, half in cases:
        kind = KINDS[kind_name]
        n = len(q)
        (c0, w), (r0, _) = SP.level1_segments(rank, world, n)
        blk = q[c0:c0 + w]
        rows_f, rows_r = s[:half], s[half:][::-1]
        lt = None
        if rank > 0:
            t = torch.zeros(len(rows_f), dtype=torch.int64)
            dist.recv(t, src=rank - 1)
            lt = [int(x) + SP.left_shift_top(kind, rank, world, n, gap) for x in t]
        Ht = _fill(kind, rows_f, blk, lt)
        if rank < world - 1:
            dist.send(torch.tensor([row[w - 1] for row in Ht], dtype=torch.int64), dst=rank + 1)
        lb = None
        if rank < world - 1:
            t = torch.zeros(len(rows_r), dtype=torch.int64)
            dist.recv(t, src=rank + 1)
            lb = [int(x) + SP.left_shift_bottom(kind, rank, world, n, gap) for x in t]
        Hb = _fill(kind, rows_r, blk[::-1], lb)
        if rank > 0:
            dist.send(torch.tensor([row[w - 1] for row in Hb], dtype=torch.int64), dst=rank - 1)
        LH = torch.zeros(n, dtype=torch.int64)
        RH = torch.zeros(n, dtype=torch.int64)
        for k in range(w):
            LH[c0 + k] = Ht[-1][k] + SP.level1_frame(kind, c0, gap)
            RH[r0 + k] = Hb[-1][k] + SP.level1_frame(kind, r0, gap)
        dist.all_reduce(LH, op=dist.ReduceOp.SUM)
        dist.all_reduce(RH, op=dist.ReduceOp.SUM)
        out.append((LH.tolist(), RH.tolist()))
    if rank == 0:
        results.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_level1_column_blocks(world):
    import torch.multiprocessing as mp
    rng = random.Random(55 + world)
    cases = []
    for kind in KINDS:
        for n, m in [(9, 7), (40, 33), (57, 64), (31, 17)]:
            q = bytes(rng.choice(b"ACGT") for _ in range(n))
            s = bytes(rng.choice(b"ACGT") for _ in range(m))
            half = 1 << ((m - 1).bit_length() - 1)   # next_pow_2(m) / 2
            cases.append((kind, q, s, half))
    ctx = mp.get_context("spawn")
    results = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_level1_worker, args=(r, world, port, cases, results)) for r in range(world)]
    for p in procs:
        p.start()
    got = results.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for (kind, q, s, half), (LH, RH) in zip(cases, got):
        k = KINDS[kind]
        want_l = _fill(k, s[:half], q, None)[-1]              # the whole forward half's bottom row
        want_r = _fill(k, s[half:][::-1], q[::-1], None)[-1]  # the whole reversed half's
        assert LH == want_l, (kind, len(q), len(s))
        assert RH == want_r, (kind, len(q), len(s))
    assert SP.level1_best_ranks(world) == (world - 1, 0)


def test_rccl_worker_cases_cover_column_blocked_level1():
    """tools/rccl_ranks.py (the 2-GPU RCCL parity worker) must include constructs whose
    level 1 is column-blocked over the ranks (blocked_rccl) as well as ones with no
    blocked level, judged by the one definition the worker asserts with
    (shard_plan.level1_blocked; checked against the engine's own choice in
    tests/test_gpu_shard_construct.py::test_level1_blocked_matches_engine)."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "rccl_ranks.py")
    spec = importlib.util.spec_from_file_location("rccl_ranks", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    blocked = [c for c in mod.CONSTRUCT_CASES if SP.level1_blocked(c[1], c[2], 2)]
    assert blocked and any(not SP.level1_blocked(c[1], c[2], 2) for c in mod.CONSTRUCT_CASES)
    assert {c[0] for c in blocked} >= {"local", "semiglobal"}
    # the engine's condition: a level (m > 128), world >= 2, n >= world
    assert SP.level1_blocked(8000, 16384, 2) and not SP.level1_blocked(100, 120, 2)
    assert not SP.level1_blocked(3, 4000, 4) and SP.level1_blocked(4, 4000, 4)
    assert not SP.level1_blocked(5000, 5000, 1)


# ------------------------- column-blocked levels >= 2 over rank subgroups (§6.2) --
def _blocked_worker(rank, world, port, levels, results):
    """Every part of a level runs over its own subgroup of ranks like level 1 over all
    of them: rank g fills its block of the part's query rows of both transposed halves
    (pure-Python stand-in fill), ships boundary columns to its neighbours INSIDE the
    subgroup, and writes its bottom rows into zeroed LH / RH at part_segments; one SUM
    all-reduce must give every part's halves' columns."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    gap = -1
    for kind_name, q, s, parts in levels:
        kind = KINDS[kind_name]
        n = len(q)
        LH = torch.zeros(n, dtype=torch.int64)
        RH = torch.zeros(n, dtype=torch.int64)
        P = len(parts)
        assert SP.blocked_level(P, world)
        for p, (off, ln, soff, mw, half) in enumerate(parts):
            r0, G = SP.part_subgroup(p, P, world)
            if not (r0 <= rank < r0 + G):
                continue
            g = rank - r0
            (c0, w), (rb, _) = SP.part_segments(rank, r0, G, off, ln)
            qp, sp_ = q[off:off + ln], s[soff:soff + mw]
            blk = qp[c0 - off:c0 - off + w]
            rows_f, rows_r = sp_[:half], sp_[half:][::-1]
            lt = None
            if g > 0:
                t = torch.zeros(len(rows_f), dtype=torch.int64)
                dist.recv(t, src=rank - 1)
                lt = [int(x) + SP.left_shift_top(kind, g, G, ln, gap) for x in t]
            Ht = _fill(kind, rows_f, blk, lt)
            if g < G - 1:
                dist.send(torch.tensor([row[w - 1] for row in Ht], dtype=torch.int64), dst=rank + 1)
            lb = None
            if g < G - 1:
                t = torch.zeros(len(rows_r), dtype=torch.int64)
                dist.recv(t, src=rank + 1)
                lb = [int(x) + SP.left_shift_bottom(kind, g, G, ln, gap) for x in t]
            Hb = _fill(kind, rows_r, blk[::-1], lb)
            if g > 0:
                dist.send(torch.tensor([row[w - 1] for row in Hb], dtype=torch.int64), dst=rank - 1)
            for k in range(w):
                LH[c0 + k] = Ht[-1][k] + SP.level1_frame(kind, c0 - off, gap)
                RH[rb + k] = Hb[-1][k] + SP.level1_frame(kind, rb - off, gap)
        dist.all_reduce(LH, op=dist.ReduceOp.SUM)
        dist.all_reduce(RH, op=dist.ReduceOp.SUM)
        out.append((LH.tolist(), RH.tolist()))
    if rank == 0:
        results.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 5])
def test_sharded_level2_column_blocks(world):
    """Level 2 (two parts) column-blocked over two rank subgroups at world 4 and 5
    (uneven subgroups 2 + 3): the assembled columns equal the whole halves' bottom rows
    of both parts, as anyseq_shard.cpp blocked_rccl / blocked_local build them."""
    import torch.multiprocessing as mp
    rng = random.Random(77 + world)
    levels = []
    for kind in KINDS:
        q = bytes(rng.choice(b"ACGT") for _ in range(37))
        s = bytes(rng.choice(b"ACGT") for _ in range(30))
        # parts (query off, len, subject off, columns, left-half width): rows split at 17
        parts = [(0, 17, 0, 15, 8), (17, 20, 15, 15, 7)]
        levels.append((kind, q, s, parts))
    ctx = mp.get_context("spawn")
    results = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_blocked_worker, args=(r, world, port, levels, results)) for r in range(world)]
    for p in procs:
        p.start()
    got = results.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for (kind, q, s, parts), (LH, RH) in zip(levels, got):
        k = KINDS[kind]
        wantL, wantR = [0] * len(q), [0] * len(q)
        for off, ln, soff, mw, half in parts:
            qp, sp_ = q[off:off + ln], s[soff:soff + mw]
            wl = _fill(k, sp_[:half], qp, None)[-1]
            wr = _fill(k, sp_[half:][::-1], qp[::-1], None)[-1]
            wantL[off:off + ln] = wl
            wantR[off:off + ln] = wr
        assert LH == wantL, (kind, world)
        assert RH == wantR, (kind, world)
    assert SP.part_subgroup(1, 2, 5) == (2, 3) and not SP.blocked_level(4, 7)

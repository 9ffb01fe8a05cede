"""GPU parity of the column-block sharded fill.

anyseq_shard_score_local runs `nshards` shards in one process on one GPU with the
same kernels, progress counters and chunked boundary-column hand-off as the RCCL
path (device copies instead of ncclSend/ncclRecv).  Scores are integers: bit-exact
against the oracle restatement of the reference CPU path.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

KINDS = ("global", "semiglobal", "local")


def rnd(rng, n):
    return "".join(rng.choice("ACGT") for _ in range(n))


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("nshards", [1, 2, 3, 4])
def test_shard_small(anyseq, oracle, kind, nshards):
    rng = random.Random(100 + nshards)
    for n, m in [(2, 9), (3, 40), (130, 200), (700, 901), (1500, 1300), (65, 4000)]:
        if m < nshards:
            continue
        q, s = rnd(rng, n), rnd(rng, m)
        assert anyseq.shard_score_local(kind, q, s, nshards) == oracle.score(kind, q, s), (kind, n, m, nshards)


@pytest.mark.parametrize("kind", KINDS)
def test_shard_multi_group_chunks(anyseq, oracle, kind, monkeypatch):
    """Several workgroups per front, several row chunks per hand-off, narrow blocks."""
    rng = random.Random(7)
    for (n, m, ns) in [(9000, 3000, 2), (5000, 5000, 4), (3000, 130, 2), (4097, 2049, 3)]:
        q, s = rnd(rng, n), rnd(rng, m)
        assert anyseq.shard_score_local(kind, q, s, ns) == oracle.score(kind, q, s), (kind, n, m, ns)


@pytest.mark.parametrize("kind", KINDS)
def test_shard_matches_single_gpu_main_inputs(anyseq, kind):
    """main.cpp-generated 16384^2 pair: sharded == single-GPU score (which is pinned elsewhere)."""
    q, s = anyseq.main_random_pair(16384, 16384)
    ref = anyseq.score(kind, q, s)
    for ns in (2, 4):
        assert anyseq.shard_score_local(kind, q, s, ns) == ref, (kind, ns)


def test_shard_similar_sequences(anyseq, oracle):
    rng = random.Random(9)
    base = rnd(rng, 3000)
    mut = list(base)
    for _ in range(60):
        mut[rng.randrange(len(mut))] = rng.choice("ACGT")
    s = "".join(mut[:1500] + list(rnd(rng, 40)) + mut[1500:])
    for kind in KINDS:
        assert anyseq.shard_score_local(kind, base, s, 3) == oracle.score(kind, base, s), kind


def test_shard_rejects_bad_shapes(anyseq):
    with pytest.raises(anyseq.AnySeqError):
        anyseq.shard_score_local("global", "A", "ACGT", 2)        # one query row: no two fronts
    with pytest.raises(anyseq.AnySeqError):
        anyseq.shard_score_local("global", "ACGT", "AC", 3)       # fewer columns than shards


@pytest.mark.parametrize("kind", KINDS)
def test_shard_local_dispatch_no_deadlock(anyseq, kind):
    """Regression (round 2): 4 concurrent in-process persistent fills of (CUs-16)/4
    workgroups filled some XCDs to 32 of 32 CUs; a fill that could not place all of its
    workgroups held back the next shard's launch and about 1 % of 4-shard runs hung until
    the 10 s spin limit.  The shard grid is XCD-aware now; 60 repetitions
    per kind (the flake would show in ~45 % of suite runs)."""
    q, s = anyseq.main_random_pair(16384, 16384)
    ref = anyseq.score(kind, q, s, gap_open=-2, gap_extend=-1)
    for _ in range(60):
        assert anyseq.shard_score_local(kind, q, s, 4, gap_open=-2, gap_extend=-1) == ref


def test_shard_max_local_count(anyseq, oracle):
    """The largest accepted local shard count under the suite's GPU_MAX_HW_QUEUES = 24
    (3N - 2 transport + fill streams + 2 <= 24: N = 8) runs, co-resident and correct;
    more shards than the device keeps co-resident (CUs/8 - 8 = 24 on MI355X) are refused
    instead of deadlocking in dispatch."""
    rng = random.Random(31)
    q, s = rnd(rng, 2000), rnd(rng, 4000)
    for kind in KINDS:
        assert anyseq.shard_score_local(kind, q, s, 8, gap_open=-2, gap_extend=-1) == \
            oracle.affine_score(kind, q, s, 2, -1, -2, -1), kind
    with pytest.raises(anyseq.AnySeqError, match="at most 24 local shards"):
        anyseq.shard_score_local("global", q, s, 25)

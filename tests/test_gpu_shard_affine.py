"""GPU parity of the AFFINE column-block sharded fill: the boundary
column carries (H, E) of the last column plus F of the last row, and the per-shard
combine joins a vertical gap across the split row.  In-process shards on one GPU
(the same kernels, counters and chunk protocol as the RCCL path); bit-exact against
the affine oracle (build-defined Gotoh, pinned by open = 0 => linear)."""
import random

import pytest

pytestmark = pytest.mark.gpu

KINDS = ("global", "semiglobal", "local")
SCHEMES = [(2, -1, -2, -1), (1, -3, -5, -2), (3, -2, -1, -3)]


def rnd(rng, n):
    return "".join(rng.choice("ACGT") for _ in range(n))


def shard(anyseq, kind, q, s, ns, sc):
    return anyseq.shard_score_local(kind, q, s, ns, match=sc[0], mismatch=sc[1], gap_open=sc[2], gap_extend=sc[3])


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("nshards", [1, 2, 3, 4])
def test_shard_affine_small(anyseq, oracle, kind, nshards):
    rng = random.Random(200 + nshards)
    for it, (n, m) in enumerate([(2, 9), (3, 40), (130, 200), (700, 901), (1500, 1300), (65, 4000)]):
        if m < nshards:
            continue
        sc = SCHEMES[it % len(SCHEMES)]
        q, s = rnd(rng, n), rnd(rng, m)
        assert shard(anyseq, kind, q, s, nshards, sc) == oracle.affine_score(kind, q, s, *sc), (kind, n, m, sc)


@pytest.mark.parametrize("kind", KINDS)
def test_shard_affine_multi_group(anyseq, oracle, kind):
    rng = random.Random(17)
    for (n, m, ns) in [(9000, 3000, 2), (5000, 5000, 4), (3000, 130, 2), (4097, 2049, 3)]:
        q, s = rnd(rng, n), rnd(rng, m)
        assert shard(anyseq, kind, q, s, ns, SCHEMES[0]) == oracle.affine_score(kind, q, s, *SCHEMES[0]), (n, m, ns)


def test_shard_affine_gap_across_boundaries(anyseq, oracle):
    """Related sequences with long indels near the block boundaries and the split row."""
    rng = random.Random(18)
    base = rnd(rng, 4000)
    s = base[:990] + base[1030:2000] + rnd(rng, 35) + base[2000:]
    for kind in KINDS:
        for ns in (2, 3, 4):
            for sc in SCHEMES:
                assert shard(anyseq, kind, base, s, ns, sc) == oracle.affine_score(kind, base, s, *sc), (kind, ns, sc)


@pytest.mark.parametrize("kind", KINDS)
def test_shard_affine_matches_single_gpu(anyseq, kind):
    q, s = anyseq.main_random_pair(16384, 16384)
    ref = anyseq.score(kind, q, s, gap_open=-2, gap_extend=-1)
    for ns in (2, 4):
        assert anyseq.shard_score_local(kind, q, s, ns, gap_open=-2, gap_extend=-1) == ref, (kind, ns)


def test_shard_received_column_never_torn(anyseq, oracle):
    """Regression (round 2): the transport's small device copies land byte by byte, and
    the fill used to poll the received words against a sentinel, so it could accept a
    half-overwritten word (seen on the box: 0x80FFFFFD = sentinel high byte + the low
    bytes of -3).  The fill now waits on per-chunk ready flags the transport writes
    after each chunk.  This repeats the failing sequence (local, 4 shards, 3 x 40,
    scheme (1,-3,-5,-2) after the other small cases), which mismatched about once in
    twelve passes before the fix."""
    for _ in range(4):
        for ns in (1, 2, 3, 4):
            for kind in KINDS:
                rng = random.Random(200 + ns)
                for it, (n, m) in enumerate([(2, 9), (3, 40), (130, 200), (700, 901)]):
                    if m < ns:
                        continue
                    sc = SCHEMES[it % len(SCHEMES)]
                    q, s = rnd(rng, n), rnd(rng, m)
                    assert shard(anyseq, kind, q, s, ns, sc) == oracle.affine_score(kind, q, s, *sc), (kind, ns, n, m)
                    assert anyseq.shard_score_local(kind, q, s, ns) == oracle.score(kind, q, s), (kind, ns, n, m)

"""GPU parity with the group hand-off ROW RING wrapped.

Genome-length matrices keep only nslots >= 2*grid+2 hand-off rows per
sub-problem; a group writes slot k % nslots and the reader puts the sentinel
back.  Here the persistent grid is cut to 2 workgroups and the ring to its
minimum (6 slots), so matrices of a few thousand rows (16+ groups) wrap it
several times: scores and construct strings must stay bit-exact with the oracle.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

KINDS = ("global", "semiglobal", "local")


def rnd(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


@pytest.fixture
def small_ring(anyseq):
    anyseq.set_option("grid", 2)
    anyseq.set_option("affine_grid", 2)
    anyseq.set_option("ring_slots", 1)     # clamped up to 2*grid+2 = 6
    yield anyseq
    anyseq.set_option("grid", 0)
    anyseq.set_option("affine_grid", 0)
    anyseq.set_option("ring_slots", 0)


@pytest.mark.parametrize("kind", KINDS)
def test_ring_linear_score(small_ring, oracle, kind):
    rng = random.Random(41)
    for n, m in [(6000, 700), (4096, 2000), (9000, 130)]:
        q, s = rnd(rng, n), rnd(rng, m)
        assert small_ring.score(kind, q, s) == oracle.score(kind, q, s), (kind, n, m)


@pytest.mark.parametrize("kind", KINDS)
def test_ring_affine_score(small_ring, oracle, kind):
    rng = random.Random(42)
    for n, m in [(5000, 600), (3000, 1500)]:
        q, s = rnd(rng, n), rnd(rng, m)
        got = small_ring.score(kind, q, s, gap_open=-2, gap_extend=-1)
        assert got == oracle.affine_score(kind, q, s, 2, -1, -2, -1), (kind, n, m)


@pytest.mark.parametrize("kind", KINDS)
def test_ring_construct(small_ring, oracle, kind):
    rng = random.Random(43)
    q, s = rnd(rng, 5000), rnd(rng, 900)
    got = getattr(small_ring, f"construct_{kind}_alignment")(q, s)
    assert got == oracle.construct(kind, q, s)


@pytest.mark.parametrize("kind", KINDS)
def test_ring_affine_construct(small_ring, oracle, kind):
    rng = random.Random(44)
    base = rnd(rng, 4000)
    q = base
    s = "".join(c if rng.random() > 0.1 else rng.choice("ACGT") for c in base[500:1500])
    v, aq, as_ = small_ring.construct(kind, q, s, gap_open=-2, gap_extend=-1)
    ov, oq, os_ = oracle.affine_construct(kind, q, s, 2, -1, -2, -1)
    assert (v, aq, as_) == (ov, oq, os_)

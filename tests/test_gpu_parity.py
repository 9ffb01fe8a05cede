"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bit-exact for scores and for the construct_* strings (integer/byte work).
"""
import random

import pytest

pytestmark = pytest.mark.gpu

KINDS = ("global", "semiglobal", "local")


def rnd(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


def abi_score(anyseq, kind, q, s):
    return getattr(anyseq, f"{kind}_alignment_score")(q, s)


def abi_construct(anyseq, kind, q, s):
    return getattr(anyseq, f"construct_{kind}_alignment")(q, s)


@pytest.mark.parametrize("kind", KINDS)
def test_score_small_random(anyseq, oracle, kind):
    rng = random.Random(11)
    for _ in range(60):
        n, m = rng.randint(1, 300), rng.randint(1, 300)
        q, s = rnd(rng, n), rnd(rng, m)
        assert abi_score(anyseq, kind, q, s) == oracle.score(kind, q, s), (kind, n, m)


@pytest.mark.parametrize("kind", KINDS)
def test_score_edge_shapes(anyseq, oracle, kind):
    rng = random.Random(12)
    sizes = [0, 1, 2, 31, 32, 33, 63, 64, 65, 127, 128, 129, 255, 256, 511, 512, 513, 1023, 1024, 1025, 2049]
    for n in sizes:
        for m in (0, 1, 63, 64, 65, 1000):
            q, s = rnd(rng, n), rnd(rng, m)
            assert abi_score(anyseq, kind, q, s) == oracle.score(kind, q, s), (kind, n, m)


@pytest.mark.parametrize("kind", KINDS)
def test_score_multi_group(anyseq, oracle, kind):
    rng = random.Random(13)
    for n, m in [(5000, 3000), (3000, 7000), (4097, 4095), (9000, 300)]:
        q, s = rnd(rng, n), rnd(rng, m)
        assert abi_score(anyseq, kind, q, s) == oracle.score(kind, q, s), (kind, n, m)


@pytest.mark.parametrize("kind", KINDS)
def test_score_bytes_and_similar(anyseq, oracle, kind):
    rng = random.Random(14)
    # raw byte equality, any byte (align.impala:130-133), and highly similar pairs
    q = bytes(rng.randrange(256) for _ in range(700))
    s = bytes(rng.randrange(256) for _ in range(900))
    assert abi_score(anyseq, kind, q, s) == oracle.score(kind, q, s)
    base = rnd(rng, 3000)
    mut = list(base)
    for _ in range(100):
        mut[rng.randrange(len(mut))] = rng.choice("ACGTN")
    mut = "".join(mut[:1200] + mut[1250:])
    assert abi_score(anyseq, kind, base, mut) == oracle.score(kind, base, mut)


@pytest.mark.parametrize("kind", KINDS)
def test_construct_bit_exact(anyseq, oracle, kind):
    rng = random.Random(21)
    cases = [(1, 1), (2, 1), (65, 65), (100, 64), (200, 129), (300, 257), (700, 1000), (1000, 700),
             (2048, 2048), (3000, 5000), (50, 3000), (3000, 130)]
    for n, m in cases:
        q, s = rnd(rng, n), rnd(rng, m)
        got = abi_construct(anyseq, kind, q, s)
        exp = oracle.construct(kind, q, s)
        assert got[0] == exp[0], (kind, n, m, "return")
        assert got[1] == exp[1], (kind, n, m, "alQuery")
        assert got[2] == exp[2], (kind, n, m, "alSubject")


@pytest.mark.parametrize("kind", KINDS)
def test_construct_random_shapes(anyseq, oracle, kind):
    rng = random.Random(22)
    for _ in range(25):
        n, m = rng.randint(0, 1500), rng.randint(1, 1500)
        q, s = rnd(rng, n), rnd(rng, m)
        got = abi_construct(anyseq, kind, q, s)
        exp = oracle.construct(kind, q, s)
        assert got == exp, (kind, n, m)


@pytest.mark.parametrize("R,NW", [(1, 3), (1, 4), (1, 7), (1, 8), (2, 8), (4, 8), (2, 4), (4, 3)])
def test_tuning_variants(anyseq, oracle, R, NW):
    rng = random.Random(30 + R * 10 + NW)
    anyseq.set_tuning(R, NW, 0)
    try:
        for kind in KINDS:
            for n, m in [(777, 1500), (5000, 2000), (64 * R * NW + 1, 999)]:
                q, s = rnd(rng, n), rnd(rng, m)
                assert abi_score(anyseq, kind, q, s) == oracle.score(kind, q, s), (R, NW, kind, n, m)
            q, s = rnd(rng, 1500), rnd(rng, 1300)
            assert abi_construct(anyseq, kind, q, s) == oracle.construct(kind, q, s), (R, NW, kind)
    finally:
        anyseq.set_tuning(1, 4, 0)


@pytest.mark.parametrize("fronts", [1, 2])
@pytest.mark.parametrize("CH", [16, 32])
def test_fronts_and_chunk(anyseq, oracle, fronts, CH):
    rng = random.Random(40 + fronts * 2 + CH)
    anyseq.set_option("fronts", fronts)
    anyseq.set_option("chunk", CH)
    try:
        for kind in KINDS:
            for n, m in [(513, 700), (2000, 1999), (4096, 64), (6001, 3000), (1024, 1)]:
                q, s = rnd(rng, n), rnd(rng, m)
                assert abi_score(anyseq, kind, q, s) == oracle.score(kind, q, s), (fronts, CH, kind, n, m)
            q, s = rnd(rng, 2500), rnd(rng, 1800)
            assert abi_construct(anyseq, kind, q, s) == oracle.construct(kind, q, s), (fronts, CH, kind)
    finally:
        anyseq.set_option("fronts", 2)
        anyseq.set_option("chunk", 32)

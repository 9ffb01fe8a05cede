"""GPU parity of LINEAR scores through the affine fill (round 5): with
`linear_via_affine` (default 1) a linear-gap score of every kind (gap open 0) runs on
fill_affine_kernel -- its code
rows, lean blocks, half-chunk hand-offs and, with `linear_affine_loop` (default), the linear
asm loop (gen_aff2 lin: one DPP and one shift move per step; X space for local) -- against
the reference-semantics linear oracle (oracle.score), bit-exact: every kind, shapes around
the band and chunk sizes, multi-group and two-front matrices, > 8 symbols (the compare
path), schemes whose mismatch does not lose, and the loop's band ends and starts
(affine_asm 97 / 3 / 1 / 0)."""
import random

import pytest

pytestmark = pytest.mark.gpu

KINDS = ("global", "semiglobal", "local")


def rnd(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


@pytest.fixture(params=[1, 0], ids=["linear-loop", "affine-loop"])
def linaff(anyseq, request):
    anyseq.set_option("linear_via_affine", 1)
    anyseq.set_option("linear_affine_loop", request.param)
    try:
        yield request.param
    finally:
        anyseq.set_option("linear_via_affine", 1)
        anyseq.set_option("linear_affine_loop", 1)


def test_linaff_random(anyseq, oracle, linaff):
    rng = random.Random(61)
    for it in range(45):
        n, m = rng.randint(1, 500), rng.randint(1, 500)
        q, s = rnd(rng, n), rnd(rng, m)
        sc = [(2, -1, -1), (1, -3, -2), (3, -2, -3), (2, 0, -1), (5, 2, -1)][it % 5]
        for kind in KINDS:
            got = anyseq.score(kind, q, s, match=sc[0], mismatch=sc[1], gap_open=0, gap_extend=sc[2])
            assert got == oracle.score(kind, q, s, *sc), (kind, n, m, sc)


def test_linaff_edges_and_multi_group(anyseq, oracle, linaff):
    rng = random.Random(62)
    for n in [1, 2, 63, 64, 65, 127, 128, 129, 511, 512, 513, 1025, 2049, 5000]:
        for m in (1, 31, 32, 33, 65, 1000, 3001):
            q, s = rnd(rng, n), rnd(rng, m)
            for kind in KINDS:
                assert anyseq.score(kind, q, s) == oracle.score(kind, q, s), (kind, n, m)
    for n, m in [(9000, 3000), (3000, 9000), (4097, 4095)]:
        q, s = rnd(rng, n), rnd(rng, m)
        for kind in KINDS:
            assert anyseq.score(kind, q, s) == oracle.score(kind, q, s), (kind, n, m)


def test_linaff_bytes_and_band_ends(anyseq, oracle, linaff):
    rng = random.Random(63)
    q = bytes(rng.randrange(256) for _ in range(701))
    s = bytes(rng.randrange(256) for _ in range(900))
    for kind in KINDS:
        assert anyseq.score(kind, q, s) == oracle.score(kind, q, s), kind
    for asm in (97, 3, 1, 0):
        anyseq.set_option("affine_asm", asm)
        try:
            for it in range(6):
                alph = ("ACGT", "ACGTNRYKMSWB")[it % 2]
                n, m = rng.randint(20, 700), rng.randint(20, 700)
                q, s = rnd(rng, n, alph), rnd(rng, m, alph)
                sc = [(2, -1, -1), (3, 1, -2), (2, 0, -1)][it % 3]
                for kind in KINDS:
                    got = anyseq.score(kind, q, s, match=sc[0], mismatch=sc[1], gap_open=0, gap_extend=sc[2])
                    assert got == oracle.score(kind, q, s, *sc), (kind, n, m, sc, alph, asm)
        finally:
            anyseq.set_option("affine_asm", 1)


def test_linear_kernel_still_covered(anyseq, oracle):
    """linear_via_affine 0: the linear fill kernel (fill_kernel) for every kind, as before
    round 5 (semiglobal scores and the linear constructs keep using it)."""
    rng = random.Random(64)
    anyseq.set_option("linear_via_affine", 0)
    try:
        for n, m in [(1, 1), (300, 517), (2049, 1000), (6000, 3001)]:
            q, s = rnd(rng, n), rnd(rng, m)
            for kind in KINDS:
                assert anyseq.score(kind, q, s) == oracle.score(kind, q, s), (kind, n, m)
    finally:
        anyseq.set_option("linear_via_affine", 1)


@pytest.mark.parametrize("force", [1, 0])
def test_semiglobal_zero_open_border(anyseq, oracle, force):
    """The zero-open left border of semiglobal fills (round 5): forced at column -1 in the
    virtual prologue (`affine_force_border` 1, the asm `pro` loop and the C++ blocks' lbrd)
    or, with 0, the masked C++ prologue as before -- affine and linear scores, one- and
    multi-group bands, bands with fewer than two full blocks (the prologue stays in C++)."""
    rng = random.Random(65)
    anyseq.set_option("affine_force_border", force)
    try:
        for n, m in [(230, 50), (700, 31), (64, 64), (3000, 2500), (9000, 300), (129, 1000)]:
            q, s = rnd(rng, n), rnd(rng, m)
            for sc in [(2, -1, -2, -1), (1, -3, -5, -2), (3, 1, -2, -1)]:
                got = anyseq.score("semiglobal", q, s, match=sc[0], mismatch=sc[1], gap_open=sc[2], gap_extend=sc[3])
                assert got == oracle.affine_score("semiglobal", q, s, *sc), (n, m, sc)
            assert anyseq.score("semiglobal", q, s) == oracle.score("semiglobal", q, s), (n, m)
    finally:
        anyseq.set_option("affine_force_border", 1)

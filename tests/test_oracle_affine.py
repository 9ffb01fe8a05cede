"""CPU checks of the build-defined affine construct oracle (oracle_affine_construct).

Affine gaps have no reference semantics (align.impala:153-166 is dead code), so
the construct is pinned by properties an optimal alignment must have, checked
against an independent textbook Gotoh (oracle.textbook_affine_score):
  * the sparse i+j+1 layout (traceback.impala:47-80) holds a valid alignment
    of exactly q[is..ie] and s[js..je] (the rectangle the oracle reports);
  * its affine score, recomputed from the alignment, equals the optimal score;
  * global covers the whole matrix; local / semiglobal rectangles start and
    end where an optimal path can.
"""
import random

import pytest

KINDS = ("global", "semiglobal", "local")
SCHEMES = [(2, -1, -2, -1), (1, -3, -5, -2), (5, -4, -10, -1), (3, -2, -1, -3), (2, -1, -1, -1)]


def rnd(rng, n, alphabet="ACGT"):
    return bytes(rng.choice(alphabet.encode()) for _ in range(n))


def dense_ops(al_q, al_s):
    pairs = [(a, b) for a, b in zip(al_q, al_s) if not (a == 32 and b == 32)]
    return pairs


def rescore(pairs, match, mismatch, go, ge):
    sc, prev = 0, None
    for a, b in pairs:
        if a == 95:
            op = "D"
        elif b == 95:
            op = "I"
        else:
            op = "M"
        if op == "M":
            sc += match if a == b else mismatch
        else:
            sc += ge + (go if prev != op else 0)
        prev = op
    return sc


def check(oracle, kind, q, s, scheme):
    m_, x_, go, ge = scheme
    score, aq, as_ = oracle.affine_construct(kind, q, s, m_, x_, go, ge)
    assert score == oracle.textbook_affine_score(kind, q, s, m_, x_, go, ge)
    i0, i1, j0, j1 = oracle.affine_last_rect()
    pairs = dense_ops(aq, as_)
    n, m = len(q), len(s)
    if not pairs:   # the empty alignment: only when nothing beats it
        assert kind != "global" or n + m == 0
        assert score <= 0 or n == 0 or m == 0
        return
    qa = bytes(a for a, _ in pairs if a != 95)
    sa = bytes(b for _, b in pairs if b != 95)
    assert qa == (q[i0:i1 + 1] if i1 >= i0 else b"") and sa == (s[j0:j1 + 1] if j1 >= j0 else b"")
    assert rescore(pairs, m_, x_, go, ge) == score
    if kind == "global":
        assert (len(qa), len(sa)) == (n, m)
    elif kind == "semiglobal":   # starts on the top row / left column, ends on the last row / column
        assert i0 == 0 or j0 == 0 or (i1 < i0 and j0 >= 0) or (j1 < j0 and i0 >= 0)
        assert i1 == n - 1 or j1 == m - 1


@pytest.mark.parametrize("kind", KINDS)
def test_affine_construct_random(oracle, kind):
    rng = random.Random(41)
    for it in range(40):
        scheme = SCHEMES[it % len(SCHEMES)]
        n, m = rng.randint(1, 200), rng.randint(1, 400)
        check(oracle, kind, rnd(rng, n), rnd(rng, m), scheme)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_construct_shapes(oracle, kind):
    rng = random.Random(42)
    for n in (0, 1, 2, 63, 64, 65, 129, 300):
        for m in (0, 1, 64, 127, 128, 129, 255, 256, 257, 700):
            check(oracle, kind, rnd(rng, n), rnd(rng, m), (2, -1, -2, -1))


@pytest.mark.parametrize("kind", KINDS)
def test_affine_construct_long_gaps(oracle, kind):
    """Gaps crossing Hirschberg column boundaries (E-state splits) and row splits."""
    rng = random.Random(43)
    core = rnd(rng, 900)
    ins = rnd(rng, 350)
    q = core[:400] + core[700:]                     # a 300-column deletion in the query
    s = core[:200] + ins + core[200:]               # a 350-column insertion in the subject
    for scheme in [(2, -1, -8, -1), (2, -1, -2, -1), (1, -1, -20, -1), (2, -1, 0, -1)]:
        check(oracle, kind, q, core, scheme)
        check(oracle, kind, core, s, scheme)
        check(oracle, kind, s, q, scheme)


def test_affine_construct_similar(oracle):
    rng = random.Random(44)
    base = rnd(rng, 1500)
    mut = bytearray(base)
    for _ in range(80):
        mut[rng.randrange(len(mut))] = rng.choice(b"ACGT")
    for kind in KINDS:
        check(oracle, kind, base, bytes(mut[100:1400]), (2, -1, -3, -1))
        check(oracle, kind, rnd(rng, 50) + base[300:900] + rnd(rng, 70), base, (2, -1, -3, -1))

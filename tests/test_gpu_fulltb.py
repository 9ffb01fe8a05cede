"""GPU parity of the reference's undeclared *_fulltb exports (export.impala:37-53,
93-109, 150-166; full-matrix traceback, global scheme for all three) against the
oracle restatement (oracle_construct_fulltb).  Bit-exact strings and score."""
import random

import pytest

pytestmark = pytest.mark.gpu

NAMES = ["construct_global_alignment_fulltb", "construct_semiglobal_alignment_fulltb",
         "construct_local_alignment_fulltb"]


def rnd(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


@pytest.mark.parametrize("name", NAMES)
def test_fulltb_shapes(anyseq, oracle, name):
    rng = random.Random(71)
    shapes = [(0, 0), (0, 7), (9, 0), (1, 1), (5, 64), (64, 5), (100, 127), (130, 128), (300, 129),
              (257, 1000), (1000, 300), (2049, 2000)]
    for n, m in shapes:
        q, s = rnd(rng, n), rnd(rng, m)
        got = getattr(anyseq, name)(q, s)
        assert got == oracle.construct_fulltb(q, s), (name, n, m)


def test_fulltb_similar_and_bytes(anyseq, oracle):
    rng = random.Random(72)
    base = rnd(rng, 3000)
    s = "".join(c if rng.random() > 0.08 else rng.choice("ACGT") for c in base)
    s = s[:1000] + s[1010:] + rnd(rng, 40)
    assert anyseq.construct_global_alignment_fulltb(base, s) == oracle.construct_fulltb(base, s)
    q = bytes(rng.randrange(256) for _ in range(500))
    t = bytes(rng.randrange(256) for _ in range(700))
    assert anyseq.construct_local_alignment_fulltb(q, t) == oracle.construct_fulltb(q, t)


def test_fulltb_large_matches_score(anyseq):
    """Size-independent property at a size the O(nm) oracle would be slow at: the
    strings re-score to the global optimum and consume every symbol."""
    q, s = anyseq.main_random_pair(8192, 8192)
    v, aq, as_ = anyseq.construct_global_alignment_fulltb(q, s)
    assert v == anyseq.global_alignment_score(q, s)
    dq, ds = anyseq.dense(aq, as_)
    assert dq.replace(b"_", b"") == q and ds.replace(b"_", b"") == s
    sc = sum(2 if a == b else -1 for a, b in zip(dq, ds) if a != 95 and b != 95) - dq.count(b"_") - ds.count(b"_")
    assert sc == v

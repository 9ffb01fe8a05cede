"""GPU parity of the inherited Hirschberg halves (option "inherit_halves").

Host-built levels (affine_device_plan 0) with every level forced to split its eligible
halves into column blocks, each block but the last recording the split column of one of the
half's next descendants (depth 1-3), and the later levels taking those descendants' halves
from the recorded columns instead of a fill.  The construct must be
bit-exact with the oracle restatement (oracle_affine_construct: every half filled), score
and both sparse strings; the stats show that halves were split and reused, so the test
covers the path it names.  Local constructs (clamped halves) never split.
"""
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCHEMES = [(2, -1, -2, -1), (1, -3, -5, -2), (5, -4, -10, -1), (3, -2, -1, -3)]


@pytest.fixture(params=[1, 2, 3], ids=["depth1", "depth2", "depth3"])
def inherit(anyseq, request):
    """Host-built levels, every level splitting; a split half records the columns of its
    next 1 / 2 / 3 descendants (option inherit_depth)."""
    anyseq.set_option("affine_device_plan", 0)
    anyseq.set_option("inherit_halves", 2)
    anyseq.set_option("inherit_depth", request.param)
    anyseq.last_inherit_stats()
    yield anyseq
    anyseq.set_option("inherit_depth", 2)
    anyseq.set_option("inherit_halves", 1)
    anyseq.set_option("affine_device_plan", 1)


def rnd(rng, n, alphabet=b"ACGT"):
    return bytes(rng.choice(alphabet) for _ in range(n))


def related(rng, n, ident=0.9):
    """A mutated copy: substitutions, short insertions and deletions (a diagonal path)."""
    a = rnd(rng, n)
    out = bytearray()
    for c in a:
        x = rng.random()
        if x < (1 - ident) * 0.6:
            out.append(rng.choice(b"ACGT"))
        elif x < (1 - ident) * 0.8:
            out += bytes([c]) + rnd(rng, rng.randint(1, 6))
        elif x < 1 - ident:
            continue
        else:
            out.append(c)
    return a, bytes(out)


def same(anyseq, oracle, kind, q, s, sc):
    g = anyseq.construct(kind, q, s, match=sc[0], mismatch=sc[1], gap_open=sc[2], gap_extend=sc[3])
    o = oracle.affine_construct(kind, q, s, *sc)
    assert g[0] == o[0], (kind, len(q), len(s), sc, "score", g[0], o[0])
    assert g[1] == o[1] and g[2] == o[2], (kind, len(q), len(s), sc, "strings")


@pytest.mark.parametrize("kind", ["global", "semiglobal"])
def test_inherit_related(inherit, oracle, kind):
    rng = random.Random(71)
    for it, (n, m) in enumerate([(2000, 2100), (3000, 2600), (1500, 4000), (4100, 1300), (2500, 2500)]):
        q, s = related(rng, n)
        s = s[:m] if len(s) >= m else s + rnd(rng, m - len(s))
        same(inherit, oracle, kind, q, s, SCHEMES[it % len(SCHEMES)])
    split, reused = inherit.last_inherit_stats()
    assert split > 0 and reused > 0, (split, reused)


@pytest.mark.parametrize("kind", ["global", "semiglobal"])
def test_inherit_random(inherit, oracle, kind):
    rng = random.Random(72)
    for it in range(16):
        n, m = rng.randint(200, 2500), rng.randint(300, 3500)
        same(inherit, oracle, kind, rnd(rng, n), rnd(rng, m), SCHEMES[it % len(SCHEMES)])
    split, reused = inherit.last_inherit_stats()
    assert split > 0, (split, reused)


@pytest.mark.parametrize("kind", ["global", "semiglobal"])
def test_inherit_shapes(inherit, oracle, kind):
    """Block counts around powers of two, ragged last blocks, thin and wide parts."""
    rng = random.Random(73)
    for n in (1, 64, 65, 300, 1000):
        for m in (257, 383, 640, 1025, 2049, 2100):
            q, s = related(rng, max(n, m))
            same(inherit, oracle, kind, q[:n], s[:m], (2, -1, -2, -1))


def test_inherit_long_gaps(inherit, oracle):
    """Paths through long horizontal / vertical gaps: the recorded column's E state and the
    second block's frame (NORMAL / EFREE borders) carry the gap across the block boundary."""
    rng = random.Random(74)
    core = rnd(rng, 3000)
    q = core[:1200] + core[2000:]
    s = core[:600] + rnd(rng, 700) + core[600:]
    for kind in ("global", "semiglobal"):
        for sc in [(2, -1, -8, -1), (2, -1, -2, -1), (1, -1, -20, -1)]:
            same(inherit, oracle, kind, q, s, sc)
            same(inherit, oracle, kind, s, q, sc)


def test_inherit_local_unsplit(inherit, oracle):
    """Local halves carry the clamp: never split, results unchanged."""
    rng = random.Random(75)
    q, s = related(rng, 2500)
    same(inherit, oracle, "local", q, s, (2, -1, -2, -1))
    assert inherit.last_inherit_stats() == (0, 0)


def test_inherit_config3_prefix(inherit):
    """configs[3]'s 262,144-bp semiglobal fixture through the host-built levels with every
    level inheriting: the same score, strings and CIGAR as the oracle-generated fixture."""
    import hashlib
    from anyseq_amd import genome
    g = json.load(open(os.path.join(GOLD, "config3_prefix.json")))
    q, s = genome.synthetic_related_pair(4_641_652, 0.9)
    q, s = q[:g["lq"]], s[:g["ls"]]
    sc = g["scoring"]
    v, aq, as_ = inherit.construct(g["kind"], q, s, match=sc["match"], mismatch=sc["mismatch"],
                                   gap_open=sc["gap_open"], gap_extend=sc["gap_extend"])
    assert v == g["score"]
    assert inherit.cigar(aq, as_) == g["cigar"]
    assert (hashlib.sha256(aq).hexdigest(), hashlib.sha256(as_).hexdigest()) == (g["sha_alq"], g["sha_als"])
    split, reused = inherit.last_inherit_stats()
    assert split > 0 and reused > 0, (split, reused)


@pytest.mark.parametrize("kind", ["global", "semiglobal"])
def test_inherit_linear_true_construct(inherit, oracle, kind):
    """Linear gaps through the extended API's true construct (construct_mode 1: the affine
    construct with gap open 0, the affine fill's linear loop) on host-built levels with
    every level splitting: bit-exact.  (Before round 6's fix the host-built levels sent gap
    open 0 to the linear fill_kernel: wrong scores, tools/lin_host_probe.py.)"""
    rng = random.Random(76)
    inherit.set_option("construct_mode", 1)
    try:
        for n, m in [(2000, 2100), (3000, 2600), (1500, 4000), (700, 900)]:
            q, s = related(rng, n)
            s = s[:m] if len(s) >= m else s + rnd(rng, m - len(s))
            for sc in ((2, -1, 0, -1), (1, -3, 0, -2)):
                same(inherit, oracle, kind, q, s, sc)
    finally:
        inherit.set_option("construct_mode", 0)
    split, reused = inherit.last_inherit_stats()
    assert split > 0 and reused > 0, (split, reused)


def test_host_built_linear_true_construct_local(inherit, oracle):
    """The local linear true construct on host-built levels (clamped halves never split)."""
    rng = random.Random(77)
    inherit.set_option("construct_mode", 1)
    try:
        for n, m in [(2000, 2100), (1500, 4000)]:
            q, s = related(rng, n)
            s = s[:m] if len(s) >= m else s + rnd(rng, m - len(s))
            for sc in ((2, -1, 0, -1), (1, -3, 0, -2)):
                same(inherit, oracle, "local", q, s, sc)
    finally:
        inherit.set_option("construct_mode", 0)

"""GPU parity of the sharded affine construct (align.impala:237-311
distributed by Hirschberg level): `nshards` virtual ranks in one process, one fill
launch per rank per level, the half fills and final blocks dealt round-robin.  It
must return exactly the single-GPU construct (which the oracle pins) -- score and
both sparse strings -- for every shard count."""
import hashlib
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KINDS = ("global", "semiglobal", "local")
SCHEMES = [(2, -1, -2, -1), (1, -3, -5, -2), (3, -2, -1, -3)]


def rnd(rng, n):
    return bytes(rng.choice(b"ACGT") for _ in range(n))


@pytest.mark.parametrize("kind", KINDS)
def test_sharded_construct_small(anyseq, oracle, kind):
    rng = random.Random(91)
    for it in range(12):
        sc = SCHEMES[it % len(SCHEMES)]
        q, s = rnd(rng, rng.randint(1, 400)), rnd(rng, rng.randint(1, 900))
        want = oracle.affine_construct(kind, q, s, *sc)
        for ns in (1, 2, 3, 4):
            got = anyseq.construct_local_sharded(kind, q, s, ns, *sc)
            assert got == want, (kind, len(q), len(s), sc, ns)


def test_sharded_construct_multi_level(anyseq):
    rng = random.Random(92)
    base = rnd(rng, 6000)
    mut = bytearray(base)
    for _ in range(300):
        mut[rng.randrange(len(mut))] = rng.choice(b"ACGT")
    for kind in KINDS:
        want = anyseq.construct(kind, base, bytes(mut[200:5800]), 2, -1, -2, -1)
        for ns in (2, 3, 8):
            assert anyseq.construct_local_sharded(kind, base, bytes(mut[200:5800]), ns, 2, -1, -2, -1) == want, (kind, ns)


def test_sharded_construct_config2(anyseq):
    """configs[2] (SW affine 65536^2) over 4 virtual ranks against the committed fixture."""
    g = json.load(open(os.path.join(GOLD, "config2_65536.json")))
    q, s = anyseq.main_random_pair(65536, 65536)
    sc = g["scoring"]
    v, aq, as_ = anyseq.construct_local_sharded(g["kind"], q, s, 4, sc["match"], sc["mismatch"], sc["gap_open"],
                                                sc["gap_extend"])
    assert v == g["score"]
    assert (hashlib.sha256(aq).hexdigest(), hashlib.sha256(as_).hexdigest()) == (g["sha_alq"], g["sha_als"])

"""GPU parity of the build-defined affine construct (anyseq_construct with gap_open < 0).

HIP path (C-ABI anyseq_construct) vs the oracle restatement
(oracle_affine_construct): score and both sparse i+j+1 strings bit-exact.  The
oracle itself is pinned by optimality/validity properties in
tests/test_oracle_affine.py (affine gaps have no reference semantics).
"""
import random

import pytest

pytestmark = pytest.mark.gpu

KINDS = ("global", "semiglobal", "local")
SCHEMES = [(2, -1, -2, -1), (1, -3, -5, -2), (5, -4, -10, -1), (3, -2, -1, -3), (2, -1, -1, -1)]


@pytest.fixture(autouse=True, params=["0", "1"], ids=["rows-unchecked", "rows-checked"])
def check_rows(request, monkeypatch):
    """Every case on the production path and with the hand-off row check after each
    planned fill (ANYSEQ_CHECK_ROWS, read per call)."""
    monkeypatch.setenv("ANYSEQ_CHECK_ROWS", request.param)
    return request.param


def rnd(rng, n, alphabet=b"ACGT"):
    return bytes(rng.choice(alphabet) for _ in range(n))


def same(anyseq, oracle, kind, q, s, sc):
    g = anyseq.construct(kind, q, s, match=sc[0], mismatch=sc[1], gap_open=sc[2], gap_extend=sc[3])
    o = oracle.affine_construct(kind, q, s, *sc)
    assert g[0] == o[0], (kind, len(q), len(s), sc, "score", g[0], o[0])
    assert g[1] == o[1] and g[2] == o[2], (kind, len(q), len(s), sc, "strings")


@pytest.mark.parametrize("kind", KINDS)
def test_affine_construct_random(anyseq, oracle, kind):
    rng = random.Random(51)
    for it in range(30):
        sc = SCHEMES[it % len(SCHEMES)]
        same(anyseq, oracle, kind, rnd(rng, rng.randint(1, 300)), rnd(rng, rng.randint(1, 700)), sc)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_construct_shapes(anyseq, oracle, kind):
    rng = random.Random(52)
    for n in (0, 1, 2, 63, 64, 65, 129, 300):
        for m in (0, 1, 64, 127, 128, 129, 255, 256, 257, 700):
            same(anyseq, oracle, kind, rnd(rng, n), rnd(rng, m), (2, -1, -2, -1))


@pytest.mark.parametrize("kind", KINDS)
def test_affine_construct_long_gaps(anyseq, oracle, kind):
    rng = random.Random(53)
    core = rnd(rng, 900)
    ins = rnd(rng, 350)
    q = core[:400] + core[700:]
    s = core[:200] + ins + core[200:]
    for sc in [(2, -1, -8, -1), (2, -1, -2, -1), (1, -1, -20, -1)]:
        same(anyseq, oracle, kind, q, core, sc)
        same(anyseq, oracle, kind, core, s, sc)
        same(anyseq, oracle, kind, s, q, sc)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_construct_multi_group(anyseq, oracle, kind):
    """Several workgroups per sub-problem, several Hirschberg levels, similar sequences."""
    rng = random.Random(54)
    base = rnd(rng, 3000)
    mut = bytearray(base)
    for _ in range(120):
        mut[rng.randrange(len(mut))] = rng.choice(b"ACGT")
    same(anyseq, oracle, kind, base, bytes(mut[100:2900]), (2, -1, -3, -1))
    same(anyseq, oracle, kind, rnd(rng, 2500), rnd(rng, 2100), (2, -1, -2, -1))
    same(anyseq, oracle, kind, rnd(rng, 60) + base[300:2000] + rnd(rng, 90), base, (1, -3, -5, -2))


@pytest.mark.parametrize("transpose", [0, 1])
@pytest.mark.parametrize("kind", KINDS)
def test_affine_construct_transposed_halves(anyseq, oracle, kind, transpose):
    """Hirschberg halves run transposed when taller than wide (affine_transpose 1, the
    default) or as they are (0): the same strings either way.  Shapes: tall, wide,
    square, and local alignments in a corner (free ends through several levels)."""
    rng = random.Random(55 + transpose)
    anyseq.set_option("affine_transpose", transpose)
    try:
        core = rnd(rng, 700)
        cases = [(rnd(rng, 3000), rnd(rng, 400)), (rnd(rng, 300), rnd(rng, 2600)), (rnd(rng, 1500), rnd(rng, 1500)),
                 (rnd(rng, 2000) + core, core + rnd(rng, 300)), (core[:500] + rnd(rng, 1800), rnd(rng, 900) + core)]
        for i, (q, s) in enumerate(cases):
            same(anyseq, oracle, kind, q, s, SCHEMES[i % len(SCHEMES)])
    finally:
        anyseq.set_option("affine_transpose", 1)


def test_affine_construct_planned_rows_stay_clean(anyseq, oracle):
    """Device-planned levels reuse one hand-off row buffer without a
    sentinel fill: every column a producer stores must get the sentinel back from its
    reader, including the band epilogue's columns past w.  Alternating shapes (odd and
    even widths, partial last chunks, several groups per half) move the per-launch row
    layout around, so a stale word left by one launch lands inside another's row."""
    rng = random.Random(58)
    for it in range(16):
        n = rng.randint(900, 2600) | (it & 1)
        m = rng.randint(900, 2600) | ((it >> 1) & 1)
        kind = KINDS[it % 3]
        same(anyseq, oracle, kind, rnd(rng, n), rnd(rng, m), SCHEMES[it % len(SCHEMES)])


@pytest.mark.parametrize("waves", [4, 7])
def test_affine_construct_row_check_fires(anyseq, oracle, monkeypatch, check_rows, waves):
    """The hand-off row invariant is checked, not timed (verdict round 3, item 1): with
    ANYSEQ_CHECK_ROWS a kernel scans every reused hand-off row after each planned fill.
    ANYSEQ_CHECK_ROWS=2 leaves one stale word past w in level 1's first half with a ring:
    the construct must fail naming that level, half and column, and the next construct
    (rows re-filled after the failure) must be right again -- with four compute waves
    per workgroup and with seven (verdict round 4, item 7)."""
    if check_rows == "0":
        pytest.skip("the check's own test runs once, under the checked parametrization")
    rng = random.Random(60)
    q, s = rnd(rng, 3001), rnd(rng, 2603)
    anyseq.set_option("affine_waves_per_group", waves)
    try:
        assert anyseq.construct("local", q, s, gap_open=-2, gap_extend=-1) == \
            oracle.affine_construct("local", q, s, 2, -1, -2, -1)
        monkeypatch.setenv("ANYSEQ_CHECK_ROWS", "2")
        with pytest.raises(anyseq.AnySeqError, match=r"hand-off row invariant broken after planned level 1: 1 "
                                                     r"non-sentinel word\(s\).*half 0, ring slot 0, column \d+"):
            anyseq.construct("local", q, s, gap_open=-2, gap_extend=-1)
        monkeypatch.setenv("ANYSEQ_CHECK_ROWS", "1")
        same(anyseq, oracle, "local", q, s, (2, -1, -2, -1))
    finally:
        anyseq.set_option("affine_waves_per_group", 0)


@pytest.mark.parametrize("virtual_best", [1, 0])
def test_affine_construct_virtual_best_border(anyseq, oracle, virtual_best):
    """Local construct halves with a free end and a NORMAL border take the best of every
    cell without the clamp; with min(match, mismatch) >= go + ge they run the virtual
    prologue, whose column -1 border cells cannot exceed cell (0,0).
    Schemes on both sides of that bound -- (2,-9,-1,-1) and (1,-6,-2,-2) keep the C++
    prologue -- and mostly-mismatching pairs, where a border cell would win if counted;
    the option off must give the same."""
    rng = random.Random(59)
    anyseq.set_option("virtual_best", virtual_best)
    try:
        for it in range(12):
            sc = [(2, -1, -2, -1), (2, -9, -1, -1), (1, -6, -2, -2), (3, -2, -1, -3)][it % 4]
            n, m = rng.randint(300, 1500), rng.randint(300, 1500)
            alph = (b"ACGT", b"AC", b"ACGTNRYK")[it % 3]
            q = rnd(rng, n, alph)
            s = rnd(rng, m, alph[::-1] if it % 2 else alph)
            same(anyseq, oracle, "local", q, s, sc)
    finally:
        anyseq.set_option("virtual_best", 1)


_NARROW_SCRIPT = r"""
import json, random, sys
sys.path.insert(0, %r)
import anyseq_amd as A
rng = random.Random(61)
rnd = lambda n: bytes(rng.choice(b"ACGT") for _ in range(n))
small = [(k, rnd(200), rnd(100)) for k in ("local", "semiglobal")]
core = rnd(300)
late = ("local", core, rnd(1500) + core + rnd(200))   # the alignment starts past column 512
cases = small + [late] + small
out = [[k, q.hex(), s.hex()] + [x if isinstance(x, int) else x.hex() for x in A.construct(k, q, s, 2, -1, -2, -1)]
       for k, q, s in cases]
print(json.dumps(out))
"""


def test_affine_construct_narrow_subject_fresh_process(oracle):
    """Advisor round 4 (high): with m <= 128 there is no Hirschberg level, so nothing on
    the device writes the level-1 score that the device-built final block table reads
    (aff_final_blocks_kernel skips every block of a local / semiglobal construct whose
    score is <= 0).  A stale word there -- a fresh buffer, or a split of 0 left by an
    earlier construct whose alignment starts past column 512 -- must not blank the
    strings: narrow constructs first in a fresh process, then after such a construct."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _NARROW_SCRIPT % root], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    for kind, qh, sh, score, aq, as_ in json.loads(r.stdout.strip().splitlines()[-1]):
        q, s = bytes.fromhex(qh), bytes.fromhex(sh)
        want = oracle.affine_construct(kind, q, s, 2, -1, -2, -1)
        assert (score, bytes.fromhex(aq), bytes.fromhex(as_)) == want, (kind, len(q), len(s))
        assert score > 0 and bytes.fromhex(aq).strip(), (kind, len(q), len(s))

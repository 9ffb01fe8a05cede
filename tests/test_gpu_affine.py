"""GPU parity for the affine-gap (Gotoh) fill: HIP path (C-ABI anyseq_score) vs the oracle.

Affine semantics are build-defined (the reference's affine_scoring_scheme,
align.impala:153-166, is dead code): oracle_affine_score in oracle/anyseq_oracle.c,
pinned on the CPU by `open == 0 => linear` and an independent textbook Gotoh
(tests/test_oracle.py).  Scores are integers: bit-exact.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

KINDS = ("global", "semiglobal", "local")
SCHEMES = [(2, -1, -2, -1), (2, -1, 0, -1), (1, -3, -5, -2), (5, -4, -10, -1), (3, -2, -1, -3)]


def rnd(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


def gpu(anyseq, kind, q, s, sc):
    return anyseq.score(kind, q, s, match=sc[0], mismatch=sc[1], gap_open=sc[2], gap_extend=sc[3])


def ora(oracle, kind, q, s, sc):
    return oracle.affine_score(kind, q, s, *sc)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_small_random(anyseq, oracle, kind):
    rng = random.Random(21)
    for it in range(60):
        sc = SCHEMES[it % len(SCHEMES)]
        n, m = rng.randint(1, 300), rng.randint(1, 300)
        q, s = rnd(rng, n), rnd(rng, m)
        assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, n, m, sc)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_edge_shapes(anyseq, oracle, kind):
    rng = random.Random(22)
    sc = (2, -1, -2, -1)
    for n in [0, 1, 2, 31, 32, 33, 63, 64, 65, 127, 128, 129, 511, 512, 513, 1023, 1024, 1025, 2049]:
        for m in (0, 1, 31, 32, 33, 63, 64, 65, 1000):
            q, s = rnd(rng, n), rnd(rng, m)
            assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, n, m)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_multi_group_two_fronts(anyseq, oracle, kind):
    """Several workgroups per problem (HBM hand-off of (G, F) rows) and the two-front split."""
    rng = random.Random(23)
    for (n, m), sc in zip([(5000, 3000), (3000, 7000), (4097, 4095), (9000, 300), (2100, 2100)],
                          [(2, -1, -2, -1), (1, -3, -5, -2), (2, -1, -3, -1), (5, -4, -10, -1), (2, -1, 0, -1)]):
        q, s = rnd(rng, n), rnd(rng, m)
        assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, n, m, sc)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_long_gaps_cross_split(anyseq, oracle, kind):
    """A long vertical gap spanning the two-front split row (opened once, not twice)."""
    rng = random.Random(24)
    core = rnd(rng, 1500)
    ins = rnd(rng, 1200)
    q = core[:700] + ins + core[700:]        # the query carries an insertion around row n/2
    s = core
    for sc in [(2, -1, -8, -1), (2, -1, -2, -1), (1, -1, -20, -1)]:
        assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, sc)
        assert gpu(anyseq, kind, s, q, sc) == ora(oracle, kind, s, q, sc), (kind, sc)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_open_zero_is_linear(anyseq, oracle, kind):
    rng = random.Random(25)
    for n, m in [(700, 900), (3000, 2500)]:
        q, s = rnd(rng, n), rnd(rng, m)
        assert anyseq.score(kind, q, s, gap_open=0, gap_extend=-1) == oracle.score(kind, q, s)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_bytes_and_similar(anyseq, oracle, kind):
    rng = random.Random(26)
    q = bytes(rng.randrange(256) for _ in range(700))
    s = bytes(rng.randrange(256) for _ in range(900))
    sc = (2, -1, -2, -1)
    assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc)
    base = rnd(rng, 3000)
    mut = list(base)
    for _ in range(150):
        mut[rng.randrange(len(mut))] = rng.choice("ACGT")
    s2 = "".join(mut)
    assert gpu(anyseq, kind, base, s2, sc) == ora(oracle, kind, base, s2, sc)


@pytest.mark.parametrize("nw", [3, 4, 7, 8])
def test_affine_waves_per_group(anyseq, oracle, nw):
    """Forced compute waves per workgroup (7: two per SIMD beside the I/O wave; 8: two per
    SIMD and no I/O wave, the groups' first bands forwarding their own input rows) give the
    same scores and constructs; 0 (the default) chooses per launch."""
    rng = random.Random(27)
    anyseq.set_option("affine_waves_per_group", nw)
    try:
        for kind in KINDS:
            q, s = rnd(rng, 2600), rnd(rng, 1900)
            sc = (2, -1, -3, -1)
            assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, nw)
            assert anyseq.construct(kind, q, s, *sc) == oracle.affine_construct(kind, q, s, *sc), (kind, nw)
    finally:
        anyseq.set_option("affine_waves_per_group", 0)


@pytest.mark.parametrize("option,value,default", [
    # (the round-4 I/O wave's options: the default build, with code rows in HBM, always runs
    # the forwarder and ignores them -- kept so that a non-GS build still runs them)
    ("io_stage", 0, 3), ("io_stage", 1, 3), ("io_stage", 2, 3),   # the I/O wave's subject staging
    ("io_poll2", 1, 0),                                           # two hand-off polls in flight
    ("io_skew", 2, 0),                                            # skewed blocks per polling pass
    ("priority", 0, -1), ("priority", 3, -1),                     # issue priority
    ("fill_events", 0, 1),                                        # no HIP events around the fills (bench's timed steps)
    ("affine_asm", 97, 1), ("affine_asm", 33, 1), ("affine_asm", 65, 1),   # round-3 ends / the start only / the end only
])
def test_affine_io_modes(anyseq, oracle, option, value, default):
    """The affine fill's I/O-wave and epilogue variants give the
    same scores and constructs: multi-group halves (HBM hand-offs through the I/O wave),
    a long subject (several staging batches) and both epilogues (the fused capture-free
    loop of bands nobody reads the last column of, the capturing one of the others)."""
    rng = random.Random(28)
    anyseq.set_option(option, value)
    try:
        for kind in KINDS:
            q, s = rnd(rng, 2600), rnd(rng, 1900)
            sc = (2, -1, -3, -1)
            assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, option, value)
            assert anyseq.construct(kind, q, s, *sc) == oracle.affine_construct(kind, q, s, *sc), (kind, option)
        q, s = rnd(rng, 700), rnd(rng, 9000)
        for kind in KINDS:
            assert gpu(anyseq, kind, q, s, (2, -1, -2, -1)) == ora(oracle, kind, q, s, (2, -1, -2, -1)), (kind, option)
    finally:
        anyseq.set_option(option, default)


@pytest.mark.parametrize("nw", [3, 4, 7])
@pytest.mark.parametrize("asm", [1, 65])
def test_affine_fused_end_every_cell_best(anyseq, oracle, nw, asm):
    """Round 5 (verdict round 4, item 1): the capture-free band end with a best of every
    cell (local scores and local constructs).  Round 4 saw local scores like 0x04000DB5
    at shapes 511x33, 1000x200 and 700x100 -- exactly those whose first band of a later
    workgroup (fed through the I/O wave) runs the asm end over a last chunk whose second
    half no hand-off poll covers (ceil(w/16) odd): a stale LDS word of an earlier
    workgroup there became the top row of cells past w, and their best won.  Shapes with
    and without that gap, three wave counts, the fused end with both band starts, and
    schemes where band 0's finite top border could seed a winner past w (mismatch far
    below the gap costs; > 8 symbols, the compare weights, with a positive mismatch):
    those keep the capturing end."""
    rng = random.Random(29)
    anyseq.set_option("affine_waves_per_group", nw)
    anyseq.set_option("affine_asm", asm)
    try:
        shapes = [(511, 33), (1000, 200), (700, 100), (1500, 64), (640, 47), (900, 81), (2600, 1900)]
        schemes = [(2, -1, -2, -1), (1, -6, -2, -1), (3, -2, -1, -3)]
        for i, (n, m) in enumerate(shapes):
            sc = schemes[i % len(schemes)]
            for alph in ("ACGT", "ACGTNRYKMSWB"):
                q, s = rnd(rng, n, alph), rnd(rng, m, alph)
                assert gpu(anyseq, "local", q, s, sc) == ora(oracle, "local", q, s, sc), (n, m, sc, alph)
                if n <= 1000:
                    assert anyseq.construct("local", q, s, *sc) == oracle.affine_construct("local", q, s, *sc), \
                        (n, m, sc, alph)
        q, s = rnd(rng, 700, "ACGTNRYKMSWB"), rnd(rng, 300, "ACGTNRYKMSWB")
        for sc in [(4, 1, -6, -1), (3, 0, -2, -2)]:   # a mismatch that does not lose
            assert gpu(anyseq, "local", q, s, sc) == ora(oracle, "local", q, s, sc), sc
            assert anyseq.construct("local", q, s, *sc) == oracle.affine_construct("local", q, s, *sc), sc
    finally:
        anyseq.set_option("affine_waves_per_group", 0)
        anyseq.set_option("affine_asm", 1)


@pytest.mark.parametrize("asm", [97, 3, 1, 0])
def test_affine_positive_mismatch(anyseq, oracle, asm):
    """Round 5: a mismatch that does not lose (> 0, or 0).  Under the local clamp the
    virtual prologue's cells are clamped to H = 0, so a diagonal step into them must not
    gain: the compare weights (> 8 symbols) gave code 0xFF the positive mismatch, and so
    did the C++ blocks' virtual columns (the asm LUT's -1 was right) -- local scores came
    out too high (468 vs 427; 89 vs 81).  Every kind, both weight paths, the asm / C++
    band ends and starts (affine_asm 97, 3: C++ epilogue, 1: fused end, 0: no asm)."""
    rng = random.Random(30)
    anyseq.set_option("affine_asm", asm)
    try:
        for it in range(24):
            sc = [(4, 1, -6, -1), (3, 0, -2, -2), (5, 2, -3, -1)][it % 3]
            alph = ("ACGT", "ACGTNRYKMSWB")[(it // 3) % 2]
            n, m = rng.randint(20, 400), rng.randint(20, 400)
            q, s = rnd(rng, n, alph), rnd(rng, m, alph)
            for kind in KINDS:
                assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, n, m, sc, alph, asm)
            if it % 4 == 0:
                assert anyseq.construct("local", q, s, *sc) == oracle.affine_construct("local", q, s, *sc), \
                    (n, m, sc, alph, asm)
    finally:
        anyseq.set_option("affine_asm", 1)


def test_affine_rejects_bad_scoring(anyseq):
    with pytest.raises(anyseq.AnySeqError):
        anyseq.score("global", "ACGT", "ACGT", gap_open=1, gap_extend=-1)
    with pytest.raises(anyseq.AnySeqError):
        anyseq.score("global", "ACGT", "ACGT", gap_open=-1, gap_extend=0)


@pytest.mark.parametrize("kind", KINDS)
def test_affine_xcd_groups(anyseq, oracle, kind):
    """XCD-local groups (round 5, FillParams::xq): the group table partitioned by XCD in
    runs of grid/8 consecutive groups and dequeued per XCD (a workgroup whose queue is
    empty takes from the others) gives the same scores and constructs: launches of 8..256
    workgroups (affine_grid), host-built and device-planned levels, tall and wide halves."""
    rng = random.Random(31)
    anyseq.set_option("xcd_groups", 1)
    try:
        for grid in (0, 64, 8):
            anyseq.set_option("affine_grid", grid)
            for n, m in ((2600, 1900), (700, 5000), (9000, 3000)):
                q, s = rnd(rng, n), rnd(rng, m)
                sc = (2, -1, -3, -1)
                assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, grid, n, m)
                assert anyseq.construct(kind, q, s, *sc) == oracle.affine_construct(kind, q, s, *sc), (kind, grid, n, m)
    finally:
        anyseq.set_option("xcd_groups", 0)
        anyseq.set_option("affine_grid", 0)


def test_affine_host_built_row_check(anyseq, oracle, monkeypatch):
    """Verdict round 4, item 7: the hand-off row check also covers host-built affine
    launches (score fronts, genome-length and sharded construct levels): with
    ANYSEQ_CHECK_ROWS every ring reused within a launch (nslots < ngroups - 1, here forced
    by an 8-workgroup grid) must be all sentinel again afterwards; =2 plants a stale word
    past w in the first such ring and the call must fail naming it, and the next call must
    be right."""
    rng = random.Random(32)
    q, s = rnd(rng, 20000), rnd(rng, 500)
    sc = (2, -1, -2, -1)
    want = ora(oracle, "local", q, s, sc)
    anyseq.set_option("affine_grid", 8)
    try:
        monkeypatch.setenv("ANYSEQ_CHECK_ROWS", "1")
        assert gpu(anyseq, "local", q, s, sc) == want
        monkeypatch.setenv("ANYSEQ_CHECK_ROWS", "2")
        with pytest.raises(anyseq.AnySeqError, match=r"hand-off row invariant broken after a host-built fill: 1 "
                                                     r"non-sentinel word\(s\)"):
            gpu(anyseq, "local", q, s, sc)
        monkeypatch.setenv("ANYSEQ_CHECK_ROWS", "1")
        assert gpu(anyseq, "local", q, s, sc) == want
        q2, s2 = rnd(rng, 6000), rnd(rng, 3000)
        assert anyseq.construct_local_sharded("local", q2, s2, 2, *sc) == anyseq.construct("local", q2, s2, *sc)
    finally:
        anyseq.set_option("affine_grid", 0)

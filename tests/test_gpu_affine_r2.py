"""GPU parity of the affine fill with TWO AND THREE ROWS PER LANE (round 5):
lane l holds rows R l .. R l + R-1 of a 64 R-row band (aff_blockn / gen_aff2 nrows), chosen
per launch for throughput-bound launches (aff_rows_for) and forced here with
`affine_rows_per_lane` 2 and 3 at four and seven compute waves.  Scores, host-built construct
levels (the device-planned levels keep one row per lane) and the column-block shards (the
left border of every row, the band's rows waited for, progress in 64-row units) against the
affine oracle, bit-exact: row counts that leave dead rows beside live ones in a lane,
band-size edges (127-129, 191-193 rows), both weight paths (LUT: <= 8 symbols; compare:
bytes), every border mode, the asm band ends and starts."""
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


# (NW 8: eight compute waves without the I/O wave, each group's first band forwarding its
# own input row -- DESIGN.md §3.5b; with one row per lane too)
@pytest.fixture(params=[(2, 7), (2, 4), (3, 7), (3, 4), (2, 8), (3, 8), (1, 8)], ids=lambda p: f"rows{p[0]}-nw{p[1]}")
def r2(anyseq, request):
    anyseq.set_option("affine_rows_per_lane", request.param[0])
    anyseq.set_option("affine_waves_per_group", request.param[1])
    anyseq.last_fill_multi_row_launches()
    try:
        yield request.param
        # the multi-row kernel actually ran (host-built fills of this test), with the rows asked for
        n, rmax = anyseq.last_fill_multi_row_launches()
        if request.param[0] > 1:
            assert n > 0 and rmax == request.param[0], (n, rmax)
    finally:
        anyseq.set_option("affine_rows_per_lane", 0)
        anyseq.set_option("affine_waves_per_group", 0)


def test_r2_small_random(anyseq, oracle, r2):
    rng = random.Random(41)
    for it in range(60):
        sc = SCHEMES[it % len(SCHEMES)]
        n, m = rng.randint(1, 400), rng.randint(1, 400)
        q, s = rnd(rng, n), rnd(rng, m)
        for kind in KINDS:
            assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, n, m, sc)


def test_r2_edge_shapes(anyseq, oracle, r2):
    rng = random.Random(42)
    sc = (2, -1, -2, -1)
    for n in [1, 2, 3, 4, 63, 64, 65, 127, 128, 129, 191, 192, 193, 255, 256, 257, 383, 384, 385, 895, 896, 897,
              1025, 2049]:
        for m in (1, 31, 32, 33, 64, 65, 1000):
            q, s = rnd(rng, n), rnd(rng, m)
            for kind in KINDS:
                assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, n, m)


def test_r2_multi_group(anyseq, oracle, r2):
    """Several workgroups per problem (HBM hand-off rows), the two-front split, long gaps."""
    rng = random.Random(43)
    for (n, m), sc in zip([(5000, 3000), (3001, 7000), (4097, 4095), (9001, 300), (2100, 2100)],
                          [(2, -1, -2, -1), (1, -3, -5, -2), (2, -1, -3, -1), (5, -4, -10, -1), (2, -1, 0, -1)]):
        q, s = rnd(rng, n), rnd(rng, m)
        for kind in KINDS:
            assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, n, m, sc)
    core = rnd(rng, 1500)
    q = core[:700] + rnd(rng, 1200) + core[700:]
    for sc in [(2, -1, -8, -1), (1, -1, -20, -1)]:
        for kind in KINDS:
            assert gpu(anyseq, kind, q, core, sc) == ora(oracle, kind, q, core, sc), (kind, sc)
            assert gpu(anyseq, kind, core, q, sc) == ora(oracle, kind, core, q, sc), (kind, sc)


def test_r2_compare_weights_and_positive_mismatch(anyseq, oracle, r2):
    """> 8 symbols (the compare path, row B's own query code) and mismatches that do not
    lose, over the asm / C++ band ends and starts (affine_asm 97, 3, 1, 0)."""
    rng = random.Random(44)
    q = bytes(rng.randrange(256) for _ in range(701))
    s = bytes(rng.randrange(256) for _ in range(900))
    for kind in KINDS:
        assert gpu(anyseq, kind, q, s, (2, -1, -2, -1)) == ora(oracle, kind, q, s, (2, -1, -2, -1)), kind
    for asm in (97, 3, 1, 0):
        anyseq.set_option("affine_asm", asm)
        try:
            for it in range(9):
                sc = [(4, 1, -6, -1), (3, 0, -2, -2), (5, 2, -3, -1)][it % 3]
                alph = ("ACGT", "ACGTNRYKMSWB")[it % 2]
                n, m = rng.randint(20, 400), rng.randint(20, 400)
                q, s = rnd(rng, n, alph), rnd(rng, m, alph)
                for kind in KINDS:
                    assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, n, m, sc, alph, asm)
        finally:
            anyseq.set_option("affine_asm", 1)


def test_r2_local_band_ends(anyseq, oracle, r2):
    """The fused band end with a best of every cell and the capturing end (local)."""
    rng = random.Random(45)
    shapes = [(511, 33), (1000, 200), (701, 100), (1500, 64), (641, 47), (900, 81), (2600, 1900)]
    schemes = [(2, -1, -2, -1), (1, -6, -2, -1), (3, -2, -1, -3)]
    for i, (n, m) in enumerate(shapes):
        sc = schemes[i % len(schemes)]
        for alph in ("ACGT", "ACGTNRYKMSWB"):
            q, s = rnd(rng, n, alph), rnd(rng, m, alph)
            assert gpu(anyseq, "local", q, s, sc) == ora(oracle, "local", q, s, sc), (n, m, sc, alph)


def test_r2_host_built_constructs(anyseq, oracle, r2):
    """Constructs through the host-built Hirschberg levels (out_col / out_col_e of both rows,
    last-row bests, transposed halves): the device plan off."""
    rng = random.Random(46)
    anyseq.set_option("affine_device_plan", 0)
    try:
        for n, m in ((2601, 1900), (700, 3001), (301, 257)):
            q, s = rnd(rng, n), rnd(rng, m)
            for kind in KINDS:
                sc = (2, -1, -3, -1)
                assert anyseq.construct(kind, q, s, *sc) == oracle.affine_construct(kind, q, s, *sc), (kind, n, m)
    finally:
        anyseq.set_option("affine_device_plan", 1)


def test_r2_shards(anyseq, oracle, r2):
    """Column-block shards: both rows' left border from the neighbour, the band's 128
    rows waited for, progress published in 64-row units."""
    rng = random.Random(47)
    for (n, m, ns) in [(130, 200, 2), (701, 901, 3), (1500, 1300, 4), (9001, 3000, 2), (4097, 2049, 3)]:
        q, s = rnd(rng, n), rnd(rng, m)
        for kind in KINDS:
            sc = (2, -1, -2, -1)
            got = anyseq.shard_score_local(kind, q, s, ns, match=sc[0], mismatch=sc[1], gap_open=sc[2],
                                           gap_extend=sc[3])
            assert got == ora(oracle, kind, q, s, sc), (kind, n, m, ns)


def test_self_forward_rows_stay_clean(anyseq, oracle, monkeypatch):
    """Eight compute waves without the I/O wave (the groups' first bands forward their own
    input rows): with a small grid every hand-off ring is reused within the launch, so the
    first bands must put the sentinel back exactly as the forwarder did -- checked after
    each host-built fill by ANYSEQ_CHECK_ROWS, at one to three rows per lane."""
    rng = random.Random(48)
    q, s = rnd(rng, 80000), rnd(rng, 700)   # (>= 53 groups of 8 bands at three rows: rings reused)
    sc = (2, -1, -2, -1)
    anyseq.set_option("affine_grid", 8)
    anyseq.set_option("affine_waves_per_group", 8)
    monkeypatch.setenv("ANYSEQ_CHECK_ROWS", "1")
    try:
        for rows in (1, 2, 3):
            anyseq.set_option("affine_rows_per_lane", rows)
            for kind in KINDS:
                assert gpu(anyseq, kind, q, s, sc) == ora(oracle, kind, q, s, sc), (kind, rows)
    finally:
        anyseq.set_option("affine_rows_per_lane", 0)
        anyseq.set_option("affine_waves_per_group", 0)
        anyseq.set_option("affine_grid", 0)

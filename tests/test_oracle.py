"""CPU tests: the oracle restatement against the golden vectors and an independent DP."""
import json
import os
import random

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
KINDS = ("global", "semiglobal", "local")


def load(name):
    return json.load(open(os.path.join(GOLD, name)))


def test_kat_scores(oracle):
    for c in load("kat.json")["scores"]:
        for k, v in c["score"].items():
            assert oracle.score(k, c["q"], c["s"]) == v, (k, c)


def test_kat_constructs(oracle):
    for c in load("kat.json")["constructs"]:
        r, aq, as_ = oracle.construct(c["kind"], c["q"], c["s"])
        assert (r, aq.decode(), as_.decode()) == (c["ret"], c["alq"], c["als"]), c["kind"]


@pytest.mark.parametrize("case", load("kat.json")["hand_constructs"], ids=lambda c: c["id"])
def test_hand_kat_constructs(oracle, case):
    """Round-2 hand-derived known answers (derivations in kat.json): hb_sum candidate order
    across two Hirschberg levels and across stride classes, compat walks that stop at
    PRED_NONE (local clamp, semiglobal border)."""
    r, aq, as_ = oracle.construct(case["kind"], case["q"], case["s"])
    assert (r, aq.decode(), as_.decode()) == (case["ret"], case["alq"], case["als"])


@pytest.mark.parametrize("case", load("kat.json")["hand_positions"], ids=lambda c: c["id"])
def test_hand_kat_semiglobal_position(oracle, case):
    """The semiglobal first-maximum position rule (scoring.impala:46-63): last row first,
    index -1 first, the column only if strictly greater."""
    assert oracle.score(case["kind"], case["q"], case["s"], with_pos=True) == (case["score"], *case["pos"])


def test_textbook_cross_check(oracle):
    rng = random.Random(5)
    for _ in range(150):
        n, m = rng.randint(0, 60), rng.randint(0, 60)
        q = "".join(rng.choice("ACGT") for _ in range(n))
        s = "".join(rng.choice("ACGT") for _ in range(m))
        for k in KINDS:
            assert oracle.score(k, q, s) == oracle.textbook_score(k, q, s), (k, q, s)


def test_textbook_multi_tile(oracle):
    # crosses the 1024x1024 tile seams of iteration_cpu.impala:1-57 (corners, seam column)
    rng = random.Random(6)
    for n, m in [(1500, 2100), (2049, 1025)]:
        q = "".join(rng.choice("ACGT") for _ in range(n))
        s = "".join(rng.choice("ACGT") for _ in range(m))
        for k in KINDS:
            assert oracle.score(k, q, s) == oracle.textbook_score(k, q, s), (k, n, m)


def test_thread_count_invariance(oracle):
    rng = random.Random(7)
    q = "".join(rng.choice("ACGT") for _ in range(2500))
    s = "".join(rng.choice("ACGT") for _ in range(3100))
    ref = {k: (oracle.score(k, q, s), oracle.construct(k, q, s)) for k in KINDS}
    for t in (1, 3, 8):
        oracle.set_threads(t)
        for k in KINDS:
            assert (oracle.score(k, q, s), oracle.construct(k, q, s)) == ref[k], (t, k)
    oracle.set_threads(4)


def test_golden_oracle_cases(oracle):
    for c in load("oracle_cases.json")["cases"]:
        for k in KINDS:
            assert oracle.score(k, c["q"], c["s"]) == c["score"][k]
            r, aq, as_ = oracle.construct(k, c["q"], c["s"])
            g = c["construct"][k]
            assert (r, aq.decode(), as_.decode()) == (g["ret"], g["alq"], g["als"])


def _dense(aq, as_):
    keep = [i for i in range(len(aq)) if not (aq[i] == 32 and as_[i] == 32)]
    return bytes(aq[i] for i in keep), bytes(as_[i] for i in keep)


def _aln_score(a, b):
    sc = 0
    for x, y in zip(a, b):
        sc += -1 if (x == 95 or y == 95) else (2 if x == y else -1)
    return sc


def test_global_construct_is_optimal(oracle):
    """The column-split Hirschberg yields an optimal global alignment of both full sequences."""
    rng = random.Random(8)
    for _ in range(20):
        n, m = rng.randint(65, 1200), rng.randint(65, 1200)
        q = "".join(rng.choice("ACGT") for _ in range(n))
        s = "".join(rng.choice("ACGT") for _ in range(m))
        _, aq, as_ = oracle.construct("global", q, s)
        dq, ds = _dense(aq, as_)
        assert dq.replace(b"_", b"") == q.encode() and ds.replace(b"_", b"") == s.encode()
        assert _aln_score(dq, ds) == oracle.score("global", q, s)


def test_no_unset_split_reads(oracle):
    rng = random.Random(9)
    for m in list(range(1, 300, 7)) + [1023, 1024, 1025, 2047, 2049, 4097]:
        n = rng.randint(0, 400)
        q = "".join(rng.choice("ACGT") for _ in range(n))
        s = "".join(rng.choice("ACGT") for _ in range(m))
        for k in KINDS:
            oracle.construct(k, q, s)   # raises on an unset split read


def test_affine_reduces_to_linear(oracle):
    rng = random.Random(10)
    for _ in range(60):
        n, m = rng.randint(0, 80), rng.randint(0, 80)
        q = "".join(rng.choice("ACGT") for _ in range(n))
        s = "".join(rng.choice("ACGT") for _ in range(m))
        for k in KINDS:
            assert oracle.affine_score(k, q, s, 2, -1, 0, -1) == oracle.score(k, q, s)
            assert (oracle.affine_score(k, q, s, 2, -1, -3, -1)
                    == oracle.textbook_affine_score(k, q, s, 2, -1, -3, -1))


def test_main_input_fingerprints(anyseq):
    """anyseq_main_random_pair reproduces main.cpp's inputs."""
    def fnv(b):
        h = 1469598103934665603
        for c in b:
            h ^= c
            h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
        return f"{h:016x}"
    for c in load("main_inputs.json")["cases"]:
        q, s = anyseq.main_random_pair(*c["args"])
        assert (len(q), len(s)) == (c["lq"], c["ls"])
        assert q[:32].decode() == c["q32"] and s[:32].decode() == c["s32"]
        assert fnv(q) == c["fnv_q"] and fnv(s) == c["fnv_s"]


def test_main_1024_golden(oracle, anyseq):
    g = load("main_1024.json")
    q, s = anyseq.main_random_pair(1024, 1024)
    for k in KINDS:
        assert oracle.score(k, q, s) == g["score"][k]
        r, aq, as_ = oracle.construct(k, q, s)
        assert (r, aq.decode(), as_.decode()) == (g["construct"][k]["ret"], g["construct"][k]["alq"],
                                                  g["construct"][k]["als"])


def test_main_65536_construct_golden(oracle, anyseq):
    """The oracle regenerates the full-size configs[1] construct pins (SHA-256 of both
    sparse strings; ~13 s at 8 threads): the fixture the GPU test compares against is
    the restatement's own output, not a stale file."""
    import hashlib
    g = load("main_65536.json")["construct"]
    q, s = anyseq.main_random_pair(65536, 65536)
    oracle.set_threads(8)
    try:
        for k in KINDS:
            r, aq, as_ = oracle.construct(k, q, s)
            assert r == g[k]["ret"]
            assert hashlib.sha256(aq).hexdigest() == g[k]["sha256_alq"]
            assert hashlib.sha256(as_).hexdigest() == g[k]["sha256_als"]
    finally:
        oracle.set_threads(4)

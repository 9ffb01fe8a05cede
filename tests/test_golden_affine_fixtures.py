"""CPU checks of the full-size affine construct fixtures (tests/golden/config*.json):
the stored CIGAR is a valid alignment of exactly q[is..ie] x s[js..je] (the stored
rectangle), its affine score recomputed here equals the stored score, and that score is
the optimum of the affine DP (oracle_affine_score over the full matrix).  The inputs are
rebuilt by the reference driver's generator (anyseq_main_random_pair, host code) and
genome.synthetic_related_pair and checked against the stored SHA-256."""
import hashlib
import json
import os
import re

import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def rescore_cigar(cigar, q, s, rect, sc):
    i, j = rect[0], rect[2]
    score, prev = 0, None
    for cnt, op in re.findall(r"(\d+)([=XID])", cigar):
        cnt = int(cnt)
        for _ in range(cnt):
            if op in "=X":
                assert (q[i] == s[j]) == (op == "="), (i, j, op)
                score += sc["match"] if op == "=" else sc["mismatch"]
                i, j = i + 1, j + 1
            elif op == "I":   # query byte against a gap
                score += sc["gap_extend"] + (sc["gap_open"] if prev != "I" else 0)
                i += 1
            else:             # subject byte against a gap
                score += sc["gap_extend"] + (sc["gap_open"] if prev != "D" else 0)
                j += 1
            prev = op if op in "ID" else None
    assert (i - 1, j - 1) == (rect[1], rect[3]), "the CIGAR does not end at the rectangle's corner"
    return score


def check(oracle, g, q, s, full_optimum=True):
    assert (sha(q), sha(s)) == (g["sha_q"], g["sha_s"])
    sc = g["scoring"]
    assert rescore_cigar(g["cigar"], q, s, g["rect"], sc) == g["score"]
    if full_optimum:
        assert oracle.affine_score(g["kind"], q, s, sc["match"], sc["mismatch"], sc["gap_open"],
                                   sc["gap_extend"]) == g["score"]


def test_config2_fixture(anyseq, oracle):
    g = json.load(open(os.path.join(GOLD, "config2_65536.json")))
    q, s = anyseq.main_random_pair(65536, 65536)
    check(oracle, g, q, s)


def test_config3_fixture(anyseq, oracle):
    path = os.path.join(GOLD, "config3_prefix.json")
    if not os.path.exists(path):
        pytest.skip("config3_prefix.json not generated")
    from anyseq_amd import genome
    g = json.load(open(path))
    q, s = genome.synthetic_related_pair(4_641_652, 0.9)
    # the 262144^2 optimum takes ~2 min single-threaded: the rescoring alone here
    check(oracle, g, q[:g["lq"]], s[:g["ls"]], full_optimum=False)


@pytest.mark.parametrize("name", ["config2_nonpow2", "config3_nonpow2"])
def test_nonpow2_fixtures(anyseq, oracle, name):
    g = json.load(open(os.path.join(GOLD, name + ".json")))
    if name.startswith("config2"):
        q, s = anyseq.main_random_pair(65536, 65536)
    else:
        from anyseq_amd import genome
        q, s = genome.synthetic_related_pair(4_641_652, 0.9)
    check(oracle, g, q[:g["lq"]], s[:g["ls"]], full_optimum=name.startswith("config2"))

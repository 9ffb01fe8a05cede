"""GPU path against the full-size affine construct fixtures (tests/golden/make_golden_affine.py):
configs[2] (local affine score + traceback of main.cpp's `-r 65536 65536` pair) and the
configs[3] workload on a 262,144-bp prefix of the synthetic genome pair (semiglobal).
Bit-exact: score, SHA-256 of both sparse i+j+1 strings, and the dense CIGAR."""
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def check(anyseq, g, q, s):
    assert (len(q), len(s), sha(q), sha(s)) == (g["lq"], g["ls"], g["sha_q"], g["sha_s"]), "inputs differ"
    sc = g["scoring"]
    v, aq, as_ = anyseq.construct(g["kind"], q, s, match=sc["match"], mismatch=sc["mismatch"],
                                  gap_open=sc["gap_open"], gap_extend=sc["gap_extend"])
    assert v == g["score"]
    assert anyseq.cigar(aq, as_) == g["cigar"]
    assert (sha(aq), sha(as_)) == (g["sha_alq"], g["sha_als"])


def test_config2_local_affine_65536(anyseq):
    g = json.load(open(os.path.join(GOLD, "config2_65536.json")))
    q, s = anyseq.main_random_pair(65536, 65536)
    check(anyseq, g, q, s)


def test_config3_semiglobal_affine_prefix(anyseq):
    path = os.path.join(GOLD, "config3_prefix.json")
    if not os.path.exists(path):
        pytest.skip("config3_prefix.json not generated")
    from anyseq_amd import genome
    g = json.load(open(path))
    q, s = genome.synthetic_related_pair(4_641_652, 0.9)
    check(anyseq, g, q[:g["lq"]], s[:g["ls"]])


@pytest.mark.parametrize("name", ["config2_nonpow2", "config3_nonpow2"])
def test_nonpow2_fixtures(anyseq, name):
    """Subject lengths whose 128-column block count is not a power of two: every level's
    parts split at their middle block (aff_part_geo, round 4), the oracle's rule."""
    g = json.load(open(os.path.join(GOLD, name + ".json")))
    if name.startswith("config2"):
        q, s = anyseq.main_random_pair(65536, 65536)
    else:
        from anyseq_amd import genome
        q, s = genome.synthetic_related_pair(4_641_652, 0.9)
    check(anyseq, g, q[:g["lq"]], s[:g["ls"]])


def test_config3_genome_length_construct(anyseq):
    """configs[3] and configs[4] at full genome length (4.64 Mbp x 4.64 Mbp, synthetic related
    pair; the oracle cannot reach this size, so parity is by properties): the construct's
    strings re-score to its score, their residues are substrings of the inputs, and the
    score equals the score-only fill's and the 2-shard column-blocked fill's (configs[4]'s
    path, in-process transport)."""
    import numpy as np
    from anyseq_amd import genome
    q, s = genome.synthetic_related_pair(4_641_652, 0.9)
    v, aq, as_ = anyseq.construct("semiglobal", q, s, gap_open=-2, gap_extend=-1)
    assert genome.affine_rescore(aq, as_) == v
    for al, seq in ((aq, q), (as_, s)):
        a = np.frombuffer(al, dtype=np.uint8)
        res = a[(a != ord(" ")) & (a != ord("_"))].tobytes()
        assert len(res) > 0.9 * len(seq) and seq.find(res) >= 0
    assert anyseq.score("semiglobal", q, s, gap_open=-2, gap_extend=-1) == v
    assert anyseq.shard_score_local("semiglobal", q, s, 2, gap_open=-2, gap_extend=-1) == v
    # the bench gate's anchor (tests/golden/config4_synthetic.json, round 6): same score
    # and, for the construct, the same strings as the single-GPU run that wrote it
    g = json.load(open(os.path.join(GOLD, "config4_synthetic.json")))
    assert (g["lq"], g["ls"], g["sha_q"], g["sha_s"]) == (len(q), len(s), sha(q), sha(s))
    assert v == g["score"] == g["construct_score"]
    assert (sha(aq), sha(as_)) == (g["construct_sha_alq"], g["construct_sha_als"])

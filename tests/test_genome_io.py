"""CPU: genome-input helpers (anyseq_amd/genome.py) against the reference's own
reader (fixtures from sequence_io.cpp, tests/golden/make_fasta_golden.py) and the
oracle (alignment re-scoring)."""
import json
import os

import pytest

from anyseq_amd import genome

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "fasta_cases.json")))["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_first_record_matches_reference_reader(tmp_path, case):
    p = tmp_path / case["name"]
    p.write_bytes(bytes.fromhex(case["content"]))
    if case["ok"]:
        h, d = genome.first_record(str(p))
        assert (h, d) == (bytes.fromhex(case["header"]), bytes.fromhex(case["data"]))
    else:
        with pytest.raises(ValueError):
            genome.first_record(str(p))


def test_synthetic_pair_is_deterministic_and_related():
    q1, s1 = genome.synthetic_related_pair(50000, 0.9)
    q2, s2 = genome.synthetic_related_pair(50000, 0.9)
    assert (q1, s1) == (q2, s2)
    assert set(q1) <= set(b"ACGT") and set(s1) <= set(b"ACGT")
    assert abs(len(s1) - len(q1)) < 500


@pytest.mark.parametrize("kind", ["global", "semiglobal", "local"])
def test_affine_rescore_equals_oracle_optimum(oracle, kind):
    q, s = genome.synthetic_related_pair(3000, 0.85, seed=7)
    v, aq, as_ = oracle.affine_construct(kind, q, s, 2, -1, -2, -1)
    assert genome.affine_rescore(aq, as_) == v

"""CPU: alignment-output adapters of the C-ABI (anyseq_alignment_dense / _cigar,
host code, no GPU) on the oracle's sparse construct outputs, checked against an
independent pure-Python conversion and against the strings' own content."""
import random

import pytest


def py_dense(aq, as_):
    keep = [i for i in range(len(aq)) if not (aq[i] == 32 and as_[i] == 32)]
    return bytes(aq[i] for i in keep), bytes(as_[i] for i in keep)


def py_cigar(dq, ds):
    out, prev, run = [], None, 0
    for a, b in zip(dq, ds):
        op = "D" if a == 95 else ("I" if b == 95 else ("=" if a == b else "X"))
        if op != prev and run:
            out.append(f"{run}{prev}")
            run = 0
        prev, run = op, run + 1
    if run:
        out.append(f"{run}{prev}")
    return "".join(out)


@pytest.mark.parametrize("kind", ["global", "semiglobal", "local"])
def test_dense_and_cigar_on_oracle_alignments(anyseq, oracle, kind):
    rng = random.Random(61)
    for n, m in [(300, 280), (700, 900), (129, 1000)]:
        q = "".join(rng.choice("ACGT") for _ in range(n))
        s = "".join(rng.choice("ACGT") for _ in range(m))
        _, aq, as_ = oracle.construct(kind, q, s)
        dq, ds = anyseq.dense(aq, as_)
        assert (dq, ds) == py_dense(aq, as_)
        cg = anyseq.cigar(aq, as_)
        assert cg == py_cigar(dq, ds)
        # the CIGAR re-derives the dense strings' consumed lengths
        import re
        ops = re.findall(r"(\d+)([=XID])", cg)
        qlen = sum(int(k) for k, o in ops if o in "=XI")
        slen = sum(int(k) for k, o in ops if o in "=XD")
        assert qlen == len(dq) - dq.count(b"_") and slen == len(ds) - ds.count(b"_")
        if kind == "global" and m > 64:
            assert qlen == n and slen == m


def test_cigar_edge_cases(anyseq):
    assert anyseq.cigar(b"", b"") == ""
    assert anyseq.cigar(b"  A", b"  A") == "1="
    assert anyseq.cigar(b"A_C", b"AGT") == "1=1D1X"
    assert anyseq.cigar(b"AAC", b"A_C") == "1=1I1="
    assert anyseq.dense(b" A  C", b" A  G") == (b"AC", b"AG")

"""Genome-scale inputs for BASELINE.json configs[3]/[4].

* ``first_record(path)`` -- the sequence main.cpp aligns for ``align -i q s``:
  the FIRST record of each file, read with the reference reader's semantics
  (main.cpp:182-189, sequence_io.cpp:62-110 fasta, :131-163 fastq, format by
  extension or first byte :205-239).  Data lines are concatenated raw: bytes are
  kept as they are (lowercase, N, a trailing CR of CRLF files), only the '\\n'
  line ends are dropped.  A FASTA record with no data raises ValueError (the
  reference throws io_format_error, and main.cpp then keeps the FILE NAME as the
  sequence -- a quirk this reader reports instead of reproducing).
* ``synthetic_related_pair(n, identity)`` -- the E. coli / S. boydii FASTAs are
  absent from the reference snapshot (.MISSING_LARGE_BLOBS:1-2), so the genome
  configs run on a synthetic pair: a uniform-ACGT query and a subject derived
  from it by substitutions and 1-base indels, so that a long alignment path
  exists as between two related genomes.
"""
from __future__ import annotations

import numpy as np

_FASTQ_EXT = (".fq", ".fnq", ".fastq")
_FASTA_EXT = (".fa", ".fna", ".fasta")


def _fmt(path: str, head: bytes) -> str:
    if path.endswith(_FASTQ_EXT):
        return "fastq"
    if path.endswith(_FASTA_EXT):
        return "fasta"
    if head[:1] == b">":
        return "fasta"
    if head[:1] == b"@":
        return "fastq"
    raise ValueError("file format not recognized")


def first_record(path: str) -> tuple[bytes, bytes]:
    """(header, data) of the first record of a FASTA/FASTQ file."""
    with open(path, "rb") as f:
        raw = f.read()
    lines = raw.split(b"\n")
    if raw.endswith(b"\n"):
        lines = lines[:-1]
    fmt = _fmt(path, raw[:1])
    if not lines:
        raise ValueError("empty file")
    if fmt == "fastq":
        if not lines[0].startswith(b"@"):
            raise ValueError("malformed fastq file - sequence header")
        return lines[0][1:], lines[1] if len(lines) > 1 else b""
    if not lines[0].startswith(b">"):
        raise ValueError("malformed fasta file - expected header char > not found")
    data = []
    for ln in lines[1:]:
        if ln.startswith(b">"):
            break
        data.append(ln)
    seq = b"".join(data)
    if not seq:
        raise ValueError("malformed fasta file - zero-length sequence")
    return lines[0][1:], seq


def synthetic_related_pair(n: int, identity: float = 0.9, seed: int = 5489) -> tuple[bytes, bytes]:
    """Uniform-ACGT query of n bases and a related subject: substitutions at rate
    0.8*(1-identity), 1-base deletions and insertions at 0.1*(1-identity) each."""
    rng = np.random.Generator(np.random.PCG64(seed))
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    q = acgt[rng.integers(0, 4, n)]
    d = 1.0 - identity
    r = rng.random(n)
    sub = r < d * 0.8
    dele = (r >= d * 0.8) & (r < d * 0.9)
    ins = (r >= d * 0.9) & (r < d)
    s = q.copy()
    s[sub] = acgt[(np.searchsorted(acgt, s[sub]) + rng.integers(1, 4, int(sub.sum()))) % 4]
    parts = np.stack([s, np.where(ins, acgt[rng.integers(0, 4, n)], 0)], axis=1).reshape(-1)
    mask = np.stack([~dele, ins], axis=1).reshape(-1)
    return q.tobytes(), parts[mask].tobytes()


def affine_rescore(aq: bytes, as_: bytes, match=2, mismatch=-1, gap_open=-2, gap_extend=-1) -> int:
    """Score of an alignment in the sparse i+j+1 layout (blank pairs dropped), a gap
    run of length k costing gap_open + k*gap_extend: checks a construct's strings
    against the fill's optimum at sizes the oracle cannot reach."""
    a = np.frombuffer(aq, dtype=np.uint8)
    b = np.frombuffer(as_, dtype=np.uint8)
    keep = ~((a == 32) & (b == 32))
    a, b = a[keep], b[keep]
    gq, gs = a == ord("_"), b == ord("_")
    col = ~(gq | gs)
    v = int(np.where(a[col] == b[col], match, mismatch).sum())
    for g in (gq, gs):
        v += int(g.sum()) * gap_extend
        starts = g & ~np.concatenate([[False], g[:-1]])
        v += int(starts.sum()) * gap_open
    return v

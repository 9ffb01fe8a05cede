#!/usr/bin/env python3
"""Genome-scale run (BASELINE.json configs[3]) on the GPU box:
python tools/genome_probe.py [n] [identity]

The E. coli / S. boydii FASTAs are not in the reference snapshot
(.MISSING_LARGE_BLOBS), so the pair is SYNTHETIC: a uniform-ACGT query of n
bases (mt19937_64-free numpy PCG64 seed 5489) and a subject derived from it by
substitutions/indels at the given identity, which gives a real alignment path
like two related genomes.  Prints the score fill and the semi-global affine
linear-memory construct (Hirschberg) with their times, and checks the construct
against the score (the alignment strings re-scored on the CPU equal the fill's
optimum).
"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import anyseq_amd as A  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_641_652
ident = float(sys.argv[2]) if len(sys.argv) > 2 else 0.9
kinds = sys.argv[3].split(",") if len(sys.argv) > 3 else ["semiglobal"]
rng = np.random.Generator(np.random.PCG64(5489))
acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
q = acgt[rng.integers(0, 4, n)]
# subject: substitutions at rate (1-ident)*0.8, 1-base indels at (1-ident)*0.1 each
r = rng.random(n)
sub = r < (1 - ident) * 0.8
dele = (r >= (1 - ident) * 0.8) & (r < (1 - ident) * 0.9)
ins = (r >= (1 - ident) * 0.9) & (r < (1 - ident))
s = q.copy()
s[sub] = acgt[(np.searchsorted(acgt, s[sub]) + rng.integers(1, 4, int(sub.sum()))) % 4]
keep = ~dele
parts = np.stack([s, np.where(ins, acgt[rng.integers(0, 4, n)], 0)], axis=1).reshape(-1)
mask = np.stack([keep, ins], axis=1).reshape(-1)
s = parts[mask]
qb, sb = q.tobytes(), s.tobytes()
cells = len(qb) * len(sb)
print(f"synthetic pair: query {len(qb)} bp, subject {len(sb)} bp, {cells / 1e12:.2f} T cells", flush=True)
T0 = time.perf_counter()


def heartbeat():   # the box treats 3 silent minutes as a hang
    while True:
        time.sleep(30)
        print(f"  ... {time.perf_counter() - T0:.0f} s", flush=True)


threading.Thread(target=heartbeat, daemon=True).start()
SC = dict(match=2, mismatch=-1, gap_open=-2, gap_extend=-1)


def rescore(aq: bytes, as_: bytes) -> int:
    """Affine score of the dense alignment (gap run costs open + len*extend)."""
    a = np.frombuffer(aq, dtype=np.uint8)
    b = np.frombuffer(as_, dtype=np.uint8)
    keep = ~((a == 32) & (b == 32))
    a, b = a[keep], b[keep]
    gq, gs = a == ord("_"), b == ord("_")
    col = ~(gq | gs)
    v = int(np.where(a[col] == b[col], SC["match"], SC["mismatch"]).sum())
    for g in (gq, gs):
        v += int(g.sum()) * SC["gap_extend"]
        starts = g & ~np.concatenate([[False], g[:-1]])
        v += int(starts.sum()) * SC["gap_open"]
    return v


for kind in kinds:
    A.last_fill_timing()
    t = time.perf_counter()
    v = A.score(kind, qb, sb, **SC)
    dt = time.perf_counter() - t
    ms, launches = A.last_fill_timing()
    print(f"score {kind} affine: {v} wall {dt:.2f} s, fill {ms / 1e3:.2f} s -> {cells / ms / 1e6:.0f} GCUPS",
          flush=True)
    t = time.perf_counter()
    cv, aq, as_ = A.construct(kind, qb, sb, **SC)
    dt = time.perf_counter() - t
    ms, launches = A.last_fill_timing()
    rs = rescore(aq, as_)
    print(f"construct {kind} affine: score {cv} (re-scored {rs}) wall {dt:.2f} s, fill {ms / 1e3:.2f} s in "
          f"{launches} launches; n*m/wall = {cells / dt / 1e9:.0f} GCUPS", flush=True)
    assert cv == v == rs, (cv, v, rs)
print("genome probe ok", flush=True)

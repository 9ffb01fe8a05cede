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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import anyseq_amd as A  # noqa: E402
from anyseq_amd import genome as G  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_641_652
ident = float(sys.argv[2]) if len(sys.argv) > 2 else 0.9
kinds = sys.argv[3].split(",") if len(sys.argv) > 3 else ["semiglobal"]
qb, sb = G.synthetic_related_pair(n, ident)
cells = len(qb) * len(sb)
print(f"synthetic pair: query {len(qb)} bp, subject {len(sb)} bp, {cells / 1e12:.2f} T cells", flush=True)
T0 = time.perf_counter()


def heartbeat():   # the box treats 3 silent minutes as a hang
    while True:
        time.sleep(30)
        print(f"  ... {time.perf_counter() - T0:.0f} s", flush=True)


threading.Thread(target=heartbeat, daemon=True).start()
SC = dict(match=2, mismatch=-1, gap_open=-2, gap_extend=-1)


rescore = G.affine_rescore


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

#!/usr/bin/env python3
"""Timing probe for the north-star configs (GPU box): python tools/perf_probe.py [n]

Prints fill-kernel time and GCUPS for the linear/affine score fills and the
wall time of the Hirschberg construct, on main.cpp's `-r n n` inputs.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import anyseq_amd as A  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
q, s = A.main_random_pair(n, n)
cells = len(q) * len(s)
AFF = dict(match=2, mismatch=-1, gap_open=-2, gap_extend=-1)
LIN = dict(match=2, mismatch=-1, gap_open=0, gap_extend=-1)

for name, sc in (("linear", LIN), ("affine", AFF)):
    for kind in ("global", "semiglobal", "local"):
        A.score(kind, q[:4096], s[:4096], **sc)
        A.last_fill_timing()
        best = 1e9
        for _ in range(3):
            v = A.score(kind, q, s, **sc)
            ms, _ = A.last_fill_timing()
            best = min(best, ms)
        print(f"score {name:6s} {kind:10s} {len(q)}x{len(s)} score={v} fill={best:.3f} ms "
              f"GCUPS={cells / best / 1e6:.0f}", flush=True)

for name, sc in (("linear", LIN), ("affine", AFF)):
    for kind in ("global", "local"):
        A.construct(kind, q[:4096], s[:4096], **sc)
        A.last_fill_timing()
        t = time.perf_counter()
        v, aq, as_ = A.construct(kind, q, s, **sc)
        dt = time.perf_counter() - t
        ms, launches = A.last_fill_timing()
        print(f"construct {name:6s} {kind:10s} score={v} wall={dt * 1e3:.1f} ms fill={ms:.1f} ms in {launches} "
              f"launches, GCUPS(n*m/wall)={cells / dt / 1e9:.0f}", flush=True)

#!/usr/bin/env python3
"""Tuning sweep on the GPU box: python tools/sweep_probe.py
Fill time of the 65536^2 score for several tuning options, and the
steady-state rate on a long matrix (pipeline ramp amortised)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import anyseq_amd as A  # noqa: E402


def run(kind, q, s, reps=3, **sc):
    A.score(kind, q[:2048], s[:2048], **sc)
    A.last_fill_timing()
    best = 1e9
    v = None
    for _ in range(reps):
        v = A.score(kind, q, s, **sc)
        ms, _ = A.last_fill_timing()
        best = min(best, ms)
    return v, best


q, s = A.main_random_pair(65536, 65536)
cells = len(q) * len(s)
AFF = dict(gap_open=-2, gap_extend=-1)
for opts in ([], [("chunk", 16)], [("waves_per_group", 8)], [("waves_per_group", 3)], [("waves_per_group", 7)],
             [("fronts", 1)], [("rows_per_lane", 2)], [("grid", 512)]):
    for k, v in opts:
        A.set_option(k, v)
    v, ms = run("global", q, s)
    print(f"linear global 64k {opts}: {ms:.3f} ms {cells / ms / 1e6:.0f} GCUPS score {v}", flush=True)
    for k, _ in opts:
        A.set_option(k, {"chunk": 32, "waves_per_group": 4, "fronts": 2, "rows_per_lane": 1, "grid": 0}[k])
for opts in ([], [("affine_waves_per_group", 3)], [("affine_grid", 512)]):
    for k, v in opts:
        A.set_option(k, v)
    for kind in ("global", "local"):
        v, ms = run(kind, q, s, **AFF)
        print(f"affine {kind} 64k {opts}: {ms:.3f} ms {cells / ms / 1e6:.0f} GCUPS score {v}", flush=True)
    for k, _ in opts:
        A.set_option(k, {"affine_waves_per_group": 4, "affine_grid": 0}[k])
# long matrix: 8192 rows x 2M columns (the ramp is a small part of the time)
ql, sl = A.main_random_pair(2_000_000, 2_000_000)
ql = ql[:8192]
c2 = len(ql) * len(sl)
for name, sc in (("linear", {}), ("affine", AFF)):
    for kind in ("global", "local"):
        v, ms = run(kind, ql, sl, reps=2, **sc)
        print(f"{name} {kind} 8192x{len(sl)}: {ms:.3f} ms {c2 / ms / 1e6:.0f} GCUPS", flush=True)

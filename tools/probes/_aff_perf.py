# Affine fill timing probe (GPU box): python tests/_aff_perf.py
import sys
sys.path.insert(0, '.')
import anyseq_amd as A
q, s = A.main_random_pair(65536, 65536)
sc = dict(match=2, mismatch=-1, gap_open=-2, gap_extend=-1)
for kind in ("local", "global"):
    for nw, grid in [(4, 0), (3, 0)]:
        A.set_option("affine_waves_per_group", nw); A.set_option("affine_grid", grid)
        A.score(kind, q[:4096], s[:4096], **sc); A.last_fill_timing()
        best = 1e9
        for _ in range(3):
            v = A.score(kind, q, s, **sc); ms, _ = A.last_fill_timing(); best = min(best, ms)
        print(f"{kind} NW={nw} grid={grid} score={v} kernel={best:.2f}ms GCUPS={len(q)*len(s)/best/1e6:.0f}", flush=True)

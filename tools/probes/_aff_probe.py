# Affine fill shape probe (GPU box): single-front timings of growing row counts.
import sys
sys.path.insert(0, '.')
import anyseq_amd as A
qq, ss = A.main_random_pair(131072, 131072)
sc = dict(match=2, mismatch=-1, gap_open=-2, gap_extend=-1)
kind = sys.argv[1] if len(sys.argv) > 1 else "global"
for fr in (1,):
    A.set_option("fronts", fr)
    for nw in (4,):
        A.set_option("affine_waves_per_group", nw)
        out = []
        for n, m in [(64, 65536), (128, 65536), (256, 65536), (512, 65536), (1024, 65536), (4096, 65536), (16384, 65536), (32768, 65536)]:
            A.score(kind, qq[:n], ss[:m], **sc); A.last_fill_timing()
            best = 1e9
            for _ in range(3):
                A.score(kind, qq[:n], ss[:m], **sc); ms, _ = A.last_fill_timing(); best = min(best, ms)
            out.append(f"{n}:{best*1e3:.0f}us")
        print(f"{kind} fronts={fr} NW={nw} | " + " ".join(out), flush=True)
A.set_option("fronts", 2)

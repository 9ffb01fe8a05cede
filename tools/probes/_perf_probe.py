import os, sys, time, itertools
sys.path.insert(0, '.')
import anyseq_amd as A
qq, ss = A.main_random_pair(262144, 262144)
def run(n, m, kind='global', reps=2):
    A.score(kind, qq[:n], ss[:m]); A.last_fill_timing()
    best = 1e9
    for _ in range(reps):
        A.score(kind, qq[:n], ss[:m]); ms, _ = A.last_fill_timing(); best = min(best, ms)
    return best
cfgs = [tuple(int(x) for x in c.split(',')) for c in sys.argv[1:]] or [(1, 4, 32)]
shapes = [(64, 65536), (512, 65536), (16384, 65536), (65536, 65536), (131072, 65536)]
for R, NW, CH in cfgs:
    A.set_tuning(R, NW, 0); A.set_option("chunk", CH)
    out = []
    for n, m in shapes:
        ms = run(n, m)
        out.append(f"{n}x{m}:{ms:.3f}ms/{n*m/ms/1e6:.0f}")
    print(f"R={R} NW={NW} CH={CH} | " + "  ".join(out), flush=True)

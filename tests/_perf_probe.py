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
cfgs = [tuple(int(x) for x in c.split(',')) for c in sys.argv[1:]] or [(1, 4), (1, 8), (2, 4), (4, 4)]
for R, NW in cfgs:
    A.set_tuning(R, NW, 0)
    print(f"--- R={R} NW={NW} X={os.environ.get('ANYSEQ_X','0')}", flush=True)
    for n, m in [(64, 65536), (512, 65536), (4096, 65536), (16384, 65536), (65536, 32768), (65536, 65536), (65536, 131072), (131072, 65536)]:
        ms = run(n, m)
        print(f"n={n:6d} m={m:6d} {ms:8.3f} ms  {n*m/ms/1e6:8.1f} GCUPS  ns/col={ms*1e6/m:6.2f}", flush=True)

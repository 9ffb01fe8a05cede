import sys, time
sys.path.insert(0, '.')
import anyseq_amd as A
q, s = A.main_random_pair(65536, 65536)
print(len(q), len(s), flush=True)
for R, NW in [(1, 8), (1, 4), (2, 8), (2, 4), (4, 8)]:
    A.set_tuning(R, NW, 0)
    A.score('global', q[:4096], s[:4096])
    A.last_fill_timing()
    t = time.time(); v = A.score('global', q, s); dt = time.time() - t
    ms, nl = A.last_fill_timing()
    print(f"R={R} NW={NW} score={v} wall={dt*1e3:.1f}ms kernel={ms:.2f}ms GCUPS={len(q)*len(s)/ms/1e6:.1f}", flush=True)

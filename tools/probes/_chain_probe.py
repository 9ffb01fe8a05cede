"""Round 5 diagnostic: the band chain of the PRODUCT build, measured from outside -- the
fill time of a 65536-column local affine score front against its number of 64-row bands
(two fronts of k bands each: 128 k query rows).  Intercept ~ one band's duration (65536
steps), slope ~ one hop (a band's end lag), split by hop kind via k around multiples of
the 4 compute waves per workgroup.  usage: _chain_probe.py [reps]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import anyseq_amd as A  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
q, s = A.main_random_pair(65536, 65536)
print("bands_per_front rows fill_ms ns_per_step_if_one_band")
for k in (1, 2, 3, 4, 5, 8, 9, 16, 17, 32, 64, 128, 256, 512):
    n = 128 * k
    A.score("local", q[:n], s, gap_open=-2, gap_extend=-1)
    best = None
    for _ in range(reps):
        A.last_fill_stats()
        A.score("local", q[:n], s, gap_open=-2, gap_extend=-1)
        ms, launches, cells = A.last_fill_stats()
        best = ms if best is None else min(best, ms)
    print(k, n, round(best, 4), round(best * 1e6 / 65536, 2), flush=True)

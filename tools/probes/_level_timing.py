"""Diagnostic: host phases per Hirschberg level of the configs[2] construct
(ANYSEQ_LEVEL_TIMING=1 prints build / launch / enqueue / wait per level)."""
import os
import sys
import time

os.environ["ANYSEQ_LEVEL_TIMING"] = "1"
sys.path.insert(0, ".")
import anyseq_amd as A  # noqa: E402

q, s = A.main_random_pair(65536, 65536)
for it in range(3):
    t = time.perf_counter()
    r = A.construct("local", q, s, gap_open=-2, gap_extend=-1)
    print(f"--- construct {1e3 * (time.perf_counter() - t):.2f} ms score {r[0]}", file=sys.stderr)

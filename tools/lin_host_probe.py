"""Probe: the linear true construct (construct_mode 1, gap open 0) on host-built affine levels
(affine_device_plan 0) under knob variants, against the oracle (round 6: found the host-built
levels launching gap open 0 on the linear fill_kernel)."""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import anyseq_amd as A  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_gpu_inherit import related, rnd  # noqa: E402

A.set_device(0)
A.set_option("construct_mode", 1)
A.set_option("inherit_halves", 0)
rng = random.Random(76)
cases = []
for n, m in [(2000, 2100), (3000, 2600), (1500, 4000), (700, 900)]:
    q, s = related(rng, n)
    s = s[:m] if len(s) >= m else s + rnd(rng, m - len(s))
    cases.append((q, s))
variants = {"devplan": [("affine_device_plan", 1)],
            "host": [("affine_device_plan", 0)],
            "host_noloop": [("affine_device_plan", 0), ("linear_affine_loop", 0)],
            "host_notr": [("affine_device_plan", 0), ("affine_transpose", 0)],
            "host_noasm": [("affine_device_plan", 0), ("affine_asm", 0)],
            "host_r1": [("affine_device_plan", 0), ("affine_rows_per_lane", 1)],
            "host_nw4": [("affine_device_plan", 0), ("affine_waves_per_group", 4)],
            "host_r1_nw4": [("affine_device_plan", 0), ("affine_rows_per_lane", 1), ("affine_waves_per_group", 4)]}
defaults = {"affine_device_plan": 1, "linear_affine_loop": 1, "affine_transpose": 1, "affine_asm": 1,
            "affine_rows_per_lane": 0, "affine_waves_per_group": 0}
for name, opts in variants.items():
    for k, v in opts:
        A.set_option(k, v)
    bad = []
    for kind in ("global", "semiglobal", "local"):
        for q, s in cases:
            for sc in ((2, -1, 0, -1), (1, -3, 0, -2)):
                g = A.construct(kind, q, s, match=sc[0], mismatch=sc[1], gap_open=0, gap_extend=sc[3])
                o = O.affine_construct(kind, q, s, *sc)
                if g != o:
                    bad.append((kind, len(q), len(s), sc, g[0], o[0]))
    print(name, "ok" if not bad else f"{len(bad)} bad: {bad[:3]}", flush=True)
    for k, v in opts:
        A.set_option(k, defaults[k])

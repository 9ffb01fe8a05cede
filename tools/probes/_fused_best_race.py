"""Round 4 diagnostic (test infrastructure: the oracle is the checker): with the masked
top row past the last chunk (tools/patches/fused_best_negtop.patch) the fused band end
with every-cell bests still fails rarely -- count failures per knob setting to localise."""
import os
import random
import sys

sys.path.insert(0, os.getcwd())
import anyseq_amd as A  # noqa: E402
from oracle import oracle as O  # noqa: E402

O.build()
sc = (2, -1, -2, -1)
rng = random.Random(7)
shapes = [(511, 33), (257, 33), (300, 33), (1000, 200), (700, 100), (1500, 64)]
cases = []
for n, m in shapes:
    for _ in range(6):
        q = "".join(rng.choice("ACGT") for _ in range(n))
        s = "".join(rng.choice("ACGT") for _ in range(m))
        cases.append((n, m, q, s, O.affine_score("local", q, s, *sc)))
settings = [("nw4 st3 a65", 4, 3, 65), ("nw4 st0 a65", 4, 0, 65), ("nw7 st3 a65", 7, 3, 65),
            ("nw4 st3 a1", 4, 3, 1), ("nw3 st3 a65", 3, 3, 65), ("nw4 st3 a97", 4, 3, 97)]
for name, nw, st, a in settings:
    A.set_option("affine_waves_per_group", nw)
    A.set_option("io_stage", st)
    A.set_option("affine_asm", a)
    bad = []
    for rep in range(3):
        for n, m, q, s, o in cases:
            g = A.score("local", q, s, match=sc[0], mismatch=sc[1], gap_open=sc[2], gap_extend=sc[3])
            if g != o:
                bad.append(f"{n}x{m}:{g}!={o}")
    print(f"{name}: {len(bad)}/{3 * len(cases)} bad", " ".join(bad[:8]), flush=True)

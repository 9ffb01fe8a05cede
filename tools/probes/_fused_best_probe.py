"""Round 4 diagnostic (test infrastructure: uses the oracle as the checker): local affine
score with the capture-free band end over shapes around the one that failed (511 x 33),
under several knobs, vs the oracle."""
import os
import random
import sys

sys.path.insert(0, os.getcwd())
import anyseq_amd as A  # noqa: E402
from oracle import oracle as O  # noqa: E402

O.build()
sc = (2, -1, -2, -1)
rng = random.Random(5)
shapes = [(511, 33), (255, 33), (257, 33), (300, 33), (511, 64), (511, 65), (511, 100), (1000, 200), (2049, 1000)]
cases = [(n, m, "".join(rng.choice("ACGT") for _ in range(n)), "".join(rng.choice("ACGT") for _ in range(m)))
         for n, m in shapes]
for opts in ({}, {"affine_waves_per_group": 7}, {"io_stage": 0}, {"affine_asm": 97}):
    for k, v in opts.items():
        A.set_option(k, v)
    res = []
    for n, m, q, s in cases:
        g = A.score("local", q, s, match=sc[0], mismatch=sc[1], gap_open=sc[2], gap_extend=sc[3])
        o = O.affine_score("local", q, s, *sc)
        res.append(f"{n}x{m}:{'ok' if g == o else f'BAD {g}!={o}'}")
    print(opts, " ".join(res), flush=True)

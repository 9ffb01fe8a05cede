import sys, random
sys.path.insert(0, '.')
import anyseq_amd as A
from oracle import oracle as O
O.build()
def rnd(rng, n): return "".join(rng.choice("ACGT") for _ in range(n))
rng = random.Random(5)
cases = [(277, 112), (64, 112), (64, 40), (128, 112), (300, 300), (64, 1000), (256, 1000), (257, 1000), (1000, 64), (3000, 2000)]
for asm in (0, 1, 2, 3):
    A.set_option("affine_asm", asm)
    for kind in ("global", "semiglobal", "local"):
        bad = []
        for (n, m) in cases:
            for sc in [(5, -4, -10, -1), (2, -1, -2, -1)]:
                q, s = rnd(rng, n), rnd(rng, m)
                g = A.score(kind, q, s, *sc); o = O.affine_score(kind, q, s, *sc)
                if g != o: bad.append((n, m, sc, g, o))
        print("asm", asm, kind, "bad:", bad[:6], flush=True)

"""Round 5 diagnostic (test infrastructure: the oracle is the checker): a local affine
score with a POSITIVE mismatch (4, 1, -6, -1) over 12 symbols (the compare weights)
came out 468 vs the oracle's 427 with the fused band end -- which settings give it?"""
import os
import random
import sys

sys.path.insert(0, os.getcwd())
import anyseq_amd as A  # noqa: E402
from oracle import oracle as O  # noqa: E402

O.build()


def rnd(rng, n, alphabet):
    return "".join(rng.choice(alphabet) for _ in range(n))


rng = random.Random(5)
cases = []
for n, m in [(700, 300), (300, 700), (64, 64), (128, 96), (200, 33)]:
    for alph in ("ACGTNRYKMSWB", "ACGT"):
        for sc in [(4, 1, -6, -1), (3, 0, -2, -2), (2, -1, -2, -1)]:
            q, s = rnd(rng, n, alph), rnd(rng, m, alph)
            cases.append((n, m, alph, sc, q, s, O.affine_score("local", q, s, *sc),
                          O.affine_score("semiglobal", q, s, *sc), O.affine_score("global", q, s, *sc)))
for asm in (97, 1, 65, 3, 99, 0):
    for nw in (3, 4, 7):
        A.set_option("affine_asm", asm)
        A.set_option("affine_waves_per_group", nw)
        bad = []
        for n, m, alph, sc, q, s, ol, osg, og in cases:
            for kind, o in (("local", ol), ("semiglobal", osg), ("global", og)):
                g = A.score(kind, q, s, *sc)
                if g != o:
                    bad.append(f"{kind[0]}{n}x{m}/{len(alph)}/{sc}:{g}!={o}")
        print(f"asm {asm} nw {nw}: {len(bad)}/{3 * len(cases)} bad", " ".join(bad[:6]), flush=True)

"""Diagnostic: the local affine case of test_affine_construct_transposed_halves[local-0]
(2700 x 1000, scheme (3, -2, -1, -3)), score and construct, for the current settings."""
import os
import random
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import anyseq_amd as A  # noqa: E402
from test_gpu_affine_construct import rnd  # noqa: E402

rng = random.Random(55)
core = rnd(rng, 700)
cases = [(rnd(rng, 3000), rnd(rng, 400)), (rnd(rng, 300), rnd(rng, 2600)), (rnd(rng, 1500), rnd(rng, 1500)),
         (rnd(rng, 2000) + core, core + rnd(rng, 300)), (core[:500] + rnd(rng, 1800), rnd(rng, 900) + core)]
q, s = cases[3]
A.set_option("affine_transpose", 0)
sc = dict(match=3, mismatch=-2, gap_open=-1, gap_extend=-3)
print(os.environ.get("ANYSEQ_AFFINE_ASM", "-"), "score", A.score("local", q, s, **sc),
      "construct", A.construct("local", q, s, **sc)[0], "T-score", A.score("local", s, q, **sc))

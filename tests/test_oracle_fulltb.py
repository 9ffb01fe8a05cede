"""CPU: the fulltb oracle (oracle_construct_fulltb, align.impala:190-216) against an
independent pure-Python full-matrix DP with the relax_global tie order
(align.impala:46-67: diagonal, then GAP_Q if strictly better, then GAP_S if
strictly better) and traceback_offset's i+j+1 layout (traceback.impala:47-80)."""
import random

import pytest


def py_fulltb(q: bytes, s: bytes, match=2, mismatch=-1, gap=-1):
    n, m = len(q), len(s)
    H = [[0] * (m + 1) for _ in range(n + 1)]
    P = [[0] * (m + 1) for _ in range(n + 1)]
    for j in range(m + 1):
        H[0][j] = j * gap
        P[0][j] = 1 if j > 0 else 0
    for i in range(1, n + 1):
        H[i][0] = i * gap
        P[i][0] = 2
        for j in range(1, m + 1):
            v, p = H[i - 1][j - 1] + (match if q[i - 1] == s[j - 1] else mismatch), 3
            if H[i][j - 1] + gap > v:
                v, p = H[i][j - 1] + gap, 1
            if H[i - 1][j] + gap > v:
                v, p = H[i - 1][j] + gap, 2
            H[i][j], P[i][j] = v, p
    aq, as_ = bytearray(b" " * (n + m)), bytearray(b" " * (n + m))
    i, j = n - 1, m - 1
    p = P[i + 1][j + 1]
    while p:
        pos = i + j + 1
        a = b = ord("_")
        if p in (3, 2):
            a = q[i]
            i -= 1
        if p in (3, 1):
            b = s[j]
            j -= 1
        aq[pos], as_[pos] = a, b
        p = P[i + 1][j + 1]
    return (H[n][m] if n + m else 0), bytes(aq), bytes(as_)


@pytest.mark.parametrize("seed", range(6))
def test_fulltb_oracle_matches_independent_dp(oracle, seed):
    rng = random.Random(seed)
    for n, m in [(0, 3), (4, 0), (1, 1), (rng.randint(1, 60), rng.randint(1, 60)), (90, 70)]:
        q = bytes(rng.choice(b"ACGT") for _ in range(n))
        s = bytes(rng.choice(b"ACGT") for _ in range(m))
        assert oracle.construct_fulltb(q, s) == py_fulltb(q, s), (n, m)

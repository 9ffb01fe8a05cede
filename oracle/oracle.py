"""Python handle on the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this module.  It wraps ``oracle/liboracle.so`` (the C restatement
of the reference CPU path, see anyseq_oracle.c for the file:line map) and adds
an independent textbook full-matrix DP used to cross-check oracle scores.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: another build of the same restatement (tests/test_oracle_asan.py: the sanitizer build)
_LIB = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")

GLOBAL, SEMIGLOBAL, LOCAL = 0, 1, 2
KINDS = {"global": GLOBAL, "semiglobal": SEMIGLOBAL, "local": LOCAL}
SCORE_MIN_VALUE = -2147483647

_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        c_i64, c_int, c_p = ctypes.c_int64, ctypes.c_int, ctypes.c_char_p
        i32p = ctypes.POINTER(ctypes.c_int32)
        L.oracle_score.restype = c_i64
        L.oracle_score.argtypes = [c_int, c_p, c_int, c_p, c_int, c_int, c_int, c_int, i32p, i32p]
        L.oracle_construct.restype = c_i64
        L.oracle_construct.argtypes = [c_int, c_p, c_int, c_p, c_int, c_int, c_int, c_int,
                                       ctypes.c_void_p, ctypes.c_void_p, i32p, c_int]
        L.oracle_set_threads.argtypes = [c_int]
        L.oracle_last_error.restype = c_int
        L.oracle_affine_score.restype = c_i64
        L.oracle_affine_score.argtypes = [c_int, c_p, c_int, c_p, c_int, c_int, c_int, c_int, c_int,
                                          i32p, i32p]
        L.oracle_affine_construct.restype = c_i64
        L.oracle_affine_construct.argtypes = [c_int, c_p, c_int, c_p, c_int, c_int, c_int, c_int,
                                              c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_construct_fulltb.restype = c_i64
        L.oracle_construct_fulltb.argtypes = [c_p, c_int, c_p, c_int, c_int, c_int, c_int,
                                              ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_affine_last_rect.argtypes = [i32p]
        _lib = L
    return _lib


def _b(x) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


def set_threads(t: int) -> None:
    lib().oracle_set_threads(int(t))


def score(kind, q, s, match=2, mismatch=-1, gap=-1, with_pos=False):
    k = KINDS[kind] if isinstance(kind, str) else kind
    q, s = _b(q), _b(s)
    pi, pj = ctypes.c_int32(-1), ctypes.c_int32(-1)
    r = lib().oracle_score(k, q, len(q), s, len(s), match, mismatch, gap,
                           ctypes.byref(pi), ctypes.byref(pj))
    if lib().oracle_last_error():
        raise RuntimeError("oracle read an unset split")
    return (r, pi.value, pj.value) if with_pos else r


def construct(kind, q, s, match=2, mismatch=-1, gap=-1, with_splits=False):
    """Returns (reference_return_value, alQuery, alSubject[, splits])."""
    k = KINDS[kind] if isinstance(kind, str) else kind
    q, s = _b(q), _b(s)
    n, m = len(q), len(s)
    aq = ctypes.create_string_buffer(max(n + m, 1))
    as_ = ctypes.create_string_buffer(max(n + m, 1))
    nb = (m + 127) // 128
    spl = (ctypes.c_int32 * max(nb, 1))()
    r = lib().oracle_construct(k, q, n, s, m, match, mismatch, gap, aq, as_, spl, nb)
    if lib().oracle_last_error():
        raise RuntimeError("oracle read an unset split")
    out = (r, aq.raw[: n + m], as_.raw[: n + m])
    if with_splits:
        out = out + (list(spl)[:nb],)
    return out


def construct_fulltb(q, s, match=2, mismatch=-1, gap=-1):
    """construct_*_alignment_fulltb (all three: global scheme, full-matrix traceback,
    export.impala:37-53,93-109,150-166): (H[n-1][m-1], alQuery, alSubject)."""
    q, s = _b(q), _b(s)
    n, m = len(q), len(s)
    aq = ctypes.create_string_buffer(max(n + m, 1))
    as_ = ctypes.create_string_buffer(max(n + m, 1))
    r = lib().oracle_construct_fulltb(q, n, s, m, match, mismatch, gap, aq, as_)
    return r, aq.raw[: n + m], as_.raw[: n + m]


def affine_score(kind, q, s, match=2, mismatch=-1, gap_open=-2, gap_extend=-1, with_pos=False):
    k = KINDS[kind] if isinstance(kind, str) else kind
    q, s = _b(q), _b(s)
    pi, pj = ctypes.c_int32(-1), ctypes.c_int32(-1)
    r = lib().oracle_affine_score(k, q, len(q), s, len(s), match, mismatch, gap_open, gap_extend,
                                  ctypes.byref(pi), ctypes.byref(pj))
    return (r, pi.value, pj.value) if with_pos else r


def affine_construct(kind, q, s, match=2, mismatch=-1, gap_open=-2, gap_extend=-1):
    """Build-defined affine alignment (anyseq_oracle.c oracle_affine_construct):
    (optimal score, alQuery, alSubject) in the sparse i+j+1 layout, len(q)+len(s) bytes each."""
    k = KINDS[kind] if isinstance(kind, str) else kind
    q, s = _b(q), _b(s)
    n, m = len(q), len(s)
    aq = ctypes.create_string_buffer(n + m + 1)
    as_ = ctypes.create_string_buffer(n + m + 1)
    r = lib().oracle_affine_construct(k, q, n, s, m, match, mismatch, gap_open, gap_extend, aq, as_)
    if lib().oracle_last_error():
        raise RuntimeError("oracle read an unset split")
    return r, aq.raw[: n + m], as_.raw[: n + m]


def affine_last_rect():
    """(is, ie, js, je): the query rows / subject columns the last affine_construct
    emitted (ie < is or je < js: none)."""
    rect = (ctypes.c_int32 * 4)()
    lib().oracle_affine_last_rect(rect)
    return tuple(rect)


# --------------------------------------------------------------------------
# Independent textbook full-matrix DP (not derived from the reference code
# layout) — used to cross-check oracle scores on small inputs.
# --------------------------------------------------------------------------
def textbook_score(kind, q, s, match=2, mismatch=-1, gap=-1):
    k = KINDS[kind] if isinstance(kind, str) else kind
    q = np.frombuffer(_b(q), dtype=np.uint8).astype(np.int64)
    s = np.frombuffer(_b(s), dtype=np.uint8).astype(np.int64)
    n, m = len(q), len(s)
    H = np.zeros((n + 1, m + 1), dtype=np.int64)
    if k == GLOBAL:
        H[0, :] = np.arange(m + 1) * gap
        H[:, 0] = np.arange(n + 1) * gap
    for i in range(1, n + 1):
        sub = np.where(s == q[i - 1], match, mismatch)
        diag = H[i - 1, :-1] + sub
        up = H[i - 1, 1:] + gap
        cand = np.maximum(diag, up)
        if k == LOCAL:
            cand = np.maximum(cand, 0)
        # left dependency: sequential scan
        row = H[i]
        prev = row[0]
        for j in range(1, m + 1):
            v = max(cand[j - 1], prev + gap)
            if k == LOCAL and v < 0:
                v = 0
            row[j] = v
            prev = v
    if k == GLOBAL:
        return int(H[n, m])
    if k == SEMIGLOBAL:
        return int(max(H[n, :].max(), H[:, m].max()))
    if n == 0 or m == 0:
        return SCORE_MIN_VALUE  # reference semantics: no slot is ever written
    return int(H[1:, 1:].max())


def textbook_affine_score(kind, q, s, match=2, mismatch=-1, gap_open=-2, gap_extend=-1):
    """Gotoh with gap(k) = open + k*extend; build-defined semantics."""
    k = KINDS[kind] if isinstance(kind, str) else kind
    q, s = _b(q), _b(s)
    n, m = len(q), len(s)
    NEG = -(1 << 40)
    go, ge = gap_open, gap_extend
    Hp = [0] * (m + 1)
    Fp = [NEG] * (m + 1)
    if k == GLOBAL:
        for j in range(1, m + 1):
            Hp[j] = go + j * ge
    best = NEG
    for i in range(1, n + 1):
        Hc = [0] * (m + 1)
        Fc = [NEG] * (m + 1)
        Hc[0] = (go + i * ge) if k == GLOBAL else 0
        E = NEG
        for j in range(1, m + 1):
            E = max(E + ge, Hc[j - 1] + go + ge)
            Fc[j] = max(Fp[j] + ge, Hp[j] + go + ge)
            d = Hp[j - 1] + (match if q[i - 1] == s[j - 1] else mismatch)
            h = max(d, E, Fc[j])
            if k == LOCAL:
                h = max(h, 0)
            Hc[j] = h
            if k == LOCAL:
                best = max(best, h)
        if k == SEMIGLOBAL and m > 0:
            best = max(best, Hc[m])
        Hp, Fp = Hc, Fc
    if k == GLOBAL:
        return Hp[m] if n > 0 else (go + m * ge if m > 0 else 0)
    if k == SEMIGLOBAL:
        last_row = Hp[1:] if n > 0 else []
        return max([0, best] + last_row)
    if n == 0 or m == 0:
        return SCORE_MIN_VALUE
    return best

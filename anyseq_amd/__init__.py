"""anyseq_amd — MI355X-native AnySeq engine, Python host mirror.

This module mirrors the reference's operator interface for the hot path — the
six ``extern "C"`` functions of ``/root/reference/src/import.h:14-41`` (defined
by ``export.impala:5-166``) — over the C-ABI library ``libanyseq.so`` built from
``anyseq_amd/csrc`` (hand-written HIP kernels for gfx950).  Same names, same
argument meaning (query, subject), same return conventions:

* ``*_alignment_score(q, s) -> int``
* ``construct_*_alignment(q, s) -> (ret, alQuery, alSubject)`` where the two
  byte strings have length ``len(q)+len(s)`` in the reference's sparse
  ``i+j+1`` layout (``traceback.impala:14-80``) and ``ret`` is the reference's
  literal return value.

There is no CPU fallback: importing this package fails loudly if the HIP
library is missing, and every call fails loudly if no GPU is usable.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ANYSEQ_LIB selects a diagnostic build of the same library (e.g. the s_memtime
# stamp build libanyseq_stamps.so); the product build is libanyseq.so.
LIB_PATH = os.environ.get("ANYSEQ_LIB") or os.path.join(_HERE, "libanyseq.so")

GLOBAL, SEMIGLOBAL, LOCAL = 0, 1, 2
KINDS = {"global": GLOBAL, "semiglobal": SEMIGLOBAL, "local": LOCAL}
INT64_MIN = -(1 << 63)

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"anyseq_amd: HIP library {LIB_PATH} is missing — build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` or `make` at the repo root")

_lib = ctypes.CDLL(LIB_PATH)


class Scoring(ctypes.Structure):
    """anyseq_scoring: gap of length k costs gap_open + k*gap_extend (open 0 = linear)."""
    _fields_ = [("match", ctypes.c_int32), ("mismatch", ctypes.c_int32),
                ("gap_open", ctypes.c_int32), ("gap_extend", ctypes.c_int32)]


ABI_SCORING = Scoring(2, -1, 0, -1)   # linear_scoring_scheme(2,-1,-1), export.impala:14

_c_i64, _c_int, _c_p, _vp = ctypes.c_int64, ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p
for _n in ("global_alignment_score", "semiglobal_alignment_score", "local_alignment_score"):
    getattr(_lib, _n).restype = _c_i64
    getattr(_lib, _n).argtypes = [_c_p, _c_int, _c_p, _c_int]
for _n in ("construct_global_alignment", "construct_semiglobal_alignment", "construct_local_alignment",
           "construct_global_alignment_fulltb", "construct_semiglobal_alignment_fulltb",
           "construct_local_alignment_fulltb"):
    getattr(_lib, _n).restype = _c_i64
    getattr(_lib, _n).argtypes = [_c_p, _c_int, _c_p, _c_int, _vp, _vp]
_lib.anyseq_score.restype = _c_int
_lib.anyseq_score.argtypes = [_c_int, ctypes.POINTER(Scoring), _c_p, _c_int, _c_p, _c_int,
                              ctypes.POINTER(_c_i64)]
_lib.anyseq_score_device.restype = _c_int
_lib.anyseq_score_device.argtypes = [_c_int, ctypes.POINTER(Scoring), _vp, _c_int, _vp, _c_int, _vp,
                                     ctypes.POINTER(_c_i64)]
_lib.anyseq_construct.restype = _c_int
_lib.anyseq_construct.argtypes = [_c_int, ctypes.POINTER(Scoring), _c_p, _c_int, _c_p, _c_int, _vp, _vp,
                                  ctypes.POINTER(_c_i64)]
_lib.anyseq_alignment_dense.restype = _c_i64
_lib.anyseq_alignment_dense.argtypes = [_c_p, _c_p, _c_i64, _vp, _vp]
_lib.anyseq_alignment_cigar.restype = _c_i64
_lib.anyseq_alignment_cigar.argtypes = [_c_p, _c_p, _c_i64, _vp, _c_i64]
_lib.anyseq_construct_device.restype = _c_int
_lib.anyseq_construct_device.argtypes = [_c_int, ctypes.POINTER(Scoring), _vp, _c_int, _vp, _c_int, _vp, _vp, _vp,
                                         ctypes.POINTER(_c_i64)]
_lib.anyseq_shard_score_local.restype = _c_int
_lib.anyseq_shard_score_local.argtypes = [_c_int, ctypes.POINTER(Scoring), _c_p, _c_int, _c_p, _c_int, _c_int,
                                          ctypes.POINTER(_c_i64)]
_lib.anyseq_construct_local_sharded.restype = _c_int
_lib.anyseq_construct_local_sharded.argtypes = [_c_int, ctypes.POINTER(Scoring), _c_p, _c_int, _c_p, _c_int, _c_int,
                                                _vp, _vp, ctypes.POINTER(_c_i64)]
_lib.anyseq_shard_construct.restype = _c_int
_lib.anyseq_shard_construct.argtypes = [_c_int, ctypes.POINTER(Scoring), _c_p, _c_int, _c_p, _c_int, _vp, _vp,
                                        ctypes.POINTER(_c_i64)]
HOST_ALLREDUCE_FN = ctypes.CFUNCTYPE(_c_int, _vp, _c_i64, _c_int, _c_int, _vp)
_lib.anyseq_shard_construct_hostcoll.restype = _c_int
_lib.anyseq_shard_construct_hostcoll.argtypes = [_c_int, ctypes.POINTER(Scoring), _c_p, _c_int, _c_p, _c_int, _c_int,
                                                 _c_int, HOST_ALLREDUCE_FN, _vp, _vp, _vp, ctypes.POINTER(_c_i64)]
_lib.anyseq_shard_unique_ids.restype = _c_int
_lib.anyseq_shard_unique_ids.argtypes = [_vp, _c_int]
_lib.anyseq_shard_init.restype = _c_int
_lib.anyseq_shard_init.argtypes = [_c_int, _c_int, _c_p, _c_int]
_lib.anyseq_shard_load.restype = _c_int
_lib.anyseq_shard_load.argtypes = [_c_p, _c_int, _c_p, _c_int, _c_int, _c_int]
_lib.anyseq_shard_score.restype = _c_int
_lib.anyseq_shard_score.argtypes = [_c_int, ctypes.POINTER(Scoring), ctypes.POINTER(_c_i64)]
_lib.anyseq_shard_finalize.restype = _c_int
_lib.anyseq_last_error.restype = _c_p
_lib.anyseq_set_device.argtypes = [_c_int]
_lib.anyseq_set_tuning.argtypes = [_c_int, _c_int, _c_int]
_lib.anyseq_set_option.restype = _c_int
_lib.anyseq_set_option.argtypes = [_c_p, _c_int]
_lib.anyseq_last_fill_timing.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_int)]
_lib.anyseq_last_fill_stats.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_int),
                                        ctypes.POINTER(_c_i64)]
_lib.anyseq_last_shard_plan.restype = _c_int
_lib.anyseq_last_fill_multi_row_launches.restype = _c_int
_lib.anyseq_last_fill_multi_row_launches.argtypes = [ctypes.POINTER(_c_int)]
_lib.anyseq_last_inherit_stats.restype = ctypes.c_int64
_lib.anyseq_last_inherit_stats.argtypes = [ctypes.POINTER(ctypes.c_int64)]
_lib.anyseq_main_random_pair.argtypes = [_c_i64, _c_i64, _vp, ctypes.POINTER(_c_i64), _vp,
                                         ctypes.POINTER(_c_i64)]


class AnySeqError(RuntimeError):
    pass


def _b(x) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


def _kind(kind) -> int:
    return KINDS[kind] if isinstance(kind, str) else int(kind)


def _err() -> str:
    return (_lib.anyseq_last_error() or b"").decode(errors="replace")


def _check_abi(v: int) -> int:
    if v == INT64_MIN:
        raise AnySeqError(_err())
    return v


# ---- the reference ABI (import.h:14-41) ---------------------------------
def global_alignment_score(query, subject) -> int:
    q, s = _b(query), _b(subject)
    return _check_abi(_lib.global_alignment_score(q, len(q), s, len(s)))


def semiglobal_alignment_score(query, subject) -> int:
    q, s = _b(query), _b(subject)
    return _check_abi(_lib.semiglobal_alignment_score(q, len(q), s, len(s)))


def local_alignment_score(query, subject) -> int:
    q, s = _b(query), _b(subject)
    return _check_abi(_lib.local_alignment_score(q, len(q), s, len(s)))


def _construct_abi(fn, query, subject):
    q, s = _b(query), _b(subject)
    L = len(q) + len(s)
    aq = ctypes.create_string_buffer(max(L, 1))
    as_ = ctypes.create_string_buffer(max(L, 1))
    r = _check_abi(fn(q, len(q), s, len(s), aq, as_))
    return r, aq.raw[:L], as_.raw[:L]


def construct_global_alignment(query, subject):
    return _construct_abi(_lib.construct_global_alignment, query, subject)


def construct_semiglobal_alignment(query, subject):
    return _construct_abi(_lib.construct_semiglobal_alignment, query, subject)


def construct_local_alignment(query, subject):
    return _construct_abi(_lib.construct_local_alignment, query, subject)


def construct_global_alignment_fulltb(query, subject):
    """Undeclared reference export (export.impala:37-53): full-matrix traceback."""
    return _construct_abi(_lib.construct_global_alignment_fulltb, query, subject)


def construct_semiglobal_alignment_fulltb(query, subject):
    """export.impala:93-109 -- runs the GLOBAL scheme, as the reference does."""
    return _construct_abi(_lib.construct_semiglobal_alignment_fulltb, query, subject)


def construct_local_alignment_fulltb(query, subject):
    """export.impala:150-166 -- runs the GLOBAL scheme, as the reference does."""
    return _construct_abi(_lib.construct_local_alignment_fulltb, query, subject)


# ---- extended API ---------------------------------------------------------
def _scoring(match=2, mismatch=-1, gap_open=0, gap_extend=-1) -> Scoring:
    return Scoring(match, mismatch, gap_open, gap_extend)


def score(kind, query, subject, match=2, mismatch=-1, gap_open=0, gap_extend=-1) -> int:
    q, s = _b(query), _b(subject)
    out = _c_i64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_score(_kind(kind), ctypes.byref(sc), q, len(q), s, len(s), ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value


def score_device(kind, q_ptr: int, n: int, s_ptr: int, m: int, stream: int = 0,
                 match=2, mismatch=-1, gap_open=0, gap_extend=-1) -> int:
    """Score device-resident sequences (e.g. torch uint8 CUDA tensors' data_ptr())."""
    out = _c_i64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_score_device(_kind(kind), ctypes.byref(sc), ctypes.c_void_p(q_ptr), n,
                                ctypes.c_void_p(s_ptr), m, ctypes.c_void_p(stream or None),
                                ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value


def construct(kind, query, subject, match=2, mismatch=-1, gap_open=0, gap_extend=-1):
    """Returns (optimal_score, alQuery, alSubject) in the sparse i+j+1 layout."""
    q, s = _b(query), _b(subject)
    L = len(q) + len(s)
    aq = ctypes.create_string_buffer(max(L, 1))
    as_ = ctypes.create_string_buffer(max(L, 1))
    out = _c_i64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_construct(_kind(kind), ctypes.byref(sc), q, len(q), s, len(s), aq, as_,
                             ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value, aq.raw[:L], as_.raw[:L]


def construct_device(kind, q_ptr: int, n: int, s_ptr: int, m: int, alq_ptr: int, als_ptr: int, stream: int = 0,
                     match=2, mismatch=-1, gap_open=0, gap_extend=-1) -> int:
    """Construct on device-resident sequences into device strings (n+m bytes each);
    returns the optimal score."""
    out = _c_i64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_construct_device(_kind(kind), ctypes.byref(sc), ctypes.c_void_p(q_ptr), n, ctypes.c_void_p(s_ptr),
                                    m, ctypes.c_void_p(alq_ptr), ctypes.c_void_p(als_ptr),
                                    ctypes.c_void_p(stream or None), ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value


def shard_score_local(kind, query, subject, nshards: int, match=2, mismatch=-1, gap_open=0, gap_extend=-1) -> int:
    """Column-block sharded score with `nshards` shards in this process on one GPU
    (the same kernels, progress counters and chunked hand-off as the RCCL path,
    with device copies as the transport) -- DESIGN.md §6."""
    q, s = _b(query), _b(subject)
    out = _c_i64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_shard_score_local(_kind(kind), ctypes.byref(sc), q, len(q), s, len(s), int(nshards),
                                     ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value


def construct_local_sharded(kind, query, subject, nshards: int, match=2, mismatch=-1, gap_open=-2, gap_extend=-1):
    """Sharded affine construct with `nshards` virtual ranks in this process on one GPU:
    the plan of the RCCL path: the leading levels column-blocked over
    rank subgroups (world >= 2 x parts, each part's query rows split over its subgroup;
    one fill per rank), the rest dealt round-robin by half and device-planned (one fill
    launch per level, every view's columns reduced between the fill and the join;
    ANYSEQ_SHARD_DEVPLAN=0: host-built, one launch per rank).  Returns (optimal_score,
    alQuery, alSubject)."""
    q, s = _b(query), _b(subject)
    L = len(q) + len(s)
    aq = ctypes.create_string_buffer(max(L, 1))
    as_ = ctypes.create_string_buffer(max(L, 1))
    out = _c_i64(0)
    sc = _scoring(match, mismatch, gap_open, gap_extend)
    if _lib.anyseq_construct_local_sharded(_kind(kind), ctypes.byref(sc), q, len(q), s, len(s), int(nshards), aq,
                                           as_, ctypes.byref(out)) != 0:
        raise AnySeqError(_err())
    return out.value, aq.raw[:L], as_.raw[:L]


def set_device(dev: int) -> None:
    _lib.anyseq_set_device(int(dev))


def set_tuning(rows_per_lane: int = 0, waves_per_group: int = 0, grid: int = -1) -> None:
    _lib.anyseq_set_tuning(rows_per_lane, waves_per_group, grid)


def set_option(name: str, value: int) -> None:
    """Engine tuning: rows_per_lane, lane_skew_extra, waves_per_group, grid, fronts."""
    if _lib.anyseq_set_option(name.encode(), int(value)) != 0:
        raise AnySeqError(f"unknown option {name}")


def last_fill_timing():
    """(milliseconds, launches) of the fill kernels since the previous call (HIP events)."""
    ms, n = ctypes.c_double(0.0), _c_int(0)
    _lib.anyseq_last_fill_timing(ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value


def last_fill_stats():
    """(milliseconds, launches, DP cells) of the fill kernels since the previous call."""
    ms, n, c = ctypes.c_double(0.0), _c_int(0), _c_i64(0)
    _lib.anyseq_last_fill_stats(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(c))
    return ms.value, n.value, c.value


def last_fill_multi_row_launches():
    """(affine fill launches since the previous call that ran two or three rows per lane,
    the most rows per lane among them); resets both."""
    r = _c_int(1)
    n = int(_lib.anyseq_last_fill_multi_row_launches(ctypes.byref(r)))
    return n, r.value


def last_inherit_stats():
    """(halves run as two column blocks recording their child's column, halves taken as
    such a recorded column instead of a fill) of this thread's affine constructs since the
    previous call (host-built levels, option "inherit_halves"); resets both."""
    r = ctypes.c_int64(0)
    n = int(_lib.anyseq_last_inherit_stats(ctypes.byref(r)))
    return n, r.value


def last_shard_plan() -> int:
    """Leading Hirschberg levels of the last sharded construct that were column-blocked
    over all ranks (0: all round-robin); resets it."""
    return int(_lib.anyseq_last_shard_plan())


def main_random_pair(minlen: int, maxlen: int):
    """The reference driver's random inputs (main.cpp:90-120,200-210): (query, subject) bytes."""
    q = ctypes.create_string_buffer(max(maxlen, 1))
    s = ctypes.create_string_buffer(max(maxlen, 1))
    n, m = _c_i64(0), _c_i64(0)
    _lib.anyseq_main_random_pair(minlen, maxlen, q, ctypes.byref(n), s, ctypes.byref(m))
    return q.raw[:n.value], s.raw[:m.value]


def dense(al_q: bytes, al_s: bytes):
    """Sparse i+j+1 layout -> dense alignment (positions blank in both dropped);
    anyseq_alignment_dense in the library."""
    al_q, al_s = _b(al_q), _b(al_s)
    n = min(len(al_q), len(al_s))
    oq, os_ = ctypes.create_string_buffer(max(n, 1)), ctypes.create_string_buffer(max(n, 1))
    k = _lib.anyseq_alignment_dense(al_q, al_s, n, oq, os_)
    if k < 0:
        raise AnySeqError("anyseq_alignment_dense failed")
    return oq.raw[:k], os_.raw[:k]


def cigar(al_q: bytes, al_s: bytes) -> str:
    """Extended CIGAR (=, X, I, D) of an alignment (sparse or dense; '_' is the gap
    symbol); anyseq_alignment_cigar in the library."""
    al_q, al_s = _b(al_q), _b(al_s)
    n = min(len(al_q), len(al_s))
    need = _lib.anyseq_alignment_cigar(al_q, al_s, n, None, 0)
    if need < 0:
        raise AnySeqError("anyseq_alignment_cigar failed")
    out = ctypes.create_string_buffer(need + 1)
    _lib.anyseq_alignment_cigar(al_q, al_s, n, out, need + 1)
    return out.value.decode()

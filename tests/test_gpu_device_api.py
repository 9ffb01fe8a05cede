"""GPU: the device-resident entry points (anyseq_score_device / anyseq_construct_device)
give the same results as the host-buffer ones, which are pinned to the oracle
elsewhere; plus the fill statistics and the genome-input helpers."""
import ctypes
import random

import pytest

pytestmark = pytest.mark.gpu

# Device buffers through the same HIP runtime the library links (/opt/rocm), not
# torch: PyTorch-ROCm bundles a second HIP/HSA runtime, and two runtimes in one
# process share the process's hardware-queue budget (conftest raises
# GPU_MAX_HW_QUEUES for the sharded tests).
_hip = ctypes.CDLL("libamdhip64.so.7")
_hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
_hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
_hip.hipFree.argtypes = [ctypes.c_void_p]
H2D, D2H = 1, 2


class DevBuf:
    def __init__(self, n, data=None):
        self.n = max(n, 1)
        self.p = ctypes.c_void_p()
        assert _hip.hipMalloc(ctypes.byref(self.p), self.n) == 0
        if data is not None:
            assert _hip.hipMemcpy(self.p, ctypes.c_char_p(bytes(data)), len(data), H2D) == 0

    def get(self, n):
        out = ctypes.create_string_buffer(max(n, 1))
        assert _hip.hipMemcpy(out, self.p, n, D2H) == 0
        return out.raw[:n]

    def __del__(self):
        _hip.hipFree(self.p)


def rnd(rng, n):
    return "".join(rng.choice("ACGT") for _ in range(n)).encode()


@pytest.mark.parametrize("kind", ["global", "semiglobal", "local"])
@pytest.mark.parametrize("gap_open", [0, -2])
def test_construct_device_matches_oracle(anyseq, oracle, kind, gap_open):
    rng = random.Random(51)
    anyseq.score("global", "A", "A")   # the engine selects the device first
    for n, m in [(700, 900), (3000, 257), (1, 1)]:
        q, s = rnd(rng, n), rnd(rng, m)
        dq, ds = DevBuf(n, q), DevBuf(m, s)
        aq, as_ = DevBuf(n + m), DevBuf(n + m)
        v = anyseq.construct_device(kind, dq.p.value, n, ds.p.value, m, aq.p.value, as_.p.value,
                                    gap_open=gap_open, gap_extend=-1)
        got = (v, aq.get(n + m), as_.get(n + m))
        if gap_open == 0:
            r, oq, os_ = oracle.construct(kind, q, s)
            want = (oracle.score(kind, q, s), oq, os_)
        else:
            want = oracle.affine_construct(kind, q, s, 2, -1, gap_open, -1)
        assert got == want, (kind, n, m, gap_open)


def test_fill_stats_count_cells(anyseq):
    rng = random.Random(52)
    q, s = rnd(rng, 5000), rnd(rng, 3000)
    anyseq.last_fill_stats()
    anyseq.score("global", q, s)
    ms, launches, cells = anyseq.last_fill_stats()
    assert launches == 1 and cells == 5000 * 3000 and ms > 0


def test_affine_rescore_matches_construct(anyseq):
    from anyseq_amd import genome
    q, s = genome.synthetic_related_pair(20000, 0.9)
    for kind in ("global", "semiglobal", "local"):
        v, aq, as_ = anyseq.construct(kind, q, s, gap_open=-2, gap_extend=-1)
        assert genome.affine_rescore(aq, as_) == v == anyseq.score(kind, q, s, gap_open=-2, gap_extend=-1)

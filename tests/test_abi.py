"""CPU tests of the C-ABI boundary: the library loads, exports every declared symbol,
and fails loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "anyseq.h")
LIB = os.path.join(ROOT, "anyseq_amd", "libanyseq.so")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"typedef[^;{]*\([^;]*;", "", txt)   # function-pointer typedefs declare no symbol
    return sorted(set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", txt)) - {"if", "sizeof"})


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    names = declared_functions()
    assert "global_alignment_score" in names and "construct_local_alignment" in names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_reference_abi_symbols_are_c_linkage():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    for n in ["construct_global_alignment", "construct_semiglobal_alignment", "construct_local_alignment",
              "global_alignment_score", "semiglobal_alignment_score", "local_alignment_score"]:
        assert re.search(rf"\sT {n}$", out, re.M), n


def test_python_mirror_names(anyseq):
    for n in ["global_alignment_score", "semiglobal_alignment_score", "local_alignment_score",
              "construct_global_alignment", "construct_semiglobal_alignment", "construct_local_alignment"]:
        assert callable(getattr(anyseq, n))


def test_fails_loudly_without_gpu(anyseq):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(anyseq.AnySeqError):
        anyseq.global_alignment_score("ACGT", "ACGT")
    with pytest.raises(anyseq.AnySeqError):
        anyseq.construct_global_alignment("ACGT", "ACGT")


def test_invalid_scoring_rejected(anyseq):
    with pytest.raises(anyseq.AnySeqError):
        anyseq.score("global", "A", "A", gap_extend=1)


@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="reference tree absent")
def test_reference_driver_links_unchanged(tmp_path):
    """main.cpp + sequence_io.cpp + alignment_io.cpp of the reference compile and link
    against libanyseq.so without modification (drop-in boundary)."""
    if not shutil.which("g++"):
        pytest.skip("no g++")
    src = "/root/reference/src"
    exe = tmp_path / "align"
    subprocess.check_call(["g++", "-std=c++14", "-O1", "-I", src, f"{src}/main.cpp", f"{src}/sequence_io.cpp",
                           f"{src}/alignment_io.cpp", "-L", os.path.dirname(LIB), "-lanyseq",
                           f"-Wl,-rpath,{os.path.dirname(LIB)}", "-o", str(exe)])
    assert exe.exists()


def test_value_range_guard_without_gpu():
    """Scores x lengths that could leave the kernels' int32 range are rejected before any
    GPU call: the error names the limit."""
    import ctypes
    import anyseq_amd as A
    sc = A._scoring(1000, -1000, -1000, -1000)
    out = ctypes.c_int64(0)
    q = b"A" * 16
    rc = A._lib.anyseq_score(0, ctypes.byref(sc), q, 200000, q, 200000, ctypes.byref(out))
    assert rc == -1
    assert b"int32 value range" in A._lib.anyseq_last_error()

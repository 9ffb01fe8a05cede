"""The reference's own driver, run on the GPU.

oracle/_ref/align is the reference's unmodified main.cpp + sequence_io.cpp +
alignment_io.cpp compiled in the build container and linked against OUR
libanyseq.so (oracle/Makefile `ref`; git-ignored, it travels with the tree).  It
calls all six import.h functions through the C ABI; the reference prints only
timings, so the check is that every call returns and the process exits cleanly.
The scores and strings of the same calls are checked bit-exactly elsewhere
(test_gpu_golden.py, main.cpp's own inputs)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALIGN = os.path.join(ROOT, "oracle", "_ref", "align")


@pytest.mark.skipif(not os.path.exists(ALIGN), reason="oracle/_ref/align not built (needs /root/reference)")
@pytest.mark.parametrize("length", [1024, 8192])
def test_reference_main_runs_on_gpu(length):
    out = subprocess.run([ALIGN, "-r", str(length), str(length)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert f"sequence lengths: {length}, {length}" in out.stdout
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("testing ")]
    names = [ln.split(" ms")[0].rsplit(" ", 1)[0][len("testing "):] for ln in lines]
    assert names == ["global score", "semiglobal score", "local score", "global alignment",
                     "semiglobal alignment", "local alignment"], out.stdout
    assert "error" not in out.stderr.lower(), out.stderr

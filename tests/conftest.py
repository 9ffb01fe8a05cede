import os
import sys

import pytest

# The sharded fill runs several concurrent streams, each needing its own hardware
# queue (anyseq_shard.cpp check_hw_queues); set before the first HIP call.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

# Device-planned Hirschberg levels: ANYSEQ_CHECK_ROWS=1 checks after every planned fill
# that the reused hand-off rows are all sentinel again.  It is off
# by default here, so the suite runs the production path; tests/test_gpu_affine_construct.py
# runs every case both ways (advisor round 4).

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def anyseq():
    import anyseq_amd
    return anyseq_amd


def loaded_libraries():
    """The in-tree shared objects this process has mapped (/proc/self/maps), each with the
    first 16 hex digits of its sha256 -- the evidence of which native code a GPU run used."""
    import hashlib
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if len(line.split()) >= 6 else ""
                if p.endswith(".so") or ".so." in p:
                    paths.add(p)
    except OSError:
        return []
    out = []
    for p in sorted(paths):
        if not os.path.realpath(p).startswith(os.path.realpath(ROOT)):
            continue
        with open(p, "rb") as f:
            out.append((os.path.relpath(p, ROOT), hashlib.sha256(f.read()).hexdigest()[:16]))
    return out


def pytest_sessionfinish(session, exitstatus):
    # ANYSEQ_MAPS_OUT=<file>: record the in-tree libraries the test process loaded
    path = os.environ.get("ANYSEQ_MAPS_OUT")
    if path:
        with open(path, "w") as f:
            for rel, digest in loaded_libraries():
                f.write(f"{rel} sha256[:16]={digest}\n")

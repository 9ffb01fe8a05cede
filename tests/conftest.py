import os
import sys

import pytest

# The sharded fill runs several concurrent streams, each needing its own hardware
# queue (anyseq_shard.cpp check_hw_queues); set before the first HIP call.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

# Device-planned Hirschberg levels: after every planned fill, check that the reused
# hand-off rows are all sentinel again (verdict round 3 item 1).
os.environ.setdefault("ANYSEQ_CHECK_ROWS", "1")

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

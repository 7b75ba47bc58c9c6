import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Several ranks of the device exchange share this process (and the GPU) in the
# multi-rank tests: each rank's stream must get a hardware queue of its own,
# or a rank's spinning exchange kernel can sit in front of its peer's kernel in
# a shared queue until the exchange deadline.  HIP's default of 4 queues per
# process is too few once torch's stream and a few leftover contexts' streams
# exist; set before anything initialises HIP (production runs one context per
# process and GPU).
os.environ["GPU_MAX_HW_QUEUES"] = "16"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as orc

    orc.build()
    return orc

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def engine():
    """One rxg context on cuda:0 for the whole GPU session.  No GPU is a failure, not a
    skip: -m gpu runs only where a GPU must be present."""
    import rxg
    eng = rxg.Engine(device=0, max_batch=1 << 16, max_bytes=64 << 20)
    yield eng
    eng.close()


@pytest.fixture(scope="session", params=["host", "device"])
def replay_engine(request):
    """A context per re-classification mode of rxg_rx_replay: small fix-ups answered from the
    host index (default) or every fix-up a GPU launch (RXG_CFG_REPLAY_ON_DEVICE).  Both must
    give the sequential reference's records."""
    import rxg
    flags = rxg.CFG_REPLAY_ON_DEVICE if request.param == "device" else 0
    eng = rxg.Engine(device=0, max_batch=1 << 16, max_bytes=64 << 20, flags=flags)
    yield eng
    eng.close()

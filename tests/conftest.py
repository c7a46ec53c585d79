import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "byzantine-agreement_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libba_hip.so")


@pytest.fixture(scope="session")
def engine():
    from ba_amd.lib import Engine
    eng = Engine(0)
    yield eng
    eng.close()

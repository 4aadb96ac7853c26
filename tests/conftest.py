import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")


def pytest_configure(config):
    # GTK_SWITCH_INTERVAL=1e-6: switch Python threads every few bytecodes, which widens every
    # check-then-act window of the threaded daemons (extender binds, plugin monitor) for a race hunt
    if os.environ.get("GTK_SWITCH_INTERVAL"):
        sys.setswitchinterval(float(os.environ["GTK_SWITCH_INTERVAL"]))
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def fixtures_dir():
    return FIXTURES

import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def oracle():
    import lhutil
    if not os.path.exists(lhutil.ORACLE_SO):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(lhutil.REPO, "oracle")])
    return lhutil.Oracle()

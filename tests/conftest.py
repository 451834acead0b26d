import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


# Batch calls compile a missing specialised module in the background and serve the call
# with the generic kernels meanwhile (the product default).  The parity tests assert which
# kernels ran, so they compile in the call instead; test_jit_compiles_in_background checks
# the default behaviour.
os.environ.setdefault("LONGHAIR_AMD_JIT_SYNC", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def oracle():
    import lhutil
    if not os.path.exists(lhutil.ORACLE_SO):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(lhutil.REPO, "oracle")])
    return lhutil.Oracle()

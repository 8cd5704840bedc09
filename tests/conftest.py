"""Shared pytest setup.  `-m gpu` tests need a HIP device; everything else runs on CPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# parity tests compare every stage array, including rank2head (not kept by default)
os.environ.setdefault("CMSBWT_KEEP_STAGES", "1")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cms-bwt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libcmsbwt.so")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def built():
    """Build the library, CLI and oracle once per session (no-op when up to date)."""
    import __graft_entry__
    __graft_entry__.build()
    return True


@pytest.fixture(scope="session")
def oracle(built):
    import oracle_lib
    return oracle_lib


@pytest.fixture(scope="session")
def engine(built):
    import cmsbwt
    e = cmsbwt.Engine(0)
    yield e
    e.close()

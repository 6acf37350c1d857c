import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="module")
def ab_ctx():
    """A device context on the A/B and test build (liblodestar_bls_ab.so, csrc/lsg_ab.h): the
    stage switches (LSG_PACKAGE_GROUP, LSG_MILLER_FUSED, LSG_MSM_MIN_GROUP, ...) are read from
    the environment there; the shipped library has none."""
    from lodestar_amd._native import AB_LIB_PATH, Context
    c = Context(0, lib=AB_LIB_PATH)
    yield c
    c.close()

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (DGS_TEST_PKG_ROOT: run the suite against a tools/variant.sh build, e.g. variants/NAME)
PKG_ROOT = os.environ.get("DGS_TEST_PKG_ROOT") or os.path.join(REPO, "diff-gaussian-sampling_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE sizes)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as orc
    orc.build()
    return orc


@pytest.fixture(scope="session")
def dgs():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import diff_gaussian_sampling
    return diff_gaussian_sampling

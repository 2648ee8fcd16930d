"""Test configuration: `gpu` marker (tests that need an MI355X), import paths, shared data."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "ssf-slam_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def dev():
    """cuda:0, which must be a gfx950.  A `-m gpu` run on a box where HIP does not enumerate
    the device FAILS here instead of skipping: a green GPU suite with zero tests run would
    claim parity it never checked (the CPU suite deselects these tests with -m "not gpu")."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the -m gpu suite needs an MI355X (gfx950)")
    arch = getattr(torch.cuda.get_device_properties(0), "gcnArchName", "")
    if not arch.startswith("gfx950"):
        pytest.fail(f"cuda:0 is {arch!r}, not gfx950")
    return torch.device("cuda", 0)

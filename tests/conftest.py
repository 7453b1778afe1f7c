import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built native extension")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def C():
    from fpga_ai_nic_amd import _ext

    return _ext.require()


@pytest.fixture(scope="session", autouse=True)
def _release_process_group():
    """A test that initialised torch.distributed in this process (a 1-rank group) leaves it up for the others; tear
    it down once at the end of the session instead of leaving that to interpreter exit."""
    yield
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()

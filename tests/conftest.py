import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-provider-ibm-cloud_amd"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.hookimpl(trylast=True)
def pytest_collection_modifyitems(config, items):
    config._gpu_selected = any(item.get_closest_marker("gpu") for item in items)


def pytest_runtestloop(session):
    """GPU runs: let torch's HIP runtime initialise before libgpusched.so
    loads its own (ROCm under /opt/rocm).  With the library first, torch's
    later init finds no device and the tests that view the library's HBM
    buffers through torch fail depending on test order."""
    if getattr(session.config, "_gpu_selected", False):
        import torch
        torch.cuda.is_available()

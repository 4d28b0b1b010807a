import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu on the MI355X box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle_lib import load_oracle
    return load_oracle()


@pytest.fixture(scope="session")
def usvlib():
    from unsynchronized_stereo_vision_proj325_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def gpu():
    """GPU tests fail loudly (never skip) when the device or native path is missing."""
    import torch
    assert torch.cuda.is_available(), "gpu-marked test needs a GPU (run with -m 'not gpu' on CPU)"
    from unsynchronized_stereo_vision_proj325_amd import _lib
    lib = _lib.load()
    import ctypes
    n = ctypes.c_int(0)
    st = lib.usv_device_check(ctypes.byref(n))
    assert st == _lib.USV_OK, f"usv_device_check -> {_lib.STATUS_NAMES.get(st, st)} ({n.value} devices)"
    return torch.device("cuda:0")

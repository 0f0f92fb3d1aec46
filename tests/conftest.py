"""Test configuration: the `gpu` marker, import paths and shared fixtures.

`-m "not gpu"` runs on CPU only: the oracle against the reference's known-answer tables, the
host-side update logic of the engine through its C-ABI (no device is touched before the first
match/sync), and the library's exported symbols. `-m gpu` runs the parity tests proper, which
call the HIP path through the C-ABI and compare with the oracle.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU is visible")
    return True

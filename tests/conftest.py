import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kotoba-whisper_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: minutes of CPU time")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gold():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            path = os.path.join(GOLD, name + ".npz")
            if not os.path.exists(path):
                pytest.skip(f"golden fixture {name} not generated")
            cache[name] = dict(np.load(path, allow_pickle=False))
        return cache[name]

    return load

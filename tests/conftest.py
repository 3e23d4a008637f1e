import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels / RCCL); run on the GPU box")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_training_compare_jax_amd.ops import _native

    _native.lib()  # must load: GPU tests never fall back to torch
    return torch.device("cuda", 0)

import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

REFERENCE = "/root/reference"  # present only in the build container, never on the GPU box


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def rt4(request):
    # GPU sessions: bring up PyTorch's HIP runtime before librt4.so's (rt4.Tracer does the same when
    # torch is already imported); torch.cuda finds no GPU if it initialises second in the process.
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    return importlib.import_module("4d_ray_tracing_amd")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib

    oracle_lib.lib()
    return oracle_lib


@pytest.fixture(scope="session")
def tracer(rt4):
    t = rt4.Tracer(device=0)
    yield t
    t.close()


@pytest.fixture(scope="session")
def tracer_lut(rt4):
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT)
    yield t
    t.close()


def reference_available():
    return os.path.isdir(os.path.join(REFERENCE, "scenes"))

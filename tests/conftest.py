import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_report_header(config):
    """Which native build the run loads: the hash embedded in the library against the
    sources' hash, and where / with which hipcc command it was compiled."""
    try:
        from rust_gpu_raytracing_amd import build as nb

        info = nb.build_info()
        return [f"rt_pathtrace build: hash {info.get('hash')} (sources {info['sources_hash']}), "
                f"host {info.get('host')}, at {info.get('built_at')}",
                f"rt_pathtrace hipcc: {info.get('command')}"]
    except Exception as e:  # the header must never break collection
        return [f"rt_pathtrace build: unavailable ({e})"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernel)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def native_lib():
    from rust_gpu_raytracing_amd import build as nb

    nb.build(verbose=False)
    from rust_gpu_raytracing_amd import _native

    return _native.load_library()


@pytest.fixture(scope="session")
def gpu():
    """Skip nothing: a gpu-marked test on a box without a GPU must fail loudly."""
    import torch

    assert torch.cuda.is_available(), "gpu test requested but no HIP device is visible"
    from rust_gpu_raytracing_amd import build as nb

    nb.build(verbose=False)
    return torch.device("cuda:0")

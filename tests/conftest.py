import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cse375-finalproj-huffman-decoding_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def gh():
    # torch first: its wheel bundles its own HIP runtime, and the process must end up with
    # one (libgaphuff then binds to the already-loaded libamdhip64; loaded the other way
    # round, torch's later HIP init reports no GPU)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    import gaphuff
    gaphuff.lib()
    return gaphuff


@pytest.fixture(scope="session")
def orc():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def gpu(gh):
    if gh.device_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    return gh

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "ecdna-evo_amd"), os.path.join(REPO, "oracle"), REPO,
          os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs on the GPU box")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def engine_mod():
    """The HIP engine. On the GPU box a missing library or device is a FAILURE, never a skip."""
    from ecdna_evo_amd import engine

    engine.lib()
    n = engine.device_count()
    assert n >= 1, "no gfx950 device visible to libecdna_ssa.so"
    return engine

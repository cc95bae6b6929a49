import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU case")


@pytest.fixture(scope="session")
def cfg():
    from distilcodec_nabeel_amd import config

    return config.default_config()


@pytest.fixture(scope="session")
def state(cfg):
    from distilcodec_nabeel_amd import weights

    return weights.synthetic_state_dict(cfg, seed=1234)


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    d = os.path.join(REPO, "tests", "golden")
    return {n: dict(np.load(os.path.join(d, f"{n}.npz"))) for n in ("e2e_batch", "e2e_3s", "e2e_real", "modules")}

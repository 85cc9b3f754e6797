import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running statistical test")


def synthetic_problem(n, p, seed=20240501, s=None, noise=1.0):
    """SURVEY.md s8(d) synthetic design: X ~ N(0,1) centred, sparse beta, y = X b + e."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, p))
    X -= X.mean(axis=0)
    s = max(5, p // 100) if s is None else s
    s = min(s, p)
    b = np.zeros(p)
    b[:s] = rng.uniform(1, 3, size=s) * rng.choice([-1.0, 1.0], size=s)
    y = X @ b + noise * rng.standard_normal(n)
    y -= y.mean()
    return np.asfortranarray(X), y, b


@pytest.fixture(scope="session")
def gpu_lib():
    import bayesbridge_amd as bb

    L = bb.library()
    if bb.device_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    bb.set_verbose(0)
    # BB_TEST_TUNING="KEY=VALUE,...": bb_set_tuning before the GPU tests (A/B of a default)
    for kv in filter(None, os.environ.get("BB_TEST_TUNING", "").split(",")):
        k, v = kv.split("=")
        bb.set_tuning(int(k), int(v))
    return bb

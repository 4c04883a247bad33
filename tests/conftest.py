import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def traces():
    d = np.load(os.path.join(GOLDEN, "model1_traces.npz"))
    train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))]
    return dict(train=np.array(train), test=d["test_cpu"], test_mean=d["test_mean"],
                test_violations=d["test_violations"], raw=d)


@pytest.fixture(scope="session")
def rt():
    import _pkg
    return _pkg.load()

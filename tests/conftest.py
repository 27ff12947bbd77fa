import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs via gpurun")
    config.addinivalue_line("markers", "slow: full-size (32 MiB shard) cases")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def gf_tables(oracle):
    """(exp, log) numpy tables of the crate's GF(2^16) (oracle restatement)."""
    import numpy as np
    L = oracle.lib()
    exp = np.array([L.oracle_gf_exp(i) for i in range(65536)], dtype=np.uint32)
    log = np.array([L.oracle_gf_log(i) for i in range(65536)], dtype=np.uint32)
    return exp, log


@pytest.fixture(scope="session")
def bfrs():
    import bfrs as B
    B.lib()
    return B


@pytest.fixture(scope="session")
def ctx(bfrs):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = bfrs.Context(0)
    yield c
    c.close()

"""Test configuration.

-m "not gpu": oracle KATs against the reference's own tables, golden fixtures, C-ABI
              load/export checks, gloo multi-process logic -- runs in the CPU container.
-m gpu:       GPU-vs-oracle parity through the C ABI (liborbg.so) on an MI355X.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def kitti_seq():
    from orb_slam2_test_amd import synthetic
    return synthetic.sequence(6, 376, 1241, seed=synthetic.DEFAULT_SEED)


@pytest.fixture(scope="session")
def ref_tables():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "ref_tables.json")) as f:
        return json.load(f)

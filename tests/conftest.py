"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs here (no GPU): the oracle against the golden fixtures and
an independent torch float64 formulation, host-side logic, the C-ABI library
(load + symbol exports, no compute) and the gloo data-parallel tests.
`-m gpu` runs on an MI355X: parity of the HIP path against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "kaldi-cnn_amd"),
          os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) checks")


@pytest.fixture(scope="session")
def kc():
    """libkcnn.so bound to cuda:0 and torch's current stream."""
    import kcnn
    kcnn.init(0)
    return kcnn


@pytest.fixture(scope="session", autouse=True)
def _oracle_threads():
    try:
        import oracle
        oracle.set_threads(min(16, os.cpu_count() or 1))
    except Exception:
        pass

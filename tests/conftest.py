"""Shared test setup.

* ``-m gpu`` tests need a real MI355X and call the engine through the C ABI.
* ``-m "not gpu"`` tests cover the oracle against the golden fixtures, host
  logic, and that libbfhip.so loads and exports every declared symbol.
The oracle (oracle/) is imported here ONLY as the checker.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import pkgload  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def pkg():
    return pkgload.load()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    return O.COracle()


@pytest.fixture(scope="session")
def O():
    import oracle as O
    return O

import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


def pkg(mod):
    return importlib.import_module("context-based-pii_amd." + mod)


@pytest.fixture(scope="session")
def compiled():
    return pkg("compiler").compile_default()


@pytest.fixture(scope="session")
def oracle_cfg():
    from oracle import pii_oracle as O
    return O.RuleConfig.load()

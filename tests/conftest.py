import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
GOLDEN = os.path.join(HERE, "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu on the MI355X box)")
    config.addinivalue_line("markers", "slow: long CPU-side oracle runs")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def streams():
    return load_golden("streams.json")


@pytest.fixture(scope="session")
def verdicts():
    return load_golden("verdicts.json")


@pytest.fixture(scope="session")
def hitsets():
    return load_golden("hitsets.json")


@pytest.fixture(scope="session")
def intermediates():
    return load_golden("intermediates.json")


@pytest.fixture(scope="session")
def long_verdicts():
    """Reference verdicts for long candidates (tests/golden/make_long.py): name -> {stream, password, verdicts}"""
    return load_golden("long_verdicts.json")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle

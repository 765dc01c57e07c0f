import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def appendix_b():
    with open(os.path.join(ROOT, "tests", "golden", "appendix_b.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # test infrastructure only
    O.build()
    return O


@pytest.fixture(scope="session")
def pj():
    import paralleljohnson_amd as pj
    return pj


@pytest.fixture(scope="session")
def ctx(pj):
    c = pj.Context(0)
    yield c
    c.close()

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libccg.so on the device)")


def _ensure_built():
    lib = os.path.join(ROOT, "consensusclustr_amd", "libccg.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "consensusclustr_amd", "csrc")])
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_built()


@pytest.fixture(scope="session")
def engine():
    from consensusclustr_amd import Engine
    eng = Engine(0)
    yield eng
    eng.close()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return load


@pytest.fixture(scope="session")
def kat():
    import json
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)

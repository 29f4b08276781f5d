import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bo-lz4-ada_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
VECTORS = os.path.join(GOLDEN, "vectors")

for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def load_digests():
    with open(os.path.join(GOLDEN, "vector_digests.json")) as fh:
        return json.load(fh)


def good_vectors():
    """Every *.lz4 with expected output (lz4test.adb:101-127 pairs *.lz4/*.bin)."""
    d = load_digests()
    return sorted(d)


def error_vectors():
    names = sorted(f[:-4] for f in os.listdir(VECTORS) if f.endswith(".err"))
    return names


def read_vector(name, ext):
    with open(os.path.join(VECTORS, f"{name}.{ext}"), "rb") as fh:
        return fh.read()


def read_eds(name):
    with open(os.path.join(VECTORS, f"{name}.eds"), "r") as fh:
        return fh.readline().rstrip("\n")


@pytest.fixture(scope="session")
def digests():
    return load_digests()

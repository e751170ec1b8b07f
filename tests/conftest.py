"""Shared test setup: import paths for the product package and the oracle
(test infrastructure), the `gpu` marker, and golden fixtures."""
import json
import os
import sys

import pytest

# torch first (its first import on a fresh box is slow, and it must own the
# process's HIP runtime before libkubecheck.so loads: see kubecheck/_lib.py)
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tla-kubernetes_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def mcout():
    return json.load(open(os.path.join(GOLDEN, "model1_mcout.json")))


@pytest.fixture(scope="session")
def fixtures():
    return json.load(open(os.path.join(GOLDEN, "oracle_fixtures.json")))


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    pyoracle.lib()
    return pyoracle

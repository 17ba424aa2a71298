"""Shared pytest setup: `gpu` marker, import paths, golden fixtures."""
import json
import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "needleman-wunsch_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ref_kats():
    return load_golden("ref_kats.json")


@pytest.fixture(scope="session")
def cli_cases():
    return load_golden("cli_cases.json")


@pytest.fixture(scope="session")
def walk_kats():
    return load_golden("walk_kats.json")

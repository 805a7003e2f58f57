"""Shared fixtures.  `gpu`-marked tests need an MI355X (run with `-m gpu`); everything else runs
on the CPU.  The oracle (oracle/liboracle_bre.so) is test infrastructure: only tests, smoke() and
bench.py's cpu_baseline leg load it."""
import importlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle():
    from oracle_lib import load_oracle

    return load_oracle()


@pytest.fixture(scope="session")
def bre():
    return importlib.import_module("beam-radiance-estimate-pbrt_amd")


@pytest.fixture(scope="session")
def synth():
    return importlib.import_module("beam-radiance-estimate-pbrt_amd.synth")


@pytest.fixture(scope="session")
def scene_mod_gpu():
    return importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")

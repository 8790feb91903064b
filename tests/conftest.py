"""Shared pytest setup.

Markers: `gpu` = needs a real MI355X (run on the GPU box with `-m gpu`); everything else runs on
the CPU here (`-m "not gpu"`).  The product libraries are the in-tree builds
(webp-decoder_amd/lib); `make` must have run (the driver's build() does it).
"""
import json
import pathlib
import sys

import pytest

# torch bundles its own HIP runtime under the same soname as /opt/rocm's: whichever loads first
# serves the whole process.  Load torch's first (as bench.py does), so that tests which allocate
# device memory with torch after libvp8g.so has run still see the GPU.
import torch  # noqa: F401,E402

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))

FIXTURES = ROOT / "tests" / "fixtures"
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session")
def manifest():
    return json.loads((GOLDEN / "manifest.json").read_text())


@pytest.fixture(scope="session")
def synth_kat():
    return json.loads((GOLDEN / "synth_kat.json").read_text())


@pytest.fixture(scope="session")
def vp8g():
    import vp8g as m
    return m

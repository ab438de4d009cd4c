"""Shared test plumbing.

`-m "not gpu"` (CPU, this container): the oracle against known answers and
golden vectors, frame bytes against the reference's nanopb, host logic, the
C-ABI library's exports, and world_size-2 gloo tests of the sharded path.
`-m gpu` (MI355X box): parity of the HIP path against the oracle, through the
C ABI.
"""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def load_pkg():
    """Import audio-network_amd/ (hyphenated directory) as audio_network_amd."""
    if "audio_network_amd" in sys.modules:
        return sys.modules["audio_network_amd"]
    spec = importlib.util.spec_from_file_location(
        "audio_network_amd", os.path.join(ROOT, "audio-network_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["audio_network_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def A():
    return load_pkg()


@pytest.fixture(scope="session")
def O():
    from oracle import oracle
    return oracle

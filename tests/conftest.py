import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "espnet-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _clear_rng_salt(request):
    """A model sets the process-wide dropout salt pointer (ea_set_rng_salt) to its own device
    buffer; op-level tests must not inherit one left by a model an earlier test freed."""
    if request.node.get_closest_marker("gpu") is not None:
        try:
            from espnet_amd._lib import lib
            lib.ea_set_rng_salt(None)
        except Exception:
            pass
    yield

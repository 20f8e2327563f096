import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu on the GPU box")


@pytest.fixture(scope="session")
def golden():
    import json
    d = os.path.join(ROOT, "tests", "golden")
    return {n[:-5]: json.load(open(os.path.join(d, n))) for n in os.listdir(d) if n.endswith(".json")}


@pytest.fixture(scope="session")
def oracle_native():
    from oracle import native
    native.lib()
    return native

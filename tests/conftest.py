import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "cuda-raytracer_amd"), os.path.join(REPO, "tools"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle, the product library and the stand-in env map once per session."""
    import oracle_lib
    import rtamd
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import make_envmap
    make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
    oracle_lib.build()
    if not os.path.exists(rtamd.LIB_PATH):
        rtamd.build()
    yield

"""__graft_entry__.build() -- what the driver runs as the build check each round -- completes and accepts the
library it built (ABI version from include/rt_abi.h).  A stale hard-coded version once made it fail after an ABI
bump while every other test passed."""
import os
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not (os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("hipcc")), reason="hipcc not found")
def test_build_entry_point():
    sys.path.insert(0, REPO)
    import __graft_entry__ as g
    g.build()

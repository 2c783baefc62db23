import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "crdt-graph_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
# the engine's test-only hooks (include/crdtm_test.h: crdtm_debug_poke, the
# level replay's injected commit failure) act only in a process that sets
# this before the library's first call
os.environ.setdefault("CRDTM_TEST_HOOKS", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: larger CPU cases")

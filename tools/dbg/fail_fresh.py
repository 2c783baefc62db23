"""Debug: a failing base batch on a fresh tree, then one op (adversarial seed 14)."""
import os
import sys
sys.path.insert(0, "crdt-graph_amd")
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from adversarial import adversarial
from crdtm import _native as N
from crdtm.tree import CRDTree, pack
from test_gpu_incremental import sub

s = pack(adversarial(14, 600, replicas=4, max_depth=3))
for mode in ("auto", "remerge", "replay", "ilr"):
    os.environ["CRDTM_INCREMENTAL"] = mode
    et = CRDTree.init(0)
    r1 = et.apply_arrays(sub(s, 0, 200), 200)
    r2 = et.apply_arrays(sub(s, 200, 201), 1)
    print(mode, (r1.code, r1.err_index, r1.path_taken, r1.flags), (r2.code, r2.err_index, r2.path_taken, r2.flags),
          flush=True)

"""Debug: config-2-shaped level replay (the parity test's stream), per batch: flags, then a host check of the state."""
import os
import sys
sys.path.insert(0, "crdt-graph_amd")
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
from crdtm import _native as N
from crdtm.tree import CRDTree
from test_gpu_incremental import sub

base, bsz, nb = 200_000, 10_000, 5
s = N.synth(n_ops=base + bsz * nb, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4, seed=0xC0FFEE02)
et = CRDTree.init(0)
cuts = [0, base] + [base + bsz * (j + 1) for j in range(nb)]
for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
    res = et.apply_arrays(sub(s, a, b), b - a)
    print(k, res.code, res.flags, res.path_taken, res.n_slots, flush=True)
    h = et.document_handles()
    print("   doc", len(h), flush=True)
    from parity_util import engine_summary
    es = engine_summary(et)
    print("   summary", es[0], es[1], flush=True)

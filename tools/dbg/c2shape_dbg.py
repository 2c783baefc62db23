"""Debug: the level replay at test_level_replay_config2_shape's shape, per batch (CRDTM_ILR_DEBUG lines)."""
import os
import sys
sys.path.insert(0, "crdt-graph_amd")
import numpy as np  # noqa: E402
from crdtm import _native as N  # noqa: E402
from crdtm.tree import CRDTree  # noqa: E402

base, bsz, nb = int(os.environ.get("BASE", 200_000)), 10_000, int(os.environ.get("NB", 5))
s = N.synth(n_ops=base + bsz * nb, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4, seed=0xC0FFEE02)
po = s["path_off"]


def sub(a, b):
    return dict(kind=s["kind"][a:b].copy(), ts=s["ts"][a:b].copy(), val=s["val"][a:b].copy(),
                path_off=(po[a:b + 1] - po[a]).astype(np.uint32), path=s["path"][po[a]:po[b]].copy())


et = CRDTree.init(0)
cuts = [0, base] + [base + bsz * (j + 1) for j in range(nb)]
for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
    res = et.apply_arrays(sub(a, b), b - a)
    print(f"batch {k} [{a},{b}) code {res.code} flags {res.flags} path {res.path_taken}", file=sys.stderr, flush=True)

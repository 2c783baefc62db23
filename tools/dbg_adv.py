"""Debug helper: engine statuses for one adversarial seed (GPU box)."""
import sys, json
sys.path[:0] = ['tests', 'crdt-graph_amd', '.']
import numpy as np
from adversarial import adversarial
from crdtm.tree import CRDTree, pack
seeds = [int(a) for a in sys.argv[1:]]
out = {}
for seed in seeds:
    n = [40, 120, 400, 1500][seed % 4]
    ops = adversarial(seed, n, replicas=2 + seed % 3, max_depth=1 + seed % 4)
    arrs = pack(ops)
    et = CRDTree.init(0)
    st = np.zeros(n, np.uint8)
    res = et.apply_arrays(arrs, n, status=st)
    out[seed] = dict(code=res.code, err=res.err_index, path=res.path_taken, guard=res.guard, st=st.tolist())
json.dump(out, open('gpurun_out/dbg_adv.json', 'w'))
print({k: (v['code'], v['err'], v['path'], v['guard']) for k, v in out.items()})

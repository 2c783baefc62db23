"""Which merge path each adversarial seed takes (GPU box diagnostic)."""
import sys, collections
sys.path[:0] = ['tests', 'crdt-graph_amd', '.']
from adversarial import adversarial
from crdtm.tree import CRDTree, pack
c = collections.Counter()
for seed in range(128):
    n = [40, 120, 400, 1500][seed % 4]
    ops = adversarial(seed, n, replicas=2 + seed % 3, max_depth=1 + seed % 4)
    et = CRDTree.init(0)
    res = et.apply_arrays(pack(ops), n)
    c[(res.path_taken, res.code)] += 1
print(sorted(c.items()))

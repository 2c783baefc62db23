"""Random op streams that stress findInsertion's tombstone walk (test data).

Deletes interleave with Adds from several replicas whose timestamps order by
replica id first (ts = replica * 2^32 + counter), so a low-replica Add after a
Delete of a high-replica node walks over a tombstone: the copy quirk of
src/Internal/Node.elm:93-104 fires often, in nested dicts too.
Anchors are picked among keys already added to the dict, so most ops are valid
and a batch rarely stops early; duplicates give AlreadyApplied.
"""
import random

from crdtm.operation import Add, Delete


def adversarial(seed, n, replicas=3, p_del=0.3, p_nest=0.35, max_depth=3, p_dup=0.03, recent=6):
    rng = random.Random(seed)
    ctr = [rng.randrange(1, 50) for _ in range(replicas)]
    dicts = {(): [0]}
    nodes = []
    ops = []
    for k in range(n):
        if nodes and rng.random() < p_del:
            pick = nodes[-recent:] if rng.random() < 0.6 else nodes
            ops.append(Delete(list(rng.choice(pick))))
            continue
        par = ()
        if nodes and rng.random() < p_nest:
            par = rng.choice(nodes[-4 * recent:])
            if len(par) >= max_depth:
                par = par[:rng.randrange(max_depth)]
        keys = dicts.setdefault(par, [0])
        anchor = rng.choice(keys[-recent:]) if rng.random() < 0.7 else rng.choice(keys)
        if len(keys) > 1 and rng.random() < p_dup:
            ts = rng.choice(keys[1:])
        else:
            r = rng.randrange(replicas)
            ctr[r] += rng.randint(1, 3)
            ts = r * (1 << 32) + ctr[r]
            keys.append(ts)
            nodes.append(par + (ts,))
        ops.append(Add(ts, list(par) + [anchor], "v%d" % k))
    return ops

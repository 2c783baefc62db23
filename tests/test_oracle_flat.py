"""The searched flat restatement (oracle/crdtree_oracle.cpp `orc_flat_replay`,
findInsertion's stop node found through a treap over the list order) against
the literal walk (`orc_flat_replay_literal`, src/Internal/Node.elm:93-104 step
by step, itself pinned against the general restatement in
tests/test_oracle_kat.py). Same return code, error index, applied count and
canonical digests on typing streams of several shapes and on random flat
batches with duplicates, missing anchors, ts 0 and negative keys. CPU only:
the searched form is what tests/test_gpu_fullsize.py runs over config 3's
10M ops."""
import ctypes as C

import numpy as np
import pytest

from crdtm import _native as N
from oracle.oracle import _ptr, lib as olib


def both(s, m):
    L = olib()
    out = []
    for f in (L.orc_flat_replay, L.orc_flat_replay_literal):
        h = np.zeros(2, np.uint64)
        w = np.zeros(2, np.uint64)
        err = C.c_int64(-1)
        na = C.c_uint64()
        rc = f(m, _ptr(s["kind"]), _ptr(s["ts"]), _ptr(s["path_off"]), _ptr(s["path"]), _ptr(s["val"]),
               C.byref(err), _ptr(h), _ptr(w), C.byref(na))
        out.append((rc, err.value, na.value, tuple(int(x) for x in h), tuple(int(x) for x in w)))
    return out


@pytest.mark.parametrize("spec", [dict(replicas=64, window=256, seed=0xC0FFEE03),
                                  dict(replicas=2, window=1, seed=7),
                                  dict(replicas=16, window=64, p_continue=0.5, seed=8),
                                  dict(replicas=200, window=32, seed=9)])
def test_searched_matches_literal_typing(spec):
    m = 150_000
    s = N.synth(n_ops=m, **spec)
    a, b = both(s, m)
    assert a == b and a[0] == 0 and a[2] == m


def random_flat(rng, m, p_dup=0.05, p_bad=0.0, p_zero=0.0, neg=False):
    """Flat Adds in a causal order: each anchors at the sentinel or at an
    earlier key; some repeat an earlier timestamp (AlreadyApplied), some
    anchor at a key no op adds (NotFound), some carry ts 0 (the sentinel)."""
    ts = np.zeros(m, np.int64)
    anc = np.zeros(m, np.int64)
    ctr = {}
    seen = []
    for i in range(m):
        if seen and rng.random() < p_dup:
            t = seen[rng.integers(len(seen))]
        elif rng.random() < p_zero:
            t = 0
        else:
            r = int(rng.integers(1, 9))
            ctr[r] = ctr.get(r, 0) + int(rng.integers(1, 3))
            t = (-1 if neg and r % 3 == 0 else 1) * (r * 2 ** 32 + ctr[r])
        ts[i] = t
        if rng.random() < p_bad:
            anc[i] = 123456789
        elif seen and rng.random() < 0.9:
            anc[i] = seen[int(rng.integers(max(0, len(seen) - 40), len(seen)))]
        else:
            anc[i] = 0
        if t != 0:
            seen.append(t)
    return dict(kind=np.zeros(m, np.uint8), ts=ts, path_off=np.arange(m + 1, dtype=np.uint32), path=anc,
                val=np.arange(m, dtype=np.uint32))


@pytest.mark.parametrize("seed", range(6))
def test_searched_matches_literal_random(seed):
    rng = np.random.default_rng(seed)
    m = 4000
    kw = [dict(), dict(p_zero=0.01), dict(neg=True), dict(p_dup=0.3), dict(p_bad=0.001), dict(neg=True, p_dup=0.2)]
    s = random_flat(rng, m, **kw[seed])
    a, b = both(s, m)
    assert a == b

"""crdtm_shard_assemble (HIP) against the torch assembly of the same records."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_native_assemble_matches_torch():
    import torch
    from crdtm import _native as N
    from crdtm import shard
    rng = np.random.default_rng(5)
    n_docs, per, world = 37, 50, 3
    recs = []
    for d in range(n_docs):
        for q in range(per):
            recs.append([(d << 32) | q, (int(rng.integers(0, 2)) << 32) | int(rng.integers(0, 1 << 31)),
                         int(rng.integers(1, 1 << 50)), int(rng.integers(0, 1 << 50))])
    rec = np.array(recs, np.int64)
    rec = rec[rng.permutation(len(rec))]
    dev = torch.device("cuda", 0)
    ctx = C.c_void_p()
    N.check(N.lib().crdtm_ctx_create(0, C.c_void_p(torch.cuda.current_stream().cuda_stream), C.byref(ctx)))
    try:
        for rank in range(world):
            t = torch.from_numpy(rec).to(dev)
            a, off_a, _ = shard.assemble(t, rank, world, n_docs, per)
            b, off_b, _ = shard.assemble(t, rank, world, n_docs, per, ctx=ctx)
            torch.cuda.synchronize()
            assert np.array_equal(off_a, off_b)
            n = int(off_a[-1])
            for k in ("kind", "ts", "path", "val"):  # (the torch path spills other ranks' records to index n)
                assert torch.equal(a[k][:n].to(torch.int64), b[k][:n].to(torch.int64)), k
            assert torch.equal(a["path_off"].to(torch.int64), b["path_off"].to(torch.int64))
    finally:
        N.lib().crdtm_ctx_destroy(ctx)

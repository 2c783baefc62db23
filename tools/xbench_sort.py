#!/usr/bin/env python3
"""Microbenchmark of the incremental merge's batch sort (radix_sort_small,
primitives.hip) through crdtm_xbench_sort_small: key distributions of a
10k-op batch, each kernel variant timed with HIP events, outputs checked
against numpy's stable argsort."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "crdt-graph_amd"))
from crdtm import _native as N  # noqa: E402

L = N.lib()
f = L.crdtm_xbench_sort_small
f.argtypes = [C.c_void_p] * 2 + [C.c_uint32] * 2 + [C.c_void_p] * 3 + [C.c_int, C.c_void_p]
rng = np.random.default_rng(1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
dists = {
    "uniform24": rng.integers(0, 1 << 24, n),
    "uniform28": rng.integers(0, 1 << 28, n),
    "few_gaps8": rng.choice(rng.integers(0, 1 << 24, 8), n),
    "few_gaps200": rng.choice(rng.integers(0, 1 << 24, 200), n),
    "window64k": (1 << 23) + rng.integers(0, 1 << 16, n),
    "one_gap": np.full(n, 12345),
}
for path in sys.argv[2:]:  # gap keys dumped by CRDTM_FI_DUMP_KEYS
    k = np.fromfile(path, dtype=np.uint32)
    dists[os.path.basename(path)] = k
    u, c = np.unique(k, return_counts=True)
    print("%s: %d keys, %d distinct, largest run %d, max %d" % (path, len(k), len(u), c.max(), k.max()))
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream()
for name, keys in dists.items():
    keys = keys.astype(np.uint32)
    n = len(keys)
    bits = 4
    while bits < 32 and int(keys.max()) >> bits:
        bits += 4
    kin = torch.from_numpy(keys.view(np.int32)).to(dev)
    vin = torch.arange(n, dtype=torch.int32, device=dev)
    ko = torch.empty_like(kin)
    vo = torch.empty_like(vin)
    want = np.argsort(keys, kind="stable")
    row = []
    cw = torch.empty(((n + 1023) // 1024) * 1024, dtype=torch.int64, device=dev)
    for which in (3, 1, 2):
        args = (kin.data_ptr(), vin.data_ptr(), n, bits, ko.data_ptr(), vo.data_ptr(), s.cuda_stream, which, cw.data_ptr())
        assert f(*args) == 0
        torch.cuda.synchronize()
        ok = np.array_equal(vo.cpu().numpy(), want) and np.array_equal(ko.cpu().numpy().view(np.uint32), keys[want])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f(*args)
        e1.record()
        torch.cuda.synchronize()
        row.append("%s %.1f us%s" % (["w4", "w4", "s4", "chunk"][which], e0.elapsed_time(e1) * 1e3 / 50, "" if ok else " WRONG"))
    print("%-12s bits %2d  %s" % (name, bits, "  ".join(row)), flush=True)

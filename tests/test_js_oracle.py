"""Differential check of the two CPU restatements of the Elm reference:
oracle/crdtree.js (persistent red-black Dicts and cons Lists, the
Elm-compiled-to-JS cost model used as bench.py's CPU baseline) against
oracle/crdtree_oracle.cpp (mutable maps, pinned by the transcribed reference
tests). Same inputs, same canonical word-dump hashes (structure and visible
order), timestamp, replicas table and log length."""
import os
import sys

import numpy as np
import pytest

from oracle import jsoracle
from parity_util import oracle_apply_arrays, oracle_summary, oracle_log
from oracle.oracle import lib as olib

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(jsoracle.node_bin() is None, reason="node not installed")


def _check(arrs, n, tmp_path, mode="chunk", chunk=10000, tag="b"):
    f = str(tmp_path / f"{tag}.bin")
    jsoracle.write_batch(f, arrs, n)
    js = jsoracle.run(f, mode=mode, chunk=chunk, canonical=True)
    doc = js["docs"][0]
    ot, rc, _ = oracle_apply_arrays(arrs, n)
    try:
        if mode == "batch" or rc != 0:
            assert doc["code"] == rc
        if rc != 0:
            return doc
        o = oracle_summary(ot)
        assert (doc["struct"][0], int(doc["struct"][1])) == o[0]
        assert (doc["visible"][0], int(doc["visible"][1])) == o[1]
        assert doc["timestamp"] == o["ts"]
        assert {int(a): int(b) for a, b in doc["replicas"]} == o["replicas"]
        assert doc["applied"] == len(oracle_log(ot, 0)[0])
        if mode == "batch":
            assert doc["last_len"] == len(oracle_log(ot, 1)[0])
    finally:
        olib().orc_free(ot)
    return doc


@pytest.mark.parametrize("seed", range(12))
def test_adversarial_js_vs_cpp(seed, tmp_path):
    """Copy quirks, nested dicts, duplicates and deletes under deleted branches."""
    from adversarial import adversarial
    from crdtm.tree import pack
    n = [60, 200, 700, 1500][seed % 4]
    ops = adversarial(seed, n, replicas=2 + seed % 3, max_depth=1 + seed % 4)
    _check(pack(ops), n, tmp_path, mode="batch")


@pytest.mark.parametrize("cfg", [
    dict(n_ops=20000, replicas=8, window=16, p_delete=0.2, p_branch=0.1, max_depth=3, seed=0xC0FFEE01),
    dict(n_ops=20000, replicas=64, window=256, seed=0xC0FFEE03),
    dict(n_ops=20000, replicas=16, p_delete=1 / 3, max_depth=12, max_children=8, deletes_last=1, seed=0xC0FFEE04),
    dict(n_ops=10000, replicas=2, window=8, p_delete=0.3, p_branch=0.05, max_depth=3, seed=0xC0FFEE01),
])
def test_synthetic_js_vs_cpp(cfg, tmp_path):
    """The bench generator's streams, applied in 10k-op Batches (mode ii): same
    final tree as one Batch."""
    from crdtm import _native as N
    s = N.synth(**cfg)
    _check(s, len(s["kind"]), tmp_path, mode="chunk", chunk=10000)


def test_batch_error_is_atomic(tmp_path):
    """A failing op aborts the Batch (tests/CRDTreeTest.elm:482-498): the JS
    restatement reports the same error code as the C++ one."""
    from crdtm.operation import Add, Delete
    from crdtm.tree import pack
    o = 1 << 32
    ops = [Add(o + 1, [0], "a"), Delete([o + 1]), Add(o + 2, [o + 9], "b")]
    doc = _check(pack(ops), len(ops), tmp_path, mode="batch")
    assert doc["code"] == 3  # OperationFailed


def test_workers_forest(tmp_path):
    """worker_threads mode (the config-5 baseline): per-document results equal
    the single-thread run."""
    from crdtm import _native as N
    s = N.synth(n_ops=300, n_docs=6, replicas=8, window=16, p_delete=0.2, seed=0xC0FFEE05)
    doc_off = np.arange(7, dtype=np.uint32) * 300
    f = str(tmp_path / "f.bin")
    jsoracle.write_batch(f, s, doc_off=doc_off)
    a = jsoracle.run(f, canonical=True, workers=1)
    b = jsoracle.run(f, canonical=True, workers=3)
    assert b["workers"] == 3 and a["ops"] == b["ops"] == 1800
    assert a["docs"] == b["docs"]

"""The Node N-API addon (crdt-graph_amd/napi): the host path an Elm
application uses through ports.

CPU: the addon builds, loads, exports the port API and fails loudly without a
GPU. GPU: JSON in -> addon -> C ABI -> HIP -> JSON out matches the oracle on
the reference's known-answer scenarios and on a synthetic stream.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADDON = os.path.join(ROOT, "crdt-graph_amd", "napi", "crdtm.node")
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None or not os.path.exists("/usr/include/node/node_api.h"),
                                reason="node / N-API headers not available")


def ensure_built():
    if not os.path.exists(ADDON):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "crdt-graph_amd")])
    assert os.path.exists(ADDON)


def test_addon_exports_and_fails_loudly_without_a_gpu():
    ensure_built()
    code = ("const a=require(%r); console.log(JSON.stringify(Object.keys(a).sort()));"
            "try { a.init(0); console.log('created'); } catch (e) { console.log(e.code); }") % ADDON
    out = subprocess.run([NODE, "-e", code], capture_output=True, text=True, timeout=60, check=True).stdout.split()
    assert json.loads(out[0]) == sorted(["init", "apply", "applySync", "operationsSince", "lastOperation", "timestamp",
                                         "lastReplicaTimestamp", "document", "release"])
    import torch
    if not torch.cuda.is_available():
        assert out[1] == "E_NODEVICE"  # no CPU fallback behind the port


def _values_of(log):
    return [(o[0], o[1], tuple(o[2]), o[3]) for o in log]


@pytest.mark.gpu
def test_addon_matches_oracle(tmp_path):
    ensure_built()
    import sys
    sys.path[:0] = [os.path.join(ROOT, "crdt-graph_amd"), ROOT, os.path.dirname(__file__)]
    from crdtm.codec import decoder, encoder
    from crdtm.operation import Batch, flatten
    from crdtm.tree import pack
    from kat_cases import SCENARIOS
    from parity_util import oracle_apply_arrays, oracle_log, oracle_summary

    cases, expect = [], []
    for name in sorted(SCENARIOS):
        replica, calls = SCENARIOS[name]
        cases.append({"replica": replica, "calls": [encoder(op) for op in calls], "since": []})
        expect.append((replica, calls))
    # a synthetic interleaved stream, as one JSON Batch (per-dict replay on the device)
    from crdtm import _native as N
    s = N.synth(n_ops=3000, replicas=4, window=16, p_delete=0.2, p_branch=0.1, max_depth=3, seed=77)
    from crdtm.operation import Add, Delete
    ops = []
    for i in range(len(s["kind"])):
        p = [int(x) for x in s["path"][s["path_off"][i]:s["path_off"][i + 1]]]
        ops.append(Add(int(s["ts"][i]), p, "v%d" % i) if s["kind"][i] == 0 else Delete(p))
    big = Batch(ops)
    adds = [o.ts for o in ops if o.kind == "add"]
    cases.append({"replica": 0, "calls": [encoder(big)], "since": [adds[10], adds[-1], 12345]})
    expect.append((0, [big]))
    # keys at the timestamp boundaries (exact JS Numbers up to 2^53 - 1), through JSON both ways
    ts_max = (1 << 53) - 1
    fs = N.synth(n_ops=500, replicas=8, window=16, seed=78)
    edge = [Add(int(fs["ts"][i]), [int(fs["path"][i])], "f%d" % i) for i in range(500)]
    a = edge[10].ts
    edge += [Add(ts_max, [a], "max"), Add((3 << 32) + 0xFFFFFFFF, [ts_max], "top"), Add(77 << 32, [a], "zero"),
             Add((5 << 32) + 999_999, [ts_max, 0], "child")]
    cases.append({"replica": 0, "calls": [encoder(Batch(edge))], "since": [ts_max, 77 << 32, (5 << 32) + 999_999]})
    expect.append((0, [Batch(edge)]))

    # the same scenarios again with every apply queued before the first is
    # awaited (the addon's per-tree FIFO keeps the reference's call order)
    for (replica, calls), case in list(zip(expect, cases))[:len(SCENARIOS)]:
        if len(calls) > 1:
            cases.append(dict(case, queued=True))
            expect.append((replica, calls))

    # oracle side first: the expected lastOperation of every call (its JSON
    # bytes are produced by Node's JSON.stringify in napi_run.js, not by this
    # package's encoder)
    from crdtm.tree import VALUES
    from oracle.oracle import lib as olib
    oracle_runs = []
    for (replica, calls), case in zip(expect, cases):
        ot = olib().orc_init(replica)
        per_call = []
        for op in calls:
            leaves = flatten(op) if op.kind == "batch" else [op]
            _, rc, oerr = oracle_apply_arrays(pack(leaves), len(leaves), is_batch=op.kind == "batch", tree=ot)
            last = None
            if rc == 0:
                olast, oisb = oracle_log(ot, 1)
                last = {"isBatch": oisb, "ops": [[k, t, list(p), VALUES.value(v) if k == 0 else None]
                                                 for k, t, p, v in olast]}
            per_call.append((rc, oerr))
            case.setdefault("expectLast", []).append(last)
        oracle_runs.append((ot, per_call))

    fin, fout = tmp_path / "in.json", tmp_path / "out.json"
    fin.write_text(json.dumps(cases))
    subprocess.run([NODE, os.path.join(ROOT, "tests", "napi_run.js"), str(fin), str(fout)], check=True, timeout=300)
    got = json.loads(fout.read_text())

    for (ot, per_call), case, res in zip(oracle_runs, cases, got):
        for (rc, oerr), text, r, want in zip(per_call, case["calls"], res["results"], res["expectLast"]):
            assert r["code"] == rc, (text[:80], r, rc)
            if rc != 0:
                assert r["errIndex"] == oerr
                continue
            # lastOperation: byte-identical to Encode.encode 0 of the oracle's lastOperation
            assert r["lastOperation"] == want, (r["lastOperation"][:200], want[:200])
        # full log and visible document against the oracle
        log = decoder(res["log"])
        olog, _ = oracle_log(ot, 0)
        assert len(flatten(log)) == len(olog)
        assert [(0 if o.kind == "add" else 1, o.ts if o.kind == "add" else 0, tuple(o.path))
                for o in flatten(log)] == [(k, t, p) for k, t, p, _ in olog]
        assert res["timestamp"] == oracle_summary(ot)["ts"]
        # operationsSince through the addon (src/CRDTree.elm:408-418)
        from parity_util import oracle_since
        for ts in case["since"]:
            got = flatten(decoder(res["since"][str(ts)]))
            want = oracle_since(ot, ts)
            assert [(0 if o.kind == "add" else 1, o.ts if o.kind == "add" else 0, tuple(o.path)) for o in got] == \
                [(k, t, p) for k, t, p, _ in want], ts

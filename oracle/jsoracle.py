"""Driver of the JavaScript restatement (oracle/crdtree.js) — TEST INFRASTRUCTURE.

Used by tests/ (differential check against the C++ restatement) and by
bench.py's cpu_baseline leg (the Elm-compiled-to-JS cost model on the host's
cores). Never imported by the product package.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = os.path.join(_HERE, "crdtree.js")


def node_bin():
    return shutil.which("node")


def _pad(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 8)


def write_batch(path, s, n=None, doc_off=None):
    """Packed batch file (the first n ops of s) read by crdtree.js `readBatch`
    (format documented there)."""
    n = len(s["kind"]) if n is None else n
    kind = np.ascontiguousarray(s["kind"][:n], np.uint8)
    off = np.ascontiguousarray(s["path_off"][:n + 1], np.uint32)
    pth = np.ascontiguousarray(s["path"], np.int64)[: int(off[n])]
    doc = np.array([0, n], np.uint32) if doc_off is None else np.ascontiguousarray(doc_off, np.uint32)
    hdr = b"CRDB" + np.uint32(1).tobytes() + np.array([n, len(pth), len(doc) - 1], np.uint64).tobytes()
    with open(path, "wb") as f:
        f.write(hdr)
        for a in (kind, np.ascontiguousarray(s["ts"][:n], np.int64), off, pth,
                  np.ascontiguousarray(s["val"][:n], np.uint32),
                  doc):
            f.write(_pad(a.tobytes()))


def run(path, mode="chunk", chunk=10000, limit=0, canonical=False, workers=1, timeout=600, heap_mb=0):
    """Run crdtree.js on a packed batch file; returns its JSON summary."""
    nb = node_bin()
    if nb is None:
        raise RuntimeError("node is not installed")
    cmd = [nb]
    if heap_mb:
        cmd.append(f"--max-old-space-size={heap_mb}")
    cmd += [SCRIPT, path, "--mode", mode, "--chunk", str(chunk), "--limit", str(limit), "--workers", str(workers)]
    if canonical:
        cmd.append("--canonical")
    out = subprocess.run(cmd, check=True, capture_output=True, timeout=timeout).stdout
    return json.loads(out.decode().strip().splitlines()[-1])

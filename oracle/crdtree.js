'use strict';
// oracle/crdtree.js
//
// TEST INFRASTRUCTURE ONLY — a second CPU restatement of the Elm reference
// (maca/crdt-replicated-tree 5.0.0), written the way elm/compiler emits Elm
// for JavaScript: persistent red-black `Dict`s (elm/core Dict.insert/get),
// cons-cell `List`s whose `++` copies its left operand (elm/core
// `_Utils_ap`), fresh node records on every update. Its two jobs:
//
//   * the CPU baseline of bench.py (SURVEY.md §8d): the reference is Elm
//     compiled to JS; no Elm compiler exists in this image, so this file is
//     the stand-in, run by `node` on the GPU box's own host cores, with the
//     same cost model (persistent path copies, the O(N^2) `lastOperation`
//     accumulator of `batch`);
//   * a differential oracle: tests/test_js_oracle.py checks it against the
//     C++ restatement (oracle/crdtree_oracle.cpp) on random streams,
//     copy-quirk streams included, through the shared canonical dump hash.
//
// Only tests/ and bench.py's cpu_baseline leg run it; the product path never
// does. Every function cites the Elm source it follows.
//
// CLI:  node oracle/crdtree.js FILE [--mode batch|chunk|op] [--chunk K]
//                            [--limit M] [--canonical] [--workers W]
// FILE is the packed batch written by oracle/jsoracle.py (format below).
// Prints one JSON object on stdout.

const fs = require('fs');
const os = require('os');

// ---------------------------------------------------------------- elm/core Dict
// Red-black tree, persistent (elm/core Dict.elm: insert / insertHelp / balance /
// get). A node is {c: RED|BLACK, k, v, l, r}; the empty dict is null.
const RED = 0, BLACK = 1;

function dictGet(key, d) {
  while (d !== null) {
    if (key < d.k) d = d.l;
    else if (key > d.k) d = d.r;
    else return d.v;
  }
  return undefined;
}

function balance(color, k, v, l, r) {
  if (r !== null && r.c === RED) {
    if (l !== null && l.c === RED) {
      return { c: RED, k, v, l: { c: BLACK, k: l.k, v: l.v, l: l.l, r: l.r }, r: { c: BLACK, k: r.k, v: r.v, l: r.l, r: r.r } };
    }
    return { c: color, k: r.k, v: r.v, l: { c: RED, k, v, l, r: r.l }, r: r.r };
  }
  if (l !== null && l.c === RED && l.l !== null && l.l.c === RED) {
    const ll = l.l;
    return { c: RED, k: l.k, v: l.v, l: { c: BLACK, k: ll.k, v: ll.v, l: ll.l, r: ll.r }, r: { c: BLACK, k, v, l: l.r, r } };
  }
  return { c: color, k, v, l, r };
}

function insertHelp(key, value, d) {
  if (d === null) return { c: RED, k: key, v: value, l: null, r: null };
  if (key < d.k) return balance(d.c, d.k, d.v, insertHelp(key, value, d.l), d.r);
  if (key > d.k) return balance(d.c, d.k, d.v, d.l, insertHelp(key, value, d.r));
  return { c: d.c, k: d.k, v: value, l: d.l, r: d.r };
}

function dictInsert(key, value, d) {
  const t = insertHelp(key, value, d);
  return t.c === RED ? { c: BLACK, k: t.k, v: t.v, l: t.l, r: t.r } : t;
}

function dictFoldl(f, d) {  // ascending keys
  if (d === null) return;
  dictFoldl(f, d.l);
  f(d.k, d.v);
  dictFoldl(f, d.r);
}

// ---------------------------------------------------------------- elm/core List
const NIL = null;
function cons(h, t) { return { h, t }; }
// _Utils_ap on lists: copies xs, shares ys
function append(xs, ys) {
  if (xs === NIL) return ys;
  const root = cons(xs.h, ys);
  let cur = root;
  for (xs = xs.t; xs !== NIL; xs = xs.t) cur = cur.t = cons(xs.h, ys);
  return root;
}
function listFromArray(a, i0, i1) {
  let l = NIL;
  for (let i = i1 - 1; i >= i0; --i) l = cons(a[i], l);
  return l;
}

// ---------------------------------------------------------------- Internal.Node
// type Node a = Root (Children a) | Node a (Children a) (Array Int) (Maybe Int)
//             | Tombstone (Array Int) (Maybe Int)          (src/Internal/Node.elm:29-32)
const ROOT = 0, NODE = 1, TOMB = 2;
// Internal.Node.Error (src/Internal/Node.elm:35-38); results are a Node or one of these
const E_NOTFOUND = 1, E_ALREADY = 2, E_INVALID = 3;

// emptyChildren = Dict.singleton 0 (Tombstone Array.empty Nothing)   (:46-48)
function emptyChildren() { return dictInsert(0, { t: TOMB, p: [], n: null }, null); }
// root (:40-43)
function nodeRoot() { return { t: ROOT, c: emptyChildren() }; }
// children (:231-241)
function children(node) { return node.t === TOMB ? null : node.c; }
// next (:244-254)
function next(node) { return node.t === ROOT ? null : node.n; }
// child ts node = children node |> Dict.get ts   (:284-286)
function child(ts, node) { return dictGet(ts, children(node)); }

// nextNode (:257-268)
function nextNode(node, c) {
  for (;;) {
    const n = next(node);
    if (n === null) return undefined;
    const x = dictGet(n, c);
    if (x === undefined) return undefined;
    if (x.t !== TOMB) return x;
    node = x;
  }
}

// updateNext (:271-281)
function updateNext(n, node) {
  if (node.t === NODE) return { t: NODE, v: node.v, c: node.c, p: node.p, n };
  if (node.t === TOMB) return { t: TOMB, p: node.p, n };
  return node;
}

// insert (:125-135): no-op on a Tombstone parent
function insert(ts, node, parent) {
  if (parent.t === NODE) return { t: NODE, v: parent.v, c: dictInsert(ts, node, parent.c), p: parent.p, n: parent.n };
  if (parent.t === TOMB) return parent;
  return { t: ROOT, c: dictInsert(ts, node, parent.c) };
}

// findInsertion (:93-104): Maybe.map2 Tuple.pair (next node) (nextNode node c);
// returns [leftKey, leftNode] — after a tombstone skip leftKey != key(leftNode)
function findInsertion(ts, n, node, c) {
  for (;;) {
    const k = next(node);
    if (k === null) return [n, node];
    const live = nextNode(node, c);
    if (live === undefined) return [n, node];
    if (ts > k) return [n, node];
    n = k;
    node = live;
  }
}

// addAfterHelp (:56-90). pArr = the op path as an array (Array.fromList p).
function addAfterHelp(pArr, ts, val, prevTs, parent) {
  if (child(ts, parent) !== undefined) return E_ALREADY;
  const found = child(prevTs, parent);
  if (found === undefined) return E_NOTFOUND;
  const lf = findInsertion(ts, prevTs, found, children(parent));
  const leftTs = lf[0], left = lf[1];
  const nodePath = pArr.slice(0, pArr.length - 1);  // Array.slice 0 -1
  nodePath.push(ts);                                 // Array.push ts
  const node = { t: NODE, v: val, c: emptyChildren(), p: nodePath, n: next(left) };
  return insert(ts, node, insert(leftTs, updateNext(ts, left), parent));
}

// deleteHelp (:112-122)
function deleteHelp(key, parent) {
  const c = child(key, parent);
  if (c === undefined) return E_NOTFOUND;
  if (c.t === NODE) return insert(key, { t: TOMB, p: c.p, n: c.n }, parent);
  return E_ALREADY;
}

// update (:138-163): rebuilds every ancestor on the way back (Result.map insert)
function update(func, p, parent) {
  if (parent.t === TOMB) return E_ALREADY;
  if (p === NIL) return E_INVALID;
  if (p.t === NIL) return func(p.h, parent);
  const found = child(p.h, parent);
  if (found === undefined) return E_INVALID;
  const r = update(func, p.t, found);
  if (typeof r === 'number') return r;
  return insert(p.h, r, parent);
}

// ---------------------------------------------------------------- CRDTree
// type Operation a = Add Int (List Int) a | Delete (List Int) | Batch (List ...)
// (src/Internal/Operation.elm:17-20). Ops: {$: 0, ts, p (List), pa (Array), v}
// / {$: 1, p, last} / {$: 2, ops (List)}.
const ADD = 0, DEL = 1, BATCH = 2;
// CRDTree.Error (src/CRDTree.elm:104-107)
const T_OK = 0, T_INVALID_PATH = 1, T_OPERATION_FAILED = 3;

// Timestamp.replicaId ts = ts // 2^32 (src/CRDTree/Timestamp.elm:16-18): Elm `//` is (a / b) | 0
function replicaId(ts) { return (ts / 4294967296) | 0; }

// init (src/CRDTree.elm:130-139)
function init(replica) {
  return { root: nodeRoot(), timestamp: replica * Math.pow(2, 32), cursor: [0], operations: NIL,
           replicas: null, last: { $: BATCH, ops: NIL } };
}

// buildPath (src/CRDTree.elm:628-632)
function buildPath(ts, pArr) {
  const r = pArr.slice(0, pArr.length - 1);
  r.push(ts);
  return r;
}

// updateTree (src/CRDTree.elm:298-325). Returns [code, tree].
function updateTree(op, pArr, ts, rec, result) {
  if (typeof result !== 'number') {
    return [T_OK, { root: result, timestamp: rec.timestamp, cursor: buildPath(ts, pArr),
                    operations: cons(op, rec.operations), replicas: dictInsert(replicaId(ts), ts, rec.replicas),
                    last: op }];
  }
  if (result === E_ALREADY) {
    return [T_OK, { root: rec.root, timestamp: rec.timestamp, cursor: rec.cursor, operations: rec.operations,
                    replicas: rec.replicas, last: { $: BATCH, ops: NIL } }];
  }
  return [result === E_INVALID ? T_INVALID_PATH : T_OPERATION_FAILED, op];
}

// Operation.toList (src/Internal/Operation.elm:58-68) / merge (:80-82)
function toList(op) { return op.$ === BATCH ? op.ops : cons(op, NIL); }
function merge(a, b) { return { $: BATCH, ops: append(toList(a), toList(b)) }; }

// incrementTimestamp (src/CRDTree.elm:337-350)
function incrementTimestamp(ts, t) {
  if (replicaId(ts) !== replicaId(t.timestamp)) return t;
  return { root: t.root, timestamp: t.timestamp + 1, cursor: t.cursor, operations: t.operations,
           replicas: t.replicas, last: t.last };
}

// applyLocal (src/CRDTree.elm:275-295)
function applyLocal(op, t) {
  if (op.$ === ADD) {
    const r = updateTree(op, op.pa, op.ts, t,
                         update((prevTs, parent) => addAfterHelp(op.pa, op.ts, op.v, prevTs, parent), op.p, t.root));
    return r[0] === T_OK ? [T_OK, incrementTimestamp(op.ts, r[1])] : r;
  }
  if (op.$ === DEL) {
    // Operation.timestamp (Delete p) = List.reverse p |> List.head, default 0 (src/Internal/Operation.elm:100-101)
    return updateTree(op, op.pa, op.last, t, update(deleteHelp, op.p, t.root));
  }
  return batch(op.ops, t);
}

// apply (src/CRDTree.elm:265-269): restore the caller's cursor
function apply(op, t) {
  const r = applyLocal(op, t);
  if (r[0] !== T_OK) return r;
  const n = r[1];
  return [T_OK, { root: n.root, timestamp: n.timestamp, cursor: t.cursor, operations: n.operations,
                  replicas: n.replicas, last: n.last }];
}

// batch (src/CRDTree.elm:224-232) with mergeOperations (:328-334): a left fold
// that stops at the first Err; lastOperation = Batch (toList acc ++ toList new)
function batch(ops, t) {
  let acc = { root: t.root, timestamp: t.timestamp, cursor: t.cursor, operations: t.operations,
              replicas: t.replicas, last: { $: BATCH, ops: NIL } };
  for (let l = ops; l !== NIL; l = l.t) {
    const r = apply(l.h, acc);
    if (r[0] !== T_OK) return r;
    const two = r[1];
    acc = { root: two.root, timestamp: two.timestamp, cursor: two.cursor, operations: two.operations,
            replicas: two.replicas, last: merge(acc.last, two.last) };
  }
  return [T_OK, acc];
}

// ---------------------------------------------------------------- canonical dumps
// Same word streams and 64-bit word-wise FNV-1a as orc_canonical
// (oracle/crdtree_oracle.cpp) and crdtm_tree_canonical.
const MASK = (1n << 64n) - 1n, FNV_OFF = 1469598103934665603n, FNV_PRIME = 1099511628211n;
function Sink() { this.h = FNV_OFF; this.n = 0; }
Sink.prototype.put = function (w) {
  this.h = ((this.h ^ BigInt.asUintN(64, BigInt(w))) * FNV_PRIME) & MASK;
  this.n++;
};

function dumpDict(d, depth, s) {
  dictFoldl((key, n) => {
    const hasNext = n.t !== ROOT && n.n !== null;
    s.put(depth); s.put(key); s.put(n.t); s.put(hasNext ? 1 : 0); s.put(hasNext ? n.n : 0);
    s.put(n.t === NODE ? n.v : 0);
    s.put(n.p.length);
    for (const x of n.p) s.put(x);
    if (n.t === NODE) dumpDict(n.c, depth + 1, s);
  }, d);
}

// visible order: Node.foldl from sentinel 0 (src/Internal/Node.elm:206-228), pre-order
function dumpVisible(c, depth, s) {
  let cur = dictGet(0, c);
  if (cur === undefined) return;
  for (;;) {
    const nx = nextNode(cur, c);
    if (nx === undefined) break;
    s.put(depth); s.put(nx.v); s.put(nx.p.length);
    for (const x of nx.p) s.put(x);
    dumpVisible(nx.c, depth + 1, s);
    cur = nx;
  }
}

function listLength(l) { let k = 0; for (; l !== NIL; l = l.t) k++; return k; }

// ---------------------------------------------------------------- packed batch file
// little endian: "CRDB" u32 version | u64 n | u64 path_total | u64 n_docs |
// u8 kind[n] | i64 ts[n] | u32 path_off[n+1] | i64 path[path_total] |
// u32 val[n] | u32 doc_off[n_docs+1]; every array padded to 8 bytes.
function pad8(x) { return (x + 7) & ~7; }
function readBatch(buf) {
  const u8 = new Uint8Array(buf.buffer, buf.byteOffset, buf.byteLength);
  const dv = new DataView(u8.buffer, u8.byteOffset, u8.byteLength);
  if (String.fromCharCode(u8[0], u8[1], u8[2], u8[3]) !== 'CRDB') throw new Error('not a CRDB file');
  const n = Number(dv.getBigUint64(8, true)), pt = Number(dv.getBigUint64(16, true));
  const nd = Number(dv.getBigUint64(24, true));
  let o = 32;
  const slice = (bytes) => { const b = u8.buffer.slice(u8.byteOffset + o, u8.byteOffset + o + bytes); o += pad8(bytes); return b; };
  const kind = new Uint8Array(slice(n));
  const ts = new BigInt64Array(slice(8 * n));
  const pathOff = new Uint32Array(slice(4 * (n + 1)));
  const path = new BigInt64Array(slice(8 * pt));
  const val = new Uint32Array(slice(4 * n));
  const docOff = new Uint32Array(slice(4 * (nd + 1)));
  return { n, kind, ts, pathOff, path, val, nd, docOff };
}

// pre-decode ops [a, b) into Elm values (untimed, like the reference's decoder)
function decodeOps(B, a, b) {
  const ops = new Array(b - a);
  for (let i = a; i < b; ++i) {
    const pa = [];
    for (let j = B.pathOff[i]; j < B.pathOff[i + 1]; ++j) pa.push(Number(B.path[j]));
    const p = listFromArray(pa, 0, pa.length);
    ops[i - a] = B.kind[i] === 0 ? { $: ADD, ts: Number(B.ts[i]), p, pa, v: B.val[i] }
                                 : { $: DEL, p, pa, last: pa.length ? pa[pa.length - 1] : 0 };
  }
  return ops;
}

// apply (Batch ops) in one call (mode "batch"), in Batches of `chunk` ops
// (mode "chunk"), or `apply op` one op at a time (mode "op"): same final tree,
// lastOperation differs. Returns the result
// and the seconds spent inside apply.
function run(ops, mode, chunk) {
  let t = init(0);
  let code = T_OK, done = 0;
  const step = mode === 'batch' ? ops.length : mode === 'op' ? 1 : chunk;
  const lists = [];
  if (mode === 'op') for (const o of ops) lists.push(o);
  else for (let i = 0; i < ops.length; i += step) lists.push({ $: BATCH, ops: listFromArray(ops, i, Math.min(ops.length, i + step)) });
  const t0 = process.hrtime.bigint();
  for (const l of lists) {
    const r = apply(l, t);
    if (r[0] !== T_OK) { code = r[0]; break; }
    t = r[1];
    done += step;
  }
  const sec = Number(process.hrtime.bigint() - t0) / 1e9;
  return { t, code, sec, done: Math.min(done, ops.length) };
}

function summary(t, code, canonical) {
  const out = { code, timestamp: t.timestamp, applied: listLength(t.operations), last_len: listLength(toList(t.last)) };
  const reps = [];
  dictFoldl((k, v) => reps.push([k, v]), t.replicas);
  out.replicas = reps;
  if (canonical) {
    const s0 = new Sink(), s1 = new Sink();
    dumpDict(t.root.c, 0, s0);
    dumpVisible(t.root.c, 0, s1);
    out.struct = [s0.n, s0.h.toString()];
    out.visible = [s1.n, s1.h.toString()];
  }
  return out;
}

function parseArgs(argv) {
  const a = { file: argv[0], mode: 'chunk', chunk: 10000, limit: 0, canonical: false, workers: 1 };
  for (let i = 1; i < argv.length; ++i) {
    const k = argv[i];
    if (k === '--mode') a.mode = argv[++i];
    else if (k === '--chunk') a.chunk = parseInt(argv[++i], 10);
    else if (k === '--limit') a.limit = parseInt(argv[++i], 10);
    else if (k === '--canonical') a.canonical = true;
    else if (k === '--workers') a.workers = parseInt(argv[++i], 10);
    else throw new Error('unknown argument ' + k);
  }
  return a;
}

function env() {
  const cpus = os.cpus();
  return { node: process.version, cpu_model: cpus.length ? cpus[0].model : '?', cpu_count: cpus.length,
           max_old_space_mb: Math.round(require('v8').getHeapStatistics().heap_size_limit / 1048576) };
}

// documents [d0, d1) of B, each applied to its own fresh tree
function runDocs(B, docs, a) {
  const decoded = docs.map((d) => {
    const lo = B.docOff[d], hi = a.limit ? Math.min(B.docOff[d + 1], B.docOff[d] + a.limit) : B.docOff[d + 1];
    return decodeOps(B, lo, hi);
  });
  return decoded;
}

function main() {
  const a = parseArgs(process.argv.slice(2));
  const { Worker } = require('worker_threads');
  if (a.workers <= 1) {
    const B = readBatch(fs.readFileSync(a.file));
    const all = [];
    for (let d = 0; d < B.nd; ++d) all.push(d);
    const decoded = runDocs(B, all, a);
    let sec = 0, ops = 0;
    const docs = [];
    for (const o of decoded) {
      const r = run(o, a.mode, a.chunk);
      sec += r.sec;
      ops += r.done;
      docs.push(summary(r.t, r.code, a.canonical));
    }
    process.stdout.write(JSON.stringify(Object.assign({ ops, seconds: sec, ops_per_s: ops / sec, workers: 1,
                                                        mode: a.mode, chunk: a.chunk, docs }, env())) + '\n');
    return;
  }
  // worker_threads, documents round-robin; the clock runs from "go" to the last "done"
  const buf = fs.readFileSync(a.file);
  const shared = new SharedArrayBuffer(buf.length);
  new Uint8Array(shared).set(buf);
  const nd = readBatch(Buffer.from(shared)).nd;
  const W = Math.max(1, Math.min(a.workers, nd));
  const workers = [];
  let ready = 0, finished = 0, ops = 0, t0 = 0n;
  const docsOut = new Array(nd);
  for (let w = 0; w < W; ++w) {
    const wk = new Worker(__filename, { workerData: { shared, w, W, args: a } });
    wk.on('message', (m) => {
      if (m.kind === 'ready') {
        if (++ready === W) { t0 = process.hrtime.bigint(); for (const x of workers) x.postMessage('go'); }
      } else if (m.kind === 'done') {
        ops += m.ops;
        m.docs.forEach((s, i) => { docsOut[m.ids[i]] = s; });
        if (++finished === W) {
          const sec = Number(process.hrtime.bigint() - t0) / 1e9;
          process.stdout.write(JSON.stringify(Object.assign({ ops, seconds: sec, ops_per_s: ops / sec, workers: W,
                                                              mode: a.mode, chunk: a.chunk, docs: a.canonical ? docsOut : [] },
                                                            env())) + '\n');
          for (const x of workers) x.terminate();
        }
      }
    });
    workers.push(wk);
  }
}

function workerMain() {
  const { parentPort, workerData } = require('worker_threads');
  const { shared, w, W, args } = workerData;
  const B = readBatch(Buffer.from(shared));
  const ids = [];
  for (let d = w; d < B.nd; d += W) ids.push(d);
  const decoded = runDocs(B, ids, args);
  parentPort.once('message', () => {
    let ops = 0;
    const docs = [];
    for (const o of decoded) {
      const r = run(o, args.mode, args.chunk);
      ops += r.done;
      if (args.canonical) docs.push(summary(r.t, r.code, true));
    }
    parentPort.postMessage({ kind: 'done', ops, ids: args.canonical ? ids : [], docs });
  });
  parentPort.postMessage({ kind: 'ready' });
}

if (!require('worker_threads').isMainThread) workerMain();
else if (require.main === module) main();

module.exports = { init, apply, batch, readBatch, decodeOps, run, summary };

'use strict';
// Runs JSON operations through the N-API addon (the Elm-ports host path) and
// prints what the Elm side would see; driven by tests/test_napi.py.
//   node tests/napi_run.js <in.json> <out.json>
// in: [{replica, calls: [jsonText, ...], since: [ts, ...]}, ...]
const fs = require('fs');
const path = require('path');
const { Tree } = require(path.join(__dirname, '..', 'crdt-graph_amd', 'napi', 'crdtm.js'));

async function main() {
  const cases = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
  const out = [];
  for (const c of cases) {
    const t = new Tree(c.replica);
    const results = [];
    if (c.queued) {
      // every apply queued before any is awaited: they must run in call order
      const rs = await Promise.all(c.calls.map((j) => t.apply(j)));
      for (const r of rs) results.push({ code: r.code, errIndex: r.errIndex, lastOperation: r.lastOperation });
    } else {
      for (let k = 0; k < c.calls.length; ++k) {
        // alternate the Promise path (off the event loop) and the synchronous one
        const r = k % 2 === 0 ? await t.apply(c.calls[k]) : t.applySync(c.calls[k]);
        results.push({ code: r.code, errIndex: r.errIndex, lastOperation: r.lastOperation });
      }
    }
    // the bytes Elm's encoder would produce for the oracle's lastOperation:
    // Encode.encode 0 = JSON.stringify, object keys in encoder order
    // (src/CRDTree/Operation.elm:109-130)
    const enc = (o) => (o[0] === 0 ? JSON.stringify({ op: 'add', path: o[2], ts: o[1], val: o[3] })
                                    : JSON.stringify({ op: 'del', path: o[2] }));
    const expectLast = (c.expectLast || []).map((e) => (e === null ? null
      : e.isBatch ? '{"op":"batch","ops":[' + e.ops.map(enc).join(',') + ']}' : enc(e.ops[0])));
    const since = {};
    for (const ts of c.since || []) since[ts] = require('../crdt-graph_amd/napi/crdtm.js').addon.operationsSince(t.h, ts);
    out.push({
      results,
      expectLast,
      log: require('../crdt-graph_amd/napi/crdtm.js').addon.operationsSince(t.h, 0),
      since,
      document: require('../crdt-graph_amd/napi/crdtm.js').addon.document(t.h),
      timestamp: t.timestamp(),
    });
    t.release();
  }
  fs.writeFileSync(process.argv[3], JSON.stringify(out));
}

main().catch((e) => {
  console.error(e);
  process.exit(1);
});

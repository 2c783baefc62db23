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
    for (let k = 0; k < c.calls.length; ++k) {
      // alternate the Promise path (off the event loop) and the synchronous one
      const r = k % 2 === 0 ? await t.apply(c.calls[k]) : t.applySync(c.calls[k]);
      results.push({ code: r.code, errIndex: r.errIndex, lastOperation: r.lastOperation });
    }
    const since = {};
    for (const ts of c.since || []) since[ts] = require('../crdt-graph_amd/napi/crdtm.js').addon.operationsSince(t.h, ts);
    out.push({
      results,
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

'use strict';
// JS side of the Elm-ports host path (INTEGRATION.md §2-3): wraps the N-API
// addon and binds an Elm application's ports to it.
//
//   port mergeRequest : Json.Encode.Value -> Cmd msg       -- CRDTree.Operation.encoder output
//   port mergeResult  : (Json.Decode.Value -> msg) -> Sub msg
//
// The reply carries {code, errIndex, lastOperation}; lastOperation decodes
// with CRDTree.Operation.decoder exactly like a remote op (code 0 = Ok,
// 1 = InvalidPath, 3 = OperationFailed (op errIndex of the flattened batch)).
const addon = require('./crdtm.node');

class Tree {
  constructor(replicaId) {
    this.h = addon.init(replicaId);
  }
  // op: an encoded Operation (JS value) or its JSON text
  apply(op) {
    return addon.apply(this.h, typeof op === 'string' ? op : JSON.stringify(op));
  }
  applySync(op) {
    return addon.applySync(this.h, typeof op === 'string' ? op : JSON.stringify(op));
  }
  operationsSince(ts) { return JSON.parse(addon.operationsSince(this.h, ts)); }
  lastOperation() { return JSON.parse(addon.lastOperation(this.h)); }
  timestamp() { return addon.timestamp(this.h); }
  lastReplicaTimestamp(rid) { return addon.lastReplicaTimestamp(this.h, rid); }
  document() { return JSON.parse(addon.document(this.h)); }
  release() { addon.release(this.h); }
}

function bindPorts(app, tree) {
  app.ports.mergeRequest.subscribe(async (opValue) => {
    const r = await tree.apply(opValue);
    app.ports.mergeResult.send({
      code: r.code,
      errIndex: r.errIndex,
      lastOperation: r.lastOperation === null ? null : JSON.parse(r.lastOperation),
    });
  });
}

module.exports = { Tree, bindPorts, addon };

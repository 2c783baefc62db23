/*
 * crdtm.h — C ABI of the MI355X-native CRDTree batch-merge engine.
 *
 * Drop-in boundary for the reference's operation-apply path
 * (maca/crdt-replicated-tree 5.0.0). Elm has no FFI; the reference-side
 * binding is an application port -> Node N-API addon -> this ABI (see
 * INTEGRATION.md). Every entry point below names the reference interface it
 * replaces. All pointers are plain C; no torch or HIP types cross the ABI
 * (streams are passed as opaque `void*`).
 *
 * Numbers: Elm `Int` runs on JS doubles, so timestamps and path elements must
 * satisfy |x| < 2^53; crdtm_apply rejects other
 * inputs with CRDTM_E_RANGE.
 */
#ifndef CRDTM_H
#define CRDTM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- op kinds: Operation a = Add Int (List Int) a | Delete (List Int)
 *      (src/Internal/Operation.elm:17-20). Batch is expressed by the
 *      is_batch flag of crdtm_apply plus flattening (nested Batches apply
 *      exactly like their flattened leaves, src/CRDTree.elm:224-232, :294-295). */
#define CRDTM_ADD 0
#define CRDTM_DELETE 1

/* ---- return codes: CRDTree.Error a = InvalidPath | NotFound | OperationFailed op
 *      (src/CRDTree.elm:104-107). Negative values are engine errors. */
#define CRDTM_OK 0
#define CRDTM_INVALID_PATH 1
#define CRDTM_NOT_FOUND 2 /* reserved: produced only by setCursor, not on this path */
#define CRDTM_OPERATION_FAILED 3
#define CRDTM_E_ARG (-1)
#define CRDTM_E_HIP (-2)
#define CRDTM_E_NOMEM (-3)
#define CRDTM_E_RANGE (-4)
#define CRDTM_E_NODEVICE (-5)
#define CRDTM_E_PARSE (-6)
#define CRDTM_E_STATE (-7) /* crdtm_tree_canonical found the state unsound: an index out of range, a reached
                              dict without a sentinel, a cyclic chain or a children dict reached twice */

/* ---- per-op status (updateTree, src/CRDTree.elm:298-325) */
#define CRDTM_ST_APPLIED 0 /* Ok: logged, lastOperation, replicas */
#define CRDTM_ST_ALREADY 1 /* Err AlreadyApplied -> Ok, nothing logged */
#define CRDTM_ST_ERROR 2   /* the first failing op (err_index) */
#define CRDTM_ST_UNREACHED 3

/* ---- which merge path served a call */
#define CRDTM_PATH_CLOSED_FORM 1 /* parallel closed form, guard held */
#define CRDTM_PATH_REPLAY 2      /* exact sequential replay on the GPU */
#define CRDTM_PATH_DICT_REPLAY 3 /* exact replay, one lane per children dict */

/* Packed op batch, structure of arrays (host or device memory; see crdtm_apply). */
typedef struct crdtm_ops {
  uint64_t n_ops;
  uint64_t n_path;    /* total path elements = path_off[n_ops] */
  uint8_t *kind;      /* [n_ops] CRDTM_ADD / CRDTM_DELETE */
  int64_t *ts;        /* [n_ops] Add timestamp (ignored for Delete) */
  uint32_t *path_off; /* [n_ops+1] CSR offsets into path */
  int64_t *path;      /* [n_path] */
  uint32_t *val;      /* [n_ops] value handle into a caller-owned value table */
  uint32_t *tree;     /* [n_ops] document id (forest calls), or NULL */
} crdtm_ops;

typedef struct crdtm_result {
  int32_t code;       /* CRDTM_OK / CRDTM_INVALID_PATH / CRDTM_OPERATION_FAILED / <0 */
  int32_t path_taken; /* CRDTM_PATH_* */
  int64_t err_index;  /* first failing op (flattened order), -1 if none */
  uint64_t n_applied;
  uint64_t n_already;
  int64_t timestamp;  /* tree timestamp after the call */
  uint64_t n_slots;   /* slots held by the device state (empty children dicts are implicit) */
  uint32_t guard;     /* bit0 ts collision, bit1 delete-before-add in a dict, bit2 replica-id drift, bit3 non-fresh tree,
                         bit4 path deeper than 64, bit5 sequential replay forced (env CRDTM_FORCE_REPLAY=1) */
  uint32_t flags;     /* CRDTM_FLAG_* */
  /* serial-work accounting: ops and dicts that went through an
   * exact in-order replay (one wave per dict, or one lane for the whole batch),
   * and the op count of the largest such replay (the merge's serial critical path) */
  uint64_t serial_ops;
  uint64_t serial_dicts;
  uint64_t serial_max;
} crdtm_result;

/* crdtm_result.flags */
#define CRDTM_FLAG_REMERGE 1 /* non-fresh tree: merged as init ++ log ++ batch on the parallel paths */
#define CRDTM_FLAG_INCREMENTAL 2 /* non-fresh flat tree, adds-only batch: merged into the document in place
                                    (incremental closed form, gaps of the base order; incr.hip) */
#define CRDTM_FLAG_INCR_WINDOWS 4 /* with INCREMENTAL: blocks of the gapped order were spread over windows */
#define CRDTM_FLAG_INCR_DENSE 8   /* with INCREMENTAL: no window could take the batch: dense merge, rebuilt */
#define CRDTM_FLAG_DICT_INCR 16   /* non-fresh tree: the batch replayed per children dict on the state itself,
                                     level by level (only the dicts it reaches; ilr.hip) */
#define CRDTM_FLAG_INCR_TOUR 32   /* with INCREMENTAL: some gap's new nodes were ordered as their tree's DFS
                                     (keys growing along its anchors) instead of replayed one by one */

typedef struct crdtm_ctx crdtm_ctx;   /* device + stream + workspace */
typedef struct crdtm_tree crdtm_tree; /* one replica's CRDTree state, resident in HBM */

/* ---- context ---- */
int crdtm_version(void);
int crdtm_device_count(int *count);
/* stream: an existing hipStream_t (as void*) to launch on, or NULL for an engine-owned stream.
 * Device inputs produced on another stream must be complete before crdtm_apply /
 * crdtm_forest_apply is called (synchronise, or create the context on that stream;
 * note that the legacy default stream's handle is NULL, i.e. "engine-owned"). */
int crdtm_ctx_create(int device, void *stream, crdtm_ctx **out);
int crdtm_ctx_destroy(crdtm_ctx *ctx);
void *crdtm_ctx_stream(crdtm_ctx *ctx);
int crdtm_ctx_sync(crdtm_ctx *ctx);

/* ---- tree state ---- */
/* CRDTree.init replicaId (src/CRDTree.elm:130-139) */
int crdtm_tree_create(crdtm_ctx *ctx, int64_t replica_id, crdtm_tree **out);
int crdtm_tree_destroy(crdtm_tree *t);
/* Reset to `init replica_id` keeping the device allocations (benchmarks, pooling). */
int crdtm_tree_reset(crdtm_tree *t, int64_t replica_id);
/* Elm values are persistent (src/CRDTree.elm:228-232): clone before apply to keep
 * the old version. O(1): the versions share the device state until one of them
 * is written (apply / reset), which then takes a private copy (copy on write).
 * Handles of one context are not used concurrently (see Threading). */
int crdtm_tree_clone(const crdtm_tree *t, crdtm_tree **out);

/* CRDTree.apply (src/CRDTree.elm:265-269): apply (Batch ops) when is_batch,
 * else the single op ops[0]. Sequential-apply semantics in array order; the
 * first failing op aborts and leaves the tree unchanged (transactional).
 * Any tree, fresh or not: a tree that holds state takes the ops in place
 * (a flat document: res->flags & CRDTM_FLAG_INCREMENTAL; per children dict
 * on the state: CRDTM_FLAG_DICT_INCR), or merges log ++ ops on the parallel
 * paths (CRDTM_FLAG_REMERGE) or, when a sequential path is needed, replays
 * ops on the existing state.
 * ops_on_device: 1 if every array of `ops` is device memory (inputs already
 * resident in HBM), 0 for host memory (copied in on the context stream).
 * status_out: optional device (ops_on_device) or host array [n_ops] of CRDTM_ST_*.
 * Asynchronous w.r.t. the host only in the sense that the result struct is
 * filled after a stream synchronisation at the end of the call. */
int crdtm_apply(crdtm_tree *t, const crdtm_ops *ops, int ops_on_device, int is_batch, uint8_t *status_out,
                crdtm_result *res);

/* ---- merge outputs (src/CRDTree.elm:353-418, :635-639) ---- */
int crdtm_tree_timestamp(const crdtm_tree *t, int64_t *out);          /* CRDTree.timestamp */
/* replicas Dict (lastReplicaTimestamp): ascending replica ids. Returns count via *n;
 * fills up to cap entries when ids/tss are non-NULL. */
int crdtm_tree_replicas(const crdtm_tree *t, int64_t *ids, int64_t *tss, uint64_t cap, uint64_t *n);
/* Operation log oldest-first (operationsSince 0) when which == 0; lastOperation's
 * op list when which == 1 (*is_batch = 0 means lastOperation is that single op).
 * Host arrays; call with NULL arrays to size (n_ops, n_path). */
int crdtm_tree_ops(const crdtm_tree *t, int which, crdtm_ops *out, int *is_batch);
/* operationsSince ts (src/CRDTree.elm:408-418 -> since, src/Internal/Operation.elm:25-53):
 * the log oldest-first from the newest logged Add whose ts == ts (inclusive) to the end;
 * no such Add -> no ops; ts == 0 -> the whole log. The search runs on the device.
 * Host arrays; NULL arrays to size, like crdtm_tree_ops. */
int crdtm_tree_ops_since(const crdtm_tree *t, int64_t ts, crdtm_ops *out);

/* ---- traversal (CRDTree.get/parent/next/prev/walk, src/CRDTree.elm:421-625;
 *      CRDTree.Node.children/head, src/CRDTree/Node.elm:96-174). get,
 *      node_info, relative and node_children run on the device (one small
 *      kernel per query over the state's own arrays and a (dict, key) -> slot
 *      index built once per tree version); only the answer is copied back.
 *      walk, whose output is document-sized, reads a host copy of the state
 *      taken once per version. A node reference is valid until the next
 *      apply/reset of the tree. */
#define CRDTM_REF_NONE UINT64_MAX                 /* Nothing */
#define CRDTM_REF_ROOT (UINT64_MAX - 1)           /* the Root node */
#define CRDTM_REF_VSENT (1ULL << 62)              /* | slot: sentinel of a live node's empty children */
#define CRDTM_REL_PARENT 0
#define CRDTM_REL_NEXT 1
#define CRDTM_REL_PREV 2
#define CRDTM_REL_HEAD 3
/* get path tree (Node.descendant from the root): *ref = node or CRDTM_REF_NONE. */
int crdtm_tree_get(const crdtm_tree *t, const int64_t *path, uint64_t len, uint64_t *ref);
/* kind 1 Node, 2 Tombstone, 3 Root; value handle (Node); next key; Node.path (up to cap words). */
int crdtm_node_info(const crdtm_tree *t, uint64_t ref, int32_t *kind, uint32_t *val, int32_t *has_next,
                    int64_t *next, int64_t *path, uint64_t cap, uint64_t *path_len);
/* parent / next / prev (src/CRDTree.elm:425-441, :560-575) and Node.head: *out or CRDTM_REF_NONE. */
int crdtm_tree_relative(const crdtm_tree *t, uint64_t ref, int which, uint64_t *out);
/* CRDTree.Node.children: the live children in chain order (head = first, last = last). */
int crdtm_node_children(const crdtm_tree *t, uint64_t ref, uint64_t *out, uint64_t cap, uint64_t *n);
/* The nodes CRDTree.walk visits, in order, when its function always Takes
 * (start = CRDTM_REF_NONE: walk ... Nothing); a walk that stops with Done
 * visits a prefix of this order. */
int crdtm_tree_walk(const crdtm_tree *t, uint64_t start, uint64_t *out, uint64_t cap, uint64_t *n);

/* Canonical dumps shared with the oracle: which 0 = every dict entry (structure),
 * 1 = visible document order. Writes up to cap words (out may be NULL), the
 * word count and a 64-bit word-wise FNV-1a hash of the words (h ^= w; h *= 0x100000001b3
 * per 64-bit word, from 0xcbf29ce484222325). Host-side read API. */
int crdtm_tree_canonical(const crdtm_tree *t, int which, int64_t *out, uint64_t cap, uint64_t *n_words,
                         uint64_t *hash);

/* Document order (north star kernel 4): for every visible node, its value handle
 * in document order (pre-order over live nodes). Device linearisation; host copy. */
int crdtm_tree_document(const crdtm_tree *t, uint32_t *vals, uint64_t cap, uint64_t *n_visible);

/* ---- forest: many independent documents in one call (config 5) ----
 * ops grouped by document, application order within a document; doc_off
 * [n_docs+1] is a host CSR over ops (ops in device memory when on_device).
 * Every document starts as `init replica_id` and takes `apply (Batch ops_d)`
 * with the exact sequential semantics. Per-document host outputs (any may be
 * NULL except doc_code): CRDTree.Error code, local err index (-1), applied
 * count, word-wise FNV-1a hash + word count of the visible-document canonical dump
 * (same words as crdtm_tree_canonical(which = 1)), final timestamp.
 * Replaces: CRDTree.apply (src/CRDTree.elm:265-269) over many trees. */
int crdtm_forest_apply(crdtm_ctx *ctx, int64_t replica_id, const crdtm_ops *ops, const uint32_t *doc_off,
                       uint64_t n_docs, int on_device, int32_t *doc_code, int64_t *doc_err, uint32_t *doc_applied,
                       uint64_t *doc_hash, uint64_t *doc_words, int64_t *doc_timestamp);

/* ---- sharding glue (config 5): records [doc << 32 | seq, kind << 32 | val, ts, anchor]
 * (int64 x 4, device, 16-byte aligned) of every replica -> the packed ops of the
 * documents this rank owns (t mod world == rank), document t at
 * [(t / world) * per_doc, ...) in causal order. out: device arrays of
 * out->n_ops (+1 for path_off) entries; records of other ranks are skipped. */
int crdtm_shard_assemble(crdtm_ctx *ctx, const int64_t *records, uint64_t n_rec, int32_t rank, int32_t world,
                         uint64_t per_doc, crdtm_ops *out);

/* ---- synthetic op streams ---- */
typedef struct crdtm_synth_params {
  uint64_t n_ops;       /* per document */
  uint64_t n_docs;      /* 1 for single-tree configs */
  uint32_t replicas;    /* remote replicas 1..R */
  uint32_t window;      /* view lag W */
  double p_delete;      /* fraction of Deletes */
  double p_branch;      /* addBranch probability (nested configs) */
  double p_continue;    /* typing: anchor after own last node */
  uint32_t max_depth;   /* 1 = flat */
  uint32_t max_children;/* 0 = unbounded (deep-tree config uses 8) */
  uint32_t deletes_last;/* 1: all Deletes after all Adds (config 4) */
  uint64_t seed;
  uint64_t doc_base;    /* forest: id of the first generated document (streams depend on seed and id) */
} crdtm_synth_params;
/* Generates host arrays owned by the engine; free with crdtm_ops_free. */
int crdtm_synth(const crdtm_synth_params *p, crdtm_ops **out);
int crdtm_ops_free(crdtm_ops *ops);

/* ---- wire format: CRDTree.Operation encoder/decoder (src/CRDTree/Operation.elm:109-159) ----
 * Decode one JSON operation (Add/Delete/Batch, nested) into flattened host ops.
 * Values are kept as canonical JSON text (JSON.stringify form) in a value
 * table: handle h -> bytes [val_off[h], val_off[h+1]) of *val_bytes.
 * *is_batch reports whether the top-level op was a Batch (unknown "op" -> Batch []). */
int crdtm_json_decode(const char *json, size_t len, crdtm_ops **ops, char **val_bytes, uint64_t **val_off,
                      uint64_t *n_vals, int *is_batch);
/* Encode ops (is_batch: as {"op":"batch","ops":[...]}, else ops[0]) byte-identically
 * to `Encode.encode 0 (encoder valueEncoder op)`; values from the value table. */
int crdtm_json_encode(const crdtm_ops *ops, int is_batch, const char *val_bytes, const uint64_t *val_off,
                      char **out, size_t *out_len);
/* JSON.stringify(JSON.parse(text)) for one value: the canonical text the
 * decoder stores in the value table (Decode.value / Encode.value round trip). */
int crdtm_json_canonical(const char *text, size_t len, char **out, size_t *out_len);
void crdtm_free(void *p);

/* ---- guard G on the per-dict replay: measured when the
 * environment variable CRDTM_GUARD_STATS=1 is set during crdtm_apply (an
 * untimed measurement run; it adds a few instructions per replayed Add).
 * An Add fails guard G when its findInsertion walk (src/Internal/Node.elm:
 * 93-104) meets a Tombstone whose key is above the Add's timestamp: a node
 * canonical RGA would pass, deleted before the Add; a dict's first such Add
 * ends the prefix a closed form could serve exactly. out[0] Adds that walked,
 * out[1] G-failing Adds, out[2] ops of the replayed dicts before each dict's
 * first G-failing Add, out[3] ops the replayed dicts reached (ops that
 * stopped at a Tombstone on their path, or no dict, are not counted). Returns 1 when the last apply of
 * this context collected them, else 0 (out zeroed). */
int crdtm_ctx_guard_stats(crdtm_ctx *ctx, uint64_t *out);

/* ---- profiling: per-kernel device time of the last apply (HIP events) ---- */
/* Returns the number of named phases; fills names (NUL-separated) and ms. */
int crdtm_ctx_profile(crdtm_ctx *ctx, int enable);
int crdtm_ctx_phase_times(crdtm_ctx *ctx, char *names, size_t names_cap, double *ms, int cap);

#ifdef __cplusplus
}
#endif
#endif /* CRDTM_H */

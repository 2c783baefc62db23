/* crdtm_napi.c — Node N-API addon: the Elm-ports host path of the merge engine.
 *
 * Elm has no FFI and packages cannot declare ports, so an
 * application routes CRDTree.apply through `port mergeRequest` -> this addon
 * -> libcrdtm.so (C ABI, include/crdtm.h) -> HIP (gfx950). Everything here is
 * marshalling: JSON text in (the reference's wire format,
 * src/CRDTree/Operation.elm:109-159), JSON text out; all semantics live
 * behind the C ABI. Values stay canonical JSON text in a per-tree value table,
 * so the lastOperation / operationsSince JSON is byte-identical to
 * `Encode.encode 0 (encoder valueEncoder op)`.
 *
 * Exports (see crdtm.js for the JS-side wrapper and the port binding):
 *   init(replicaId)                 -> tree handle        CRDTree.init (src/CRDTree.elm:130-139)
 *   apply(tree, json)               -> Promise<result>    CRDTree.apply (src/CRDTree.elm:265-269), off the event loop
 *   applySync(tree, json)           -> result
 *   operationsSince(tree, ts)       -> json               CRDTree.operationsSince (src/CRDTree.elm:408-418)
 *   lastOperation(tree)             -> json               CRDTree.lastOperation (src/CRDTree.elm:371-373)
 *   timestamp(tree)                 -> number             CRDTree.timestamp (src/CRDTree.elm:385-387)
 *   lastReplicaTimestamp(tree, rid) -> number             src/CRDTree.elm:637-639
 *   document(tree)                  -> json array         visible values in document order
 *   release(tree)
 * result = {code, errIndex, applied, already, timestamp, path, lastOperation}
 * (code 0 = Ok, 1 = InvalidPath, 3 = OperationFailed at op errIndex of the
 * flattened batch). No CPU fallback: without a GPU, init throws E_NODEVICE.
 */
#include <node_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crdtm.h"

struct job;

typedef struct {
  crdtm_tree *t;
  char *vb;          /* value bytes (canonical JSON texts, concatenated) */
  uint64_t vb_len, vb_cap;
  uint64_t *vo;      /* handle h -> [vo[h], vo[h+1]) */
  uint64_t nv, vo_cap;
  /* async applies of this tree run one at a time in call order (the
   * reference's applies are sequential): a FIFO touched only on the JS thread */
  struct job *qhead, *qtail;
  int busy;
} tree_h;

static crdtm_ctx *g_ctx = NULL;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER; /* one merge at a time: the context's stream and workspace */

static const char *code_name(int rc) {
  switch (rc) {
    case CRDTM_E_ARG: return "E_ARG";
    case CRDTM_E_HIP: return "E_HIP";
    case CRDTM_E_NOMEM: return "E_NOMEM";
    case CRDTM_E_RANGE: return "E_RANGE";
    case CRDTM_E_NODEVICE: return "E_NODEVICE";
    case CRDTM_E_PARSE: return "E_PARSE";
    default: return "E_UNKNOWN";
  }
}

static napi_value throw_rc(napi_env env, const char *what, int rc) {
  char msg[128];
  snprintf(msg, sizeof msg, "crdtm: %s failed: %s", what, code_name(rc));
  napi_throw_error(env, code_name(rc), msg);
  return NULL;
}

/* ---- value table ---- */
static int vt_reserve(tree_h *h, uint64_t more_bytes, uint64_t more_vals) {
  if (h->vb_len + more_bytes > h->vb_cap) {
    uint64_t c = h->vb_cap ? h->vb_cap : 4096;
    while (c < h->vb_len + more_bytes) c *= 2;
    char *p = realloc(h->vb, c);
    if (!p) return CRDTM_E_NOMEM;
    h->vb = p;
    h->vb_cap = c;
  }
  if (h->nv + more_vals + 1 > h->vo_cap) {
    uint64_t c = h->vo_cap ? h->vo_cap : 1024;
    while (c < h->nv + more_vals + 1) c *= 2;
    uint64_t *p = realloc(h->vo, c * sizeof(uint64_t));
    if (!p) return CRDTM_E_NOMEM;
    h->vo = p;
    h->vo_cap = c;
  }
  return CRDTM_OK;
}

/* ---- one merge: decode, remap value handles into the tree's table, apply,
 *      encode lastOperation ---- */
typedef struct job {
  tree_h *h;
  napi_ref tree_ref; /* async: keeps the tree external alive until the job is done */
  struct job *next;  /* the tree's FIFO */
  char *json;
  size_t len;
  int rc;            /* engine error (< 0) */
  crdtm_result res;
  char *last;        /* lastOperation JSON on success */
  size_t last_len;
  napi_async_work work;
  napi_deferred def;
} job;
typedef job job_t;

static int encode_log(tree_h *h, int which, int64_t since, int use_since, char **out, size_t *out_len) {
  crdtm_ops o;
  memset(&o, 0, sizeof o);
  int isb = 1;
  int rc = use_since ? crdtm_tree_ops_since(h->t, since, &o) : crdtm_tree_ops(h->t, which, &o, &isb);
  if (rc) return rc;
  const uint64_t n = o.n_ops, np = o.n_path;
  o.kind = malloc(n + 1);
  o.ts = malloc((n + 1) * sizeof(int64_t));
  o.path_off = malloc((n + 1) * sizeof(uint32_t));
  o.path = malloc((np + 1) * sizeof(int64_t));
  o.val = malloc((n + 1) * sizeof(uint32_t));
  o.tree = NULL;
  if (!o.kind || !o.ts || !o.path_off || !o.path || !o.val) rc = CRDTM_E_NOMEM;
  if (!rc) rc = use_since ? crdtm_tree_ops_since(h->t, since, &o) : crdtm_tree_ops(h->t, which, &o, &isb);
  if (!rc) rc = crdtm_json_encode(&o, use_since ? 1 : isb, h->vb, h->vo, out, out_len);
  free(o.kind);
  free(o.ts);
  free(o.path_off);
  free(o.path);
  free(o.val);
  return rc;
}

static void run_merge(job_t *j) {
  tree_h *h = j->h;
  crdtm_ops *ops = NULL;
  char *vals = NULL;
  uint64_t *voff = NULL, nv = 0;
  int is_batch = 0;
  pthread_mutex_lock(&g_mu);
  j->rc = crdtm_json_decode(j->json, j->len, &ops, &vals, &voff, &nv, &is_batch);
  if (!j->rc) j->rc = vt_reserve(h, voff[nv], nv);
  if (!j->rc) {
    const uint64_t base = h->nv;
    memcpy(h->vb + h->vb_len, vals, voff[nv]);
    for (uint64_t k = 0; k < nv; ++k) h->vo[base + k] = h->vb_len + voff[k];
    h->vb_len += voff[nv];
    h->nv += nv;
    h->vo[h->nv] = h->vb_len;
    for (uint64_t i = 0; i < ops->n_ops; ++i)
      if (ops->kind[i] == CRDTM_ADD) ops->val[i] += (uint32_t)base;
    j->rc = crdtm_apply(h->t, ops, 0, is_batch, NULL, &j->res);
  }
  if (!j->rc && j->res.code == CRDTM_OK) j->rc = encode_log(h, 1, 0, 0, &j->last, &j->last_len);
  pthread_mutex_unlock(&g_mu);
  crdtm_ops_free(ops);
  crdtm_free(vals);
  crdtm_free(voff);
}

static napi_value result_object(napi_env env, job_t *j) {
  napi_value o, v;
  napi_create_object(env, &o);
  napi_create_int32(env, j->res.code, &v);
  napi_set_named_property(env, o, "code", v);
  napi_create_int64(env, j->res.err_index, &v);
  napi_set_named_property(env, o, "errIndex", v);
  napi_create_int64(env, (int64_t)j->res.n_applied, &v);
  napi_set_named_property(env, o, "applied", v);
  napi_create_int64(env, (int64_t)j->res.n_already, &v);
  napi_set_named_property(env, o, "already", v);
  napi_create_int64(env, j->res.timestamp, &v);
  napi_set_named_property(env, o, "timestamp", v);
  napi_create_int32(env, j->res.path_taken, &v);
  napi_set_named_property(env, o, "path", v);
  if (j->last) napi_create_string_utf8(env, j->last, j->last_len, &v);
  else napi_get_null(env, &v);
  napi_set_named_property(env, o, "lastOperation", v);
  return o;
}

static void job_free(job_t *j) {
  crdtm_free(j->last);
  free(j->json);
  free(j);
}

/* ---- argument helpers ---- */
static tree_h *get_tree(napi_env env, napi_value v) {
  void *p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p || !((tree_h *)p)->t) {
    napi_throw_type_error(env, "E_ARG", "crdtm: not a live tree handle");
    return NULL;
  }
  return (tree_h *)p;
}

static char *get_string(napi_env env, napi_value v, size_t *len) {
  size_t n = 0;
  if (napi_get_value_string_utf8(env, v, NULL, 0, &n) != napi_ok) {
    napi_throw_type_error(env, "E_ARG", "crdtm: expected a JSON string");
    return NULL;
  }
  char *s = malloc(n + 1);
  if (!s) return NULL;
  napi_get_value_string_utf8(env, v, s, n + 1, &n);
  *len = n;
  return s;
}

static napi_value ret_string(napi_env env, char *s, size_t n) {
  napi_value v;
  napi_create_string_utf8(env, s, n, &v);
  crdtm_free(s);
  return v;
}

static void tree_finalize(napi_env env, void *data, void *hint) {
  (void)env;
  (void)hint;
  tree_h *h = data;
  /* (no job can be in flight: every queued job holds a reference to the external) */
  pthread_mutex_lock(&g_mu);
  if (h->t) crdtm_tree_destroy(h->t);
  h->t = NULL;
  pthread_mutex_unlock(&g_mu);
  free(h->vb);
  free(h->vo);
  free(h);
}

/* ---- exports ---- */
static napi_value js_init(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  int64_t rid = 0;
  if (argc > 0) napi_get_value_int64(env, argv[0], &rid);
  pthread_mutex_lock(&g_mu);
  int rc = g_ctx ? CRDTM_OK : crdtm_ctx_create(0, NULL, &g_ctx);
  tree_h *h = NULL;
  if (!rc) {
    h = calloc(1, sizeof *h);
    rc = h ? crdtm_tree_create(g_ctx, rid, &h->t) : CRDTM_E_NOMEM;
  }
  if (!rc) rc = vt_reserve(h, 0, 0);
  if (!rc) h->vo[0] = 0;
  pthread_mutex_unlock(&g_mu);
  if (rc) {
    if (h) tree_finalize(env, h, NULL);
    return throw_rc(env, "init", rc);
  }
  napi_value out;
  napi_create_external(env, h, tree_finalize, NULL, &out);
  return out;
}

static job_t *make_job(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  if (argc < 2) {
    napi_throw_type_error(env, "E_ARG", "crdtm: apply(tree, json)");
    return NULL;
  }
  tree_h *h = get_tree(env, argv[0]);
  if (!h) return NULL;
  job_t *j = calloc(1, sizeof *j);
  j->h = h;
  j->json = get_string(env, argv[1], &j->len);
  if (!j->json) {
    free(j);
    return NULL;
  }
  return j;
}

static napi_value js_apply_sync(napi_env env, napi_callback_info info) {
  job_t *j = make_job(env, info);
  if (!j) return NULL;
  if (j->h->busy) {  /* would overtake queued async applies of this tree */
    job_free(j);
    napi_throw_error(env, "E_BUSY", "crdtm: applySync while async applies of this tree are pending");
    return NULL;
  }
  run_merge(j);
  if (j->rc) {
    const int rc = j->rc;
    job_free(j);
    return throw_rc(env, "apply", rc);
  }
  napi_value o = result_object(env, j);
  job_free(j);
  return o;
}

static void async_exec(napi_env env, void *data) {
  (void)env;
  run_merge(data);
}

static void start_next(napi_env env, tree_h *h);

static void async_done(napi_env env, napi_status status, void *data) {
  job_t *j = data;
  tree_h *h = j->h;
  if (status != napi_ok || j->rc) {
    napi_value err, msg;
    char m[128];
    snprintf(m, sizeof m, "crdtm: apply failed: %s", code_name(j->rc ? j->rc : CRDTM_E_ARG));
    napi_create_string_utf8(env, m, NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, j->def, err);
  } else {
    napi_resolve_deferred(env, j->def, result_object(env, j));
  }
  napi_delete_async_work(env, j->work);
  napi_ref ref = j->tree_ref;
  job_free(j);
  h->busy = 0;
  start_next(env, h);          /* the next queued apply of this tree, if any */
  napi_delete_reference(env, ref);  /* (last: may let the tree be collected) */
}

/* Queue the tree's oldest pending job on the libuv pool (JS thread only). */
static void start_next(napi_env env, tree_h *h) {
  if (h->busy || !h->qhead) return;
  job_t *j = h->qhead;
  h->qhead = j->next;
  if (!h->qhead) h->qtail = NULL;
  h->busy = 1;
  napi_queue_async_work(env, j->work);
}

static napi_value js_apply(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  job_t *j = make_job(env, info);
  if (!j) return NULL;
  napi_value promise, name;
  napi_create_reference(env, argv[0], 1, &j->tree_ref);
  napi_create_promise(env, &j->def, &promise);
  napi_create_string_utf8(env, "crdtm.apply", NAPI_AUTO_LENGTH, &name);
  napi_create_async_work(env, NULL, name, async_exec, async_done, j, &j->work);
  tree_h *h = j->h;
  if (h->qtail) h->qtail->next = j;
  else h->qhead = j;
  h->qtail = j;
  start_next(env, h);
  return promise;
}

static napi_value js_ops_since(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  tree_h *h = argc > 0 ? get_tree(env, argv[0]) : NULL;
  if (!h) return NULL;
  int64_t ts = 0;
  if (argc > 1) napi_get_value_int64(env, argv[1], &ts);
  char *s = NULL;
  size_t n = 0;
  pthread_mutex_lock(&g_mu);
  int rc = encode_log(h, 0, ts, 1, &s, &n);
  pthread_mutex_unlock(&g_mu);
  if (rc) return throw_rc(env, "operationsSince", rc);
  return ret_string(env, s, n);
}

static napi_value js_last_operation(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  tree_h *h = argc > 0 ? get_tree(env, argv[0]) : NULL;
  if (!h) return NULL;
  char *s = NULL;
  size_t n = 0;
  pthread_mutex_lock(&g_mu);
  int rc = encode_log(h, 1, 0, 0, &s, &n);
  pthread_mutex_unlock(&g_mu);
  if (rc) return throw_rc(env, "lastOperation", rc);
  return ret_string(env, s, n);
}

static napi_value js_timestamp(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  tree_h *h = argc > 0 ? get_tree(env, argv[0]) : NULL;
  if (!h) return NULL;
  int64_t ts = 0;
  int rc = crdtm_tree_timestamp(h->t, &ts);
  if (rc) return throw_rc(env, "timestamp", rc);
  napi_value v;
  napi_create_int64(env, ts, &v);
  return v;
}

static napi_value js_last_replica_ts(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  tree_h *h = argc > 0 ? get_tree(env, argv[0]) : NULL;
  if (!h) return NULL;
  int64_t rid = 0;
  if (argc > 1) napi_get_value_int64(env, argv[1], &rid);
  uint64_t n = 0;
  int rc = crdtm_tree_replicas(h->t, NULL, NULL, 0, &n);
  int64_t out = 0;
  if (!rc && n) {
    int64_t *ids = malloc(n * sizeof(int64_t)), *tss = malloc(n * sizeof(int64_t));
    rc = crdtm_tree_replicas(h->t, ids, tss, n, &n);
    for (uint64_t k = 0; !rc && k < n; ++k)
      if (ids[k] == rid) out = tss[k];
    free(ids);
    free(tss);
  }
  if (rc) return throw_rc(env, "lastReplicaTimestamp", rc);
  napi_value v;
  napi_create_int64(env, out, &v);
  return v;
}

static napi_value js_document(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  tree_h *h = argc > 0 ? get_tree(env, argv[0]) : NULL;
  if (!h) return NULL;
  pthread_mutex_lock(&g_mu);
  uint64_t nvis = 0;
  int rc = crdtm_tree_document(h->t, NULL, 0, &nvis);
  uint32_t *vals = NULL;
  if (!rc && nvis) {
    vals = malloc(nvis * sizeof(uint32_t));
    rc = vals ? crdtm_tree_document(h->t, vals, nvis, &nvis) : CRDTM_E_NOMEM;
  }
  pthread_mutex_unlock(&g_mu);
  if (rc) {
    free(vals);
    return throw_rc(env, "document", rc);
  }
  size_t cap = 2, len = 0;
  for (uint64_t k = 0; k < nvis; ++k) cap += h->vo[vals[k] + 1] - h->vo[vals[k]] + 1;
  char *s = malloc(cap + 1);
  s[len++] = '[';
  for (uint64_t k = 0; k < nvis; ++k) {
    const uint64_t b = h->vo[vals[k]], e = h->vo[vals[k] + 1];
    if (k) s[len++] = ',';
    memcpy(s + len, h->vb + b, e - b);
    len += e - b;
  }
  s[len++] = ']';
  napi_value v;
  napi_create_string_utf8(env, s, len, &v);
  free(s);
  free(vals);
  return v;
}

static napi_value js_release(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
  tree_h *h = argc > 0 ? get_tree(env, argv[0]) : NULL;
  if (!h) return NULL;
  if (h->busy || h->qhead) {
    napi_throw_error(env, "E_BUSY", "crdtm: release while async applies of this tree are pending");
    return NULL;
  }
  pthread_mutex_lock(&g_mu);
  crdtm_tree_destroy(h->t);
  h->t = NULL;
  pthread_mutex_unlock(&g_mu);
  return NULL;
}

#define EXPORT(name, fn)                                         \
  do {                                                           \
    napi_value f;                                                \
    napi_create_function(env, name, NAPI_AUTO_LENGTH, fn, NULL, &f); \
    napi_set_named_property(env, exports, name, f);              \
  } while (0)

static napi_value module_init(napi_env env, napi_value exports) {
  EXPORT("init", js_init);
  EXPORT("apply", js_apply);
  EXPORT("applySync", js_apply_sync);
  EXPORT("operationsSince", js_ops_since);
  EXPORT("lastOperation", js_last_operation);
  EXPORT("timestamp", js_timestamp);
  EXPORT("lastReplicaTimestamp", js_last_replica_ts);
  EXPORT("document", js_document);
  EXPORT("release", js_release);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, module_init)

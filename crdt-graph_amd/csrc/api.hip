// api.hip — the C ABI (include/crdtm.h) over the gfx950 merge engine.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "engine.h"
#include "../../include/crdtm_test.h"  // (test-only entry points, gated by CRDTM_TEST_HOOKS)

using namespace crdtm;

namespace {

constexpr uint64_t FNV_OFF = 1469598103934665603ULL, FNV_PRIME = 1099511628211ULL;

struct Sink {
  int64_t* out;
  uint64_t cap;
  uint64_t n = 0;
  uint64_t h = FNV_OFF;
  void put(int64_t w) {
    if (out && n < cap) out[n] = w;
    h ^= static_cast<uint64_t>(w);  // word-wise FNV-1a over 64-bit words (same as the oracle)
    h *= FNV_PRIME;
    ++n;
  }
};

// Host copy of a tree state (read APIs only: canonical dumps and egress).
struct HostTree {
  std::vector<long long> key;
  std::vector<uint32_t> next, src, child, dict;
  std::vector<uint8_t> flags;
  std::vector<uint32_t> d_sent;
  std::vector<uint8_t> l_kind;
  std::vector<long long> l_ts;
  std::vector<uint32_t> l_val, l_off;
  std::vector<long long> l_path;
  std::vector<std::vector<uint32_t>> members;
};

template <class T>
int d2h(std::vector<T>& v, const T* p, uint64_t n) {
  v.resize(n);
  if (n) HIP_CHECK(hipMemcpy(v.data(), p, n * sizeof(T), hipMemcpyDeviceToHost));
  return CRDTM_OK;
}

int fetch(const crdtm_tree* t, HostTree& h, bool members) {
  HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
  const uint64_t S = t->n_slots, D = t->n_dicts;
  int r;
  if ((r = d2h(h.key, t->d.s_key, S)) || (r = d2h(h.next, t->d.s_next, S)) || (r = d2h(h.src, t->d.s_src, S)) ||
      (r = d2h(h.child, t->d.s_child, S)) || (r = d2h(h.dict, t->d.s_dict, S)) ||
      (r = d2h(h.flags, t->d.s_flags, S)) || (r = d2h(h.d_sent, t->d.d_sent, D)) ||
      (r = d2h(h.l_kind, t->d.l_kind, t->log_n)) || (r = d2h(h.l_ts, t->d.l_ts, t->log_n)) ||
      (r = d2h(h.l_val, t->d.l_val, t->log_n)) || (r = d2h(h.l_off, t->d.l_off, t->log_n + 1)) ||
      (r = d2h(h.l_path, t->d.l_path, t->log_npath)))
    return r;
  if (members) {
    h.members.assign(D, {});
    for (uint64_t s = 0; s < S; ++s) h.members[h.dict[s]].push_back(static_cast<uint32_t>(s));
  }
  return CRDTM_OK;
}

void put_path(const HostTree& h, uint32_t src, Sink& s) {
  if (src == NONE) {
    s.put(0);
    return;
  }
  const uint32_t b = h.l_off[src], e = h.l_off[src + 1];
  const uint32_t L = e - b;  // node path = op path without its last element, then ts
  s.put(static_cast<int64_t>(L));
  for (uint32_t j = b; j + 1 < e; ++j) s.put(h.l_path[j]);
  s.put(h.l_ts[src]);
}

void dump_dict(const HostTree& h, uint32_t d, int64_t depth, Sink& s) {
  std::vector<uint32_t> m = h.members[d];
  std::sort(m.begin(), m.end(), [&](uint32_t a, uint32_t b) { return h.key[a] < h.key[b]; });
  for (uint32_t x : m) {
    const bool tomb = h.flags[x] & F_TOMB;
    s.put(depth);
    s.put(h.key[x]);
    s.put(tomb ? 2 : 1);
    const uint32_t nx = h.next[x];
    s.put(nx != NONE ? 1 : 0);
    s.put(nx != NONE ? h.key[nx] : 0);
    s.put(tomb ? 0 : static_cast<int64_t>(h.l_val[h.src[x]]));
    put_path(h, h.src[x], s);
    if (tomb) continue;
    if (h.child[x] != NONE) {
      dump_dict(h, h.child[x], depth + 1, s);
    } else {  // implicit children {0: Tombstone [] Nothing}: its sentinel entry
      const int64_t sent[] = {depth + 1, 0, 2, 0, 0, 0, 0};
      for (int64_t w : sent) s.put(w);
    }
  }
}

void dump_visible(const HostTree& h, uint32_t d, int64_t depth, Sink& s) {
  uint32_t cur = h.d_sent[d];
  for (;;) {
    uint32_t nx = h.next[cur];
    while (nx != NONE && (h.flags[nx] & F_TOMB)) nx = h.next[nx];
    if (nx == NONE) break;
    s.put(depth);
    s.put(static_cast<int64_t>(h.l_val[h.src[nx]]));
    put_path(h, h.src[nx], s);
    if (h.child[nx] != NONE) dump_visible(h, h.child[nx], depth + 1, s);
    cur = nx;
  }
}

// The per-op kernels load 4 ops per lane with 16-byte vector loads; device
// inputs that are not aligned for that are staged into the (aligned) arena.
int align_ops(crdtm_ctx* c, OpsDev& o) {
  auto mis = [](const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) != 0; };
  hipStream_t s = c->stream;
  const uint64_t n = o.n;
  if (mis(o.kind, 4)) {
    auto* k = c->ws.alloc<uint8_t>(n + 1);
    HIP_CHECK(hipMemcpyAsync(k, o.kind, n, hipMemcpyDeviceToDevice, s));
    o.kind = k;
  }
  if (mis(o.ts, 16)) {
    auto* t = c->ws.alloc<long long>(n + 1);
    HIP_CHECK(hipMemcpyAsync(t, o.ts, n * 8, hipMemcpyDeviceToDevice, s));
    o.ts = t;
  }
  if (mis(o.off, 16)) {
    auto* f = c->ws.alloc<uint32_t>(n + 1);
    HIP_CHECK(hipMemcpyAsync(f, o.off, (n + 1) * 4, hipMemcpyDeviceToDevice, s));
    o.off = f;
  }
  if (mis(o.path, 16)) {
    auto* p = c->ws.alloc<long long>(o.n_path + 1);
    if (o.n_path) HIP_CHECK(hipMemcpyAsync(p, o.path, o.n_path * 8, hipMemcpyDeviceToDevice, s));
    o.path = p;
  }
  if (mis(o.val, 16)) {
    auto* v = c->ws.alloc<uint32_t>(n + 1);
    HIP_CHECK(hipMemcpyAsync(v, o.val, n * 4, hipMemcpyDeviceToDevice, s));
    o.val = v;
  }
  return CRDTM_OK;
}

uint64_t arena_need(uint64_t n, uint64_t np, const crdtm_tree* t) {
  const uint64_t slots = t->cap.slots + 2 * n + 1024;
  return 640 * n + 16 * np + 48 * slots + 32 * t->cap.dicts + (64ULL << 20);
}

int ensure_arena(crdtm_ctx* c, uint64_t bytes) {
  if (c->ws.cap >= bytes) return CRDTM_OK;
  HIP_CHECK(hipStreamSynchronize(c->stream));
  HIP_CHECK(hipStreamSynchronize(c->side));
  if (c->ws.base) HIP_CHECK(hipFree(c->ws.base));
  c->ws.base = nullptr;
  c->ws.cap = 0;
  const uint64_t cap = bytes + bytes / 4;
  HIP_CHECK(hipMalloc(&c->ws.base, cap));
  c->ws.cap = cap;
  return CRDTM_OK;
}

}  // namespace

extern "C" {

int crdtm_version(void) { return 1; }

int crdtm_device_count(int* count) {
  if (!count) return CRDTM_E_ARG;
  if (hipGetDeviceCount(count) != hipSuccess) {
    *count = 0;
    return CRDTM_E_NODEVICE;
  }
  return CRDTM_OK;
}

int crdtm_ctx_create(int device, void* stream, crdtm_ctx** out) {
  if (!out) return CRDTM_E_ARG;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return CRDTM_E_NODEVICE;
  if (device < 0 || device >= nd) return CRDTM_E_ARG;
  HIP_CHECK(hipSetDevice(device));
  auto* c = new crdtm_ctx;
  c->device = device;
  if (stream) {
    c->stream = static_cast<hipStream_t>(stream);
  } else {
    HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
  }
  HIP_CHECK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
  HIP_CHECK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&c->ev_sync, hipEventDisableTiming));
  HIP_CHECK(hipMalloc(&c->dres, sizeof(DevResult)));
  HIP_CHECK(hipHostMalloc(&c->hres, sizeof(DevResult), hipHostMallocDefault));
  HIP_CHECK(hipMalloc(&c->crange, RID_SLOTS * sizeof(uint2)));
  HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->crange), -1, 2ULL * RID_SLOTS, c->stream));
  HIP_CHECK(hipMemset2DAsync(reinterpret_cast<char*>(c->crange) + 4, 8, 0, 4, RID_SLOTS, c->stream));
  c->ws.scan_cap = 1u << 20;
  HIP_CHECK(hipMalloc(&c->ws.scan_status, (c->ws.scan_cap + 2) * sizeof(unsigned long long)));
  HIP_CHECK(hipMemsetAsync(c->ws.scan_status, 0, (c->ws.scan_cap + 2) * sizeof(unsigned long long), c->stream));
  c->ws.scan_ticket = reinterpret_cast<uint32_t*>(c->ws.scan_status + c->ws.scan_cap);
  c->ws.scan_err = &c->dres->scan_err;
  HIP_CHECK(hipMemsetAsync(c->dres, 0, sizeof(DevResult), c->stream));
  HIP_CHECK(hipMalloc(&c->rtab, REPLICA_SLOTS * sizeof(uint32_t)));
  HIP_CHECK(hipMemsetAsync(c->rtab, 0, REPLICA_SLOTS * sizeof(uint32_t), c->stream));
  int r = ensure_arena(c, 64ULL << 20);
  if (r) return r;
  HIP_CHECK(hipStreamSynchronize(c->stream));
  *out = c;
  return CRDTM_OK;
}

int crdtm_ctx_destroy(crdtm_ctx* c) {
  if (!c) return CRDTM_OK;
  hipStreamSynchronize(c->stream);
  c->clear_marks();
  if (c->ws.base) hipFree(c->ws.base);
  hipFree(c->dres);
  hipHostFree(c->hres);
  if (c->pin) hipHostFree(c->pin);
  hipFree(c->crange);
  if (c->fl_rec) hipFree(c->fl_rec);
  hipFree(c->ws.scan_status);
  hipFree(c->rtab);
  if (c->gstat_dev) hipFree(c->gstat_dev);
  if (c->own_stream) hipStreamDestroy(c->stream);
  hipStreamSynchronize(c->side);
  hipStreamDestroy(c->side);
  hipEventDestroy(c->ev_fork);
  hipEventDestroy(c->ev_join);
  hipEventDestroy(c->ev_sync);
  delete c;
  return CRDTM_OK;
}

void* crdtm_ctx_stream(crdtm_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int crdtm_ctx_sync(crdtm_ctx* c) {
  if (!c) return CRDTM_E_ARG;
  HIP_CHECK(hipStreamSynchronize(c->stream));
  return CRDTM_OK;
}

static int init_root(crdtm_tree* t) {
  // init: Root {0: Tombstone [] Nothing} (src/Internal/Node.elm:41-48)
  const long long k0 = 0;
  const uint32_t none = NONE, zero = 0;
  const uint8_t fl = F_TOMB | F_SENT;
  HIP_CHECK(hipMemcpy(t->d.s_key, &k0, sizeof(k0), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(t->d.s_next, &none, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(t->d.s_src, &none, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(t->d.s_child, &none, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(t->d.s_dict, &zero, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(t->d.s_flags, &fl, 1, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(t->d.d_sent, &zero, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(t->d.d_owner, &none, 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(t->d.l_off, &zero, 4, hipMemcpyHostToDevice));
  return CRDTM_OK;
}

int crdtm_tree_create(crdtm_ctx* c, int64_t replica_id, crdtm_tree** out) {
  if (!c || !out) return CRDTM_E_ARG;
  HIP_CHECK(hipSetDevice(c->device));
  auto* t = new crdtm_tree;
  t->ctx = c;
  TreeCaps need;
  need.slots = 1024;
  need.dicts = 512;
  need.log = 1024;
  need.lpath = 4096;
  need.doc = 1024;
  int r = grow_tree(t, need);
  if (r || (r = init_root(t))) return r;
  t->n_slots = 1;
  t->n_dicts = 1;
  t->timestamp = replica_id * TWO32;  // replicaId * 2 ^ 32 (src/CRDTree.elm:137)
  t->doc_valid = true;
  t->doc_n = 0;
  *out = t;
  return CRDTM_OK;
}

int crdtm_tree_reset(crdtm_tree* t, int64_t replica_id) {
  if (!t) return CRDTM_E_ARG;
  if (t->store && t->store.use_count() > 1) {  // other versions keep the shared arrays
    int r = unshare_tree(t, false);
    if (r || (r = init_root(t))) return r;
  }
  // slot 0 / dict 0 / l_off[0] keep their init values: only the root
  // sentinel's `next` can change, and only to a slot we now drop.
  // (stream-ordered, no host wait: every later read of the state synchronises)
  // (the result block's init rides on this launch: a merge that follows
  // skips its own, crdtm_ctx::dres_ready)
  // (env CRDTM_DRES_FOLD=0: off, A/B)
  static const bool fold = [] {
    const char* e = getenv("CRDTM_DRES_FOLD");
    return !(e && e[0] == '0');
  }();
  hipLaunchKernelGGL(k_reset_root, dim3(1), dim3(fold ? 64 : 1), 0, t->ctx->stream, t->d.s_next,
                     fold ? t->ctx->dres : nullptr);
  HIP_CHECK(hipGetLastError());
  t->ctx->dres_ready = fold;
  t->n_slots = 1;
  t->n_dicts = 1;
  t->log_n = 0;
  t->log_npath = 0;
  t->doc_n = 0;
  t->doc_valid = true;
  t->doc_gapped = false;
  t->max_depth = 0;
  t->timestamp = replica_id * TWO32;
  t->replicas.clear();
  t->last_begin = t->last_end = 0;
  t->last_is_batch = 1;
  t->flat_clean = true;
  t->kidx_valid = false;
  t->ilr_valid = false;
  ++t->version;
  return CRDTM_OK;
}

int crdtm_tree_destroy(crdtm_tree* t) {
  if (!t) return CRDTM_OK;
  hipStreamSynchronize(t->ctx->stream);
  t->store.reset();  // frees the arrays unless another version still shares them
  delete t;
  return CRDTM_OK;
}

// A new version handle sharing the state's device arrays (O(1)); the first
// write to either handle gives it a private copy (Elm persistence,
// src/CRDTree.elm:228-232: the old value stays valid after apply).
int crdtm_tree_clone(const crdtm_tree* t, crdtm_tree** out) {
  if (!t || !out) return CRDTM_E_ARG;
  if (t->doc_gapped) {  // the order lives in t's own index: write the shared `doc` from it first
    auto* tw = const_cast<crdtm_tree*>(t);
    crdtm_ctx* c = t->ctx;
    HIP_CHECK(hipSetDevice(c->device));
    int r = ensure_arena(c, arena_need(0, 0, tw) + 64 * (t->n_slots + t->n_dicts));
    if (r) return r;
    try {
      if ((r = linearize(tw))) return r;
    } catch (const ArenaOverflow&) {
      return CRDTM_E_NOMEM;
    }
  }
  auto* u = new crdtm_tree;
  u->ctx = t->ctx;
  u->d = t->d;
  u->cap = t->cap;
  u->store = t->store;
  u->n_slots = t->n_slots;
  u->n_dicts = t->n_dicts;
  u->log_n = t->log_n;
  u->log_npath = t->log_npath;
  u->doc_n = t->doc_n;
  u->doc_valid = t->doc_valid;
  u->max_depth = t->max_depth;
  u->timestamp = t->timestamp;
  u->replicas = t->replicas;
  u->last_begin = t->last_begin;
  u->last_end = t->last_end;
  u->last_is_batch = t->last_is_batch;
  u->flat_clean = t->flat_clean;  // (the key index stays with `t`: each handle builds its own)
  *out = u;
  return CRDTM_OK;
}

// Linearise inside apply when the batch is at least 1/16 of the document
// (env CRDTM_LINEARIZE=eager|lazy overrides).
static bool linearize_eagerly(const crdtm_tree* t, uint64_t n) {
  const char* e = getenv("CRDTM_LINEARIZE");
  if (e && !strcmp(e, "eager")) return true;
  if (e && !strcmp(e, "lazy")) return false;
  return 16 * n >= t->n_slots;
}

int crdtm_apply(crdtm_tree* t, const crdtm_ops* ops, int ops_on_device, int is_batch, uint8_t* status_out,
                crdtm_result* res) {
  if (!t || !ops || !res) return CRDTM_E_ARG;
  ++t->version;
  std::memset(res, 0, sizeof(*res));
  res->err_index = -1;
  if (!is_batch && ops->n_ops != 1) return CRDTM_E_ARG;
  if (ops->n_ops >= 0x7FFFFFF0ULL) return CRDTM_E_ARG;
  crdtm_ctx* c = t->ctx;
  HIP_CHECK(hipSetDevice(c->device));
  if (int ru = unshare_tree(t, true)) return ru;  // this version is about to be written
  c->clear_marks();
  c->gstat_valid = 0;
  const uint64_t n = ops->n_ops;
  uint64_t np = ops->n_path;
  if (!ops_on_device && n) np = ops->path_off[n];
  // a fresh tree (the closed form and the per-dict replay only run on one)
  // is restored on an engine error; other paths commit after their last check
  const bool fresh = t->n_slots == 1 && t->log_n == 0;
  const int64_t ts_before = t->timestamp;
  int r = CRDTM_OK;
  // an incremental merge may run over log ++ batch (merge.hip apply_batch)
  const uint64_t n_need = fresh ? n : n + t->log_n, np_need = fresh ? np : np + t->log_npath;
  for (int attempt = 0; attempt < 4; ++attempt) {
    r = ensure_arena(c, arena_need(n_need, np_need, t) << attempt);
    if (r) return r;
    c->ws.reset();
    try {
      OpsDev o;
      o.n = static_cast<uint32_t>(n);
      o.n_path = np;
      uint8_t* st_dev = nullptr;
      if (ops_on_device) {
        o.kind = ops->kind;
        o.ts = reinterpret_cast<const long long*>(ops->ts);
        o.off = ops->path_off;
        o.path = reinterpret_cast<const long long*>(ops->path);
        o.val = ops->val;
        st_dev = status_out;
        if ((r = align_ops(c, o))) return r;
      } else {
        hipStream_t s = c->stream;
        auto* kind = c->ws.alloc<uint8_t>(n + 1);
        auto* ts = c->ws.alloc<long long>(n + 1);
        auto* off = c->ws.alloc<uint32_t>(n + 1);
        auto* path = c->ws.alloc<long long>(np + 1);
        auto* val = c->ws.alloc<uint32_t>(n + 1);
        if (n) {
          HIP_CHECK(hipMemcpyAsync(kind, ops->kind, n, hipMemcpyHostToDevice, s));
          HIP_CHECK(hipMemcpyAsync(ts, ops->ts, n * 8, hipMemcpyHostToDevice, s));
          HIP_CHECK(hipMemcpyAsync(off, ops->path_off, (n + 1) * 4, hipMemcpyHostToDevice, s));
          if (np) HIP_CHECK(hipMemcpyAsync(path, ops->path, np * 8, hipMemcpyHostToDevice, s));
          HIP_CHECK(hipMemcpyAsync(val, ops->val, n * 4, hipMemcpyHostToDevice, s));
        }
        o.kind = kind;
        o.ts = ts;
        o.off = off;
        o.path = path;
        o.val = val;
        if (status_out) st_dev = c->ws.alloc<uint8_t>(n + 1);
      }
      g_prof = c->profile ? c : nullptr;
      r = apply_batch(t, o, st_dev, res);
      g_prof = nullptr;
      if (r == CRDTM_OK && status_out && !ops_on_device && n) {
        HIP_CHECK(hipMemcpyAsync(status_out, st_dev, n, hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(hipStreamSynchronize(c->stream));
      }
      break;
    } catch (const ArenaOverflow&) {
      HIP_CHECK(hipStreamSynchronize(c->stream));
      HIP_CHECK(hipStreamSynchronize(c->side));  // (side-stream work may read the old arena)
      r = CRDTM_E_NOMEM;
    }
  }
  if (r != CRDTM_OK) {
    if (fresh && crdtm_tree_reset(t, replica_of(ts_before)) == CRDTM_OK) t->timestamp = ts_before;
    res->code = r;
    return r;
  }
  if (res->code == CRDTM_OK) {
    // lastOperation: the op itself, or Batch of the applied ops; an
    // AlreadyApplied single op leaves Batch [] (src/CRDTree.elm:318-319)
    t->last_is_batch = (is_batch || res->n_applied == 0) ? 1 : 0;
    // The document order (north-star kernel 4): the closed forms compute it
    // as they merge; a replay's state is linearised here, inside the call
    // (and inside a timed bench step), when the batch is large against the
    // document — linearising is O(document), so a small edit leaves it to
    // the first read (crdtm_tree_document, clone), which linearises then.
    // The batch is committed at this point: a failure here only leaves the
    // order to that first read.
    if (!t->doc_valid && n && linearize_eagerly(t, n)) {
      r = ensure_arena(c, arena_need(0, 0, t) + 64 * (t->n_slots + t->n_dicts));
      g_prof = c->profile ? c : nullptr;
      try {
        if (r == CRDTM_OK) r = linearize(t);
      } catch (const ArenaOverflow&) {
        r = CRDTM_E_NOMEM;
      }
      g_prof = nullptr;
      if (r != CRDTM_OK) {
        r = CRDTM_OK;
      }
    }
  }
  res->timestamp = t->timestamp;
  res->n_slots = t->n_slots;
  if (c->profile) {
    HIP_CHECK(hipStreamSynchronize(c->stream));
    c->collect_phases();
  }
  return res->code < 0 ? res->code : CRDTM_OK;
}

int crdtm_tree_timestamp(const crdtm_tree* t, int64_t* out) {
  if (!t || !out) return CRDTM_E_ARG;
  *out = t->timestamp;
  return CRDTM_OK;
}

int crdtm_tree_replicas(const crdtm_tree* t, int64_t* ids, int64_t* tss, uint64_t cap, uint64_t* n) {
  if (!t || !n) return CRDTM_E_ARG;
  uint64_t i = 0;
  for (const auto& kv : t->replicas) {
    if (ids && tss && i < cap) {
      ids[i] = kv.first;
      tss[i] = kv.second;
    }
    ++i;
  }
  *n = i;
  return CRDTM_OK;
}

// Copy log entries [b, e) out as a crdtm_ops (sizes only when out->kind is NULL).
static int copy_log_range(const crdtm_tree* t, uint64_t b, uint64_t e, crdtm_ops* out) {
  const uint64_t n = e - b;
  std::vector<uint32_t> off(n + 1);
  HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
  if (n + 1) HIP_CHECK(hipMemcpy(off.data(), t->d.l_off + b, (n + 1) * 4, hipMemcpyDeviceToHost));
  const uint64_t pb = off[0], pe = off[n];
  const bool fill = out->kind != nullptr;
  out->n_ops = n;
  out->n_path = pe - pb;
  if (!fill) return CRDTM_OK;
  if (n) {
    HIP_CHECK(hipMemcpy(out->kind, t->d.l_kind + b, n, hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(out->ts, t->d.l_ts + b, n * 8, hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(out->val, t->d.l_val + b, n * 4, hipMemcpyDeviceToHost));
  }
  for (uint64_t i = 0; i <= n; ++i) out->path_off[i] = off[i] - static_cast<uint32_t>(pb);
  if (pe > pb) HIP_CHECK(hipMemcpy(out->path, t->d.l_path + pb, (pe - pb) * 8, hipMemcpyDeviceToHost));
  return CRDTM_OK;
}

int crdtm_tree_ops(const crdtm_tree* t, int which, crdtm_ops* out, int* is_batch) {
  if (!t || !out) return CRDTM_E_ARG;
  const uint64_t b = which == 0 ? 0 : t->last_begin;
  const uint64_t e = which == 0 ? t->log_n : t->last_end;
  if (is_batch) *is_batch = which == 0 ? 1 : t->last_is_batch;
  return copy_log_range(t, b, e, out);
}

// since (src/Internal/Operation.elm:25-53): the newest logged Add with this ts
__global__ void k_since(const uint8_t* kind, const long long* ts, uint64_t n, long long want, uint32_t* end) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    if (kind[i] == CRDTM_ADD && ts[i] == want) atomicMax(end, static_cast<uint32_t>(i + 1));
}

int crdtm_tree_ops_since(const crdtm_tree* t, int64_t ts, crdtm_ops* out) {
  if (!t || !out) return CRDTM_E_ARG;
  crdtm_ctx* c = t->ctx;
  HIP_CHECK(hipSetDevice(c->device));
  if (ts == 0) return copy_log_range(t, 0, t->log_n, out);  // operationsSince 0: the whole log
  uint32_t* end = &c->dres->since_end;
  c->dres_ready = false;
  HIP_CHECK(hipMemsetAsync(end, 0, sizeof(uint32_t), c->stream));
  if (t->log_n)
    hipLaunchKernelGGL(k_since, dim3(grid_for(t->log_n)), dim3(BLOCK), 0, c->stream, t->d.l_kind, t->d.l_ts,
                       t->log_n, static_cast<long long>(ts), end);
  uint32_t h = 0;
  HIP_CHECK(hipMemcpyAsync(&h, end, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(hipStreamSynchronize(c->stream));
  if (h == 0) return copy_log_range(t, 0, 0, out);  // no such Add: []
  return copy_log_range(t, h - 1, t->log_n, out);
}

// Every index of the state in range (a read API walks them on the host):
// the first violation goes to stderr with CRDTM_STATE_DEBUG set.
static int check_state(const HostTree& h, uint64_t S, uint64_t D, uint64_t L) {
  static const bool verbose = getenv("CRDTM_STATE_DEBUG") != nullptr;
  auto bad = [&](const char* what, uint64_t s, uint64_t v) {
    if (verbose) fprintf(stderr, "crdtm state: slot %llu %s %llu (S %llu D %llu L %llu)\n",
                         static_cast<unsigned long long>(s), what, static_cast<unsigned long long>(v),
                         static_cast<unsigned long long>(S), static_cast<unsigned long long>(D),
                         static_cast<unsigned long long>(L));
    return CRDTM_E_STATE;
  };
  for (uint64_t s = 0; s < S; ++s) {
    if (h.dict[s] >= D) return bad("dict", s, h.dict[s]);
    if (h.next[s] != NONE && (h.next[s] >= S || h.dict[h.next[s]] != h.dict[s])) return bad("next", s, h.next[s]);
    if (h.child[s] != NONE && h.child[s] >= D) return bad("child", s, h.child[s]);
    if (h.src[s] != NONE && h.src[s] >= L) return bad("src", s, h.src[s]);
  }
  for (uint64_t d = 0; d < D; ++d)
    if (h.d_sent[d] != NONE && h.d_sent[d] >= S) return bad("sentinel of dict", d, h.d_sent[d]);
  // the dicts the dumps reach (live members' children, from the root): each
  // once, with a sentinel, its chain inside it and finite
  if (!D) return CRDTM_OK;
  std::vector<uint8_t> seen(D, 0);
  std::vector<uint32_t> todo{0}, ncount(D, 0), moff(D + 1, 0), mem(S);
  for (uint64_t s = 0; s < S; ++s) ++ncount[h.dict[s]];
  for (uint64_t d = 0; d < D; ++d) moff[d + 1] = moff[d] + ncount[d];
  {
    std::vector<uint32_t> fill(moff.begin(), moff.end() - 1);
    for (uint64_t s = 0; s < S; ++s) mem[fill[h.dict[s]]++] = static_cast<uint32_t>(s);
  }
  seen[0] = 1;
  while (!todo.empty()) {
    const uint32_t d = todo.back();
    todo.pop_back();
    if (h.d_sent[d] == NONE) return bad("reached dict without a sentinel", d, d);
    if (h.dict[h.d_sent[d]] != d || !(h.flags[h.d_sent[d]] & F_SENT))  // (its own sentinel slot)
      return bad("sentinel slot of dict", d, h.d_sent[d]);
    uint64_t steps = 0;
    for (uint32_t q = h.d_sent[d]; q != NONE; q = h.next[q])
      if (++steps > ncount[d]) return bad("chain cycle in dict", d, q);
    for (uint32_t j = moff[d]; j < moff[d + 1]; ++j) {  // (the structure dump walks every member)
      const uint32_t q = mem[j];
      if ((h.flags[q] & F_TOMB) || h.child[q] == NONE) continue;
      if (seen[h.child[q]]) return bad("children dict reached twice", q, h.child[q]);
      seen[h.child[q]] = 1;
      todo.push_back(h.child[q]);
    }
  }
  return CRDTM_OK;
}

int crdtm_tree_canonical(const crdtm_tree* t, int which, int64_t* out, uint64_t cap, uint64_t* n_words,
                         uint64_t* hash) {
  if (!t) return CRDTM_E_ARG;
  HostTree h;
  int r = fetch(t, h, false);
  if (r) return r;
  if ((r = check_state(h, t->n_slots, t->n_dicts, t->log_n))) return r;
  if (which == 0) {
    h.members.assign(t->n_dicts, {});
    for (uint64_t s2 = 0; s2 < t->n_slots; ++s2) h.members[h.dict[s2]].push_back(static_cast<uint32_t>(s2));
  }
  Sink s{out, cap};
  if (which == 0) dump_dict(h, 0, 0, s);
  else dump_visible(h, 0, 0, s);
  if (n_words) *n_words = s.n;
  if (hash) *hash = s.h;
  return CRDTM_OK;
}

__global__ void k_doc_vals(const uint32_t* doc, uint64_t n, const uint32_t* src, const uint32_t* lval,
                           uint32_t* out) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = lval[src[doc[i]]];
}

int crdtm_tree_document(const crdtm_tree* tc, uint32_t* vals, uint64_t cap, uint64_t* n_visible) {
  if (!tc || !n_visible) return CRDTM_E_ARG;
  auto* t = const_cast<crdtm_tree*>(tc);
  crdtm_ctx* c = t->ctx;
  HIP_CHECK(hipSetDevice(c->device));
  int r = ensure_arena(c, arena_need(0, 0, t) + 64 * (t->n_slots + t->n_dicts));
  if (r) return r;
  try {
    if ((r = linearize(t))) return r;
    *n_visible = t->doc_n;
    if (vals && t->doc_n) {
      c->ws.reset();
      uint32_t* tmp = c->ws.alloc<uint32_t>(t->doc_n);
      hipLaunchKernelGGL(k_doc_vals, dim3(grid_for(t->doc_n)), dim3(BLOCK), 0, c->stream, t->d.doc, t->doc_n,
                         t->d.s_src, t->d.l_val, tmp);
      const uint64_t m = std::min<uint64_t>(cap, t->doc_n);
      HIP_CHECK(hipMemcpyAsync(vals, tmp, m * 4, hipMemcpyDeviceToHost, c->stream));
      HIP_CHECK(hipStreamSynchronize(c->stream));
    }
  } catch (const ArenaOverflow&) {
    return CRDTM_E_NOMEM;
  }
  return CRDTM_OK;
}

int crdtm_debug_poke(crdtm_tree* t, int field, uint64_t index, uint32_t value) {
  if (!t || !test_hooks()) return CRDTM_E_ARG;
  uint32_t* a = field == 0 ? t->d.s_next : field == 1 ? t->d.s_child : field == 2 ? t->d.s_dict
              : field == 3 ? t->d.d_sent : nullptr;
  const uint64_t lim = field == 3 ? t->n_dicts : t->n_slots;
  if (!a || index >= lim) return CRDTM_E_ARG;
  if (int ru = unshare_tree(t, true)) return ru;
  HIP_CHECK(hipSetDevice(t->ctx->device));
  HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
  HIP_CHECK(hipMemcpy(a + index, &value, sizeof(value), hipMemcpyHostToDevice));
  ++t->version;  // (the host caches of this version are stale)
  // (and no merge path may trust the device indexes of the poked state)
  t->kidx_valid = false;
  t->ilr_valid = false;
  t->flat_clean = false;
  return CRDTM_OK;
}

int crdtm_ctx_guard_stats(crdtm_ctx* c, uint64_t* out) {
  if (!c || !out) return CRDTM_E_ARG;
  for (int k = 0; k < 4; ++k) out[k] = c->gstat_valid ? c->gstat[k] : 0;
  return c->gstat_valid;
}

int crdtm_ctx_profile(crdtm_ctx* c, int enable) {
  if (!c) return CRDTM_E_ARG;
  c->profile = enable != 0;
  return CRDTM_OK;
}

int crdtm_ctx_phase_times(crdtm_ctx* c, char* names, size_t names_cap, double* ms, int cap) {
  if (!c) return CRDTM_E_ARG;
  size_t pos = 0;
  int k = 0;
  for (auto& p : c->phases) {
    if (k < cap) {
      if (ms) ms[k] = p.second;
      if (names && pos + p.first.size() + 1 <= names_cap) {
        std::memcpy(names + pos, p.first.c_str(), p.first.size() + 1);
        pos += p.first.size() + 1;
      }
    }
    ++k;
  }
  return k;
}

int crdtm_forest_apply(crdtm_ctx* c, int64_t replica_id, const crdtm_ops* ops, const uint32_t* doc_off,
                       uint64_t n_docs, int on_device, int32_t* doc_code, int64_t* doc_err, uint32_t* doc_applied,
                       uint64_t* doc_hash, uint64_t* doc_words, int64_t* doc_timestamp) {
  if (!c || !ops || !doc_off || !doc_code) return CRDTM_E_ARG;
  HIP_CHECK(hipSetDevice(c->device));
  const uint64_t n = ops->n_ops;
  if (doc_off[n_docs] != n || n >= 0x7FFFFFF0ULL) return CRDTM_E_ARG;
  uint64_t np = ops->n_path;
  if (!on_device && n) np = ops->path_off[n];
  int r = ensure_arena(c, forest_ws_bytes(doc_off, n_docs, n, np));
  if (r) return r;
  c->ws.reset();
  c->clear_marks();
  try {
    OpsDev o;
    o.n = static_cast<uint32_t>(n);
    o.n_path = np;
    if (on_device) {
      o.kind = ops->kind;
      o.ts = reinterpret_cast<const long long*>(ops->ts);
      o.off = ops->path_off;
      o.path = reinterpret_cast<const long long*>(ops->path);
      o.val = ops->val;
      if ((r = align_ops(c, o))) return r;
    } else {
      hipStream_t s = c->stream;
      auto* kind = c->ws.alloc<uint8_t>(n + 1);
      auto* ts = c->ws.alloc<long long>(n + 1);
      auto* off = c->ws.alloc<uint32_t>(n + 1);
      auto* path = c->ws.alloc<long long>(np + 1);
      auto* val = c->ws.alloc<uint32_t>(n + 1);
      if (n) {
        HIP_CHECK(hipMemcpyAsync(kind, ops->kind, n, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(ts, ops->ts, n * 8, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(off, ops->path_off, (n + 1) * 4, hipMemcpyHostToDevice, s));
        if (np) HIP_CHECK(hipMemcpyAsync(path, ops->path, np * 8, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(val, ops->val, n * 4, hipMemcpyHostToDevice, s));
      }
      o.kind = kind;
      o.ts = ts;
      o.off = off;
      o.path = path;
      o.val = val;
    }
    g_prof = c->profile ? c : nullptr;
    r = forest_apply(c, replica_id, o, doc_off, n_docs, doc_code, doc_err, doc_applied, doc_hash, doc_words,
                     doc_timestamp);
    g_prof = nullptr;
  } catch (const ArenaOverflow&) {
    return CRDTM_E_NOMEM;
  }
  if (c->profile) {
    HIP_CHECK(hipStreamSynchronize(c->stream));
    c->collect_phases();
  }
  return r;
}

void crdtm_free(void* p) { std::free(p); }

}  // extern "C"

// ---------------------------------------------------------------------------
// Traversal API (src/CRDTree.elm:421-625, src/CRDTree/Node.elm:96-174).
// Point queries (get, node info, parent / next / prev / head, children) run
// on the device, over the state's own arrays plus a (dict, key) -> slot hash
// built in parallel once per tree version: one single-lane kernel per query
// follows the reference's lookups, and only the answer crosses PCIe. `walk`,
// whose output is the size of the document, reads a host copy of the state
// (fetched once per version). Both run the same rules, written once over a
// view of the state (TvDev / TvHost). Node references: a slot index of the
// current state, CRDTM_REF_ROOT, or the implicit sentinel of a live node's
// still-empty children dict (CRDTM_REF_VSENT | slot); valid until the next
// apply. Semantics follow the reference literally: a node's parent is found
// from its *path* (a dict sentinel's path is [] so its parent is the root),
// `next` follows next *keys* in that parent's children skipping Tombstones,
// `prev` scans the parent's chain from its sentinel (Tombstones included),
// `walk` starts after its start node and after the head of every node it
// descends into.
// ---------------------------------------------------------------------------
namespace {

constexpr uint64_t REF_NONE = CRDTM_REF_NONE, REF_ROOT = CRDTM_REF_ROOT, REF_VSENT = CRDTM_REF_VSENT;

// children dict of a node: kind 0 = empty (Tombstone), 1 = dict id, 2 = implicit {0: sentinel} of owner slot
struct DictRef {
  int kind;
  uint64_t v;
};

template <class V>
__host__ __device__ bool tv_ref_ok(const V& c, uint64_t r) {
  if (r == REF_ROOT) return true;
  if (r & REF_VSENT) {
    const uint64_t s = r & ~REF_VSENT;
    return s < c.S && !(c.flags(s) & F_TOMB) && c.child(s) == NONE;
  }
  return r < c.S;
}

template <class V>
__host__ __device__ bool tv_is_tomb(const V& c, uint64_t r) {
  return r != REF_ROOT && ((r & REF_VSENT) || (c.flags(r) & F_TOMB));
}

template <class V>
__host__ __device__ DictRef tv_children(const V& c, uint64_t r) {
  if (r == REF_ROOT) return {1, 0};
  if (tv_is_tomb(c, r)) return {0, 0};
  const uint32_t ch = c.child(r);
  return ch == NONE ? DictRef{2, r} : DictRef{1, ch};
}

template <class V>
__host__ __device__ uint64_t tv_lookup(const V& c, const DictRef& d, long long key) {
  if (d.kind == 0) return REF_NONE;
  if (d.kind == 2) return key == 0 ? (REF_VSENT | d.v) : REF_NONE;
  const uint32_t s = c.find(static_cast<uint32_t>(d.v), key);
  return s == NONE ? REF_NONE : s;
}

template <class V>
__host__ __device__ bool tv_next_key(const V& c, uint64_t r, long long* k) {
  if (r == REF_ROOT || (r & REF_VSENT)) return false;
  const uint32_t nx = c.next(r);
  if (nx == NONE) return false;
  *k = c.key(nx);
  return true;
}

// nextNode (src/Internal/Node.elm:257-268) in dict d
template <class V>
__host__ __device__ uint64_t tv_next_node(const V& c, uint64_t r, const DictRef& d) {
  long long k;
  for (uint64_t x = r;;) {
    if (!tv_next_key(c, x, &k)) return REF_NONE;
    x = tv_lookup(c, d, k);
    if (x == REF_NONE) return REF_NONE;
    if (!tv_is_tomb(c, x)) return x;
  }
}

// Node.descendant from the root (src/Internal/Node.elm:289-299) along keys p(0..n-1)
template <class V, class P>
__host__ __device__ uint64_t tv_descend(const V& c, const P& p, uint64_t n) {
  if (n == 0) return REF_NONE;
  uint64_t r = REF_ROOT;
  for (uint64_t j = 0; j < n && r != REF_NONE; ++j) r = tv_lookup(c, tv_children(c, r), p(j));
  return r;
}

// Node.path: the Add's path without its last element, then the node's ts
// (empty for the root and sentinels); the parent is `get` of all but the last
template <class V>
__host__ __device__ uint64_t tv_path_len(const V& c, uint64_t r) {
  if (r == REF_ROOT || (r & REF_VSENT)) return 0;
  const uint32_t src = c.src(r);
  return src == NONE ? 0 : c.loff(src + 1) - c.loff(src);
}
template <class V>
__host__ __device__ long long tv_path_at(const V& c, uint64_t r, uint64_t j) {
  const uint32_t src = c.src(r);
  const uint32_t b = c.loff(src), e = c.loff(src + 1);
  return b + j + 1 < e ? c.lpath(b + j) : c.lts(src);
}

template <class V>
__host__ __device__ uint64_t tv_parent(const V& c, uint64_t r) {  // src/CRDTree.elm:425-441
  const uint64_t L = tv_path_len(c, r);
  if (L <= 1) return REF_ROOT;
  return tv_descend(c, [&](uint64_t j) { return tv_path_at(c, r, j); }, L - 1);
}

template <class V>
__host__ __device__ uint64_t tv_next_of(const V& c, uint64_t r) {  // src/CRDTree.elm:560-566
  const uint64_t par = tv_parent(c, r);
  if (par == REF_NONE) return REF_NONE;
  return tv_next_node(c, r, tv_children(c, par));
}

template <class V>
__host__ __device__ uint64_t tv_prev_of(const V& c, uint64_t r) {  // src/CRDTree.elm:569-575 (Node.find)
  const uint64_t par = tv_parent(c, r);
  if (par == REF_NONE) return REF_NONE;
  const DictRef d = tv_children(c, par);
  uint64_t left = tv_lookup(c, d, 0);
  long long k;
  while (left != REF_NONE && tv_next_key(c, left, &k)) {
    const uint64_t x = tv_lookup(c, d, k);
    if (x == REF_NONE) return REF_NONE;
    if (tv_next_of(c, x) == r) return x;
    left = x;
  }
  return REF_NONE;
}

template <class V>
__host__ __device__ uint64_t tv_head_of(const V& c, uint64_t r) {  // src/CRDTree/Node.elm:165-167
  const DictRef d = tv_children(c, r);
  const uint64_t s0 = tv_lookup(c, d, 0);
  return s0 == REF_NONE ? REF_NONE : tv_next_node(c, s0, d);
}

// ---- the device view: the state's arrays + the per-version slot hash ----
struct TvDev {
  TreeDev T;
  SlotHash H;
  uint64_t S;
  __device__ uint8_t flags(uint64_t s) const { return T.s_flags[s]; }
  __device__ uint32_t child(uint64_t s) const { return T.s_child[s]; }
  __device__ uint32_t next(uint64_t s) const { return T.s_next[s]; }
  __device__ long long key(uint64_t s) const { return T.s_key[s]; }
  __device__ uint32_t src(uint64_t s) const { return T.s_src[s]; }
  __device__ uint32_t loff(uint32_t i) const { return T.l_off[i]; }
  __device__ long long lpath(uint32_t j) const { return T.l_path[j]; }
  __device__ long long lts(uint32_t i) const { return T.l_ts[i]; }
  __device__ uint32_t lval(uint32_t i) const { return T.l_val[i]; }
  __device__ uint32_t find(uint32_t d, long long k) const { return slothash_find(H, d, k); }
};

struct TravOut {
  uint64_t ref;
  uint64_t n;
  int64_t next;
  int32_t ok, kind, has_next;
  uint32_t val;
};

enum : int { TQ_GET = 0, TQ_INFO = 1, TQ_REL = 2, TQ_CHILDREN = 3 };

__global__ void __launch_bounds__(BLOCK) k_trav_index(TreeDev T, uint32_t S, SlotHash H) {
  GRID_STRIDE(s, S) slothash_put_par(H, T.s_dict[s], T.s_key[s], s);
}

// One query on one lane (the reference's lookups are a dependent chain).
__global__ void k_trav(TvDev v, int q, uint64_t ref, int which, const long long* path, uint64_t len, TravOut* out,
                       uint64_t* list, uint64_t list_cap, long long* pbuf, uint64_t pcap) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  TravOut o{};
  o.ok = 1;
  if (q == TQ_GET) {
    o.ref = tv_descend(v, [&](uint64_t j) { return path[j]; }, len);
    *out = o;
    return;
  }
  if (!tv_ref_ok(v, ref)) {
    o.ok = 0;
    *out = o;
    return;
  }
  if (q == TQ_INFO) {
    const bool tomb = tv_is_tomb(v, ref);
    o.kind = ref == REF_ROOT ? 3 : (tomb ? 2 : 1);
    o.val = (ref == REF_ROOT || tomb) ? 0u : v.lval(v.src(ref));
    long long k = 0;
    o.has_next = tv_next_key(v, ref, &k) ? 1 : 0;
    o.next = o.has_next ? k : 0;
    o.n = tv_path_len(v, ref);
    for (uint64_t j = 0; j < o.n && j < pcap; ++j) pbuf[j] = tv_path_at(v, ref, j);
  } else if (q == TQ_REL) {
    switch (which) {
      case CRDTM_REL_PARENT: o.ref = tv_parent(v, ref); break;
      case CRDTM_REL_NEXT: o.ref = tv_next_of(v, ref); break;
      case CRDTM_REL_PREV: o.ref = tv_prev_of(v, ref); break;
      case CRDTM_REL_HEAD: o.ref = tv_head_of(v, ref); break;
      default: o.ok = 0;
    }
  } else {  // CRDTree.Node.children: the live children in chain order
    const DictRef d = tv_children(v, ref);
    const uint64_t s0 = tv_lookup(v, d, 0);
    uint64_t n = 0;
    for (uint64_t x = s0 == REF_NONE ? REF_NONE : tv_next_node(v, s0, d); x != REF_NONE; x = tv_next_node(v, x, d)) {
      if (n < list_cap) list[n] = x;
      ++n;
    }
    o.n = n;
  }
  *out = o;
}

// Per-tree device traversal state: the slot hash of one version, query
// scratch, a pinned result block.
struct DevTrav {
  uint64_t version = ~0ULL;
  SlotHash H{nullptr, nullptr, nullptr, 0};
  uint64_t hcap = 0;
  TravOut* out = nullptr;
  TravOut* hout = nullptr;
  uint64_t* list = nullptr;
  uint64_t list_cap = 0;
  long long* buf = nullptr;  // query path in / node path out
  uint64_t buf_cap = 0;
  ~DevTrav() {
    void* ps[] = {H.dict, H.key, H.slot, out, list, buf};
    for (void* p : ps)
      if (p) hipFree(p);
    if (hout) hipHostFree(hout);
  }
};

int dev_trav(const crdtm_tree* tc, DevTrav*& out) {
  auto* t = const_cast<crdtm_tree*>(tc);
  hipStream_t s = t->ctx->stream;
  HIP_CHECK(hipSetDevice(t->ctx->device));
  auto* c = static_cast<DevTrav*>(t->dtrav.get());
  if (!c) {
    auto p = std::make_shared<DevTrav>();
    HIP_CHECK(hipMalloc(&p->out, sizeof(TravOut)));
    HIP_CHECK(hipHostMalloc(&p->hout, sizeof(TravOut), hipHostMallocDefault));
    t->dtrav = p;
    c = p.get();
  }
  if (c->version != t->version) {
    const uint64_t S = t->n_slots;
    uint64_t H = 1024;
    while (H < 2 * S) H <<= 1;
    if (H > c->hcap) {
      void* ps[] = {c->H.dict, c->H.key, c->H.slot};
      for (void* p : ps)
        if (p) HIP_CHECK(hipFree(p));
      HIP_CHECK(hipMalloc(&c->H.dict, H * sizeof(uint32_t)));
      HIP_CHECK(hipMalloc(&c->H.key, H * sizeof(long long)));
      HIP_CHECK(hipMalloc(&c->H.slot, H * sizeof(uint32_t)));
      c->hcap = H;
    }
    c->H.mask = static_cast<uint32_t>(H - 1);
    HIP_CHECK(hipMemsetAsync(c->H.slot, 0xFF, H * sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_trav_index, dim3(grid_for(S)), dim3(BLOCK), 0, s, t->d, static_cast<uint32_t>(S), c->H);
    HIP_CHECK(hipGetLastError());
    c->version = t->version;
  }
  out = c;
  return CRDTM_OK;
}

template <class T>
int dev_room(T*& p, uint64_t& cap, uint64_t need) {
  if (need <= cap) return CRDTM_OK;
  if (p) HIP_CHECK(hipFree(p));
  p = nullptr;
  const uint64_t n = need + need / 2 + 64;
  HIP_CHECK(hipMalloc(&p, n * sizeof(T)));
  cap = n;
  return CRDTM_OK;
}

// Runs one query; the answer lands in c->hout (and c->list / c->buf on the device).
int dev_query(const crdtm_tree* t, int q, uint64_t ref, int which, const int64_t* path, uint64_t len, uint64_t lcap,
              uint64_t pcap, DevTrav*& c) {
  int r = dev_trav(t, c);
  if (r) return r;
  hipStream_t s = t->ctx->stream;
  if ((r = dev_room(c->buf, c->buf_cap, std::max(len, pcap) + 1))) return r;
  if ((r = dev_room(c->list, c->list_cap, lcap + 1))) return r;
  if (len) HIP_CHECK(hipMemcpyAsync(c->buf, path, len * 8, hipMemcpyHostToDevice, s));
  TvDev v{t->d, c->H, t->n_slots};
  hipLaunchKernelGGL(k_trav, dim3(1), dim3(64), 0, s, v, q, ref, which, c->buf, len, c->out, c->list, lcap, c->buf,
                     pcap);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(c->hout, c->out, sizeof(TravOut), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return CRDTM_OK;
}

// ---- the host view (walk): a copy of the state fetched once per version ----
struct PairHash {
  size_t operator()(const std::pair<uint32_t, long long>& p) const {
    return std::hash<long long>()(p.second * 0x9E3779B97F4A7C15LL ^ static_cast<long long>(p.first));
  }
};

struct TravCache {
  uint64_t version = ~0ULL;
  HostTree h;
  std::unordered_map<std::pair<uint32_t, long long>, uint32_t, PairHash> index;  // (dict, key) -> slot
};

struct TvHost {
  const TravCache* c;
  uint64_t S;
  uint8_t flags(uint64_t s) const { return c->h.flags[s]; }
  uint32_t child(uint64_t s) const { return c->h.child[s]; }
  uint32_t next(uint64_t s) const { return c->h.next[s]; }
  long long key(uint64_t s) const { return c->h.key[s]; }
  uint32_t src(uint64_t s) const { return c->h.src[s]; }
  uint32_t loff(uint32_t i) const { return c->h.l_off[i]; }
  long long lpath(uint32_t j) const { return c->h.l_path[j]; }
  long long lts(uint32_t i) const { return c->h.l_ts[i]; }
  uint32_t lval(uint32_t i) const { return c->h.l_val[i]; }
  uint32_t find(uint32_t d, long long k) const {
    auto it = c->index.find({d, k});
    return it == c->index.end() ? NONE : it->second;
  }
};

int trav_cache(const crdtm_tree* tc, TravCache*& out) {
  auto* t = const_cast<crdtm_tree*>(tc);
  auto* c = static_cast<TravCache*>(t->trav.get());
  if (!c) {
    t->trav = std::make_shared<TravCache>();
    c = static_cast<TravCache*>(t->trav.get());
  }
  if (c->version != t->version) {
    c->h = HostTree();
    int r = fetch(t, c->h, false);
    // the walk follows the copy's indices on the host: an unsound state is
    // CRDTM_E_STATE here, like crdtm_tree_canonical, never a wild read
    if (!r) r = check_state(c->h, t->n_slots, t->n_dicts, t->log_n);
    if (r) {
      c->h = HostTree();
      c->version = ~0ULL;
      return r;
    }
    c->index.clear();
    c->index.reserve(c->h.key.size() * 2);
    for (uint32_t sl = 0; sl < c->h.key.size(); ++sl) c->index[{c->h.dict[sl], c->h.key[sl]}] = sl;
    c->version = t->version;
  }
  out = c;
  return CRDTM_OK;
}

// walkHelp (src/CRDTree.elm:602-625) with a function that always Takes; an
// explicit stack instead of recursion (documents nest arbitrarily deep)
void walk_from(const TvHost& c, uint64_t left, const DictRef& sib, std::vector<uint64_t>& out) {
  std::vector<std::pair<uint64_t, DictRef>> st{{left, sib}};
  while (!st.empty()) {
    auto [l, d] = st.back();
    st.pop_back();
    const uint64_t node = tv_next_node(c, l, d);
    if (node == REF_NONE) continue;
    out.push_back(node);
    st.push_back({node, d});  // then the siblings after node
    const uint64_t h = tv_head_of(c, node);
    if (h != REF_NONE) st.push_back({h, tv_children(c, node)});  // first: node's children after its head
  }
}

int put_refs(const std::vector<uint64_t>& v, uint64_t* out, uint64_t cap, uint64_t* n) {
  for (uint64_t k = 0; out && k < v.size() && k < cap; ++k) out[k] = v[k];
  if (n) *n = v.size();
  return CRDTM_OK;
}

}  // namespace

extern "C" {

int crdtm_tree_get(const crdtm_tree* t, const int64_t* path, uint64_t len, uint64_t* ref) {
  if (!t || !ref || (len && !path)) return CRDTM_E_ARG;
  DevTrav* c;
  int r = dev_query(t, TQ_GET, 0, 0, path, len, 0, 0, c);
  if (r) return r;
  *ref = c->hout->ref;
  return CRDTM_OK;
}

int crdtm_node_info(const crdtm_tree* t, uint64_t ref, int32_t* kind, uint32_t* val, int32_t* has_next,
                    int64_t* next, int64_t* path, uint64_t cap, uint64_t* path_len) {
  if (!t) return CRDTM_E_ARG;
  DevTrav* c;
  const uint64_t pcap = path ? cap : 0;
  int r = dev_query(t, TQ_INFO, ref, 0, nullptr, 0, 0, pcap, c);
  if (r) return r;
  const TravOut o = *c->hout;
  if (!o.ok) return CRDTM_E_ARG;
  if (kind) *kind = o.kind;
  if (val) *val = o.val;
  if (has_next) *has_next = o.has_next;
  if (next) *next = o.next;
  if (path && o.n && cap) HIP_CHECK(hipMemcpy(path, c->buf, std::min(o.n, cap) * 8, hipMemcpyDeviceToHost));
  if (path_len) *path_len = o.n;
  return CRDTM_OK;
}

int crdtm_tree_relative(const crdtm_tree* t, uint64_t ref, int which, uint64_t* out) {
  if (!t || !out) return CRDTM_E_ARG;
  DevTrav* c;
  int r = dev_query(t, TQ_REL, ref, which, nullptr, 0, 0, 0, c);
  if (r) return r;
  if (!c->hout->ok) return CRDTM_E_ARG;
  *out = c->hout->ref;
  return CRDTM_OK;
}

int crdtm_node_children(const crdtm_tree* t, uint64_t ref, uint64_t* out, uint64_t cap, uint64_t* n) {
  if (!t) return CRDTM_E_ARG;
  DevTrav* c;
  const uint64_t lcap = out ? cap : 0;
  int r = dev_query(t, TQ_CHILDREN, ref, 0, nullptr, 0, lcap, 0, c);
  if (r) return r;
  const TravOut o = *c->hout;
  if (!o.ok) return CRDTM_E_ARG;
  if (out && o.n && lcap)
    HIP_CHECK(hipMemcpy(out, c->list, std::min(o.n, lcap) * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (n) *n = o.n;
  return CRDTM_OK;
}

int crdtm_tree_walk(const crdtm_tree* t, uint64_t start, uint64_t* out, uint64_t cap, uint64_t* n) {
  if (!t) return CRDTM_E_ARG;
  TravCache* tc;
  int r = trav_cache(t, tc);
  if (r) return r;
  const TvHost c{tc, tc->h.key.size()};
  std::vector<uint64_t> v;
  uint64_t s = start;
  if (s == REF_NONE) s = tv_head_of(c, REF_ROOT);  // walk ... Nothing: from the root's head
  else if (!tv_ref_ok(c, s)) return CRDTM_E_ARG;
  if (s != REF_NONE) {
    const uint64_t par = tv_parent(c, s);
    if (par != REF_NONE) walk_from(c, s, tv_children(c, par), v);
  }
  return put_refs(v, out, cap, n);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Sharding glue (config 5): after the all-gather of the
// replicas' op logs, put every record of a document this rank owns at its
// place in the document's causal stream, as packed ops (one pass).
// ---------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(BLOCK) k_shard_assemble(const long long* __restrict__ rec, uint64_t n_rec,
                                                          uint32_t rank, uint32_t world, uint64_t per_doc,
                                                          uint64_t n_out, uint8_t* kind, uint32_t* val, long long* ts,
                                                          long long* path, uint32_t* path_off) {
  for (uint64_t r = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; r < n_rec;
       r += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const longlong2 a = reinterpret_cast<const longlong2*>(rec)[2 * r];
    const longlong2 b = reinterpret_cast<const longlong2*>(rec)[2 * r + 1];
    const uint64_t doc = static_cast<uint64_t>(a.x) >> 32, seq = static_cast<uint64_t>(a.x) & 0xFFFFFFFFull;
    if (doc % world != rank || seq >= per_doc) continue;
    const uint64_t dst = (doc / world) * per_doc + seq;
    if (dst >= n_out) continue;
    kind[dst] = static_cast<uint8_t>(static_cast<uint64_t>(a.y) >> 32);
    val[dst] = static_cast<uint32_t>(a.y);
    ts[dst] = b.x;
    path[dst] = b.y;
  }
  for (uint64_t q = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; q <= n_out;
       q += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    path_off[q] = static_cast<uint32_t>(q);  // flat documents: one path element per op
}
}  // namespace

extern "C" {

int crdtm_shard_assemble(crdtm_ctx* c, const int64_t* records, uint64_t n_rec, int32_t rank, int32_t world,
                         uint64_t per_doc, crdtm_ops* out) {
  if (!c || !out || world <= 0 || rank < 0 || rank >= world || (n_rec && !records)) return CRDTM_E_ARG;
  if ((reinterpret_cast<uintptr_t>(records) & 15) != 0) return CRDTM_E_ARG;
  HIP_CHECK(hipSetDevice(c->device));
  hipLaunchKernelGGL(k_shard_assemble, dim3(grid_for(std::max<uint64_t>(n_rec, out->n_ops + 1))), dim3(BLOCK), 0,
                     c->stream, reinterpret_cast<const long long*>(records), n_rec, static_cast<uint32_t>(rank),
                     static_cast<uint32_t>(world), per_doc, out->n_ops, out->kind, out->val,
                     reinterpret_cast<long long*>(out->ts), reinterpret_cast<long long*>(out->path), out->path_off);
  HIP_CHECK(hipGetLastError());
  return CRDTM_OK;
}

}  // extern "C"

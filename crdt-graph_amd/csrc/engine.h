// engine.h — crdtm engine internals: workspace arena, context, tree state,
// and the host-side launch entry points of each kernel family.
#pragma once

#include <memory>
#include <stdexcept>

#include "kernels.h"

namespace crdtm {

struct ArenaOverflow : std::runtime_error {
  size_t need;
  explicit ArenaOverflow(size_t n) : std::runtime_error("arena overflow"), need(n) {}
};

// Bump allocator over one device allocation, reset per call. Overflow throws
// (host side, before any tree mutation); the API layer grows and retries.
struct Arena {
  char* base = nullptr;
  size_t cap = 0;
  size_t used = 0;
  size_t high = 0;
  template <class T>
  T* alloc(uint64_t n) {
    size_t b = (static_cast<size_t>(n) * sizeof(T) + 255) & ~static_cast<size_t>(255);
    if (b == 0) b = 256;
    if (used + b > cap) throw ArenaOverflow(used + b);
    T* p = reinterpret_cast<T*>(base + used);
    used += b;
    if (used > high) high = used;
    return p;
  }
  void reset() { used = 0; }
  // single-pass scans (scan.h): status words tagged with a per-call epoch, so
  // the pool is zeroed once at context creation and never again
  unsigned long long* scan_status = nullptr;
  uint64_t scan_cap = 0;
  uint32_t* scan_ticket = nullptr;
  uint32_t scan_epoch = 0;
  uint32_t* scan_err = nullptr;  // device word every scan reports an exhausted look-back to (DevResult::scan_err)
};

enum : uint8_t { F_TOMB = 1, F_ORPHAN = 2, F_SENT = 4 };

constexpr uint32_t HOST_RANGES = 4096;  // replica ranges scanned on the host

// Device-resident CRDTree state (the "replay representation"): one slot per
// dict entry. Slot s lives in dict s_dict[s] under key s_key[s]; s_next is the
// slot of the entry named by its `next` key (Elm keeps the key; within a dict
// the two are interchangeable); s_src is the op-log index of the Add whose
// path and value the entry carries (a findInsertion copy carries the copied
// node's source); s_child is the children dict of a live Node,
// or NONE for a live Node whose children are still the initial
// {0: Tombstone} (implicit until something descends into it).
struct TreeDev {
  long long* s_key = nullptr;
  uint32_t* s_next = nullptr;
  uint32_t* s_src = nullptr;
  uint32_t* s_child = nullptr;
  uint32_t* s_dict = nullptr;
  uint8_t* s_flags = nullptr;
  uint32_t* d_sent = nullptr;   // dict -> sentinel slot
  uint32_t* d_owner = nullptr;  // dict -> owning slot (NONE for the root dict)
  // operation log, oldest first
  uint8_t* l_kind = nullptr;
  long long* l_ts = nullptr;
  uint32_t* l_val = nullptr;
  uint32_t* l_off = nullptr;
  long long* l_path = nullptr;
  // document order from the last closed-form merge (vis rank -> slot)
  uint32_t* doc = nullptr;
};

struct TreeCaps {
  uint64_t slots = 0, dicts = 0, log = 0, lpath = 0, doc = 0;
};

// Owner of a tree state's device arrays. Versions (crdtm_tree_clone) share
// one store until one of them is mutated (copy on write, api.hip unshare):
// a kept version costs nothing until the next apply to either handle.
struct DevStore {
  TreeDev d;
  ~DevStore();
};

}  // namespace crdtm

struct crdtm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // a second stream for work off the critical path (the flat merge's log
  // copy), forked from and joined back into `stream` with these events
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_sync = nullptr;  // recorded after each result read; the host spins on it (sync_read)
  crdtm::Arena ws;
  // guard-G statistics of the last apply's per-dict replay (CRDTM_GUARD_STATS=1, pdr.hip)
  unsigned long long* gstat_dev = nullptr;
  uint64_t gstat[4] = {0, 0, 0, 0};
  int gstat_valid = 0;
  crdtm::DevResult* dres = nullptr;  // device
  crdtm::DevResult* hres = nullptr;  // pinned host
  // dres holds k_dres_init's values: crdtm_tree_reset's launch set them, and
  // nothing has touched dres since (the flat speculation then skips its own
  // init launch); cleared by every apply, every result read and ops_since
  bool dres_ready = false;
  // pinned host staging for bulk per-call transfers (the forest's per-document
  // tables and results: one DMA each way instead of a pageable copy per array)
  char* pin = nullptr;
  size_t pin_cap = 0;
  uint32_t* rtab = nullptr;          // replica table [REPLICA_SLOTS], 0 = empty (kept clean between calls)
  uint2* crange = nullptr;           // replica counter ranges [RID_SLOTS] {min, max}, kept clean between calls
  // flat merge: slot -> anchor code tagged with the merge's epoch (merge.hip
  // FlatRec); a slot carrying another epoch holds no Add, so no clearing pass
  uint2* fl_rec = nullptr;
  uint64_t fl_cap = 0;
  uint32_t fl_epoch = 0;
  bool profile = false;
  // profiling: one {name, begin, end} event pair per kernel launch
  struct Mark {
    std::string name;
    hipEvent_t begin, end;
  };
  std::vector<Mark> marks;
  hipEvent_t pending = nullptr;  // begin event of the launch in flight
  std::vector<std::pair<std::string, double>> phases;
  void clear_marks() {
    for (auto& m : marks) {
      hipEventDestroy(m.begin);
      hipEventDestroy(m.end);
    }
    marks.clear();
    if (pending) hipEventDestroy(pending);
    pending = nullptr;
  }
  void collect_phases() {  // after a stream synchronisation
    phases.clear();
    for (auto& m : marks) {
      float ms = 0;
      hipEventElapsedTime(&ms, m.begin, m.end);
      phases.emplace_back(m.name, ms);
    }
  }
};

namespace crdtm {
// Index of a clean flat tree for the incremental closed form (incr.hip), owned
// by one tree handle: key -> slot (hash), and the document order as a gapped
// array of blocks (FI_CAP positions each, a quarter full when built):
// slot ids and keys per position (padding positions hold the key +inf),
// entries per block, the smallest key per 64 positions and per 4096, and
// slot -> position. An adds-only batch shifts entries inside the blocks it
// lands in only; a block that would overflow spreads an aligned window of
// up to 64 blocks evenly (a packed-memory array), and only a window that
// cannot take it rebuilds the layout.
struct KeyIndex {
  unsigned long long* keys = nullptr;  // ts ^ INT64_MIN, 0 = empty (TsHash layout)
  uint32_t* vals = nullptr;
  uint32_t mask = 0;
  uint32_t* bent = nullptr;  // [nbk * FI_CAP] slot per position
  long long* bdk = nullptr;  // [nbk * FI_CAP] key per position, +inf = padding
  uint32_t* bcnt = nullptr;  // [nbk] entries per block (>= 1)
  uint32_t* bfirst = nullptr;  // [nbk] a batch's new nodes of the block: sorted range
  uint32_t* bend = nullptr;    //   [bfirst, bend) (both 0 between batches)
  uint32_t* bwin = nullptr;  // [nbk] level + 1 of the rebalance window over the block (0 between batches)
  long long* bmin = nullptr; // [nbk FI_CAP / 64] smallest key per 64 positions
  long long* smin = nullptr; // smallest key per 4096 positions
  long long* tmin = nullptr; // smallest key per 64 superblocks (262,144 positions)
  uint64_t bcap = 0;         // blocks the arrays hold
  uint32_t nbk = 0;          // blocks in use
  uint32_t* rank = nullptr;  // slot -> position
  uint64_t rcap = 0;
  uint32_t* doc2 = nullptr;  // the next dense order (a rebuild's merge)
  uint64_t doc2_cap = 0;
  bool ord_ready = false;  // the blocks describe the tree's document
  ~KeyIndex();
};
// Index of a tree state for the incremental per-dict replay (ilr.hip), owned
// by one tree handle: (dict, key) -> slot hash and per-dict member lists of
// the state, kept current by the replay's own commits (any other commit
// drops it), plus per-slot event times of the batch in flight.
struct IlrIndex {
  SlotHash H{};
  uint32_t hcap = 0;           // hash entries (power of two)
  uint64_t hused = 0;          // entries in use
  uint32_t* dhead = nullptr;   // [dcap] first member slot of each dict
  uint32_t* mnext = nullptr;   // [scap] next member of the slot's dict
  uint32_t* ev = nullptr;      // [4 * scap] per slot: created / deleted / refilled at op, old children (NONE)
  uint32_t* xmap = nullptr;    // [scap] source slot -> its copy, during one deep copy
  uint32_t* dsrc = nullptr;    // [dcap] a dict filled by a deferred copy its lane reads back: the source
  uint4* rec = nullptr;        // [scap] per slot {next, flags, key lo, key hi}: one load per findInsertion step
  uint64_t dcap = 0, scap = 0;
  // the chain order snapshot (chain_snapshot) of the slots [0, snapE) as of
  // `snap_age` batches ago: the walks check every link against the state,
  // so an older snapshot is still exact, its checked runs only shorter
  uint32_t* snapR = nullptr;
  uint32_t* snapG = nullptr;
  uint64_t snap_cap = 0;
  uint32_t snapE = 0, snap_age = 0;
  ~IlrIndex();
};
}  // namespace crdtm

struct crdtm_tree {
  crdtm_ctx* ctx = nullptr;
  crdtm::TreeDev d;
  crdtm::TreeCaps cap;
  uint64_t n_slots = 0, n_dicts = 0, log_n = 0, log_npath = 0, doc_n = 0;
  bool doc_valid = false;
  // the document order is current in kidx's blocks, `doc` is not (incr.hip);
  // linearize() writes `doc` from them
  bool doc_gapped = false;
  uint32_t max_depth = 0;
  int64_t timestamp = 0;
  std::map<int64_t, int64_t> replicas;
  uint64_t last_begin = 0, last_end = 0;
  int last_is_batch = 1;
  std::shared_ptr<crdtm::DevStore> store;  // owns d's arrays; shared by versions until written
  uint64_t version = 0;              // bumped by every state change (apply, reset)
  // incremental re-merge (merge.hip apply_batch): while set, the engine runs
  // the fresh-tree paths over log ++ batch; own-replica Adds of the log are
  // not counted again (own_bias), and no path may write the state before its
  // last check (no speculation, no sequential replay: R_INCR instead)
  bool remerge = false;
  int64_t own_bias = 0;
  // a single root dict of live nodes only (no tombstone, orphan or copy) with
  // `doc` covering every node: the incremental flat closed form (incr.hip) may
  // merge an adds-only batch into it; kidx = its key index while kidx_valid
  bool flat_clean = true;
  std::unique_ptr<crdtm::KeyIndex> kidx;
  bool kidx_valid = false;
  // incremental per-dict replay index (ilr.hip), valid while ilr_valid
  std::unique_ptr<crdtm::IlrIndex> ilr;
  bool ilr_valid = false;
  std::shared_ptr<void> trav;        // traversal cache (api.hip), valid for `version`
  std::shared_ptr<void> dtrav;       // device traversal index (api.hip), valid for `version`
};

namespace crdtm {

// primitives.hip
int scan_excl_u32(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* total, Arena& ws, hipStream_t st);
int segmented_sort(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items,
                   const long long* sort_key, Arena& ws, hipStream_t st, DevResult* dres);
// same, ordering items by descending id (timestamp-slot numbering); segment
// `skip` is left alone (the caller orders it)
int segmented_sort_desc_id(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items, Arena& ws,
                           hipStream_t st, DevResult* dres, uint32_t skip);
// same, explicit keys, segment `skip` left alone (the caller orders it)
int segmented_sort_skip(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items,
                        const long long* sort_key, Arena& ws, hipStream_t st, DevResult* dres, uint32_t skip);
// same, ascending op index (per-dict op lists of pdr.hip)
int segmented_sort_asc_id(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items, Arena& ws,
                          hipStream_t st, DevResult* dres);
// stable LSD radix sort of (key, value) pairs by the low `bits` key bits (primitives.hip)
int radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, const uint32_t* n_dev, uint32_t n_max,
                     uint32_t bits, Arena& ws, hipStream_t st, uint32_t** out_k, uint32_t** out_v,
                     uint32_t* inv = nullptr);
// forest.hip: the flat documents of a forest (slot map + wave replay; fb[d] = 1
// leaves document d to k_forest); vt holds FL_SLOTS (value, ts) pairs per document
constexpr uint32_t FL_SLOTS = 1024;
// Several fills in one launch (primitives.hip k_fill_batch): each region a
// 4-byte aligned pointer, its byte count and a 32-bit pattern (a byte fill
// passes the byte replicated), instead of one hipMemsetAsync per region.
struct FillList {
  static constexpr int MAX = 8;
  void* p[MAX];
  uint64_t bytes[MAX];
  uint32_t pat[MAX];
  int n = 0;
  bool overflow = false;  // (an add past MAX: launch() returns E_ARG, nothing was written past the arrays)
  void add(void* q, uint64_t b, uint32_t v) {
    if (n >= MAX) {
      overflow = true;
      return;
    }
    p[n] = q;
    bytes[n] = b;
    pat[n] = v;
    ++n;
  }
  int launch(hipStream_t s);  // (runs and clears the list; more than MAX regions: E_ARG)
};
// the same for n <= RS_SMALL_MAX pairs (primitives.hip), into (kout, vout); values below
// 2^16, ties of key in value order (stable when the values are the input positions);
// cw: scratch of n rounded up to 1,024 words for the chunked sort (nullptr: one workgroup)
constexpr uint32_t RS_SMALL_MAX = 16384;
int radix_sort_small(const uint32_t* kin, const uint32_t* vin, uint32_t n, uint32_t bits, uint32_t* kout,
                     uint32_t* vout, hipStream_t st, unsigned long long* cw = nullptr);
// ent[e] = {succ, wbits}: see primitives.hip / listrank.h (list_rank_fused)
int list_rank(const uint2* ent, uint64_t n, uint32_t head, unsigned long long* excl, Arena& ws, hipStream_t st);
int list_rank_packed(const uint2* ent, uint64_t n, uint32_t head, unsigned long long* excl, Arena& ws,
                     hipStream_t st);
int list_rank_unpacked(const uint32_t* succ, const unsigned long long* w, uint64_t n, uint32_t head,
                       unsigned long long* excl, Arena& ws, hipStream_t st);

// Device view of one batch of ops.
struct OpsDev {
  uint32_t n = 0;
  uint64_t n_path = 0;
  const uint8_t* kind = nullptr;
  const long long* ts = nullptr;
  const uint32_t* off = nullptr;
  const long long* path = nullptr;
  const uint32_t* val = nullptr;
};

// K1 results handed to the per-dict replay (pdr.hip)
struct PdrIn {
  TsIndex ix;
  const uint32_t* tag;     // PDR_REACHED, the tombstoned node the path stopped at, TAG_LAZY, or NONE
  const uint32_t* cur;     // leaf dict owner (n = root)
  const uint32_t* leaf;    // leaf target: node, SENT_T or MISS_T
  const uint32_t* addpar;  // Adds: dict owner
  const uint32_t* dtime;   // node -> first Delete that tombstoned it
  uint32_t maxlen;
};

// Test hooks (crdtm_debug_poke, fault injection, debug dumps) act only when
// the process sets CRDTM_TEST_HOOKS=1; a production caller never reaches them.
inline bool test_hooks() {
  static const bool on = [] {
    const char* e = getenv("CRDTM_TEST_HOOKS");
    return e && e[0] == '1';
  }();
  return on;
}

// internal: a path that cannot run inside an incremental re-merge asks the
// caller to replay the batch incrementally on the untouched state instead
constexpr int R_INCR = 1 << 20;

// merge.hip
int sync_read(crdtm_ctx* c);
// replicas[replicaId t] := t over the applied ops (st) into `rep`; collected by take_replicas after a sync
// (zeroed: the caller's own kernel has cleared DevResult::n_replica_out / n_rep_list)
int replica_fold(crdtm_ctx* c, const OpsDev& o, const uint8_t* st, long long* rep, Arena& ws, hipStream_t s,
                 bool zeroed = false);
// forest.hip (FL_SLOTS above)
int forest_flat_launch(const OpsDev& o, const uint32_t* doff, uint32_t n_docs, long long ts0, uint32_t* opw,
                       uint16_t* sent, uint8_t* fb, longlong2* vt, int32_t* code, uint32_t* err, uint32_t* applied,
                       unsigned long long* vhash, unsigned long long* vwords, long long* tstamp,
                       uint32_t* overflow, hipStream_t s);
int replica_fold_into(crdtm_ctx* c, const OpsDev& o, const uint8_t* st, long long* rep, uint32_t* rlist,
                      hipStream_t s, bool zeroed = false);
int take_replicas(crdtm_tree* t, const long long* rep_dev);
// incr.hip: adds-only flat batch into a clean flat tree; *handled = false leaves it to apply_batch
int finc_apply(crdtm_tree* t, const OpsDev& o, uint8_t* st_out, crdtm_result* res, bool* handled);
// ilr.hip: a batch into a tree that holds state, replayed per children dict on the
// state itself; *handled = false leaves it to the re-merge (nothing written)
int ilr_apply(crdtm_tree* t, const OpsDev& o, uint8_t* st_out, crdtm_result* res, bool* handled);
bool ilr_wanted(const crdtm_tree* t, uint32_t n);
// merge.hip helpers shared with ilr.hip
void launch_pre(crdtm_ctx* c, const OpsDev& o, hipStream_t s);
// Resets the context's replica range table entries 0..nr-1 (nr = 0: the
// ones k_pre touched, read from the DevResult — valid only until the next
// DevResult reset, so callers pass nr once they have read max_replica).
void range_reset(crdtm_ctx* c, uint32_t nr);
// Launches range_reset when a merge leaves by any path. (`armed` is cleared
// when the merge reset the table itself, stream-ordered before its final
// result read, and set again if it had to rebuild it)
struct RangeReset {
  crdtm_ctx* c;
  bool armed = true;
  uint32_t nr = 0;
  void now() {
    range_reset(c, nr);
    armed = false;
  }
  ~RangeReset() {
    if (armed) now();
  }
};
__global__ void k_dres_init(DevResult* d);
__global__ void k_path_range(OpsDev o, DevResult* dres);
__global__ void k_post_flags(OpsDev o, const uint8_t* st, uint32_t* appl, uint32_t* plen);
__global__ void k_log(OpsDev o, const uint8_t* st, TreeDev T, uint32_t log_base, uint32_t lpath_base,
                      const uint32_t* appl, const uint32_t* plen);
__global__ void k_log_tail(TreeDev T, uint32_t log_base, const uint32_t* n_app, uint32_t lpath_base,
                           const uint32_t* np);
__global__ void k_status_out(const uint8_t* st, uint32_t n, uint32_t err, uint8_t* out);
__global__ void k_replay_index(TreeDev T, uint32_t n_slots, SlotHash H, uint32_t* dhead, uint32_t* mnext);
__global__ void k_reset_root(uint32_t* s_next, DevResult* d);
// each group's first position in sorted keys (NONE: no group) (merge.hip)
__global__ void k_doc_gstart(const uint32_t* sk, uint32_t m, uint32_t* gs);
int post_pass(crdtm_tree* t, const OpsDev& o, const uint8_t* st, Arena& ws);
// pdr.hip
int pdr_apply(crdtm_tree* t, const OpsDev& o, const PdrIn& in, uint8_t* st, crdtm_result* res, bool* handled);
// merge.hip
int grow_tree(crdtm_tree* t, const TreeCaps& need);
// copy on write (DevStore): a private copy of the state before it is written
int unshare_tree(crdtm_tree* t, bool keep_contents);
int apply_batch(crdtm_tree* t, const OpsDev& ops, uint8_t* status_dev, crdtm_result* res);
int linearize(crdtm_tree* t);  // fills t->d.doc / t->doc_n from the tree state
// chain positions of the state's dict entries, every dict's chain
// consecutive (R: slot -> position, NONE for an orphan; G: position -> slot),
// both sized n_slots
int chain_snapshot(crdtm_tree* t, uint32_t* R, uint32_t* G, Arena& ws, hipStream_t s);
int fi_materialize(crdtm_tree* t);  // incr.hip: `doc` from the gapped order (doc_gapped)
int forest_apply(crdtm_ctx* c, int64_t replica_id, const OpsDev& o, const uint32_t* doc_off_host, uint64_t n_docs,
                 int32_t* code, int64_t* err, uint32_t* applied, uint64_t* vhash, uint64_t* vwords, int64_t* tstamp);
uint64_t forest_ws_bytes(const uint32_t* doc_off_host, uint64_t n_docs, uint64_t n_ops, uint64_t n_path);
void mark_begin(crdtm_ctx* c, hipStream_t st);
void mark(crdtm_ctx* c, const char* name, hipStream_t st);
// Profiling hook: when the current context profiles, every launch is
// bracketed by two HIP events on the launch stream, so each kernel's device
// time is measured on its own (no host gaps between launches).
extern thread_local crdtm_ctx* g_prof;
inline void prof_begin(hipStream_t st) {
  if (g_prof) mark_begin(g_prof, st);
}
inline void prof_mark(const char* name, hipStream_t st) {
  if (g_prof) mark(g_prof, name, st);
}
// Host wait for everything queued on stream s by polling an event (a
// blocking stream synchronisation sleeps and wakes ~15 us late, idling the
// device between the phases of a merge). One event per host thread and
// device (the caller has made the stream's device current); the poll loop
// pauses between queries so a waiting thread does not hammer the runtime.
inline void spin_pause() { __builtin_ia32_pause(); }
inline int stream_wait(hipStream_t s) {
  constexpr int MAXDEV = 64;
  static thread_local hipEvent_t ev[MAXDEV] = {};
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= MAXDEV) {
    HIP_CHECK(hipStreamSynchronize(s));
    return CRDTM_OK;
  }
  if (!ev[dev]) HIP_CHECK(hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming));
  HIP_CHECK(hipEventRecord(ev[dev], s));
  for (;;) {
    const hipError_t e = hipEventQuery(ev[dev]);
    if (e == hipSuccess) return CRDTM_OK;
    if (e != hipErrorNotReady) HIP_CHECK(e);
    spin_pause();
  }
}

#define LAUNCH(k, grid, block, shm, st, ...)                    \
  do {                                                          \
    ::crdtm::prof_begin(st);                                    \
    hipLaunchKernelGGL(k, grid, block, shm, st, __VA_ARGS__);   \
    ::crdtm::prof_mark(#k, st);                                 \
  } while (0)

}  // namespace crdtm

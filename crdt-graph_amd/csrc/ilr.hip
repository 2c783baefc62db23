// ilr.hip — incremental merge into a tree that already holds state, replayed
// per children dict on the state itself ("ILR": incremental level replay).
//
// `apply batch state` (src/CRDTree.elm:265-269) applies the batch's ops in
// order with the literal addAfterHelp / findInsertion / deleteHelp semantics
// (src/Internal/Node.elm:56-163). Ops that land in different children dicts
// interact only through path resolution (update, :138-163): an op's path
// crosses the nodes of shallower dicts. So the batch is grouped by the dict
// it lands in — ops with path length L and the same owner key path[L-2] (the
// root dict for L = 1) — and replayed level by level (L = 1, 2, ...), one
// lane per group and the group's ops in batch order, on the tree state's own
// slots. When level L runs, every shallower dict holds its whole batch, so an
// op i resolves its path "as of op i" through per-slot event times recorded
// by the shallower levels: a node created by op j exists for i only if j < i,
// one deleted by op j is a Tombstone for i only if j < i (its children stay
// in place until the commit, for the ops before the Delete), one the copy
// quirk re-filled at op j is live (with the copied children) only if j < i.
// Inside a group's dict only that group writes, so the dict is exactly at
// op i when op i runs.
//
// Paths are resolved for all ops of a level in parallel before its lanes run
// (the lanes then only touch their own dicts). A copy quirk whose copied
// node has batch activity below it needs the node's children as of the
// quirk: it becomes a deferred copy, made by the lane that owns those
// children at the next level when it passes the quirk's op; the lanes of
// ops landing in the copy run in a second phase of that level. A slot may
// carry a Delete and a re-fill (either order).
//
// What this order cannot decide sends the batch to the re-merge (merge.hip
// apply_batch_paths; nothing is written): a slot with three events, an op
// landing under a deleted-then-refilled node before its Delete, a deferred
// copy whose source has no lane or activity two levels down, a lane that is
// both the source and the target of deferred copies. Any error (the first
// failing op in batch order is exact: each op only sees earlier ops) rolls
// the state back
// through per-group undo logs. Each group takes its Adds' slots from a range
// reserved for it (a prefix sum over the groups; an Add that does not apply
// leaves a dead slot in a dict nothing reaches); materialised sentinels,
// deep copies and dicts come from device counters. The slots' sources are op
// indices (tagged) until the commit turns them into log indices. Per batch:
// O(batch) work — grouping, the levels, and a commit that visits only the
// new slots and the undo entries; the (dict, key) -> slot hash, the dict
// member lists and the event times persist with the tree handle.
//
// Visibility: the groups of one level run as concurrent workgroups spread
// over the XCDs, whose L2s are not coherent with each other inside a kernel.
// So nothing one lane writes is read by another lane of the same launch: a
// lane writes only the slots of its own dict (and of dicts it creates), and
// the slots it creates go to a table of its own (per group, in the arena),
// published into the shared (dict, key) hash by a separate kernel after the
// level. During a level the shared hash is read-only.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "engine.h"
#include "scan.h"

namespace crdtm {

IlrIndex::~IlrIndex() {
  if (H.dict) hipFree(H.dict);
  if (H.key) hipFree(H.key);
  if (H.slot) hipFree(H.slot);
  if (dhead) hipFree(dhead);
  if (mnext) hipFree(mnext);
  if (ev) hipFree(ev);
  if (xmap) hipFree(xmap);
  if (dsrc) hipFree(dsrc);
  if (snapR) hipFree(snapR);
  if (snapG) hipFree(snapG);
  if (rec) hipFree(rec);
}

constexpr uint32_t ILR_TAG = 0x80000000u;  // s_src of this batch: ILR_TAG | op index
constexpr uint32_t ILR_MAXL = 64;          // deeper paths: the re-merge
constexpr uint32_t EVW = 4;                // event words per slot
constexpr uint32_t EV_CRE = 0, EV_DEL = 1, EV_CPY = 2, EV_OCH = 3;
constexpr uint32_t IMPLICIT = 0xFFFFFFFEu;  // a live node's children still the implicit {0: Tombstone}
constexpr uint32_t ST_CONFLICT = 0xFF;     // (prep: the batch goes to the re-merge)
constexpr uint32_t LV_PTOT = ILR_MAXL + 1, LV_QTOT = ILR_MAXL + 2, LV_N = ILR_MAXL + 4;
constexpr uint32_t ILR_JOBS = 4;  // deferred copies one lane makes
constexpr uint32_t COPY_POOL = 32;  // slots a lane takes from the counter at a time (copies, sentinels)
constexpr uint32_t PT_LDS = 2048;   // private tables up to this size live in LDS (32 KB)
constexpr uint32_t ILR_LREC = 1024;  // LDS mirror of a lane's first reserved slots' records (16 KB)

// conflict reasons (DevResult::ilr_why) and overflow reasons (ilr_overflow)
enum : uint32_t {
  IW_EVENTS = 1,      // a slot with a third event
  IW_COPY_BELOW = 2,  // a deferred copy two levels down, or with no lane at its level
  IW_REFILL = 4,      // an op lands under a deleted-then-refilled node before the Delete
  IW_CHAIN = 8,       // a lane both source and target of deferred copies (or > ILR_JOBS)
  IW_DEPTH = 16,      // a deep copy deeper than ILR_MAXL
  IW_PENDING = 32     // a copy of a dict a deferred copy of this batch makes
};
// dsrc of a dict a deferred copy fills (other lanes never read such a dict
// in the batch: its filling lane may run in the same launch)
constexpr uint32_t DS_PENDING = 0xFFFFFFFEu;
enum : uint32_t { IO_SLOTS = 1, IO_DICTS = 2, IO_UNDO = 4, IO_PRIV = 8, IO_JOBS = 16 };
enum : uint32_t { IF_NEXT = 0, IF_SRC = 1, IF_CHILD = 2, IF_FLAGS = 3 };
enum : uint32_t { GF_SRC = 1, GF_DST = 2 };

// per group of m ops with `adds` Adds: private table entries (at most half
// used: its nodes and materialised sentinels), undo triples and their offset
__host__ __device__ inline uint32_t ilr_pcap(uint32_t adds) {
  uint32_t p = 16;
  while (p < 2 * (adds + 2)) p <<= 1;
  return p;
}
__host__ __device__ inline uint32_t ilr_ucap(uint32_t m) { return 3 * m + 8; }
__host__ __device__ inline uint64_t ilr_uoff(uint32_t gbeg, uint32_t g) { return 3ULL * gbeg + 8ULL * g; }

// a level's ops, resolved before its lanes (per sorted position)
// (everything a lane needs of an op, packed so it loads the next op's while
// it works on this one)
struct IlrPrep {
  uint4* w1;  // {op index, kind | res << 8, landing dict (or IMPLICIT), its owner slot (NONE: the root dict)}
              //   res: ST_APPLIED (lands), ST_ALREADY / ST_INVALID (stops on the way), ST_CONFLICT
  uint4* w2;  // {ts lo, ts hi, last path key lo, hi} (the anchor / the Delete's target)
  uint2* w3;  // {slot of ts in d, slot of the last key in d} before this level (NONE: absent)
};

struct IlrJobs {
  uint32_t* own;   // the copied node (its children as of `at` are copied)
  uint32_t* dst;   // the copy's dict (children of the re-filled slot)
  uint32_t* at;    // the quirk's op
  uint32_t* next;  // per group list
  uint32_t* head;  // [groups] first job of the group that owns the source
  uint8_t* same;   // the copy's ops are in the source's group (its lane looks the copy up through xmap)
  uint8_t* gflag;  // [groups] GF_SRC / GF_DST
  uint32_t* freel; // jobs whose source no op of the level reaches (one lane copies them first)
  uint32_t cap;
};

struct IlrArgs {
  TreeDev T;
  SlotHash H;
  uint32_t* dhead;
  uint32_t* mnext;
  uint32_t* ev;  // [EVW * scap]
  uint32_t* xmap;
  uint4* rec;    // [scap] {next, flags, key}: a copy of the walked fields (IlrIndex::rec)
  uint32_t scap;
  uint32_t committed;  // slots of the state before the batch
  uint32_t cap_slots, cap_dicts;
  uint32_t hash_limit;  // entries the shared hash may hold
  // (depth, key) of every node some op's path crosses (activity below a node)
  const unsigned long long* tk;
  uint32_t tk_mask;
  long long ts0;
  DevResult* dr;
  // per group: its private table (dict, key) -> slot over pk/pd/ps[poff[g], + pcap[g])
  long long* pk;
  uint32_t* pd;
  uint32_t* ps;
  const uint32_t* poff;
  const uint32_t* pcap;
  // per group: its reserved Add slots [committed + qoff[g], + qn[g])
  const uint32_t* qoff;
  const uint32_t* qn;
  // per group: undo triples (slot, field, old) at ilr_uoff, ucnt[g] used
  uint32_t* undo;
  uint32_t* ucnt;
  uint32_t grave;  // the dead dict of this batch's unused reserved slots
  IlrPrep P;
  IlrJobs J;
  // chain order of the state at the batch's start (chain_snapshot, merge.hip):
  // slot -> position and position -> slot (nullptr: none taken)
  const uint32_t* R;
  const uint32_t* G;
  uint32_t E;
  uint32_t* dsrc;    // [dicts] a copy made by a same-group deferred copy: its source dict (else NONE)
  uint32_t dnew;     // dicts of the state before the batch
  unsigned long long* stats;  // (CRDTM_ILR_STATS: per group ops, walk steps, tombstone skips, quirks, marks, ticks)
  // (CRDTM_ILR_OFF: bits switching lane shortcuts off, for bisecting — 1 the
  // LDS private table, 2 the LDS records, 4 the record cache, 8 the recent
  // keys, 16 the member-head cache)
  uint32_t off;
};

__device__ __forceinline__ unsigned long long ilr_tk_key(uint32_t depth, long long key) {
  return ((static_cast<unsigned long long>(depth) << 54) | (static_cast<unsigned long long>(key + TWO53))) + 1ULL;
}
__device__ __forceinline__ uint32_t ilr_hash64(unsigned long long k, uint32_t mask) {
  return static_cast<uint32_t>(mix64(k)) & mask;
}
__device__ void ilr_set_insert(unsigned long long* t, uint32_t mask, unsigned long long k) {
  uint32_t p = ilr_hash64(k, mask);
  for (;;) {
    const unsigned long long prev = atomicCAS(&t[p], 0ULL, k);
    if (prev == 0ULL || prev == k) return;
    p = (p + 1) & mask;
  }
}
// position of key k in an insert-only set, or NONE
__device__ uint32_t ilr_set_pos(const unsigned long long* t, uint32_t mask, unsigned long long k) {
  uint32_t p = ilr_hash64(k, mask);
  for (;;) {
    const unsigned long long v = t[p];
    if (v == k) return p;
    if (v == 0ULL) return NONE;
    p = (p + 1) & mask;
  }
}
__device__ __forceinline__ bool ilr_set_has(const unsigned long long* t, uint32_t mask, unsigned long long k) {
  return ilr_set_pos(t, mask, k) != NONE;
}

// Slot s as of op i, from the events of the shallower levels: 0 = a live node
// (its children dict in *child, NONE = implicit), 1 = a Tombstone, 2 = not
// created yet, 3 = undecidable. *hi = min(*hi, the next event after i).
__device__ __forceinline__ uint32_t ilr_slot_state(const IlrArgs& a, uint32_t s, uint32_t i, uint32_t* child,
                                                   uint32_t* hi) {
  const uint32_t* e = a.ev + static_cast<uint64_t>(EVW) * s;
  const uint32_t cr = e[EV_CRE], de = e[EV_DEL], cp = e[EV_CPY];
  if (cr != NONE && cr > i) *hi = min(*hi, cr);
  if (de != NONE && de > i) *hi = min(*hi, de);
  if (cp != NONE && cp > i) *hi = min(*hi, cp);
  if (cr != NONE && cr > i) return 2;
  bool live;
  uint32_t c = a.T.s_child[s];
  if (de != NONE && cp != NONE) {
    if (de < cp) {  // deleted, then re-filled by the copy quirk: its old children before the Delete
      live = i < de || i > cp;
      if (i < de) c = e[EV_OCH];
    } else {  // re-filled, then deleted
      live = i > cp && i < de;
    }
  } else if (de != NONE) {
    live = i < de;
  } else if (cp != NONE) {
    live = i > cp;
  } else {
    live = !(a.T.s_flags[s] & F_TOMB);
  }
  *child = c;
  return live ? 0u : 1u;
}

// One group's lane: the Replayer's literal semantics (merge.hip) on the
// shared state, with event times, reserved slots, a private table and an
// undo log of its own.
struct IlrLane {
  IlrArgs a;
  bool bad;  // overflow or conflict: the batch goes to the re-merge
  uint32_t depth;  // of the group's dicts (= the level)
  long long* pk;
  uint32_t* pd;
  uint32_t* ps;
  uint32_t pmask, pused;
  uint32_t qnext, qend;
  uint32_t* un;
  uint32_t ucap, ucnt;
  // this lane's reserved slots' records mirrored in LDS (the walks of a busy
  // dict run mostly over the text its own earlier ops inserted)
  uint4* lrec;
  uint32_t lbase, lcnt;
  // slots for deep copies, taken from the counter COPY_POOL at a time
  uint32_t cpnext, cpend;
  // the head of the member list of the dict this lane last wrote
  uint32_t hd_d, hd_v;
  // and the last record read from the state (a typist's next character
  // walks from the entry the previous one stopped at: a global load after
  // this op's stores waits for them)
  uint32_t cs;
  uint4 cr;
  __device__ uint4 getrec(uint32_t s) {
    if (s - lbase < lcnt) return lrec[s - lbase];
    if (s == cs && !(a.off & 4)) return cr;
    cr = a.rec[s];
    cs = s;
    return cr;
  }
  __device__ void rec_next(uint32_t s, uint32_t v) {
    a.rec[s].x = v;
    if (s - lbase < lcnt) lrec[s - lbase].x = v;
    if (s == cs) cr.x = v;
  }
  __device__ void rec_flags(uint32_t s, uint32_t v) {
    a.rec[s].y = v;
    if (s - lbase < lcnt) lrec[s - lbase].y = v;
    if (s == cs) cr.y = v;
  }

  __device__ uint32_t& ev(uint32_t s, uint32_t k) { return a.ev[static_cast<uint64_t>(EVW) * s + k]; }
  // (the lanes of a group's wave all run the replay on the same values: one
  // lane makes each atomic and the others take its result)
  __device__ static uint32_t wave_add(uint32_t* p, uint32_t v) {
    uint32_t r = 0;
    if ((threadIdx.x & 63) == 0) r = atomicAdd(p, v);
    return __shfl(r, 0);
  }
  __device__ void conflict(uint32_t why) {
    if ((threadIdx.x & 63) == 0) {
      atomicOr(&a.dr->ilr_why, why);
      atomicOr(&a.dr->ilr_conflict, 1u);
    }
    bad = true;
  }
  __device__ void overflow(uint32_t why) {
    if ((threadIdx.x & 63) == 0) atomicOr(&a.dr->ilr_overflow, why);
    bad = true;
  }
  // (dict, key) -> slot among the slots this lane created in this level
  __device__ uint32_t pfind(uint32_t d, long long k) const {
    for (uint32_t p = slothash_pos(d, k, pmask);; p = (p + 1) & pmask) {
      const uint32_t v = ps[p];
      if (v == NONE) return NONE;
      if (pd[p] == d && pk[p] == k) return v;
    }
  }
  // a dict this lane filled by a deferred copy: its entries are the source's
  // as of the copy (through xmap) or this lane's own later slots
  __device__ uint32_t copy_src(uint32_t d) const {
    if (d < a.dnew) return NONE;
    const uint32_t v = a.dsrc[d];
    return v == DS_PENDING ? NONE : v;
  }
  // a dict of this batch made by a deferred copy (pending or done)
  __device__ bool job_made(uint32_t d) const { return d >= a.dnew && a.dsrc[d] != NONE; }
  __device__ uint32_t via_copy(uint32_t d, uint32_t src, long long k) const {
    uint32_t s = pfind(src, k);
    if (s == NONE) s = slothash_find(a.H, src, k);
    if (s == NONE) return NONE;
    const uint32_t x = a.xmap[s];
    return (x < a.scap && a.T.s_dict[x] == d && a.T.s_key[x] == k) ? x : NONE;
  }
  // ... then the shared hash (everything before this level, or this phase)
  __device__ uint32_t find(uint32_t d, long long k) const {
    uint32_t v = pfind(d, k);
    if (v != NONE) return v;
    const uint32_t src = copy_src(d);
    if (src != NONE && (v = via_copy(d, src, k)) != NONE) return v;
    return slothash_find(a.H, d, k);
  }
  __device__ void log_undo(uint32_t s, uint32_t field, uint32_t old) {
    if (s >= a.committed) return;
    if (ucnt >= ucap) {
      overflow(IO_UNDO);
      return;
    }
    un[3 * ucnt] = s;
    un[3 * ucnt + 1] = field;
    un[3 * ucnt + 2] = old;
    ++ucnt;
  }
  __device__ void set_next(uint32_t s, uint32_t old, uint32_t v) {
    log_undo(s, IF_NEXT, old);
    a.T.s_next[s] = v;
    rec_next(s, v);
  }
  __device__ void set_src(uint32_t s, uint32_t v) { log_undo(s, IF_SRC, a.T.s_src[s]); a.T.s_src[s] = v; }
  __device__ void set_child(uint32_t s, uint32_t v) { log_undo(s, IF_CHILD, a.T.s_child[s]); a.T.s_child[s] = v; }
  __device__ void set_flags(uint32_t s, uint32_t old, uint32_t v) {
    log_undo(s, IF_FLAGS, old);
    a.T.s_flags[s] = static_cast<uint8_t>(v);
    rec_flags(s, v);
  }

  // a new slot: an Add's from the group's reserved range, others from the counter
  __device__ uint32_t take_slot(bool reserved, bool bulk = false) {
    uint32_t s;
    if (reserved && qnext < qend) {
      s = qnext++;
    } else if (!bulk) {
      s = wave_add(&a.dr->ilr_slots, 1u);
    } else {
      if (cpnext == cpend) {
        cpnext = wave_add(&a.dr->ilr_slots, COPY_POOL);
        cpend = cpnext + COPY_POOL;
      }
      s = cpnext++;
    }
    if (s >= a.cap_slots || s >= a.scap || s + 1 > a.hash_limit) {
      overflow(IO_SLOTS);
      return NONE;
    }
    return s;
  }
  // a slot nothing will use: a dead entry of the batch's dead dict
  __device__ void put_dead(uint32_t x) {
    a.T.s_key[x] = x;
    a.T.s_dict[x] = a.grave;
    a.T.s_next[x] = NONE;
    a.T.s_src[x] = NONE;
    a.T.s_child[x] = NONE;
    a.T.s_flags[x] = F_TOMB | F_ORPHAN;
    a.rec[x] = make_uint4(NONE, F_TOMB | F_ORPHAN, x, 0u);
    *reinterpret_cast<uint4*>(a.ev + static_cast<uint64_t>(EVW) * x) = make_uint4(NONE, NONE, NONE, NONE);
    a.mnext[x] = NONE;
  }
  // the pool's unused slots (they were counted: the commit keeps them)
  __device__ void retire_pool() {
    const uint32_t e = min(min(cpend, a.cap_slots), a.scap);
    for (uint32_t x = cpnext; x < e; ++x) put_dead(x);
    cpnext = cpend;
  }
  // slot s into dict d (a dict this lane writes); `priv`: later ops of this
  // lane may look it up (its nodes and sentinels; copies are reached by
  // other lanes only, through the shared hash)
  __device__ void put_slot(uint32_t s, uint32_t d, long long key, uint32_t next, uint32_t src, uint32_t child,
                           uint8_t flags, uint32_t at, bool priv) {
    a.T.s_key[s] = key;
    a.T.s_dict[s] = d;
    a.T.s_next[s] = next;
    a.T.s_src[s] = src;
    a.T.s_child[s] = child;
    a.T.s_flags[s] = flags;
    const uint4 r4 = make_uint4(next, flags, static_cast<uint32_t>(key), static_cast<uint32_t>(key >> 32));
    a.rec[s] = r4;
    if (s - lbase < lcnt) lrec[s - lbase] = r4;
    if (s == cs) cr = r4;
    static_assert(EVW == 4 && EV_CRE == 0 && EV_DEL == 1 && EV_CPY == 2 && EV_OCH == 3, "one 16-byte store");
    *reinterpret_cast<uint4*>(a.ev + static_cast<uint64_t>(EVW) * s) = make_uint4(at, NONE, NONE, NONE);
    if (priv) {
      if (2 * (pused + 1) > pmask + 1) {
        overflow(IO_PRIV);
        return;
      }
      uint32_t p = slothash_pos(d, key, pmask);
      while (ps[p] != NONE) p = (p + 1) & pmask;
      pd[p] = d;
      pk[p] = key;
      ps[p] = s;
      ++pused;
    }
    a.mnext[s] = (d == hd_d && !(a.off & 16)) ? hd_v : a.dhead[d];
    a.dhead[d] = s;
    hd_d = d;
    hd_v = s;
  }
  __device__ uint32_t new_dict(uint32_t owner) {
    const uint32_t d = wave_add(&a.dr->ilr_dicts, 1u);
    if (d >= a.cap_dicts) {
      overflow(IO_DICTS);
      return NONE;
    }
    a.dhead[d] = NONE;
    hd_d = d;
    hd_v = NONE;
    a.dsrc[d] = NONE;
    a.T.d_owner[d] = owner;
    a.T.d_sent[d] = NONE;
    return d;
  }
  // a sentinel into dict dd (emptyChildren, src/Internal/Node.elm:46-48)
  __device__ bool put_sentinel(uint32_t dd, uint32_t at, bool priv) {
    const uint32_t ss = take_slot(false);
    if (ss == NONE) return false;
    put_slot(ss, dd, 0, NONE, NONE, NONE, F_TOMB | F_SENT, at, priv);
    a.T.d_sent[dd] = ss;
    return !bad;
  }
  // the children dict of live node s, created on first use: its sentinel
  // only; it has always been there for earlier ops (no creation time)
  __device__ uint32_t materialise(uint32_t s) {
    const uint32_t dd = new_dict(s);
    if (dd == NONE || !put_sentinel(dd, NONE, true)) return NONE;
    set_child(s, dd);
    return bad ? NONE : dd;
  }
  // Persistent copy of dict `src` (at depth d0) and every dict below it into
  // `dst` (depth-first over an explicit stack). Nothing below a copied
  // member may have batch activity (its children would be needed as of
  // `at`, from a later level). xmap maps each source slot to its copy.
  // With `defer`, a member of `src` itself with activity below gets an empty
  // children dict and a deferred copy for the next level instead.
  __device__ void deep_copy(uint32_t src, uint32_t dst, uint32_t at, uint32_t d0, bool defer = false) {
    uint32_t stk_s[ILR_MAXL], stk_d[ILR_MAXL], stk_m[ILR_MAXL];
    // a dict without a sentinel is the target of a deferred copy still to
    // run (a quirk re-filled a slot whose children are such a copy): its
    // contents as of `at` are not there yet
    if (a.T.d_sent[src] == NONE || job_made(src)) {
      conflict(IW_PENDING);
      return;
    }
    int sp = 0;
    stk_s[0] = src;
    stk_d[0] = dst;
    stk_m[0] = a.dhead[src];
    while (sp >= 0 && !bad) {
      const uint32_t sd = stk_s[sp], dd = stk_d[sp], m = stk_m[sp];
      if (m == NONE) {  // every member copied: the `next` links inside the copy
        for (uint32_t q = a.dhead[sd]; q != NONE; q = a.mnext[q]) {
          const uint32_t nx = a.T.s_next[q];
          if (nx != NONE) {
            a.T.s_next[a.xmap[q]] = a.xmap[nx];
            rec_next(a.xmap[q], a.xmap[nx]);
          }
        }
        --sp;
        continue;
      }
      stk_m[sp] = a.mnext[m];
      const uint8_t fl = a.T.s_flags[m];
      const uint32_t nm = take_slot(false, true);
      if (nm == NONE) return;
      put_slot(nm, dd, a.T.s_key[m], NONE, a.T.s_src[m], NONE, fl, at, false);
      a.xmap[m] = nm;
      if (fl & F_SENT) a.T.d_sent[dd] = nm;
      const uint32_t c = a.T.s_child[m];
      const bool below = !(fl & F_TOMB) && ilr_set_has(a.tk, a.tk_mask, ilr_tk_key(d0 + sp, a.T.s_key[m]));
      if (below) {
        if (!defer || sp != 0) {
          conflict(IW_COPY_BELOW);
          return;
        }
        const uint32_t nc = new_dict(nm);
        if (nc == NONE || !add_job(m, nc, at)) return;
        a.T.s_child[nm] = nc;
        continue;
      }
      if (c != NONE && !(fl & F_TOMB)) {  // (a Tombstone has no children, :237-238)
        const uint32_t nc = new_dict(nm);
        if (nc == NONE) return;
        a.T.s_child[nm] = nc;
        if (sp + 1 >= static_cast<int>(ILR_MAXL)) {  // (deeper than any path the engine accepts)
          conflict(IW_DEPTH);
          return;
        }
        if (a.T.d_sent[c] == NONE || job_made(c)) {
          conflict(IW_PENDING);
          return;
        }
        ++sp;
        stk_s[sp] = c;
        stk_d[sp] = nc;
        stk_m[sp] = a.dhead[c];
      }
    }
  }
  // a deferred copy of node's children as of op `at`, for the next level
  __device__ bool add_job(uint32_t node, uint32_t dst, uint32_t at) {
    const uint32_t j = wave_add(&a.dr->ilr_jobs, 1u);
    if (j >= a.J.cap) {
      overflow(IO_JOBS);
      return false;
    }
    a.J.own[j] = node;
    a.J.dst[j] = dst;
    a.J.at[j] = at;
    a.dsrc[dst] = DS_PENDING;
    return true;
  }
  // run a deferred copy: node's children (a dict of this lane, now exactly as
  // of op `at`, or one no op of this level reaches) into dict dst; `same`:
  // this lane's later ops land in the copy (they find it through xmap)
  __device__ void run_job(uint32_t node, uint32_t dst, uint32_t at, bool same) {
    const uint32_t c = a.T.s_child[node];
    if (c == NONE) {
      put_sentinel(dst, at, same);
      return;
    }
    if (same) a.dsrc[dst] = c;
    deep_copy(c, dst, at, depth, true);
  }
};

// ---- grouping ----
// per op: its group key in the group hash (L, owner key), the sort key
// (L << gbits | group slot), the crossed (depth, key) pairs; empty paths are
// InvalidPath (update [], src/Internal/Node.elm:147-148) and sort first
__global__ void __launch_bounds__(BLOCK) k_ilr_group(OpsDev o, unsigned long long* gk, uint32_t gmask, uint32_t gbits,
                                                     unsigned long long* tk, uint32_t tk_mask, uint32_t* skey,
                                                     uint32_t* sval, uint8_t* st, DevResult* dr) {
  GRID_STRIDE(i, o.n) {
    const uint32_t b = o.off[i], L = o.off[i + 1] - b;
    sval[i] = i;
    if (L == 0) {
      st[i] = ST_INVALID;
      atomicMin(&dr->err_index, i);
      skey[i] = 0;
      continue;
    }
    const long long owner = L >= 2 ? o.path[b + L - 2] : 0;
    const unsigned long long k = ilr_tk_key(L, owner);
    uint32_t p = ilr_hash64(k, gmask);
    for (;;) {
      const unsigned long long prev = atomicCAS(&gk[p], 0ULL, k);
      if (prev == 0ULL || prev == k) break;
      p = (p + 1) & gmask;
    }
    skey[i] = (L << gbits) | p;
    for (uint32_t l = 0; l + 1 < L; ++l) ilr_set_insert(tk, tk_mask, ilr_tk_key(l + 1, o.path[b + l]));
  }
}

// group boundaries over the sorted keys: flag[k] = 1 at a group's first op
// (levels >= 1); addf[k] = 1 for an Add of a group (addf[n] = 0)
__global__ void __launch_bounds__(BLOCK) k_ilr_gflag(const uint32_t* sk, const uint32_t* sv, uint32_t n, uint32_t gbits,
                                                     OpsDev o, uint32_t* flag, uint32_t* addf) {
  GRID_STRIDE(k, n + 1) {
    if (k == n) {
      addf[n] = 0;
      continue;
    }
    const bool grp = (sk[k] >> gbits) != 0;
    flag[k] = (grp && (k == 0 || sk[k] != sk[k - 1])) ? 1u : 0u;
    addf[k] = (grp && o.kind[sv[k]] == CRDTM_ADD) ? 1u : 0u;
  }
}
// group j = [gbeg[j], gend[j]) of the sorted ops: its start, and the end of
// the group before it (the last group ends at n); groups per level; group
// hash slot -> group
__global__ void __launch_bounds__(BLOCK) k_ilr_glist(const uint32_t* sk, uint32_t n, uint32_t gbits,
                                                     const uint32_t* flag, const uint32_t* gidx, const uint32_t* ngrp,
                                                     uint32_t* gbeg, uint32_t* gend, uint32_t* lvcnt,
                                                     uint32_t* slot2grp) {
  const uint32_t G = *ngrp;
  GRID_STRIDE(k, n) {
    if (!flag[k]) continue;
    const uint32_t j = gidx[k];
    gbeg[j] = k;
    if (j > 0) gend[j - 1] = k;
    if (j + 1 == G) gend[j] = n;
    atomicAdd(&lvcnt[sk[k] >> gbits], 1u);
    slot2grp[sk[k] & ((1u << gbits) - 1u)] = j;
  }
}
// per group: ops per level, the largest group, its Adds (reserved slots) and
// private table size (adds: exclusive prefix of addf)
__global__ void __launch_bounds__(BLOCK) k_ilr_gsize(const uint32_t* sk, uint32_t n, uint32_t gbits,
                                                     const uint32_t* flag, const uint32_t* gidx, const uint32_t* gend,
                                                     const uint32_t* adds, uint32_t* lvcnt, uint32_t* lvops,
                                                     uint32_t* qn, uint32_t* pcap) {
  GRID_STRIDE(k, n) {
    if (!flag[k]) continue;
    const uint32_t j = gidx[k], e = gend[j], L = sk[k] >> gbits;
    atomicAdd(&lvops[L], e - k);
    atomicMax(&lvcnt[ILR_MAXL + 3], e - k);  // (the largest group)
    const uint32_t a = adds[e] - adds[k];
    qn[j] = a;
    pcap[j] = ilr_pcap(a);
    atomicMax(&lvops[LV_N + L], a);  // (per level: the most Adds of a group, for its launch's LDS)
  }
}

// ---- a level's paths, in parallel: each op's prefix as of the op
// (update, src/Internal/Node.elm:138-163) and its landing lookups ----
__global__ void __launch_bounds__(BLOCK) k_ilr_prep(IlrArgs a, OpsDev o, const uint32_t* vs, uint32_t p0,
                                                    uint32_t p1) {
  for (uint32_t k = p0 + blockIdx.x * blockDim.x + threadIdx.x; k < p1; k += gridDim.x * blockDim.x) {
    const uint32_t i = vs[k];
    const uint32_t b = o.off[i], L = o.off[i + 1] - b;
    uint32_t d = 0, own = NONE, res = ST_APPLIED, hi = NONE, last = 0;
    for (uint32_t l = 0; l + 1 < L; ++l) {
      const long long key = o.path[b + l];
      if (d == IMPLICIT) {  // the implicit children hold only the sentinel 0 (a Tombstone)
        res = key == 0 ? ST_ALREADY : ST_INVALID;
        break;
      }
      const uint32_t sl = slothash_find(a.H, d, key);  // (shallower dicts: all in the shared hash)
      if (sl == NONE) {
        res = ST_INVALID;
        break;
      }
      uint32_t c = NONE;
      const uint32_t sv = ilr_slot_state(a, sl, i, &c, &hi);
      if (sv == 2) {
        res = ST_INVALID;
        break;
      }
      if (sv == 1) {
        res = ST_ALREADY;
        break;
      }
      own = sl;
      last = l + 1;
      d = c == NONE ? IMPLICIT : c;
    }
    uint32_t pts = NONE, pkk = NONE;
    if (res == ST_APPLIED && own != NONE && last + 1 == L) {
      // landing under a deleted-then-refilled node before its Delete: its
      // old children, which the lanes cannot tell from its new ones
      const uint32_t* e = a.ev + static_cast<uint64_t>(EVW) * own;
      if (e[EV_DEL] != NONE && e[EV_CPY] != NONE && i < e[EV_DEL]) {
        atomicOr(&a.dr->ilr_why, IW_REFILL);
        atomicOr(&a.dr->ilr_conflict, 1u);
        res = ST_CONFLICT;
      }
    }
    if (res == ST_APPLIED && d != IMPLICIT) {
      const long long kk = o.path[b + L - 1];
      if (o.kind[i] == CRDTM_ADD) pts = slothash_find(a.H, d, o.ts[i]);
      pkk = slothash_find(a.H, d, kk);
    }
    const unsigned long long tsu = static_cast<unsigned long long>(o.ts[i]);
    const unsigned long long kku = static_cast<unsigned long long>(L ? o.path[b + L - 1] : 0);
    a.P.w1[k] = make_uint4(i, static_cast<uint32_t>(o.kind[i]) | (res << 8), d, own);
    a.P.w2[k] = make_uint4(static_cast<uint32_t>(tsu), static_cast<uint32_t>(tsu >> 32), static_cast<uint32_t>(kku),
                           static_cast<uint32_t>(kku >> 32));
    a.P.w3[k] = make_uint2(pts, pkk);
  }
}

// ---- the deferred copies made at level L - 1, to the lanes of level L ----
__global__ void __launch_bounds__(BLOCK) k_ilr_jobs(IlrArgs a, uint32_t L, const unsigned long long* gk,
                                                    uint32_t gmask, const uint32_t* slot2grp, const uint32_t* jlo_p,
                                                    const uint32_t* jhi_p, uint32_t* nfree, uint32_t* mark_slots) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *mark_slots = a.dr->ilr_slots;  // (the level's first slot)
  const uint32_t jlo = *jlo_p, jhi = min(*jhi_p, a.J.cap);
  for (uint32_t j = jlo + blockIdx.x * blockDim.x + threadIdx.x; j < jhi; j += gridDim.x * blockDim.x) {
    const uint32_t node = a.J.own[j], dst = a.J.dst[j];
    const uint32_t ps = ilr_set_pos(gk, gmask, ilr_tk_key(L, a.T.s_key[node]));
    const uint32_t gs = ps == NONE ? NONE : slot2grp[ps];
    const uint32_t pd = ilr_set_pos(gk, gmask, ilr_tk_key(L, a.T.s_key[a.T.d_owner[dst]]));
    const uint32_t gd = pd == NONE ? NONE : slot2grp[pd];
    a.J.same[j] = gd != NONE && gd == gs;
    if (gd != NONE && gd != gs) atomicOr(reinterpret_cast<uint32_t*>(a.J.gflag) + (gd >> 2), GF_DST << (8 * (gd & 3)));
    if (gs == NONE) {  // nothing of this level lands in node's children: copied first, by one lane
      a.J.freel[atomicAdd(nfree, 1u)] = j;
      continue;
    }
    // (a same-group copy too: the lane reads its list only with the flag set)
    atomicOr(reinterpret_cast<uint32_t*>(a.J.gflag) + (gs >> 2), GF_SRC << (8 * (gs & 3)));
    a.J.next[j] = atomicExch(&a.J.head[gs], j);
  }
}

// the level's deferred copies whose source no op of the level reaches, one
// lane in order (their sources are the state before the level)
__global__ void __launch_bounds__(64) k_ilr_free(IlrArgs args, uint32_t L, const uint32_t* nfree, uint32_t* empty) {
  if (threadIdx.x != 0) return;
  IlrLane R;
  R.a = args;
  R.bad = false;
  R.depth = L;
  R.pk = nullptr;
  R.pd = nullptr;
  R.ps = empty;  // (a table with no entries)
  R.pmask = 0;
  R.pused = 0;
  R.qnext = R.qend = 0;
  R.un = nullptr;
  R.ucap = R.ucnt = 0;
  R.lrec = nullptr;
  R.lbase = 0;
  R.lcnt = 0;
  R.cpnext = R.cpend = 0;
  R.hd_d = NONE;
  R.hd_v = NONE;
  R.cs = NONE;
  R.cr = make_uint4(NONE, 0u, 0u, 0u);
  const uint32_t nf = min(*nfree, args.J.cap);
  for (uint32_t q = 0; q < nf && !R.bad; ++q) {
    const uint32_t j = args.J.freel[q];
    R.run_job(args.J.own[j], args.J.dst[j], args.J.at[j], false);
  }
  if (!R.bad) R.retire_pool();
}

// ---- one level, one phase: one lane per group ----
// phase 1: every group that receives no deferred copy (it makes those it
// owns); phase 2: the groups landing in deferred copies
// (LDS sized per launch from the level's largest group: lrn record mirror
// entries and ptn private table entries; a level of small groups keeps
// more of them resident per CU)
__global__ void __launch_bounds__(64) k_ilr_level(IlrArgs args, OpsDev o, const uint32_t* vs, const uint32_t* gbeg,
                                                  const uint32_t* gend, uint32_t g0, uint32_t L, uint32_t phase,
                                                  uint8_t* st, uint32_t lrn, uint32_t ptn) {
  // (one wave per group: every lane runs the replay on the same values; the
  // lanes part ways only in the chain-order walk below)
  const uint32_t g = g0 + blockIdx.x;
  const uint32_t gf = args.J.gflag[g];
  if ((gf & GF_DST) ? phase != 2 : phase != 1) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t kb = gbeg[g], ke = gend[g];
  extern __shared__ uint4 ilr_dyn[];
  uint4* lrec = ilr_dyn;                                                 // [lrn]
  long long* tpk = reinterpret_cast<long long*>(lrec + lrn);            // [ptn]
  uint32_t* tpd = reinterpret_cast<uint32_t*>(tpk + ptn);              // [ptn]
  uint32_t* tps = tpd + ptn;                                           // [ptn]
  const uint32_t pc = args.pcap[g];
  const bool plds = pc <= ptn && !(args.off & 1);
  if (plds) {
    for (uint32_t q = lane; q < pc; q += 64) tps[q] = NONE;
    wave_sync();  // (one wave per workgroup)
  }
  IlrLane R;
  R.a = args;
  R.bad = false;
  R.depth = L;
  R.pk = plds ? tpk : args.pk + args.poff[g];
  R.pd = plds ? tpd : args.pd + args.poff[g];
  R.ps = plds ? tps : args.ps + args.poff[g];
  R.pmask = pc - 1;
  R.pused = 0;
  R.qnext = args.committed + args.qoff[g];
  R.qend = R.qnext + args.qn[g];
  R.un = args.undo + 3 * ilr_uoff(kb, g);
  R.ucap = ilr_ucap(ke - kb);
  R.ucnt = 0;
  R.lrec = lrec;
  R.lbase = R.qnext;
  R.lcnt = (args.off & 2) ? 0u : min(args.qn[g], lrn);
  R.cpnext = R.cpend = 0;
  R.hd_d = NONE;
  R.hd_v = NONE;
  R.cs = NONE;
  const bool pre = phase == 1;  // (phase 2: the copies changed the landing dicts after the prep)
  if ((gf & (GF_SRC | GF_DST)) == (GF_SRC | GF_DST)) R.conflict(IW_CHAIN);
  // the deferred copies this lane makes, by op
  uint32_t jat[ILR_JOBS], jown[ILR_JOBS], jdst[ILR_JOBS], nj = 0;
  bool jsame[ILR_JOBS];
  for (uint32_t j = (gf & GF_SRC) ? args.J.head[g] : NONE; j != NONE && !R.bad; j = args.J.next[j]) {
    if (nj == ILR_JOBS) {
      R.conflict(IW_CHAIN);
      break;
    }
    jat[nj] = args.J.at[j];
    jown[nj] = args.J.own[j];
    jdst[nj] = args.J.dst[j];
    jsame[nj] = args.J.same[j];
    for (uint32_t q = 0; q < nj; ++q)  // (two copies of one source: xmap holds one)
      if (jsame[nj] && jown[q] == jown[nj]) R.conflict(IW_CHAIN);
    ++nj;
  }
  auto run_jobs_before = [&](uint32_t i) {
    for (;;) {
      uint32_t best = NONE, bj = 0;
      for (uint32_t q = 0; q < nj; ++q)
        if (jat[q] < i && jat[q] < best) {
          best = jat[q];
          bj = q;
        }
      if (best == NONE || R.bad) return;
      R.run_job(jown[bj], jdst[bj], jat[bj], jsame[bj]);
      jat[bj] = NONE;
    }
  };
  const long long id0 = replica_of(args.ts0);
  uint32_t app = 0, alr = 0, own_ok = 0, err = NONE;
  // the last slots this lane created in dict rdict (typing anchors at its own
  // previous character): key -> slot
  uint32_t rdict = NONE;
  long long rk0 = 0, rk1 = 0, rk2 = 0, rk3 = 0;
  uint32_t rs0 = NONE, rs1 = NONE, rs2 = NONE, rs3 = NONE;
  auto recent = [&](long long k) -> uint32_t {
    if (args.off & 8) return NONE;
    return (rs0 != NONE && rk0 == k) ? rs0 : (rs1 != NONE && rk1 == k) ? rs1 : (rs2 != NONE && rk2 == k) ? rs2
           : (rs3 != NONE && rk3 == k) ? rs3 : NONE;
  };
  unsigned long long n_walk = 0, n_skip = 0, n_quirk = 0, n_mark = 0;
  const unsigned long long t0 = wall_clock64();
  uint4 c1 = args.P.w1[kb], c2 = args.P.w2[kb];
  uint2 c3 = args.P.w3[kb];
  for (uint32_t k = kb; k < ke && !R.bad; ++k) {
    uint4 n1 = c1, n2 = c2;
    uint2 n3 = c3;
    if (k + 1 < ke) {  // the next op's record, in flight while this op runs
      n1 = args.P.w1[k + 1];
      n2 = args.P.w2[k + 1];
      n3 = args.P.w3[k + 1];
    }
    const uint32_t i = c1.x;
    const uint8_t kind = static_cast<uint8_t>(c1.y & 0xFFu);
    const uint32_t res = c1.y >> 8;
    const long long ts = static_cast<long long>((static_cast<unsigned long long>(c2.y) << 32) | c2.x);
    const long long kk = static_cast<long long>((static_cast<unsigned long long>(c2.w) << 32) | c2.z);
    const uint32_t pre_ts = c3.x, pre_kk = c3.y;
    uint32_t d = c1.z, ownr = c1.w;
    c1 = n1;
    c2 = n2;
    c3 = n3;
    if (nj) run_jobs_before(i);
    if (R.bad) break;
    uint8_t s = ST_APPLIED;
    if (res == ST_CONFLICT) {
      R.bad = true;
      break;
    }
    if (res != ST_APPLIED) {
      s = static_cast<uint8_t>(res);
    } else {
      bool usepre = pre && (d == IMPLICIT || R.copy_src(d) == NONE);
      if (d == IMPLICIT) {  // (materialised by this lane since the prep?)
        const uint32_t c = args.T.s_child[ownr];
        if (c != NONE) {
          d = c;
          usepre = false;
        }
      }
      if (d == IMPLICIT) {
        // the empty children {0: Tombstone}: only an Add after the sentinel
        // changes it (then the dict is created); ts 0 or Delete 0: AlreadyApplied
        if (kind == CRDTM_ADD && ts != 0 && kk == 0) {
          d = R.materialise(ownr);
          if (d == NONE) break;
          usepre = false;
        } else {
          s = (kk == 0 || (kind == CRDTM_ADD && ts == 0)) ? ST_ALREADY : ST_NOTFOUND;
        }
      }
      if (s == ST_APPLIED) {
        if (d != rdict) {
          rdict = d;
          rs0 = rs1 = rs2 = rs3 = NONE;
        }
        // (a dict this lane filled by a same-group copy holds entries the
        // shared hash does not have yet: R.find goes through xmap)
        auto lookup = [&](long long key, uint32_t prek) -> uint32_t {
          if (!usepre) return R.find(d, key);
          const uint32_t v = R.pfind(d, key);
          return v != NONE ? v : prek;
        };
        if (kind == CRDTM_DELETE) {  // deleteHelp (:112-122)
          uint32_t t = recent(kk);
          if (t == NONE) t = lookup(kk, pre_kk);
          if (t == NONE) {
            s = ST_NOTFOUND;
          } else {
            const uint8_t tf = args.T.s_flags[t];
            if (tf & F_TOMB) {
              s = ST_ALREADY;
            } else if (R.ev(t, EV_DEL) != NONE) {  // (deleted, re-filled, deleted: a third event)
              R.conflict(IW_EVENTS);
              break;
            } else {
              R.set_flags(t, tf, tf | F_TOMB);
              R.ev(t, EV_DEL) = i;  // children drop at the commit
            }
          }
        } else if (lookup(ts, pre_ts) != NONE) {  // addAfterHelp (:56-90)
          s = ST_ALREADY;
        } else {
          uint32_t found = recent(kk);
          if (found == NONE) found = lookup(kk, pre_kk);
          if (found == NONE) {
            s = ST_NOTFOUND;
          } else {
            // findInsertion (:93-104): ls = the slot of the key it returns
            // (one 16-byte record per step: rn's next, flags and key)
            uint32_t node = found, ls = found, rn = R.getrec(found).x;
            for (;;) {
              // The chain from node in the batch-start snapshot's order, 64
              // entries at a time, each link checked against the state (a
              // link this batch changed ends the run): the walk's steps over
              // the checked run are decided together; only where the run
              // ends or breaks does the walk take single steps.
              if (args.R && node < args.E && args.R[node] != NONE) {
                const uint32_t pos = args.R[node] + 1 + lane;
                const uint32_t ck = pos < args.E ? args.G[pos] : NONE;  // c_{lane+1}
                const uint4 rc = ck != NONE ? args.rec[ck] : make_uint4(NONE, F_TOMB, 0u, 0u);
                uint32_t nprev = __shfl_up(rc.x, 1);  // next(c_lane)
                if (lane == 0) nprev = rn;            // next(c_0 = node)
                const unsigned long long mlink = __ballot(ck != NONE && nprev == ck);
                const uint32_t V = ~mlink ? static_cast<uint32_t>(__builtin_ctzll(~mlink)) : 64u;
                // positions 0..V are the chain from node; bit p below is position p
                const bool valid = lane < V;  // position lane + 1
                const long long kc = static_cast<long long>((static_cast<unsigned long long>(rc.w) << 32) | rc.z);
                const unsigned long long mlive = __ballot(valid && !(rc.y & F_TOMB)) << 1;
                const unsigned long long mkey = __ballot(valid && ts > kc);          // compare at position lane + 1
                const unsigned long long mend = __ballot(lane <= V && nprev == NONE);  // next(position lane) is none
                const unsigned long long vis = mlive | 1ULL;  // visited: node, then every live entry
                unsigned long long cand = vis & (mkey | mend);
                if (mend) {  // the chain ends in the run: no live entry after the last visited one
                  const uint32_t e = static_cast<uint32_t>(__builtin_ctzll(mend));
                  const unsigned long long upto = e >= 63 ? ~0ULL : ((2ULL << e) - 1ULL);
                  cand |= 1ULL << (63 - __builtin_clzll(vis & upto));
                }
                auto slot_at = [&](uint32_t p) -> uint32_t { return p == 0 ? node : __shfl(ck, p - 1); };
                auto next_at = [&](uint32_t p) -> uint32_t { return __shfl(nprev, p); };
                if (cand) {  // the walk stops at the first candidate
                  const uint32_t S = static_cast<uint32_t>(__builtin_ctzll(cand));
                  if (S > 0) {
                    const unsigned long long below = vis & ((1ULL << S) - 1ULL);
                    ls = slot_at(static_cast<uint32_t>(63 - __builtin_clzll(below)) + 1);
                    node = slot_at(S);
                    n_walk += __builtin_popcountll(below);
                  }
                  rn = next_at(S);
                  break;
                }
                // no stop in the run: the walk passes every visited entry up
                // to the last one (which needs what follows the run)
                const unsigned long long inrun = vis & (V >= 63 ? ~0ULL : ((2ULL << V) - 1ULL));
                const uint32_t Lv = static_cast<uint32_t>(63 - __builtin_clzll(inrun));
                if (Lv > 0) {
                  const unsigned long long below = inrun & ((1ULL << Lv) - 1ULL);
                  ls = slot_at(static_cast<uint32_t>(63 - __builtin_clzll(below)) + 1);
                  node = slot_at(Lv);
                  rn = next_at(Lv);
                  n_walk += __builtin_popcountll(below);
                  continue;
                }
              }
              ++n_walk;
              if (rn == NONE) break;
              const uint4 r = R.getrec(rn);
              uint32_t live = rn;
              uint4 lr = r;
              while (lr.y & F_TOMB) {
                live = lr.x;
                ++n_skip;
                if (live == NONE) break;
                lr = R.getrec(live);
              }
              if (live == NONE) break;
              const long long rk = static_cast<long long>((static_cast<unsigned long long>(r.w) << 32) | r.z);
              if (ts > rk) break;
              ls = rn;
              node = live;
              rn = lr.x;
            }
            const uint32_t x = R.take_slot(true);
            if (x == NONE) break;
            const uint8_t lsf = static_cast<uint8_t>(R.getrec(ls).y);
            // x is reachable from the dict's sentinel iff its predecessor is
            R.put_slot(x, d, ts, rn, ILR_TAG | i, NONE, (lsf & F_ORPHAN) ? F_ORPHAN : 0, i, true);
            if (R.bad) break;
            if (ls == node) {
              R.set_next(node, rn, x);
            } else {
              // the copy quirk: slot ls := copy of node with
              // next = ts; the entries after it up to node drop off the chain
              if (R.ev(ls, EV_CPY) != NONE) {  // (re-filled, deleted, re-filled: a third event)
                R.conflict(IW_EVENTS);
                break;
              }
              ++n_quirk;
              if (!(lsf & F_ORPHAN)) {
                for (uint32_t q = args.T.s_next[ls]; q != NONE; q = args.T.s_next[q]) {
                  const uint8_t qf = args.T.s_flags[q];
                  ++n_mark;
                  R.set_flags(q, qf, qf | F_ORPHAN);
                  if (q == node) break;
                }
              }
              const uint32_t c = args.T.s_child[node];
              if (R.ev(ls, EV_DEL) != NONE) R.ev(ls, EV_OCH) = args.T.s_child[ls];  // (its children before the Delete)
              R.set_src(ls, args.T.s_src[node]);
              R.set_flags(ls, lsf, (args.T.s_flags[node] & ~F_ORPHAN) | (lsf & F_ORPHAN));
              R.set_next(ls, args.T.s_next[ls], x);
              R.ev(ls, EV_CPY) = i;
              // its children are node's as of op i: now, unless the batch
              // reaches below node — then the lane owning node's children
              // makes the copy at the next level when it passes op i
              uint32_t nc = NONE;
              if (ilr_set_has(args.tk, args.tk_mask, ilr_tk_key(L, args.T.s_key[node]))) {
                nc = R.new_dict(ls);
                if (nc == NONE) break;
                const uint32_t j = IlrLane::wave_add(&args.dr->ilr_jobs, 1u);
                if (j >= args.J.cap) {
                  R.overflow(IO_JOBS);
                  break;
                }
                args.J.own[j] = node;
                args.J.dst[j] = nc;
                args.J.at[j] = i;
                args.dsrc[nc] = DS_PENDING;
              } else if (c != NONE) {
                nc = R.new_dict(ls);
                if (nc == NONE) break;
                R.deep_copy(c, nc, i, L + 1);
                if (R.bad) break;
              }
              R.set_child(ls, nc);
            }
            rk3 = rk2; rs3 = rs2;
            rk2 = rk1; rs2 = rs1;
            rk1 = rk0; rs1 = rs0;
            rk0 = ts; rs0 = x;
          }
        }
      }
    }
    if (R.bad) break;
    st[i] = s;
    if (s == ST_APPLIED) ++app;
    else if (s == ST_ALREADY) ++alr;
    else err = min(err, i);
    // incrementTimestamp (src/CRDTree.elm:337-343): Ok Adds of the own replica
    if ((s == ST_APPLIED || s == ST_ALREADY) && kind == CRDTM_ADD && replica_of(ts) == id0) ++own_ok;
  }
  if (nj && !R.bad) run_jobs_before(NONE);
  if (args.stats) {
    unsigned long long* q = args.stats + 8ULL * g;
    q[0] = ke - kb;
    q[1] = n_walk;
    q[2] = n_skip;
    q[3] = n_quirk;
    q[4] = n_mark;
    q[5] = wall_clock64() - t0;
    q[6] = L;
    q[7] = 0;
  }
  args.ucnt[g] = R.ucnt;
  if (!R.bad) {
    // reserved slots no Add took, pool slots no copy took: dead entries of
    // the batch's dead dict
    for (uint32_t x = R.qnext; x < R.qend; ++x) R.put_dead(x);
    R.retire_pool();
  }
  if (lane == 0) {
    if (app) atomicAdd(&args.dr->n_applied, app);
    if (alr) atomicAdd(&args.dr->n_already, alr);
    if (own_ok) atomicAdd(&args.dr->own_ok_adds, own_ok);
    if (err != NONE) atomicMin(&args.dr->err_index, err);
  }
}

// counters before a phase: slots (publish start) and deferred copies
__global__ void k_ilr_mark(const DevResult* d, uint32_t* slots, uint32_t* jobs) {
  if (slots) *slots = d->ilr_slots;
  if (jobs) *jobs = d->ilr_jobs;
}
// after a phase: its slots into the shared hash — the reserved ranges of
// its groups (one block each) and what the counter gave since the mark
// (skipped once the batch overflowed or conflicted: it is rolled back and
// the index rebuilt)
__global__ void __launch_bounds__(BLOCK) k_ilr_publish(TreeDev T, SlotHash H, const uint32_t* qoff, const uint32_t* qn,
                                                       const uint8_t* gflag, uint32_t g0, uint32_t cnt,
                                                       uint32_t phase, uint32_t committed, const uint32_t* mark,
                                                       const DevResult* d, uint32_t cap, uint32_t* mark_slots,
                                                       uint32_t* mark_jobs) {
  // (the next phase's first slot, or the level's last deferred copy: the
  // counters as this phase left them)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (mark_slots) *mark_slots = d->ilr_slots;
    if (mark_jobs) *mark_jobs = d->ilr_jobs;
  }
  if (d->ilr_overflow || d->ilr_conflict) return;
  if (blockIdx.x < cnt) {
    const uint32_t g = g0 + blockIdx.x;
    if ((gflag[g] & GF_DST) ? phase != 2 : phase != 1) return;
    const uint32_t a0 = committed + qoff[g];
    for (uint32_t j = threadIdx.x; j < qn[g]; j += blockDim.x)
      slothash_put_par(H, T.s_dict[a0 + j], T.s_key[a0 + j], a0 + j);
    return;
  }
  const uint32_t b0 = *mark, b1 = min(d->ilr_slots, cap);
  for (uint32_t s = b0 + (blockIdx.x - cnt) * blockDim.x + threadIdx.x; s < b1; s += (gridDim.x - cnt) * blockDim.x)
    slothash_put_par(H, T.s_dict[s], T.s_key[s], s);
}

// undo of one level's groups, each newest first (launched deepest level first:
// a field two levels wrote — an owner's children — gets its oldest value)
__global__ void __launch_bounds__(BLOCK) k_ilr_rollback(TreeDev T, const uint32_t* undo, const uint32_t* ucnt,
                                                        const uint32_t* gbeg, uint32_t g0, uint32_t cnt) {
  GRID_STRIDE(j, cnt) {
    const uint32_t g = g0 + j;
    const uint32_t* u = undo + 3 * ilr_uoff(gbeg[g], g);
    for (uint32_t e = ucnt[g]; e-- > 0;) {
      const uint32_t s = u[3 * e], f = u[3 * e + 1], v = u[3 * e + 2];
      if (f == IF_NEXT) T.s_next[s] = v;
      else if (f == IF_SRC) T.s_src[s] = v;
      else if (f == IF_CHILD) T.s_child[s] = v;
      else T.s_flags[s] = static_cast<uint8_t>(v);
    }
  }
}

// commit, for the slots the batch touched — the new ones [lo, hi) and the
// state's slots in the undo logs: sources tagged with an op index take its
// log index; a node the batch left deleted drops its children (children
// Tombstone = Dict.empty, src/Internal/Node.elm:237-238)
__device__ __forceinline__ void ilr_fix_slot(TreeDev& T, uint32_t s, const uint32_t* logidx, uint32_t log_base,
                                             const uint32_t* ev) {
  const uint32_t src = T.s_src[s];
  if (src != NONE && (src & ILR_TAG)) T.s_src[s] = log_base + logidx[src & ~ILR_TAG];
  if (ev[static_cast<uint64_t>(EVW) * s + EV_DEL] != NONE && (T.s_flags[s] & F_TOMB)) T.s_child[s] = NONE;
}
__global__ void __launch_bounds__(BLOCK) k_ilr_fix(TreeDev T, uint32_t lo, uint32_t hi, const uint32_t* undo,
                                                   uint32_t nu, const uint32_t* logidx, uint32_t log_base,
                                                   const uint32_t* ev) {
  const uint32_t nn = hi - lo;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nn + nu; j += gridDim.x * blockDim.x) {
    if (j < nn) {
      ilr_fix_slot(T, lo + j, logidx, log_base, ev);
    } else {
      const uint32_t s = undo[3ULL * (j - nn)], f = undo[3ULL * (j - nn) + 1];
      if (s != NONE && (f == IF_SRC || f == IF_FLAGS))
        ilr_fix_slot(T, s, logidx, log_base, ev);  // (the entries of one slot: same result, any order)
    }
  }
}
// then the event times back to NONE (a separate pass: the fix reads them)
__global__ void __launch_bounds__(BLOCK) k_ilr_ev_reset(uint32_t lo, uint32_t hi, const uint32_t* undo, uint32_t nu,
                                                        uint32_t* ev) {
  const uint32_t nn = hi - lo;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nn + nu; j += gridDim.x * blockDim.x) {
    const uint32_t s = j < nn ? lo + j : undo[3ULL * (j - nn)];
    if (s == NONE) continue;
    for (uint32_t w = 0; w < EVW; ++w) ev[static_cast<uint64_t>(EVW) * s + w] = NONE;
  }
}

__global__ void k_ilr_counters(DevResult* d, TreeDev T, uint32_t* dhead, uint32_t* dsrc, uint32_t committed,
                               const uint32_t* qtot, uint32_t grave) {
  d->ilr_slots = committed + *qtot;
  d->ilr_dicts = grave + 1;
  d->ilr_conflict = 0;
  d->ilr_overflow = 0;
  d->ilr_why = 0;
  d->ilr_jobs = 0;
  T.d_owner[grave] = NONE;  // (no owner: never alive)
  T.d_sent[grave] = NONE;
  dhead[grave] = NONE;
  dsrc[grave] = NONE;
}

__global__ void __launch_bounds__(BLOCK) k_ilr_rec(TreeDev T, uint32_t S, uint4* rec) {
  GRID_STRIDE(s, S) {
    const unsigned long long k = static_cast<unsigned long long>(T.s_key[s]);
    rec[s] = make_uint4(T.s_next[s], T.s_flags[s], static_cast<uint32_t>(k), static_cast<uint32_t>(k >> 32));
  }
}

static uint32_t pow2_ge(uint64_t x) {
  uint32_t p = 1024;
  while (p < x && p < (1u << 31)) p <<= 1;
  return p;
}

bool ilr_wanted(const crdtm_tree* t, uint32_t n) {
  const char* e = getenv("CRDTM_INCREMENTAL");
  if (e && (!strcmp(e, "replay") || !strcmp(e, "remerge"))) return false;
  if (e && !strcmp(e, "ilr")) return true;
  // per-dict replay on the state: worth it when the state outweighs the batch
  // (the re-merge's parallel work grows with log + batch)
  return t->n_slots >= 4ULL * n && t->max_depth <= ILR_MAXL;
}

// (re)build the index of the state: hash sized for the slot capacity
static int ilr_build(crdtm_tree* t) {
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  if (!t->ilr) t->ilr.reset(new IlrIndex);
  IlrIndex& X = *t->ilr;
  X.snapE = 0;  // (a rebuilt index describes another state: the next level replay takes a fresh snapshot)
  X.snap_age = 0;
  const uint32_t H = pow2_ge(2 * t->cap.slots);
  if (X.hcap < H) {
    HIP_CHECK(hipStreamSynchronize(s));
    if (X.H.dict) hipFree(X.H.dict);
    if (X.H.key) hipFree(X.H.key);
    if (X.H.slot) hipFree(X.H.slot);
    X.H.dict = nullptr;
    X.H.key = nullptr;
    X.H.slot = nullptr;
    HIP_CHECK(hipMalloc(&X.H.dict, H * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.H.key, H * sizeof(long long)));
    HIP_CHECK(hipMalloc(&X.H.slot, H * sizeof(uint32_t)));
    X.hcap = H;
    X.H.mask = H - 1;
  }
  if (X.dcap < t->cap.dicts) {
    HIP_CHECK(hipStreamSynchronize(s));
    if (X.dhead) hipFree(X.dhead);
    if (X.dsrc) hipFree(X.dsrc);
    X.dhead = nullptr;
    X.dsrc = nullptr;
    HIP_CHECK(hipMalloc(&X.dhead, t->cap.dicts * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.dsrc, t->cap.dicts * sizeof(uint32_t)));
    X.dcap = t->cap.dicts;
  }
  if (X.scap < t->cap.slots) {
    HIP_CHECK(hipStreamSynchronize(s));
    if (X.mnext) hipFree(X.mnext);
    if (X.ev) hipFree(X.ev);
    if (X.xmap) hipFree(X.xmap);
    if (X.rec) hipFree(X.rec);
    X.mnext = nullptr;
    X.ev = nullptr;
    X.xmap = nullptr;
    X.rec = nullptr;
    HIP_CHECK(hipMalloc(&X.mnext, t->cap.slots * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.ev, EVW * t->cap.slots * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.xmap, t->cap.slots * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.rec, t->cap.slots * sizeof(uint4)));
    X.scap = t->cap.slots;
  }
  HIP_CHECK(hipMemsetAsync(X.H.slot, 0xFF, X.hcap * sizeof(uint32_t), s));
  HIP_CHECK(hipMemsetAsync(X.dhead, 0xFF, X.dcap * sizeof(uint32_t), s));
  HIP_CHECK(hipMemsetAsync(X.ev, 0xFF, EVW * X.scap * sizeof(uint32_t), s));
  LAUNCH(k_replay_index, dim3(grid_for(t->n_slots)), dim3(BLOCK), 0, s, t->d, static_cast<uint32_t>(t->n_slots), X.H,
         X.dhead, X.mnext);
  LAUNCH(k_ilr_rec, dim3(grid_for(t->n_slots)), dim3(BLOCK), 0, s, t->d, static_cast<uint32_t>(t->n_slots), X.rec);
  X.hused = t->n_slots;
  t->ilr_valid = true;
  return CRDTM_OK;
}

int ilr_apply(crdtm_tree* t, const OpsDev& o, uint8_t* st_out, crdtm_result* res, bool* handled) {
  *handled = false;
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  DevResult* dr = c->dres;
  const uint32_t n = o.n;
  const size_t mark0 = ws.used;
  int r;
  // ranges and the longest path (one host round trip)
  LAUNCH(k_dres_init, dim3(1), dim3(64), 0, s, dr);
  launch_pre(c, o, s);
  RangeReset keep_clean{c};  // (k_pre fills the context's replica ranges; nothing here reads them)
  if (o.n_path)
    LAUNCH(k_path_range, dim3(std::min<uint32_t>(grid_for(o.n_path / 2 + 1), 1024)), dim3(BLOCK), 0, s, o, dr);
  if ((r = sync_read(c))) return r;
  keep_clean.nr = c->hres->max_replica + 1;
  keep_clean.now();
  if (c->hres->bad_range) return CRDTM_E_RANGE;  // (the state is untouched)
  const uint32_t maxlen = c->hres->max_len;
  if (maxlen > ILR_MAXL) return CRDTM_OK;
  // capacity: new nodes and their dicts, the dead dict, room for deep copies
  // (an overflow sends the batch to the re-merge)
  TreeCaps need = t->cap;
  const uint64_t extra = 1024 + n / 2;
  need.slots = std::max<uint64_t>(need.slots, t->n_slots + 2ULL * n + extra);
  need.dicts = std::max<uint64_t>(need.dicts, t->n_dicts + n + extra);
  need.log = std::max<uint64_t>(need.log, t->log_n + n + 1);
  need.lpath = std::max<uint64_t>(need.lpath, t->log_npath + o.n_path + 1);
  if (need.slots > t->cap.slots || need.dicts > t->cap.dicts || need.log > t->cap.log || need.lpath > t->cap.lpath) {
    if ((r = grow_tree(t, need))) return r;
  }
  IlrIndex* X = t->ilr.get();
  if (!t->ilr_valid || !X || X->scap < t->cap.slots || X->dcap < t->cap.dicts || X->hcap < 2 * t->cap.slots) {
    if ((r = ilr_build(t))) return r;
    X = t->ilr.get();
  }
  // ---- groups: (L, owner key), sorted by level, batch order inside ----
  const uint32_t gsz = pow2_ge(2ULL * n + 16);
  uint32_t gbits = 0;
  while ((1u << gbits) < gsz) ++gbits;
  unsigned long long* gk = ws.alloc<unsigned long long>(gsz);
  uint32_t* slot2grp = ws.alloc<uint32_t>(gsz);
  const uint32_t tsz = pow2_ge(2ULL * o.n_path + 16);
  unsigned long long* tk = ws.alloc<unsigned long long>(tsz);
  uint32_t* sk[2] = {ws.alloc<uint32_t>(n + 1), ws.alloc<uint32_t>(n + 1)};
  uint32_t* sv[2] = {ws.alloc<uint32_t>(n + 1), ws.alloc<uint32_t>(n + 1)};
  uint8_t* st = ws.alloc<uint8_t>(n + 1);
  uint32_t* nd = ws.alloc<uint32_t>(2);
  uint32_t* flag = ws.alloc<uint32_t>(n + 1);
  uint32_t* gidx = ws.alloc<uint32_t>(n + 1);
  uint32_t* gbeg = ws.alloc<uint32_t>(n + 1);
  uint32_t* gend = ws.alloc<uint32_t>(n + 1);
  uint32_t* qn = ws.alloc<uint32_t>(n + 2);
  uint32_t* qoff = ws.alloc<uint32_t>(n + 2);
  uint32_t* pcap = ws.alloc<uint32_t>(n + 2);
  uint32_t* poff = ws.alloc<uint32_t>(n + 2);
  uint32_t* ucnt = ws.alloc<uint32_t>(n + 1);
  uint32_t* lvcnt = ws.alloc<uint32_t>(3 * LV_N);  // groups per level, totals; ops per level; most Adds per level
  FillList fl;  // (one launch for the batch's cleared arrays)
  fl.add(gk, gsz * sizeof(unsigned long long), 0u);
  fl.add(slot2grp, gsz * sizeof(uint32_t), NONE);
  fl.add(tk, tsz * sizeof(unsigned long long), 0u);
  fl.add(lvcnt, 3 * LV_N * sizeof(uint32_t), 0u);
  fl.add(qn, (n + 2) * sizeof(uint32_t), 0u);
  fl.add(pcap, (n + 2) * sizeof(uint32_t), 0u);
  fl.add(nd, sizeof(uint32_t), n);
  if ((r = fl.launch(s))) return r;
  LAUNCH(k_ilr_group, dim3(grid_for(n)), dim3(BLOCK), 0, s, o, gk, gsz - 1, gbits, tk, tsz - 1, sk[0], sv[0], st, dr);
  uint32_t *ks = nullptr, *vs = nullptr;
  if ((r = radix_sort_pairs(sk[0], sv[0], sk[1], sv[1], nd, n, gbits + 7, ws, s, &ks, &vs))) return r;
  uint32_t* addf = ws.alloc<uint32_t>(n + 1);
  uint32_t* adds = ws.alloc<uint32_t>(n + 1);
  LAUNCH(k_ilr_gflag, dim3(grid_for(n + 1)), dim3(BLOCK), 0, s, ks, vs, n, gbits, o, flag, addf);
  if ((r = scan_excl_u32(flag, gidx, n, &dr->ilr_groups, ws, s))) return r;
  if ((r = scan_excl_u32(addf, adds, n + 1, nullptr, ws, s))) return r;
  LAUNCH(k_ilr_glist, dim3(grid_for(n)), dim3(BLOCK), 0, s, ks, n, gbits, flag, gidx, &dr->ilr_groups, gbeg, gend,
         lvcnt, slot2grp);
  LAUNCH(k_ilr_gsize, dim3(grid_for(n)), dim3(BLOCK), 0, s, ks, n, gbits, flag, gidx, gend, adds, lvcnt,
         lvcnt + LV_N, qn, pcap);
  // reserved slot ranges and private tables: offsets and totals (in lvcnt)
  if ((r = scan_excl_u32(qn, qoff, n + 1, lvcnt + LV_QTOT, ws, s))) return r;
  if ((r = scan_excl_u32(pcap, poff, n + 1, lvcnt + LV_PTOT, ws, s))) return r;
  const uint32_t grave = static_cast<uint32_t>(t->n_dicts);
  LAUNCH(k_ilr_counters, dim3(1), dim3(1), 0, s, dr, t->d, X->dhead, X->dsrc, static_cast<uint32_t>(t->n_slots),
         lvcnt + LV_QTOT, grave);
  static_assert(sizeof(DevResult::ilr_levels) >= 3 * LV_N * sizeof(uint32_t), "staging room");
  uint32_t* hl = c->hres->ilr_levels;  // (pinned)
  HIP_CHECK(hipMemcpyAsync(hl, lvcnt, 3 * LV_N * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (int rw = stream_wait(s)) return rw;
  uint32_t lv[3 * LV_N];
  memcpy(lv, hl, sizeof(lv));
  uint32_t G = 0, nops = 0;
  for (uint32_t L = 1; L <= ILR_MAXL; ++L) {
    G += lv[L];
    nops += lv[LV_N + L];
  }
  const uint32_t ptot = lv[LV_PTOT];
  long long* pk = ws.alloc<long long>(ptot);
  uint32_t* pd = ws.alloc<uint32_t>(ptot);
  uint32_t* ps = ws.alloc<uint32_t>(ptot);
  const uint64_t nu = 3ULL * n + 8ULL * G + 8;  // undo triples (ilr_uoff layout)
  uint32_t* undo = ws.alloc<uint32_t>(3 * nu);
  uint32_t* marks = ws.alloc<uint32_t>(4 * (ILR_MAXL + 2));
  const uint32_t jcap = n / 2 + 64;
  IlrJobs J;
  J.own = ws.alloc<uint32_t>(jcap);
  J.dst = ws.alloc<uint32_t>(jcap);
  J.at = ws.alloc<uint32_t>(jcap);
  J.next = ws.alloc<uint32_t>(jcap);
  J.head = ws.alloc<uint32_t>(G + 1);
  J.same = ws.alloc<uint8_t>(jcap);
  J.gflag = ws.alloc<uint8_t>(G + 4);
  J.freel = ws.alloc<uint32_t>(jcap);
  J.cap = jcap;
  uint32_t* empty = ws.alloc<uint32_t>(16);
  // the commit's arrays are taken before the first level changes the state
  // in place: past that point an arena overflow would leave it half written
  uint32_t* appl = ws.alloc<uint32_t>(n + 1);
  uint32_t* plen = ws.alloc<uint32_t>(n + 1);
  long long* rep = ws.alloc<long long>(2 * static_cast<uint64_t>(n) + 2);
  uint32_t* rlist = ws.alloc<uint32_t>(std::min<uint64_t>(n, REPLICA_SLOTS) + 1);
  IlrPrep P;
  P.w1 = ws.alloc<uint4>(n + 1);
  P.w2 = ws.alloc<uint4>(n + 1);
  P.w3 = ws.alloc<uint2>(n + 1);
  fl.add(ps, static_cast<size_t>(ptot) * sizeof(uint32_t), NONE);
  fl.add(undo, 3 * nu * sizeof(uint32_t), NONE);
  fl.add(marks, 4 * (ILR_MAXL + 2) * sizeof(uint32_t), 0u);
  fl.add(J.head, (G + 1) * sizeof(uint32_t), NONE);
  fl.add(J.gflag, G + 4, 0u);
  fl.add(empty, 16 * sizeof(uint32_t), NONE);
  if ((r = fl.launch(s))) return r;
  // ---- the levels ----
  IlrArgs a;
  a.T = t->d;
  a.H = X->H;
  a.dhead = X->dhead;
  a.mnext = X->mnext;
  a.ev = X->ev;
  a.xmap = X->xmap;
  a.rec = X->rec;
  a.scap = static_cast<uint32_t>(X->scap);
  a.committed = static_cast<uint32_t>(t->n_slots);
  a.cap_slots = static_cast<uint32_t>(t->cap.slots);
  a.cap_dicts = static_cast<uint32_t>(t->cap.dicts);
  a.hash_limit = X->hcap / 2;
  a.tk = tk;
  a.tk_mask = tsz - 1;
  a.ts0 = t->timestamp;
  a.dr = dr;
  a.pk = pk;
  a.pd = pd;
  a.ps = ps;
  a.poff = poff;
  a.pcap = pcap;
  a.qoff = qoff;
  a.qn = qn;
  a.undo = undo;
  a.ucnt = ucnt;
  a.grave = grave;
  a.P = P;
  a.J = J;
  // the chain order of the state, when a lane has enough ops for long walks
  // (env CRDTM_ILR_SNAPSHOT=0: never)
  const char* snap_env = getenv("CRDTM_ILR_SNAPSHOT");
  const uint32_t snap_min = snap_env ? static_cast<uint32_t>(atoi(snap_env)) : 64u;
  a.R = nullptr;
  a.G = nullptr;
  a.E = 0;
  // (kept with the index and rebuilt every CRDTM_ILR_SNAP_EVERY batches: a
  // snapshot some batches old covers the slots it knew, and a link a later
  // batch changed only ends a checked run early -- but the busy lane walks
  // where the text changed: incr_cfg2 23.7 ms per 10 batches rebuilt every
  // batch, 23.9 every 4, 25.4 every 8, 27.0 never, so 1 by default)
  static const uint32_t snap_every = [] {
    const char* e = getenv("CRDTM_ILR_SNAP_EVERY");
    const int v = e ? atoi(e) : 1;
    return static_cast<uint32_t>(v >= 1 ? v : 1);
  }();
  if (snap_min && lv[ILR_MAXL + 3] >= snap_min) {
    const uint64_t E = t->n_slots;
    if (!X->snapR || !X->snapE || X->snap_age + 1 >= snap_every || X->snapE > E) {
      if (X->snap_cap < E + 1) {
        if (X->snapR) hipFree(X->snapR);
        if (X->snapG) hipFree(X->snapG);
        X->snapR = X->snapG = nullptr;
        X->snap_cap = 0;
        const uint64_t cap = 2 * (E + 1) + 4096;
        HIP_CHECK(hipMalloc(&X->snapR, cap * sizeof(uint32_t)));
        HIP_CHECK(hipMalloc(&X->snapG, cap * sizeof(uint32_t)));
        X->snap_cap = cap;
      }
      if ((r = chain_snapshot(t, X->snapR, X->snapG, ws, s))) return r;
      X->snapE = static_cast<uint32_t>(E);
      X->snap_age = 0;
    } else {
      ++X->snap_age;
    }
    a.R = X->snapR;
    a.G = X->snapG;
    a.E = X->snapE;
  }
  a.dsrc = X->dsrc;
  a.dnew = grave;
  const char* off_env = getenv("CRDTM_ILR_OFF");
  a.off = off_env ? static_cast<uint32_t>(atoi(off_env)) : 0u;
  static const bool want_stats = getenv("CRDTM_ILR_STATS") != nullptr;
  a.stats = nullptr;
  if (want_stats) {
    a.stats = ws.alloc<unsigned long long>(8ULL * (G + 1));
    HIP_CHECK(hipMemsetAsync(a.stats, 0, 8ULL * (G + 1) * sizeof(unsigned long long), s));
  }
  uint32_t g0 = 0, levels = 0, p0 = n - nops;  // (empty paths sort first)
  uint32_t lv_g0[ILR_MAXL + 2] = {};
  // marks: [4 L] slots before phase 1 (and the free copies), [4 L + 1] before
  // phase 2, [4 L + 2] jobs after level L, [4 L + 3] free copies of level L
  for (uint32_t L = 1; L <= maxlen; ++L) {
    const uint32_t cnt = lv[L], m = lv[LV_N + L];
    lv_g0[L] = g0;
    uint32_t* mk = marks + 4 * L;
    if (L == 1) LAUNCH(k_ilr_mark, dim3(1), dim3(1), 0, s, dr, mk, nullptr);
    if (L > 1) {  // (which also takes the level's slots mark)
      LAUNCH(k_ilr_jobs, dim3(16), dim3(BLOCK), 0, s, a, L, gk, gsz - 1, slot2grp, marks + 4 * (L - 1) - 2,
             marks + 4 * (L - 1) + 2, mk + 3, mk);
      LAUNCH(k_ilr_free, dim3(1), dim3(64), 0, s, a, L, mk + 3, empty);
    }
    if (cnt) {
      // the level's LDS from its largest group (mirror: its Adds; private
      // table: ilr_pcap of them, when that fits PT_LDS)
      const uint32_t amax = lv[2 * LV_N + L];
      const uint32_t lrn = std::max<uint32_t>(64u, std::min<uint32_t>(ILR_LREC, (amax + 63) & ~63u));
      const uint32_t pcm = ilr_pcap(amax);
      const uint32_t ptn = std::max<uint32_t>(64u, pcm <= PT_LDS ? pcm : PT_LDS);
      const size_t lv_lds = lrn * sizeof(uint4) + ptn * (sizeof(long long) + 2 * sizeof(uint32_t));
      LAUNCH(k_ilr_prep, dim3(grid_for(m, BLOCK, 1024)), dim3(BLOCK), 0, s, a, o, vs, p0, p0 + m);
      for (uint32_t ph = 1; ph <= 2; ++ph) {
        LAUNCH(k_ilr_level, dim3(cnt), dim3(64), lv_lds, s, a, o, vs, gbeg, gend, g0, L, ph, st, lrn, ptn);
        // (phase 1's publish takes phase 2's slots mark, phase 2's the level's jobs mark)
        LAUNCH(k_ilr_publish, dim3(cnt + 64), dim3(BLOCK), 0, s, a.T, a.H, qoff, qn, J.gflag, g0, cnt, ph,
               a.committed, mk + ph - 1, dr, a.cap_slots, ph == 1 ? mk + 1 : nullptr, ph == 2 ? mk + 2 : nullptr);
      }
      ++levels;
    } else {  // (only free copies: their slots into the shared hash)
      LAUNCH(k_ilr_publish, dim3(64), dim3(BLOCK), 0, s, a.T, a.H, qoff, qn, J.gflag, g0, 0u, 1u, a.committed, mk,
             dr, a.cap_slots, nullptr, mk + 2);
    }
    g0 += cnt;
    p0 += m;
  }
  if ((r = sync_read(c))) return r;
  DevResult h = *c->hres;
  if (h.ilr_slots > a.cap_slots || h.ilr_slots > a.scap || h.ilr_slots > a.hash_limit)
    h.ilr_overflow |= IO_SLOTS;  // (slots counted by a pool but never taken lie beyond the room)
  const long long new_ts = t->timestamp + h.own_ok_adds;
  const bool drift = replica_of(new_ts) != replica_of(t->timestamp);
  static const bool debug = getenv("CRDTM_ILR_DEBUG") != nullptr;
  if (debug)
    fprintf(stderr,
            "ilr: n=%u groups=%u levels=%u jobs=%u conflict=%u why=%#x overflow=%#x drift=%d err=%d slots+%u\n", n,
            G, levels, h.ilr_jobs, h.ilr_conflict, h.ilr_why, h.ilr_overflow, drift ? 1 : 0,
            h.err_index == NONE ? -1 : static_cast<int>(h.err_index),
            h.ilr_slots - static_cast<uint32_t>(t->n_slots));
  if (a.stats) {  // the slowest groups: ops, walk steps, tombstone skips, quirks, orphan marks, us
    std::vector<unsigned long long> hs(8ULL * G);
    HIP_CHECK(hipMemcpy(hs.data(), a.stats, hs.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    std::vector<uint32_t> ord(G);
    for (uint32_t g = 0; g < G; ++g) ord[g] = g;
    std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return hs[8 * x + 5] > hs[8 * y + 5]; });
    unsigned long long tw = 0, ts = 0, to = 0;
    for (uint32_t g = 0; g < G; ++g) {
      tw += hs[8 * g + 1];
      ts += hs[8 * g + 2];
      to += hs[8 * g];
    }
    fprintf(stderr, "ilr stats: ops %llu walk %llu skip %llu\n", to, tw, ts);
    for (uint32_t q = 0; q < std::min<uint32_t>(G, 6); ++q) {
      const unsigned long long* v = &hs[8 * ord[q]];
      fprintf(stderr, "  L%llu ops %llu walk %llu skip %llu quirk %llu mark %llu (%llu)  %.1f us\n", v[6], v[0],
              v[1], v[2], v[3], v[4], v[7], v[5] / 100.0);
    }
  }
  // every level's changes, undone deepest level first
  auto rollback = [&]() {
    for (uint32_t L = maxlen; L >= 1; --L)
      if (lv[L])
        LAUNCH(k_ilr_rollback, dim3(grid_for(lv[L])), dim3(BLOCK), 0, s, t->d, undo, ucnt, gbeg, lv_g0[L], lv[L]);
    t->ilr_valid = false;  // (its hash, member lists and event times hold the batch)
  };
  if (h.ilr_conflict || h.ilr_overflow || drift || h.err_index != NONE) {
    rollback();
    if (h.ilr_conflict || h.ilr_overflow || drift) {  // the re-merge decides
      HIP_CHECK(hipStreamSynchronize(s));
      ws.used = mark0;
      return CRDTM_OK;
    }
    // the first failing op in batch order (every op saw only earlier ops)
    *handled = true;
    res->path_taken = CRDTM_PATH_DICT_REPLAY;
    res->flags |= CRDTM_FLAG_DICT_INCR;
    uint8_t est = 0;
    HIP_CHECK(hipMemcpyAsync(&est, st + h.err_index, 1, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    res->code = est == ST_INVALID ? CRDTM_INVALID_PATH : CRDTM_OPERATION_FAILED;
    res->err_index = h.err_index;
    if (st_out) LAUNCH(k_status_out, dim3(grid_for(n)), dim3(BLOCK), 0, s, st, n, h.err_index, st_out);
    return CRDTM_OK;
  }
  // ---- commit: log (applied ops in order), sources, dropped children, replicas ----
  // Until k_ilr_fix runs, the level changes can still be undone: a failure
  // there (an arena overflow in a scan's workspace, which crdtm_apply retries
  // with a larger arena, or an error) rolls the state back first.
  // (test hook, env CRDTM_ILR_FAIL_COMMIT=<token>: the first commit that
  // sees a new token fails here with an arena overflow, so the tests can
  // check the rollback and crdtm_apply's retry)
  static thread_local std::string fail_token;
  try {
    const char* fe = test_hooks() ? getenv("CRDTM_ILR_FAIL_COMMIT") : nullptr;
    if (fe && fe[0] && fail_token != fe) {
      fail_token = fe;
      throw ArenaOverflow(ws.cap + 1);
    }
    LAUNCH(k_post_flags, dim3(grid_for(n)), dim3(BLOCK), 0, s, o, st, appl, plen);
    if (!(r = scan_excl_u32(appl, appl, n, &dr->log_n, ws, s))) r = scan_excl_u32(plen, plen, n, &dr->log_npath, ws, s);
  } catch (const ArenaOverflow&) {
    rollback();
    throw;
  }
  if (r) {
    rollback();
    return r;
  }
  *handled = true;
  LAUNCH(k_log, dim3(grid_for(n)), dim3(BLOCK), 0, s, o, st, t->d, static_cast<uint32_t>(t->log_n),
         static_cast<uint32_t>(t->log_npath), appl, plen);
  LAUNCH(k_log_tail, dim3(1), dim3(1), 0, s, t->d, static_cast<uint32_t>(t->log_n), &dr->log_n,
         static_cast<uint32_t>(t->log_npath), &dr->log_npath);
  const uint32_t lo = static_cast<uint32_t>(t->n_slots), hi = h.ilr_slots;
  const uint32_t fx = grid_for(static_cast<uint64_t>(hi - lo) + nu, BLOCK, 4096);
  LAUNCH(k_ilr_fix, dim3(fx), dim3(BLOCK), 0, s, t->d, lo, hi, undo, static_cast<uint32_t>(nu), appl,
         static_cast<uint32_t>(t->log_n), X->ev);
  LAUNCH(k_ilr_ev_reset, dim3(fx), dim3(BLOCK), 0, s, lo, hi, undo, static_cast<uint32_t>(nu), X->ev);
  // (past k_ilr_fix only a device error can fail: the state is then lost
  // with the device context, and the index is dropped)
  if (!(r = replica_fold_into(c, o, st, rep, rlist, s)) && st_out)
    LAUNCH(k_status_out, dim3(grid_for(n)), dim3(BLOCK), 0, s, st, n, NONE, st_out);
  if (r || (r = sync_read(c)) || (r = take_replicas(t, rep))) {
    t->ilr_valid = false;
    return r;
  }
  X->hused = h.ilr_slots;
  t->n_slots = h.ilr_slots;
  t->n_dicts = h.ilr_dicts;
  t->last_begin = t->log_n;
  t->log_n += c->hres->log_n;
  t->log_npath += c->hres->log_npath;
  t->last_end = t->log_n;
  t->timestamp = new_ts;
  if (t->max_depth < maxlen) t->max_depth = maxlen;
  t->doc_valid = false;
  t->flat_clean = false;
  t->kidx_valid = false;
  res->path_taken = CRDTM_PATH_DICT_REPLAY;
  res->flags |= CRDTM_FLAG_DICT_INCR;
  res->n_applied = h.n_applied;
  res->n_already = h.n_already;
  res->serial_dicts = G;
  res->serial_ops = n;
  res->serial_max = levels;
  res->code = CRDTM_OK;
  return CRDTM_OK;
}

}  // namespace crdtm

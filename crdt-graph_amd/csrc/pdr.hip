// pdr.hip — per-dict exact replay (PDR) for fresh trees whose dicts see
// Deletes before later Adds, the batches the closed form's guard rejects
// (G_DEL_BEFORE_ADD; configs 1-2 of BASELINE.json).
//
// The reference applies a batch one op at a time (src/CRDTree.elm:224-232,
// :275-295). Ops in different children dicts only interact through path
// resolution: an op's path crosses keys of ancestor dicts, and a key stays
// bound to its original node until that node's first Delete — except when
// findInsertion's copy quirk (src/Internal/Node.elm:93-104)
// later re-fills the tombstoned slot with a copy of a live sibling. So:
//
//  1. K1 (merge.hip, level-synchronous lookup) resolves every path as if no
//     slot were ever re-filled, and tags each op with "reached its leaf dict"
//     or the tombstoned node where the path stopped (Work.tag);
//  2. one wave per children dict replays that dict's reached ops in batch
//     order with the reference's literal addAfter/findInsertion/delete
//     semantics, on a slot state held in LDS (P2);
//  3. an op whose path stopped at a key re-filled before it ran would have
//     descended into the copy: conflict, and the batch goes to the sequential
//     replay (P3). Otherwise every status is exact;
//  4. assembly (P5): the surviving dicts are the original dicts whose owner
//     chain is live and un-copied, plus one snapshot per copied slot — the
//     deep copy (Replayer::deep_copy, merge.hip) of the source dict as of the
//     copy time, rebuilt by replaying the source dict's op prefix (nested
//     level by level). Slots are numbered by scans and written into TreeDev.
//
// Slot numbering inside a dict: the dict's keys are the timestamps of the
// Adds that reach it first (no collision: one dict per timestamp), so slot r
// = rank of the key among them (sentinel = 0) and findInsertion's key test
// `ts > key(rn)` becomes `r > rn`. A slot is one 32-bit word: next slot (24
// bits) | flags (8 bits). What a copy carries (source node, children view)
// lives in side arrays written only when the quirk fires.
//
// Regions: original dict D (D = owner op index, n = root) owns positions
// [rbase[D], rbase[D+1]): olist holds the dict's ops in batch order there (a
// NONE pad last, the sort needs unique keys); rop[rbase[D] + r] is the Add
// that created slot r; the slot words of rank r live at base[I] + r for each
// instance I of D (the original, then its snapshots).

#include <cstdlib>

#include "engine.h"

namespace crdtm {

#ifdef PDR_STATS  // walk statistics of the replay (debug builds only)
__device__ unsigned long long g_pdr_stats[8];
__device__ bool pdr_stat_on;  // (unused)
#define PDR_STAT(k) do { ++g_stc[k]; } while (0)
#define PDR_CAT(c) (q_cat = (c))
#else
#define PDR_STAT(k) do { } while (0)
#define PDR_CAT(c) do { } while (0)
#endif

// A wave-uniform load of data no kernel writes while this one runs, through
// the scalar data cache (counted by lgkmcnt: it does not wait for the wave's
// outstanding vector stores the way a vector load does)
typedef const __attribute__((address_space(4))) uint32_t* ConstU32;
__device__ __forceinline__ uint32_t ld_scalar(const uint32_t* p, uint32_t i) { return ((ConstU32)p)[i]; }

constexpr uint32_t PM = 0xFFFFFFu;  // slot index mask; PM = end of chain
enum : uint32_t { SF_TOMB = 1u << 24, SF_ORPHAN = 2u << 24, SF_COPY = 4u << 24, SF_MADE = 8u << 24 };
constexpr uint32_t OW_NF = PM;           // op word code: the target/anchor is missing (NotFound)
constexpr uint32_t PDR_SMALL = 4096;     // slots per dict held in static LDS

struct PdrInst {       // per instance: originals 0..n (n = root), snapshots n+1+j
  uint32_t* base;      // first slot position
  uint32_t* src;       // snapshots: source original dict
  uint32_t* bound;     // snapshots: replay the ops < bound
  uint32_t* pi;        // snapshots: parent instance
  uint32_t* pl;        // snapshots: parent slot (rank)
};

struct PdrCtx {
  OpsDev o;
  TsIndex ix;
  const uint32_t* leaf;
  const uint32_t* rbase;   // [n + 2]
  const uint32_t* cbase;   // [n + 2] key counts, scanned: K_D = cbase[D+1] - cbase[D]
  const uint32_t* olist;   // per region position: op index (batch order)
  const unsigned long long* opw;  // per region position: op word
  uint32_t* rankof;        // per op: slot (rank) of the Add's key in its dict, 0 = not a key
  uint32_t* rop;           // per region position: Add op of rank r
  uint32_t* tcopy;         // node op -> first op whose copy quirk re-filled its key's slot
  uint32_t* S;             // per slot position: next | flags
  uint32_t* qsrc;          // per slot position, COPY slots: node carried
  uint32_t* qcd;           // ... its children: original dict
  uint32_t* qcb;           // ... as of op index (NONE: current)
  uint32_t* ch;            // assembly: snapshot instance of a slot's children
  uint32_t* inst;          // per slot position: instance (NONE: unused room)
  uint4* log;              // per original dict (4 entries per region position): slot writes in op order
  uint32_t* logn;          // per dict: entries logged, NONE = no log (small dict or room exhausted)
  uint32_t* ilog;          // per instance: snapshots rebuilt from the log -> prefix length, else NONE
  uint32_t log_min;        // slots a dict needs to keep a change log
  uint32_t* where;         // per slot position: pdr_blocked's compaction scratch
  uint32_t blk_spare;      // 0, or (tests) blocks beyond a repacked chain before pdr_blocked compacts
  // guard-G statistics (env CRDTM_GUARD_STATS=1; nullptr: off). An Add fails
  // guard G when its findInsertion walk meets a Tombstone whose key is above
  // its own timestamp — a node that canonical RGA would pass and that was
  // deleted before the Add: the first such Add of a
  // dict ends the prefix the closed form could serve exactly.
  unsigned long long* gcount;  // [0] Adds that walked, [1] G-failing ones, [2] ops before each dict's first failure,
                               // [3] ops the dicts' replays reached
  PdrInst I;
};

// Change log of an original dict's replay: {op, slot | kind << 30, a, b};
// kind 0: slot word := a; kind 1: copy payload (node carried a, children dict
// b); kind 2: children as-of op a. A snapshot as of op b is the last write per
// slot among the entries with op < b, found in parallel (k_pdr_snap_*).
constexpr uint32_t PDR_LOG_MIN = 512;  // smaller dicts re-replay their snapshots (env CRDTM_PDR_LOG_MIN)
constexpr uint32_t PDR_LANE = 32;      // dicts of at most this many slots replay on one lane (k_pdr_lane)

__device__ __forceinline__ uint32_t pdr_kcount(const PdrCtx& p, uint32_t D) { return p.cbase[D + 1] - p.cbase[D]; }

__device__ __forceinline__ uint32_t pdr_first_op(const PdrCtx& p, uint32_t D) {
  const uint32_t b = p.rbase[D];
  return p.rbase[D + 1] - b > 1 ? p.olist[b] : NONE;
}

// ---- P1: group the reached ops by leaf dict ----
__global__ void __launch_bounds__(BLOCK) k_pdr_init(uint32_t n, uint32_t* cnt, uint32_t* fill, uint32_t* ccnt,
                                                    uint32_t* cfill, uint32_t* rankof, uint32_t* tcopy) {
  GRID_STRIDE(i, n + 2) {
    cnt[i] = 0;
    fill[i] = 0;
    ccnt[i] = 0;
    cfill[i] = 0;
    if (i < n) {
      rankof[i] = 0;
      tcopy[i] = NONE;
    }
  }
}

__device__ __forceinline__ bool pdr_is_key(const OpsDev& o, const TsIndex& ix, uint32_t i) {
  if (o.kind[i] != CRDTM_ADD) return false;
  const long long ts = o.ts[i];
  return ts != 0 && tsindex_find(ix, ts) == i;
}

// region size: one position per reached op + 1 (sentinel slot / list pad);
// the root dict always exists
__global__ void __launch_bounds__(BLOCK) k_pdr_size(uint32_t n, uint32_t* cnt) {
  GRID_STRIDE(d, n + 1) {
    const uint32_t c = cnt[d];
    cnt[d] = (c || d == n) ? c + 1 : 0u;
  }
}

// Grouping without atomics (replaces k_pdr_count / k_pdr_scatter, which
// took two random device atomics per op): a stable radix sort of the ops by
// dict (key NONE: not reached) keeps each dict's ops in batch order; the
// group sizes come from the sorted keys, and a scan over the sorted positions
// of "this op is a key" (the first Add of its timestamp) numbers the keys
// inside each dict.
// (val = the op | is-a-key << 31, decided here in op order: coalesced kinds
// and timestamps; op indices stay below 2^31)
__global__ void __launch_bounds__(BLOCK) k_pdr_keys(OpsDev o, TsIndex ix, const uint32_t* tag, const uint32_t* cur,
                                                    uint32_t* key, uint32_t* val, uint32_t* nitems) {
  const uint32_t n = o.n;
  if (blockIdx.x == 0 && threadIdx.x == 0) *nitems = n;
  GRID_STRIDE(i, n) {
    const bool reached = tag[i] == PDR_REACHED;
    key[i] = reached ? cur[i] : NONE;
    val[i] = i | ((reached && pdr_is_key(o, ix, i)) ? 0x80000000u : 0u);
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_kflag(uint32_t n, const uint32_t* sv, uint32_t* kf) {
  GRID_STRIDE(k, n + 1) kf[k] = k < n ? sv[k] >> 31 : 0u;
}

// per dict (at its last sorted position): ops (into rbase) and keys (into cbase)
__global__ void __launch_bounds__(BLOCK) k_pdr_gcount(uint32_t m, const uint32_t* sk, const uint32_t* gs,
                                                      const uint32_t* X, uint32_t* cnt, uint32_t* ccnt) {
  GRID_STRIDE(k, m) {
    const uint32_t d = sk[k];
    if (d == NONE || (k + 1 < m && sk[k + 1] == d)) continue;
    cnt[d] = k + 1 - gs[d];
    ccnt[d] = X[k + 1] - X[gs[d]];
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_place(uint32_t m, const uint32_t* sk, const uint32_t* sv,
                                                     const uint32_t* gs, const uint32_t* X, const uint32_t* rbase,
                                                     const uint32_t* cbase, uint32_t* olist, uint32_t* carr) {
  GRID_STRIDE(k, m) {
    const uint32_t d = sk[k];
    if (d == NONE) continue;
    const uint32_t g = gs[d], i = sv[k] & 0x7FFFFFFFu;
    olist[rbase[d] + (k - g)] = i;  // the pad (NONE) stays last
    if (X[k + 1] != X[k]) carr[cbase[d] + (X[k] - X[g])] = i;
  }
}

// keys sorted by ts within each dict -> ranks
__global__ void __launch_bounds__(BLOCK) k_pdr_rank(uint32_t kt, const uint32_t* carr, const uint32_t* cur,
                                                    const uint32_t* cbase, const uint32_t* rbase, uint32_t* rankof,
                                                    uint32_t* rop) {
  GRID_STRIDE(k, kt) {
    const uint32_t i = carr[k];
    const uint32_t d = cur[i];
    const uint32_t r = k - cbase[d] + 1;
    rankof[i] = r;
    rop[rbase[d] + r] = i;
  }
}

// op word: bit 63 = Delete; Add: anchor code << 24 | own rank (0 = key
// already present -> AlreadyApplied); Delete: target code (0 = the sentinel
// -> AlreadyApplied). Codes: 0 sentinel, OW_NF missing, else a rank.
__global__ void __launch_bounds__(BLOCK) k_pdr_opw(uint32_t R0, const uint32_t* olist, OpsDev o,
                                                   const uint32_t* leaf, const uint32_t* rankof,
                                                   unsigned long long* opw) {
  GRID_STRIDE(k, R0) {
    const uint32_t i = olist[k];
    if (i == NONE) continue;
    const uint32_t a = leaf[i];
    uint32_t code;
    if (a == SENT_T) code = 0;
    else if (a == MISS_T || a >= i) code = OW_NF;
    else code = rankof[a];  // a node of the same dict that came first: a key
    unsigned long long w;
    if (o.kind[i] == CRDTM_DELETE) w = (1ULL << 63) | code;
    else w = (static_cast<unsigned long long>(code) << 24) | rankof[i];
    opw[k] = w;
  }
}

// A slot word read by the whole wave (same address): moved to a scalar
// register, so the walk's tests and branches are scalar instructions.
__device__ __forceinline__ uint32_t ld_uniform(const uint32_t* S, uint32_t k) {
  return __builtin_amdgcn_readfirstlane(S[k]);
}

// nextNode's tombstone skip (src/Internal/Node.elm:257-268) from chain entry
// p (slot word wp): the first live entry from p on, or PM; *wp becomes its
// word. Tombstone runs through consecutive ranks are crossed 64 ranks at a
// time (wave-uniform: every lane runs it with the same p).
#ifdef PDR_STATS
#define STC_PARAM , unsigned long long* g_stc
#define STC_ARG , g_stc
#else
#define STC_PARAM
#define STC_ARG
#endif
__device__ __forceinline__ uint32_t pdr_next_live(const uint32_t* S, uint32_t K, uint32_t lane, uint32_t p,
                                                  uint32_t& wp STC_PARAM) {
  while (p != PM && (wp & SF_TOMB)) {
    PDR_STAT(2);
    const uint32_t q = wp & PM;
    if (q == p + 1) {
      const uint32_t e = p + lane;
      const bool in = e <= K;
      const uint32_t a = in ? S[e] : 0u;
      const unsigned long long lb = __ballot(in && (a & PM) == e + 1);
      const unsigned long long vb = __ballot(in && (a & SF_MADE) && !(a & SF_TOMB));
      const uint32_t m = lb == ~0ULL ? 64u : static_cast<uint32_t>(__builtin_ctzll(~lb));
      const uint32_t M = m < 63u ? m : 63u;
      const unsigned long long lv = vb & ((M == 63u ? ~0ULL : ((2ULL << M) - 1ULL)) & ~1ULL);
      if (lv) {
        const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(lv));
        wp = __builtin_amdgcn_readlane(a, j);
        return p + j;
      }
      p = __builtin_amdgcn_readlane(a, M) & PM;
    } else {
      p = q;
    }
    if (p == PM) break;
    wp = __builtin_amdgcn_readfirstlane(S[p]);
  }
  return p;
}

__device__ __forceinline__ void pdr_gstat_flush(const PdrCtx& p, uint32_t adds, uint32_t fails, uint32_t prefix,
                                                uint32_t ops) {
  if (ops) atomicAdd(&p.gcount[3], static_cast<unsigned long long>(ops));
  if (adds) atomicAdd(&p.gcount[0], static_cast<unsigned long long>(adds));
  if (fails) atomicAdd(&p.gcount[1], static_cast<unsigned long long>(fails));
  if (prefix) atomicAdd(&p.gcount[2], static_cast<unsigned long long>(prefix));
}

// ---- P2: the serial replay of one dict (instance) on one wave ----
// All lanes run the loop with identical values (wave-uniform control flow,
// broadcast LDS reads); S points to LDS (or to the region for huge dicts).
// MODE: 0 a snapshot instance, 1 an original dict, 2 an original dict with
// the guard-G statistics (CRDTM_GUARD_STATS=1: separate code, so the timed
// replay carries no trace of them)
template <int MODE>
__device__ void pdr_serial(const PdrCtx& p, uint8_t* st, uint32_t I, uint32_t* S) {
  constexpr bool ORIG = MODE >= 1, GST = MODE == 2;
  const uint32_t lane = threadIdx.x;
  const uint32_t D = ORIG ? I : p.I.src[I];
  const uint32_t bound = ORIG ? NONE : p.I.bound[I];
  const uint32_t base = p.I.base[I];
  const uint32_t K = pdr_kcount(p, D);
  const uint32_t rb = p.rbase[D];
#ifdef PDR_STATS
  unsigned long long g_stc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long t_start = clock64();
#endif
  for (uint32_t r = lane; r <= K; r += 64) S[r] = r == 0 ? (PM | SF_TOMB | SF_MADE) : PM;
  wave_sync();  // (one wave per workgroup)
  const uint32_t ob = rb, oe = p.rbase[D + 1] - 1;
  // change log (original dicts big enough to be worth rebuilding snapshots from)
  const bool logging = ORIG && p.log != nullptr && K + 1 >= p.log_min;
  const uint32_t lcap = 4 * (oe + 1 - rb);
  uint4* const lg = logging ? p.log + 4ULL * rb : nullptr;
  uint32_t ln = 0;
  auto logw = [&](uint32_t i, uint32_t k, uint32_t kind, uint32_t a, uint32_t b) {
    if (logging) {
      if (ln < lcap) lg[ln] = make_uint4(i, k | (kind << 30), a, b);  // uniform store (no divergence)
      ++ln;
    }
  };
  // op words stream through registers 64 at a time; the next chunk is loaded
  // while this one replays (the loads do not depend on the slot state)
  uint32_t nx_i = ob + lane < oe ? p.olist[ob + lane] : NONE;
  unsigned long long nx_w = ob + lane < oe ? p.opw[ob + lane] : 0ULL;
  constexpr bool gst = GST;
  uint32_t g_adds = 0, g_fail = 0, g_first = NONE;  // (guard-G statistics)
  for (uint32_t k0 = ob; k0 < oe; k0 += 64) {
    const uint32_t my_i = nx_i;
    const unsigned long long my_w = nx_w;
    const uint32_t kn = k0 + 64 + lane;
    nx_i = kn < oe ? p.olist[kn] : NONE;
    nx_w = kn < oe ? p.opw[kn] : 0ULL;
    const uint32_t cnt = min(64u, oe - k0);
    for (uint32_t j = 0; j < cnt; ++j) {
      const uint32_t i = __builtin_amdgcn_readlane(my_i, j);
      const uint32_t wlo = __builtin_amdgcn_readlane(static_cast<uint32_t>(my_w), j);
      const uint32_t whi = __builtin_amdgcn_readlane(static_cast<uint32_t>(my_w >> 32), j);
      if (!ORIG && i >= bound) goto replay_done;  // (a snapshot stops at its bound; an original dict has none)
      uint8_t s;
      if (whi >> 31) {  // deleteHelp
        const uint32_t t = wlo & PM;
        if (t == 0) {
          s = ST_ALREADY;
        } else {
          const uint32_t wt = t == OW_NF ? 0u : ld_uniform(S, t);
          if (!(wt & SF_MADE)) {
            s = ST_NOTFOUND;
          } else if (wt & SF_TOMB) {
            s = ST_ALREADY;
          } else {
            S[t] = wt | SF_TOMB;
            logw(i, t, 0, wt | SF_TOMB, 0);
            s = ST_APPLIED;
          }
        }
      } else {  // addAfterHelp
        const uint32_t x = wlo & PM;
        const uint32_t an = ((wlo >> 24) | (whi << 8)) & PM;
        if (x == 0) {
          s = ST_ALREADY;
        } else if (an == OW_NF || !(ld_uniform(S, an) & SF_MADE)) {
          s = ST_NOTFOUND;
        } else {
          PDR_STAT(4);
          uint32_t node = an, nk = an;  // findInsertion
          uint32_t wn = ld_uniform(S, node);
          bool gfail = false;  // a Tombstone above x met by the walk (guard G)
          for (;;) {
            const uint32_t rn = wn & PM;
            if (rn == PM) break;
            // ts > key(rn) stops the walk whatever follows rn: decided before
            // rn's word is read (one dependent read fewer at every stop)
            if (x > rn) break;
            PDR_STAT(0);
            if (rn == node + 1 && x < rn) {
              PDR_STAT(1);
              // Window step. The chain runs through consecutive ranks from
              // node (node -> node+1 -> ...), so every key ahead is larger
              // than x: the walk visits each live entry of the run and goes
              // on (nextNode skips the run's tombstones); lane l reads rank
              // node+l. Afterwards node = the last visited entry and the
              // copy quirk's n = the rank after the entry visited before it.
              const uint32_t e = node + lane;
              const bool in = e <= K;
              const uint32_t a = in ? S[e] : 0u;
              const unsigned long long lb = __ballot(in && (a & PM) == e + 1);
              const unsigned long long vb = __ballot(in && (a & SF_MADE) && !(a & SF_TOMB));
              const uint32_t m = lb == ~0ULL ? 64u : static_cast<uint32_t>(__builtin_ctzll(~lb));  // >= 1
              const uint32_t M = m < 63u ? m : 63u;  // ranks node..node+M are chained
              const unsigned long long chained = (M == 63u ? ~0ULL : ((2ULL << M) - 1ULL)) & ~1ULL;
              const unsigned long long vis = vb & chained;
              if (vis) {
                const uint32_t vs = 63u - static_cast<uint32_t>(__builtin_clzll(vis));
                if constexpr (GST)
                  if (chained & ~vb & ((2ULL << vs) - 1ULL)) gfail = true;  // crossed a Tombstone (above x)
                const unsigned long long rest = (vis & ~(1ULL << vs)) | 1ULL;
                nk = node + (63u - static_cast<uint32_t>(__builtin_clzll(rest))) + 1u;
                wn = __builtin_amdgcn_readlane(a, vs);
                node += vs;
                continue;
              }
              // ranks node+1..node+M are tombstones: the next live entry lies past them
              if constexpr (GST) gfail = true;  // (all above x: crossed, or passed over by the stop)
              uint32_t p = __builtin_amdgcn_readlane(a, M) & PM;
              uint32_t wl = p == PM ? 0u : ld_uniform(S, p);
              p = pdr_next_live(S, K, lane, p, wl STC_ARG);
              if (p == PM) break;  // only tombstones follow: stop here
              nk = node + 1u;      // (x < node + 1: the walk goes on)
              node = p;
              wn = wl;
              continue;
            }
            uint32_t wl = ld_uniform(S, rn);
            if constexpr (GST)
              if ((wl & SF_TOMB) && x < rn) gfail = true;  // a Tombstone above x: crossed or stopped before
            const uint32_t live = pdr_next_live(S, K, lane, rn, wl STC_ARG);
            if (live == PM) break;
            nk = rn;
            node = live;
            wn = wl;
          }
          if (gst) {
            ++g_adds;
            if (gfail) {
              ++g_fail;
              g_first = min(g_first, k0 + j);
            }
          }
          const uint32_t wk = nk == node ? wn : ld_uniform(S, nk);
          S[x] = (wn & PM) | (wk & SF_ORPHAN) | SF_MADE;
          logw(i, x, 0, (wn & PM) | (wk & SF_ORPHAN) | SF_MADE, 0);
          if (nk == node) {
            S[node] = (wn & ~PM) | x;
            logw(i, node, 0, (wn & ~PM) | x, 0);
          } else {
            PDR_STAT(3);
            // copy quirk: slot nk := copy of node, next = x; the entries after
            // nk up to node drop off the chain when nk was on it
            if (!(wk & SF_ORPHAN)) {
              for (uint32_t q = wk & PM; q != PM;) {
                const uint32_t wq = ld_uniform(S, q);
                S[q] = wq | SF_ORPHAN;
                logw(i, q, 0, wq | SF_ORPHAN, 0);
                if (q == node) break;
                q = wq & PM;
              }
              wn |= SF_ORPHAN;
            }
            S[nk] = x | (wn & ~PM & ~SF_ORPHAN) | (wk & SF_ORPHAN) | SF_COPY;
            logw(i, nk, 0, x | (wn & ~PM & ~SF_ORPHAN) | (wk & SF_ORPHAN) | SF_COPY, 0);
            uint32_t cs, cd, cb;
            if (wn & SF_COPY) {
              cs = p.qsrc[base + node];
              cd = p.qcd[base + node];
              cb = p.qcb[base + node];
            } else {
              cs = cd = p.rop[rb + node];
              cb = bound;
            }
            p.qsrc[base + nk] = cs;
            p.qcd[base + nk] = cd;
            p.qcb[base + nk] = min(cb, i);
            logw(i, nk, 1, cs, cd);
            logw(i, nk, 2, min(cb, i), 0);
            if (ORIG && lane == 0) atomicMin(&p.tcopy[p.rop[rb + nk]], i);
          }
          s = ST_APPLIED;
        }
      }
      if (ORIG) st[i] = s;  // uniform store
    }
  }
replay_done:
#ifdef PDR_STATS
  if (ORIG && lane == 0 && K > 28000)
    printf("pdr big dict K=%u ops=%u adds %llu steps %llu windows %llu tomb %llu quirks %llu cycles %lld\n", K,
           p.rbase[D + 1] - p.rbase[D], g_stc[4], g_stc[0], g_stc[1], g_stc[2], g_stc[3], clock64() - t_start);
#endif
  if (ORIG && lane == 0) p.logn[D] = (logging && ln <= lcap) ? ln : NONE;
  if (gst && lane == 0) pdr_gstat_flush(p, g_adds, g_fail, (g_first == NONE ? oe : g_first) - ob, oe - ob);
  wave_sync();  // (one wave per workgroup)
  if (S != p.S + base) {
    for (uint32_t r = lane; r <= K; r += 64) p.S[base + r] = S[r];
  }
  for (uint32_t r = lane; r <= K; r += 64) p.inst[base + r] = I;
}

template <int MODE>
__global__ void __launch_bounds__(64) k_pdr_small(PdrCtx p, const uint32_t* list, uint8_t* st) {
  __shared__ uint32_t S[PDR_SMALL];
  pdr_serial<MODE>(p, st, list[blockIdx.x], S);
}

template <int MODE>
__global__ void __launch_bounds__(64) k_pdr_big(PdrCtx p, const uint32_t* list, uint8_t* st) {
  extern __shared__ uint32_t S_dyn[];
  pdr_serial<MODE>(p, st, list[blockIdx.x], S_dyn);
}

template <int MODE>
__global__ void __launch_bounds__(64) k_pdr_huge(PdrCtx p, const uint32_t* list, uint8_t* st) {
  const uint32_t I = list[blockIdx.x];
  pdr_serial<MODE>(p, st, I, p.S + p.I.base[I]);
}

// ---- P2b: the same replay over a blocked chain order (big dicts) ----
// pdr_serial follows the chain one `next` at a time: ~13 dependent steps per
// Add in config 2's two 39k-op dicts (walks cross other replicas' typing
// runs), ~470 cycles each. Here the dict's chain (from its sentinel) is also
// kept in order as a list of 64-entry blocks in LDS, one entry per lane
// {rank:15, tombstone:1}, so findInsertion's walk (src/Internal/Node.elm:
// 93-104) is decided 64 positions at a time with ballots: the compare
// positions are the entries right after the anchor or after a live entry
// (the walk compares `ts` with the raw next key of every node it visits and
// moves to the next live node), the walk stops at the first compare position
// whose rank is below x's, or where nothing live follows (Nothing from
// nextNode), and the copy quirk's key n is the entry at the compare position
// that led to the stop node. Every rank's flags and block live in LDS too
// (wf), so an op touches global memory only with stores: the slot words S
// (exact, as in pdr_serial: the assembly and the change log read them) and
// the log. (A global load would wait for every store before it: gfx9's vmcnt
// counts both.) Adds anchored at an orphan (off the chain, rare) walk the
// slot words like pdr_serial and then edit the blocks.
constexpr uint32_t BLK_E = 64;          // entries per block (one per lane)
constexpr uint32_t BLK_KMAX = 32766;    // ranks fit 15 bits; bit 15 = tombstone
constexpr uint32_t BE_T = 0x8000u;
constexpr uint32_t BE_NONE = 0xFFFFu;   // an empty lane
constexpr uint32_t BLK_MIN = PDR_SMALL;  // smaller dicts keep pdr_serial (env CRDTM_PDR_BLK_MIN)
constexpr uint32_t BLK_FILL = 56;        // entries per block after a compaction
// wf[rank]: block (11 bits, WB_NONE = off the chain) | MADE | TOMB | ORPHAN | COPY
constexpr uint32_t WB_NONE = 0x7FFu, WF_MADE = 1u << 11, WF_TOMB = 1u << 12, WF_ORPH = 1u << 13, WF_COPY = 1u << 14;
// block meta word: entries (8 bits) | next block << 8 (WB_NONE = the last block)

__device__ __forceinline__ uint32_t wf_sflags(uint32_t w) {  // the slot-word flags of a wf entry
  return ((w & WF_MADE) ? SF_MADE : 0u) | ((w & WF_TOMB) ? SF_TOMB : 0u) | ((w & WF_ORPH) ? SF_ORPHAN : 0u) |
         ((w & WF_COPY) ? SF_COPY : 0u);
}

template <int MODE>
__device__ void pdr_blocked(const PdrCtx& p, uint8_t* st, uint32_t I, uint32_t* lds, uint32_t lds_words) {
  constexpr bool ORIG = MODE >= 1, GST = MODE == 2;
  const uint32_t lane = threadIdx.x;
  const uint32_t D = ORIG ? I : p.I.src[I];
  const uint32_t bound = ORIG ? NONE : p.I.bound[I];
  const uint32_t base = p.I.base[I];
  const uint32_t K = pdr_kcount(p, D);
  const uint32_t rb = p.rbase[D];
  uint16_t* const wf = reinterpret_cast<uint16_t*>(lds);
  const uint32_t wf_words = (K + 2) / 2;
  uint32_t* const meta = lds + wf_words;
  uint32_t nbmax = min(WB_NONE, (lds_words - wf_words) / (1 + BLK_E / 2));
  if (p.blk_spare)  // (tests: few spare blocks, so compactions happen)
    nbmax = min(nbmax, (K + 1 + BLK_FILL - 1) / BLK_FILL + p.blk_spare);
  uint16_t* const ent = reinterpret_cast<uint16_t*>(meta + nbmax);
  uint32_t* const S = p.S + base;
  uint32_t* const tmp = p.where + base;  // compaction scratch
  for (uint32_t r = lane; r <= K; r += 64) {
    S[r] = r == 0 ? (PM | SF_TOMB | SF_MADE) : PM;
    wf[r] = static_cast<uint16_t>(r == 0 ? (0u | WF_MADE | WF_TOMB) : WB_NONE);
  }
  if (lane == 0) {
    ent[0] = static_cast<uint16_t>(BE_T);  // the sentinel (rank 0, a Tombstone)
    meta[0] = 1u | (WB_NONE << 8);
  }
  uint32_t nb = 1;
#ifdef PDR_STATS
  unsigned long long g_stc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long q_cnt[5] = {0, 0, 0, 0, 0}, q_cyc[5] = {0, 0, 0, 0, 0}, q_walk = 0;
#endif
  wave_sync();  // (one wave per workgroup)
  const uint32_t ob = rb, oe = p.rbase[D + 1] - 1;
  const bool logging = ORIG && p.log != nullptr && K + 1 >= p.log_min;
  const uint32_t lcap = 4 * (oe + 1 - rb);
  uint4* const lg = logging ? p.log + 4ULL * rb : nullptr;
  uint32_t ln = 0;
  auto logw = [&](uint32_t i, uint32_t k, uint32_t kind, uint32_t a, uint32_t b) {
    if (logging) {
      if (ln < lcap && lane == 0) lg[ln] = make_uint4(i, k | (kind << 30), a, b);
      ++ln;
    }
  };
  auto wfu = [&](uint32_t r) -> uint32_t { return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(wf[r])); };
  auto setwf = [&](uint32_t r, uint32_t v) {
    if (lane == 0) wf[r] = static_cast<uint16_t>(v);
  };
  auto load_blk = [&](uint32_t b, uint32_t& cnt, uint32_t& nxb) -> uint32_t {  // this lane's entry, BE_NONE past the end
    const uint32_t v = ent[b * BLK_E + lane];  // (issued with the meta read)
    const uint32_t m = __builtin_amdgcn_readfirstlane(meta[b]);
    cnt = m & 0xFFu;
    nxb = m >> 8;
    return lane < cnt ? v : BE_NONE;
  };
  auto idx_of = [&](uint32_t e, uint32_t r) -> uint32_t {
    const unsigned long long m = __ballot(e != BE_NONE && (e & 0x7FFFu) == r);
    return m ? static_cast<uint32_t>(__builtin_ctzll(m)) : BLK_E;
  };
  auto rk = [&](uint32_t e, uint32_t j) -> uint32_t { return __builtin_amdgcn_readlane(e, j) & 0x7FFFu; };
  // the first entry after block b's end, along the chain (PM: none)
  auto first_after = [&](uint32_t nxb) -> uint32_t {
    for (uint32_t bb = nxb; bb != WB_NONE;) {
      const uint32_t m = __builtin_amdgcn_readfirstlane(meta[bb]);
      if (m & 0xFFu) return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ent[bb * BLK_E])) & 0x7FFFu;
      bb = m >> 8;
    }
    return PM;
  };
  // repack the whole chain BLK_FILL entries per block (when a split finds no free block)
  auto compact = [&]() {
    uint32_t pos = 0;
    for (uint32_t b = 0; b != WB_NONE;) {
      uint32_t cnt, nxb;
      const uint32_t e = load_blk(b, cnt, nxb);
      if (lane < cnt) tmp[pos + lane] = e;
      pos += cnt;
      b = nxb;
    }
    __threadfence();  // the scratch writes land before they are read back (and no stale L1 lines)
    const uint32_t nbn = (pos + BLK_FILL - 1) / BLK_FILL;
    for (uint32_t k = 0; k < nbn; ++k) {
      const uint32_t len = min(BLK_FILL, pos - k * BLK_FILL);
      const uint32_t e = lane < len ? tmp[k * BLK_FILL + lane] : BE_NONE;
      if (lane < len) {
        ent[k * BLK_E + lane] = static_cast<uint16_t>(e);
        const uint32_t r = e & 0x7FFFu;
        wf[r] = static_cast<uint16_t>((wf[r] & ~WB_NONE) | k);
      }
      if (lane == 0) meta[k] = len | ((k + 1 < nbn ? k + 1 : WB_NONE) << 8);
    }
    nb = nbn;
  };
  // v becomes the entry after rank `prev`, which sits at index i of block b (e, cnt, nxb: block b loaded)
  auto blk_insert_e = [&](uint32_t prev, uint32_t b, uint32_t i, uint32_t v, uint32_t e, uint32_t cnt,
                          uint32_t nxb) {
    if (cnt == BLK_E) {
      if (nb >= nbmax) {  // no free block: repack, then find prev again
        compact();
        PDR_STAT(3);
        b = wfu(prev) & WB_NONE;
        e = load_blk(b, cnt, nxb);
        i = idx_of(e, prev);
      }
    }
    if (cnt == BLK_E) {  // split: the upper half moves to a fresh block
      const uint32_t b2 = nb++;
      PDR_STAT(2);
      if (lane >= 32) {
        ent[b2 * BLK_E + lane - 32] = static_cast<uint16_t>(e);
        const uint32_t r = e & 0x7FFFu;
        wf[r] = static_cast<uint16_t>((wf[r] & ~WB_NONE) | b2);
      }
      if (lane == 0) {
        meta[b2] = 32u | (nxb << 8);
        meta[b] = 32u | (b2 << 8);
      }
      const bool hi = i >= 32;  // the insert goes to the new upper block
      if (hi) {
        b = b2;
        i -= 32;
        e = __shfl_down(e, 32, 64);
      } else {
        nxb = b2;
      }
      if (lane >= 32) e = BE_NONE;
      cnt = 32;
    }
    if (lane > i && lane < cnt) ent[b * BLK_E + lane + 1] = static_cast<uint16_t>(e);
    if (lane == i + 1) ent[b * BLK_E + lane] = static_cast<uint16_t>(v);
    if (lane == 0) {
      meta[b] = (cnt + 1) | (nxb << 8);
      const uint32_t r = v & 0x7FFFu;
      wf[r] = static_cast<uint16_t>((wf[r] & ~WB_NONE) | b);
    }
  };
  auto blk_insert = [&](uint32_t prev, uint32_t v) {
    const uint32_t b = wfu(prev) & WB_NONE;
    uint32_t cnt, nxb;
    const uint32_t e = load_blk(b, cnt, nxb);
    blk_insert_e(prev, b, idx_of(e, prev), v, e, cnt, nxb);
  };
  // copy quirk: the chain entries after rank `after` up to and including
  // rank `last` drop off the chain (orphans): off the blocks, ORPHAN in wf
  // and in their slot words (+ log)
  auto blk_orphan_after = [&](uint32_t after, uint32_t last, uint32_t op) {
    uint32_t b = wfu(after) & WB_NONE;
    uint32_t cnt, nxb;
    uint32_t e = load_blk(b, cnt, nxb);
    uint32_t s0 = idx_of(e, after) + 1;
    for (;;) {
      const unsigned long long mr = __ballot(lane >= s0 && lane < cnt && (e & 0x7FFFu) == last);
      const uint32_t end = mr ? static_cast<uint32_t>(__builtin_ctzll(mr)) + 1u : cnt;
      const uint32_t k = end > s0 ? end - s0 : 0u;
      const uint32_t succ_last = end < cnt ? rk(e, end) : first_after(nxb);
      const uint32_t en = __shfl_down(e, 1, 64);
      if (lane >= s0 && lane < end) {
        const uint32_t q = e & 0x7FFFu;
        const uint32_t nq = lane + 1 < end ? (en & 0x7FFFu) : succ_last;
        const uint32_t w = (wf[q] | WF_ORPH) | WB_NONE;
        wf[q] = static_cast<uint16_t>(w);
        const uint32_t wq = nq | wf_sflags(w);
        S[q] = wq;
        if (logging && ln + (lane - s0) < lcap) lg[ln + (lane - s0)] = make_uint4(op, q, wq, 0u);
      }
      ln += logging ? k : 0u;
      if (k) {
        if (lane >= end && lane < cnt) ent[b * BLK_E + lane - k] = static_cast<uint16_t>(e);
        if (lane == 0) meta[b] = (cnt - k) | (nxb << 8);
      }
      if (mr || nxb == WB_NONE) break;
      b = nxb;
      s0 = 0;
      e = load_blk(b, cnt, nxb);
    }
  };
  uint32_t nx_i = ob + lane < oe ? p.olist[ob + lane] : NONE;
  unsigned long long nx_w = ob + lane < oe ? p.opw[ob + lane] : 0ULL;
  constexpr bool gst = GST;
  uint32_t g_adds = 0, g_fail = 0, g_first = NONE;  // (guard-G statistics, as in pdr_serial)
  for (uint32_t k0 = ob; k0 < oe; k0 += 64) {
    const uint32_t my_i = nx_i;
    const unsigned long long my_w = nx_w;
    const uint32_t kn = k0 + 64 + lane;
    nx_i = kn < oe ? p.olist[kn] : NONE;
    nx_w = kn < oe ? p.opw[kn] : 0ULL;
    const uint32_t cntop = min(64u, oe - k0);
    for (uint32_t jo = 0; jo < cntop; ++jo) {
      const uint32_t i = __builtin_amdgcn_readlane(my_i, jo);
      const uint32_t wlo = __builtin_amdgcn_readlane(static_cast<uint32_t>(my_w), jo);
      const uint32_t whi = __builtin_amdgcn_readlane(static_cast<uint32_t>(my_w >> 32), jo);
      if (!ORIG && i >= bound) goto replay_done;  // (a snapshot stops at its bound; an original dict has none)
#ifdef PDR_STATS
      const long long q_t0 = clock64();
      uint32_t q_cat = 4;
#endif
      uint8_t s;
      if (whi >> 31) {  // deleteHelp
        PDR_CAT(0);
        const uint32_t t = wlo & PM;
        const uint32_t w = (t == 0 || t == OW_NF) ? 0u : wfu(t);
        if (t == 0) {
          s = ST_ALREADY;
        } else if (!(w & WF_MADE)) {
          s = ST_NOTFOUND;
        } else if (w & WF_TOMB) {
          s = ST_ALREADY;
        } else {
          const uint32_t b = w & WB_NONE;
          uint32_t nxt;
          if (b != WB_NONE) {  // on the chain: the entry becomes a Tombstone
            uint32_t cnt, nxb;
            const uint32_t e = load_blk(b, cnt, nxb);
            const uint32_t j = idx_of(e, t);
            if (lane == j) ent[b * BLK_E + lane] = static_cast<uint16_t>(e | BE_T);
            nxt = j + 1 < cnt ? rk(e, j + 1) : first_after(nxb);
          } else {  // an orphan: its next key lives in its slot word only
            nxt = ld_uniform(S, t) & PM;
          }
          setwf(t, w | WF_TOMB);
          const uint32_t wt = nxt | wf_sflags(w | WF_TOMB);
          if (lane == 0) S[t] = wt;
          logw(i, t, 0, wt, 0);
          s = ST_APPLIED;
        }
      } else {  // addAfterHelp
        const uint32_t x = wlo & PM;
        const uint32_t an = ((wlo >> 24) | (whi << 8)) & PM;
        const uint32_t wa = (x == 0 || an == OW_NF) ? 0u : wfu(an);
        if (x == 0) {
          s = ST_ALREADY;
        } else if (!(wa & WF_MADE)) {
          s = ST_NOTFOUND;
        } else {
          // an anchor on the chain walks the blocks; an orphan anchor (off the
          // chain, rare) first follows the slot words as pdr_serial does, and
          // once a live step lands on a chain entry the rest of the walk is the
          // block walk anchored there
          uint32_t an_w = an, wa_w = wa;
          bool ow = (wa & WB_NONE) == WB_NONE;
          uint32_t o_node = an, o_nk = an, o_wn = 0;
          bool o_gfail = false;
          if (ow) {
            o_wn = ld_uniform(S, an);
            for (;;) {
              const uint32_t rn = o_wn & PM;
              if (rn == PM) break;
              if (x > rn) break;  // (decided before rn's word is read)
              uint32_t wl = ld_uniform(S, rn);
              if constexpr (GST)
                if ((wl & SF_TOMB) && x < rn) o_gfail = true;
              const uint32_t live = pdr_next_live(S, K, lane, rn, wl STC_ARG);
              if (live == PM) break;
              o_nk = rn;
              o_node = live;
              o_wn = wl;
              if (live == rn) {
                const uint32_t wv = wfu(live);
                if ((wv & WB_NONE) != WB_NONE) {
                  an_w = live;
                  wa_w = wv;
                  ow = false;
                  break;
                }
              }
            }
          }
          if (!ow) {
            // ---- findInsertion over the blocks ----
            const uint32_t ba = wa_w & WB_NONE;
            uint32_t b = ba, cnt, nxb;
            uint32_t e = load_blk(b, cnt, nxb);
            const uint32_t i0 = idx_of(e, an_w);
            uint32_t s0 = i0 + 1;
            bool carry = true;        // the entry before the window: live or the anchor
            uint32_t prev_r = an_w;     // that entry
            uint32_t nkc = an_w;        // the compare entry that led to the latest node
            bool at_anchor = true;    // no node visited yet
            uint32_t node, nk, nxt;   // result (nxt: the rank after node, PM = none)
            uint32_t cur_b = b, cur_e = e, cur_cnt = cnt, cur_nxb = nxb, node_i = i0;  // node's block (when loaded)
            bool gfail = o_gfail;  // a Tombstone above x met by the walk (guard G)
            for (;;) {
              const bool valid = lane >= s0 && lane < cnt;
              const unsigned long long ml = __ballot(valid && !(e & BE_T));
              const unsigned long long mkey = __ballot(valid && (e & 0x7FFFu) < x);
              const unsigned long long mval = __ballot(valid);
              unsigned long long mc = (ml << 1) & mval;
              if (carry && s0 < cnt) mc |= 1ULL << s0;
              const unsigned long long m1 = mc & mkey;
              const int j1 = m1 ? __builtin_ctzll(m1) : -1;
              int j2 = -1;
              if (ml) {
                const int ll = 63 - __builtin_clzll(ml);
                if (static_cast<uint32_t>(ll) + 1 < cnt) j2 = ll + 1;
              } else if (carry && s0 < cnt) {
                j2 = static_cast<int>(s0);
              }
              int j = -1;
              if (j1 >= 0 && (j2 < 0 || j1 <= j2)) {
                j = j1;
              } else if (j2 >= 0) {  // nothing live after j2 in this block: anything live further on?
                bool any = false;
                for (uint32_t bb = nxb; bb != WB_NONE && !any;) {
                  uint32_t c2, n2;
                  const uint32_t e2 = load_blk(bb, c2, n2);
                  any = __ballot(lane < c2 && !(e2 & BE_T)) != 0;
                  PDR_STAT(1);
                  bb = n2;
                }
                if (!any) j = j2;  // nextNode is Nothing: stop
              }
              if (j >= 0) {
                const uint32_t uj = static_cast<uint32_t>(j);
                // compare entries passed before the stop are above x; the stop
                // entry is above x only when nothing live follows it
                if constexpr (GST) {
                  const unsigned long long mtomb = mval & ~ml;
                  if ((mc & mtomb & ((1ULL << uj) - 1ULL)) || (((mtomb & ~mkey) >> uj) & 1ULL)) gfail = true;
                }
                nxt = rk(e, uj);
                if (uj == s0) {  // node = the entry before the window
                  node = prev_r;
                  nk = at_anchor ? an_w : nkc;
                  if (b != ba || !at_anchor) {  // node sits in an earlier block: reload at insert
                    cur_b = WB_NONE;
                  } else {
                    cur_b = b;
                    cur_e = e;
                    cur_cnt = cnt;
                    cur_nxb = nxb;
                    node_i = i0;
                  }
                } else {
                  node = rk(e, uj - 1);
                  const unsigned long long mcl = mc & ((2ULL << (uj - 1)) - 1ULL);
                  nk = mcl ? rk(e, 63u - static_cast<uint32_t>(__builtin_clzll(mcl))) : nkc;
                  cur_b = b;
                  cur_e = e;
                  cur_cnt = cnt;
                  cur_nxb = nxb;
                  node_i = uj - 1;
                }
                break;
              }
              if constexpr (GST)
                if (mc & mval & ~ml) gfail = true;  // (no stop in this block: every compare entry passed)
              if (mc) nkc = rk(e, 63u - static_cast<uint32_t>(__builtin_clzll(mc)));
              if (cnt > s0) {
                carry = (ml >> (cnt - 1)) & 1ULL;
                prev_r = rk(e, cnt - 1);
                at_anchor = false;
              }
              if (nxb == WB_NONE) {  // the chain ends: `next node` is Nothing
                node = prev_r;
                nk = at_anchor ? an_w : nkc;
                nxt = PM;
                if (cnt > s0 || (at_anchor && b == ba)) {
                  cur_b = b;
                  cur_e = e;
                  cur_cnt = cnt;
                  cur_nxb = nxb;
                  node_i = cnt > s0 ? cnt - 1 : i0;
                } else {
                  cur_b = WB_NONE;
                }
                break;
              }
              b = nxb;
              s0 = 0;
              e = load_blk(b, cnt, nxb);
              PDR_STAT(0);
            }
#ifdef PDR_STATS
            q_walk += clock64() - q_t0;
            PDR_STAT(4);
#endif
            if (gst) {
              ++g_adds;
              if (gfail) {
                ++g_fail;
                g_first = min(g_first, k0 + jo);
              }
            }
            // ---- the two inserts (src/Internal/Node.elm:87-89) ----
            const uint32_t wx = nxt | SF_MADE;
            if (lane == 0) S[x] = wx;
            setwf(x, WF_MADE | WB_NONE);
            logw(i, x, 0, wx, 0);
            const uint32_t wnode = wfu(node);
            PDR_CAT(nk == node ? 1 : 2);
            if (nk == node) {
              const uint32_t wn = wf_sflags(wnode) | x;
              if (lane == 0) S[node] = wn;
              logw(i, node, 0, wn, 0);
              if (cur_b != WB_NONE) blk_insert_e(node, cur_b, node_i, x, cur_e, cur_cnt, cur_nxb);
              else blk_insert(node, x);
            } else {
              // copy quirk: slot nk := copy of node with next = x;
              // the entries after nk up to node drop off the chain
              blk_orphan_after(nk, node, i);
              const uint32_t wk = x | SF_MADE | SF_COPY;
              if (lane == 0) S[nk] = wk;
              setwf(nk, (wfu(nk) & WB_NONE) | WF_MADE | WF_COPY);
              logw(i, nk, 0, wk, 0);
              uint32_t cs, cd, cb;
              if (wnode & WF_COPY) {
                cs = p.qsrc[base + node];
                cd = p.qcd[base + node];
                cb = p.qcb[base + node];
              } else {
                cs = cd = ld_scalar(p.rop, rb + node);
                cb = bound;
              }
              if (lane == 0) {
                p.qsrc[base + nk] = cs;
                p.qcd[base + nk] = cd;
                p.qcb[base + nk] = min(cb, i);
              }
              logw(i, nk, 1, cs, cd);
              logw(i, nk, 2, min(cb, i), 0);
              if (ORIG && lane == 0) atomicMin(&p.tcopy[ld_scalar(p.rop, rb + nk)], i);
              {  // nk's entry is live again (a copy of node)
                const uint32_t bk = wfu(nk) & WB_NONE;
                uint32_t c3, n3;
                const uint32_t e3 = load_blk(bk, c3, n3);
                const uint32_t jk = idx_of(e3, nk);
                if (lane == jk) ent[bk * BLK_E + lane] = static_cast<uint16_t>(e3 & 0x7FFFu);
                blk_insert_e(nk, bk, jk, x, e3 & (lane == jk ? 0x7FFFu : 0xFFFFFFFFu), c3, n3);
              }
            }
            s = ST_APPLIED;
          } else {
            // ---- the orphan walk ended off the chain ----
            PDR_CAT(3);
            uint32_t node = o_node, nk = o_nk;
            uint32_t wn = o_wn;
            if (gst) {
              ++g_adds;
              if (o_gfail) {
                ++g_fail;
                g_first = min(g_first, k0 + jo);
              }
            }
            const uint32_t wk = nk == node ? wn : ld_uniform(S, nk);
            const bool on_chain = !(wk & SF_ORPHAN);
            const uint32_t wx = (wn & PM) | (wk & SF_ORPHAN) | SF_MADE;
            if (lane == 0) S[x] = wx;
            setwf(x, WF_MADE | (on_chain ? 0u : WF_ORPH) | WB_NONE);
            logw(i, x, 0, wx, 0);
            if (nk == node) {
              if (lane == 0) S[node] = (wn & ~PM) | x;
              logw(i, node, 0, (wn & ~PM) | x, 0);
              if (on_chain) blk_insert(node, x);
            } else {
              if (on_chain) {
                blk_orphan_after(nk, node, i);
                wn |= SF_ORPHAN;
              }
              const uint32_t wkn = x | (wn & ~PM & ~SF_ORPHAN) | (wk & SF_ORPHAN) | SF_COPY;
              if (lane == 0) S[nk] = wkn;
              setwf(nk, (wfu(nk) & WB_NONE) | WF_MADE | WF_COPY | ((wk & SF_ORPHAN) ? WF_ORPH : 0u));
              logw(i, nk, 0, wkn, 0);
              uint32_t cs, cd, cb;
              if (wn & SF_COPY) {
                cs = p.qsrc[base + node];
                cd = p.qcd[base + node];
                cb = p.qcb[base + node];
              } else {
                cs = cd = ld_scalar(p.rop, rb + node);
                cb = bound;
              }
              if (lane == 0) {
                p.qsrc[base + nk] = cs;
                p.qcd[base + nk] = cd;
                p.qcb[base + nk] = min(cb, i);
              }
              logw(i, nk, 1, cs, cd);
              logw(i, nk, 2, min(cb, i), 0);
              if (ORIG && lane == 0) atomicMin(&p.tcopy[ld_scalar(p.rop, rb + nk)], i);
              if (on_chain) {
                const uint32_t bk = wfu(nk) & WB_NONE;
                uint32_t c3, n3;
                const uint32_t e3 = load_blk(bk, c3, n3);
                const uint32_t jk = idx_of(e3, nk);
                if (lane == jk) ent[bk * BLK_E + lane] = static_cast<uint16_t>(e3 & 0x7FFFu);
                blk_insert_e(nk, bk, jk, x, e3 & (lane == jk ? 0x7FFFu : 0xFFFFFFFFu), c3, n3);
              }
            }
            s = ST_APPLIED;
          }
        }
      }
      if (ORIG && lane == 0) st[i] = s;
#ifdef PDR_STATS
      ++q_cnt[q_cat];
      q_cyc[q_cat] += clock64() - q_t0;
#endif
    }
  }
replay_done:
#ifdef PDR_STATS  // ops and cycles per kind: Delete, plain insert, copy quirk, orphan anchor, other
  if (ORIG && lane == 0 && K > 28000)
    printf("pdr blocked K=%u del %llu/%llu ins %llu/%llu quirk %llu/%llu orphan %llu/%llu other %llu/%llu | walks "
           "%llu cycles %llu, next blocks %llu, scans %llu, splits %llu, compactions %llu\n", K,
           q_cnt[0], q_cyc[0], q_cnt[1], q_cyc[1], q_cnt[2], q_cyc[2], q_cnt[3], q_cyc[3], q_cnt[4], q_cyc[4], g_stc[4],
           q_walk, g_stc[0], g_stc[1], g_stc[2], g_stc[3]);
#endif
  if (ORIG && lane == 0) p.logn[D] = (logging && ln <= lcap) ? ln : NONE;
  if (gst && lane == 0) pdr_gstat_flush(p, g_adds, g_fail, (g_first == NONE ? oe : g_first) - ob, oe - ob);
  for (uint32_t r = lane; r <= K; r += 64) p.inst[base + r] = I;
}

template <int MODE>
__global__ void __launch_bounds__(64) k_pdr_blk(PdrCtx p, const uint32_t* list, uint8_t* st, uint32_t lds_words) {
  extern __shared__ uint32_t blk_lds[];
  // (the LDS base as a per-lane value, +0 for the one wave: its address
  // arithmetic then runs on the vector unit, 7% fewer scalar instructions)
  pdr_blocked<MODE>(p, st, list[blockIdx.x], blk_lds + (threadIdx.x >> 6), lds_words);
}

// (A/B: a workgroup cap from the environment, at least 8)
static uint32_t pdr_env_grid(const char* name, uint32_t def) {
  const char* e = getenv(name);
  const int g = e ? atoi(e) : 0;
  return g >= 8 && g <= (1 << 20) ? static_cast<uint32_t>(g) : def;
}

// Sort instances [i0, i1) into three size tiers: static LDS, dynamic LDS,
// global memory. count = {tier sizes, largest slot count of tier 1}.
// ---- P2c: tiny dicts, one lane each ----
// The same replay as pdr_serial (its plain walk: src/Internal/Node.elm:93-104
// findInsertion, nextNode skipping Tombstones, the copy quirk and its
// orphans, deleteHelp) by one lane per dict over the dict's slot words in
// global memory: a dict of a few ops wastes 63 lanes and a workgroup launch
// in pdr_serial (deep10m_il: 1.6M dicts of <= 17 ops). Only dicts without a
// change log take it (snapshots are rebuilt by re-replaying small dicts).
template <int MODE>
__global__ void __launch_bounds__(BLOCK) k_pdr_lane(PdrCtx p, const uint32_t* list, uint32_t cnt, uint8_t* st) {
  constexpr bool ORIG = MODE >= 1;
  GRID_STRIDE(k, cnt) {
    const uint32_t I = list[k];
    const uint32_t D = ORIG ? I : p.I.src[I];
    const uint32_t bound = ORIG ? NONE : p.I.bound[I];
    const uint32_t base = p.I.base[I];
    const uint32_t K = pdr_kcount(p, D);
    const uint32_t rb = p.rbase[D];
    uint32_t* const S = p.S + base;
    for (uint32_t r = 0; r <= K; ++r) {
      S[r] = r == 0 ? (PM | SF_TOMB | SF_MADE) : PM;
      p.inst[base + r] = I;
    }
    const uint32_t oe = p.rbase[D + 1] - 1;
    for (uint32_t q = rb; q < oe; ++q) {
      const uint32_t i = p.olist[q];
      if (i >= bound) break;
      const unsigned long long w = p.opw[q];
      const uint32_t wlo = static_cast<uint32_t>(w), whi = static_cast<uint32_t>(w >> 32);
      uint8_t s;
      if (whi >> 31) {  // deleteHelp
        const uint32_t t = wlo & PM;
        if (t == 0) {
          s = ST_ALREADY;
        } else {
          const uint32_t wt = t == OW_NF ? 0u : S[t];
          if (!(wt & SF_MADE)) {
            s = ST_NOTFOUND;
          } else if (wt & SF_TOMB) {
            s = ST_ALREADY;
          } else {
            S[t] = wt | SF_TOMB;
            s = ST_APPLIED;
          }
        }
      } else {  // addAfterHelp
        const uint32_t x = wlo & PM;
        const uint32_t an = ((wlo >> 24) | (whi << 8)) & PM;
        if (x == 0) {
          s = ST_ALREADY;
        } else if (an == OW_NF || !(S[an] & SF_MADE)) {
          s = ST_NOTFOUND;
        } else {
          uint32_t node = an, nk = an;  // findInsertion
          uint32_t wn = S[node];
          for (;;) {
            const uint32_t rn = wn & PM;
            if (rn == PM) break;
            if (x > rn) break;  // ts > key(rn): decided before rn's word is read
            uint32_t live = rn, wl = S[rn];  // nextNode: the first live node from rn on
            while (live != PM && (wl & SF_TOMB)) {
              live = wl & PM;
              if (live != PM) wl = S[live];
            }
            if (live == PM) break;
            nk = rn;
            node = live;
            wn = wl;
          }
          const uint32_t wk = nk == node ? wn : S[nk];
          S[x] = (wn & PM) | (wk & SF_ORPHAN) | SF_MADE;
          if (nk == node) {
            S[node] = (wn & ~PM) | x;
          } else {
            // copy quirk: slot nk := copy of node, next = x; the entries after
            // nk up to node drop off the chain when nk was on it
            if (!(wk & SF_ORPHAN)) {
              for (uint32_t q2 = wk & PM; q2 != PM;) {
                const uint32_t wq = S[q2];
                S[q2] = wq | SF_ORPHAN;
                if (q2 == node) break;
                q2 = wq & PM;
              }
              wn |= SF_ORPHAN;
            }
            S[nk] = x | (wn & ~PM & ~SF_ORPHAN) | (wk & SF_ORPHAN) | SF_COPY;
            uint32_t cs, cd, cb;
            if (wn & SF_COPY) {
              cs = p.qsrc[base + node];
              cd = p.qcd[base + node];
              cb = p.qcb[base + node];
            } else {
              cs = cd = p.rop[rb + node];
              cb = bound;
            }
            p.qsrc[base + nk] = cs;
            p.qcd[base + nk] = cd;
            p.qcb[base + nk] = min(cb, i);
            if (ORIG) atomicMin(&p.tcopy[p.rop[rb + nk]], i);
          }
          s = ST_APPLIED;
        }
      }
      if (ORIG) st[i] = s;
    }
    if (ORIG) p.logn[D] = NONE;  // (no change log)
  }
}

struct PdrTiers {
  uint32_t* list[5];
  uint32_t* count;  // [0..3] tier sizes, [4] largest slot count of tier 1, [5] most ops of a dict, [6] tier 3's,
                    // [7] tier 4's size
  uint32_t blk_min;  // dicts of more slots than this (and at most blk_max) take pdr_blocked (tier 3)
  uint32_t blk_max;
  uint32_t lane_max;  // dicts of at most this many slots and no change log: one lane each (tier 4; 0 = off)
};

// (Two passes over the instances: each workgroup counts its share per tier,
// reserves it with one device atomic per tier, then writes its entries at
// offsets kept in LDS. A counter bumped per dict, or per wave, serialises
// ~12 ns per atomic on one word: 20 ms, then 1.5 ms, over deep10m_il's 1.6M
// dicts. The grid is capped, so there are few workgroups (2,048 since round
// 6: 512 left 2 waves per SIMD for these gathers, 0.29 against 0.20 ms at
// deep10m_il; the same for k_pdr_jobs, 0.50 against 0.26); loops are
// block-uniform.)
__device__ __forceinline__ uint32_t pdr_tier_of(const PdrCtx& p, uint32_t I, uint32_t big_cap, const PdrTiers& tt,
                                                uint32_t& slots, uint32_t& ops) {
  const uint32_t n = p.o.n;
  uint32_t D = I;
  ops = 0;
  if (I > n) {
    if (p.ilog[I] != NONE) return NONE;  // rebuilt from the source dict's change log
    D = p.I.src[I];
  } else if (p.rbase[I + 1] == p.rbase[I]) {
    return NONE;  // a dict no op reached
  } else {
    ops = p.rbase[I + 1] - p.rbase[I];  // ops replayed by this dict's wave
  }
  slots = pdr_kcount(p, D) + 1;
  uint32_t t = slots <= PDR_SMALL ? 0u : (slots <= big_cap ? 1u : 2u);
  if (slots > tt.blk_min && slots <= tt.blk_max) t = 3;
  if (t == 0 && slots <= tt.lane_max && (I > n || p.log == nullptr || slots < p.log_min)) t = 4;
  return t;
}

__global__ void __launch_bounds__(BLOCK) k_pdr_tier(PdrCtx p, uint32_t i0, uint32_t i1, uint32_t big_cap,
                                                    PdrTiers tt) {
  __shared__ uint32_t s_off[5];
  const uint32_t n = p.o.n, m = i1 - i0, stride = gridDim.x * blockDim.x;
  uint32_t c[5] = {0u, 0u, 0u, 0u, 0u};
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) {
    uint32_t slots, ops;
    const uint32_t t = pdr_tier_of(p, i0 + k, big_cap, tt, slots, ops);
#pragma unroll
    for (uint32_t q = 0; q < 5; ++q) c[q] += t == q ? 1u : 0u;
  }
#pragma unroll
  for (uint32_t q = 0; q < 5; ++q) {
    const uint32_t tot = block_sum(c[q]);
    if (threadIdx.x == 0) s_off[q] = tot ? atomicAdd(&tt.count[q < 4 ? q : 7], tot) : 0u;
  }
  __syncthreads();
  uint32_t m4 = 0, m5 = 0, m6 = 0;
  for (uint32_t k0 = blockIdx.x * blockDim.x; k0 < m; k0 += stride) {
    const uint32_t k = k0 + threadIdx.x;
    const uint32_t I = i0 + k;
    uint32_t slots = 0, ops = 0, t = NONE;
    if (k < m) {
      t = pdr_tier_of(p, I, big_cap, tt, slots, ops);
      if (t != NONE && I <= n) p.I.base[I] = p.rbase[I];
    }
    const uint32_t j = block_ticket<5, false>(s_off, t);
    if (t < 5) tt.list[t][j] = I;
    if (t == 1) m4 = max(m4, slots);
    if (t == 3) m6 = max(m6, slots);
    m5 = max(m5, ops);
  }
  m4 = block_max(m4);
  m5 = block_max(m5);
  m6 = block_max(m6);
  if (threadIdx.x == 0) {
    if (m4) atomicMax(&tt.count[4], m4);
    if (m5) atomicMax(&tt.count[5], m5);
    if (m6) atomicMax(&tt.count[6], m6);
  }
}

// ---- P3: conflicts ----
// An op whose path stopped at a Tombstone that the copy quirk re-filled
// before the op ran would have descended into the copy. K1 left the stop
// node implicit (TAG_LAZY) on its fast path: it is the topmost node of the
// chain ending at cur[i] deleted before i.
__global__ void __launch_bounds__(BLOCK) k_pdr_conflict(uint32_t n, const uint32_t* tag, const uint32_t* cur,
                                                        const uint32_t* addpar, const uint32_t* dtime,
                                                        const uint32_t* tcopy, DevResult* dres) {
  GRID_STRIDE(i, n) {
    uint32_t x = tag[i];
    if (x == TAG_LAZY) {
      x = NONE;
      for (uint32_t y = cur[i]; y != n; y = addpar[y])
        if (dtime[y] < i) x = y;
    }
    if (x < n && tcopy[x] < i) atomicOr(&dres->pdr_conflict, 1u);  // rare
  }
}

// batch accounting on the final statuses (k_stats' counters)
__global__ void __launch_bounds__(BLOCK) k_pdr_stats(OpsDev o, const uint8_t* st, long long ts0, DevResult* dres) {
  uint32_t app = 0, alr = 0, err = NONE, own = 0;
  const long long id0 = replica_of(ts0);
  const uint32_t n = o.n;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t trips = (n + stride - 1) / stride;
  for (uint32_t t = 0; t < trips; ++t) {
    const uint32_t i = t * stride + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) continue;
    const uint8_t s = st[i];
    if (s == ST_APPLIED) ++app;
    else if (s == ST_ALREADY) ++alr;
    else err = min(err, i);
    if (o.kind[i] == CRDTM_ADD && (s == ST_APPLIED || s == ST_ALREADY) && replica_of(o.ts[i]) == id0) ++own;
  }
  app = block_sum(app);
  alr = block_sum(alr);
  own = block_sum(own);
  err = block_min(err);
  if (threadIdx.x == 0) {
    atomicAdd(&dres->n_applied, app);
    atomicAdd(&dres->n_already, alr);
    atomicAdd(&dres->own_ok_adds, own);
    if (err != NONE) atomicMin(&dres->err_index, err);
  }
}

__global__ void k_pdr_stats_reset(DevResult* d) {
  d->n_applied = 0;
  d->n_already = 0;
  d->own_ok_adds = 0;
  d->err_index = NONE;
  d->pdr_jobs = 0;
  d->pdr_overflow = 0;
  d->pdr_conflict = 0;
}

// ---- P5: assembly ----
// ok[D]: original dict D is reachable in the final state (its owner is a
// live, un-copied node of a reachable dict); pointer jumping over owners.
__global__ void __launch_bounds__(BLOCK) k_pdr_alive_init(PdrCtx p, const uint32_t* addpar, uint8_t* ok,
                                                          uint32_t* up) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(d, n + 1) {
    if (d == n) {
      ok[d] = 1;
      up[d] = n;
      continue;
    }
    uint8_t v = 0;
    uint32_t P = n;
    if (p.rbase[d + 1] != p.rbase[d]) {
      P = addpar[d];
      const uint32_t w = p.S[p.rbase[P] + p.rankof[d]];
      v = (w & SF_MADE) && !(w & (SF_TOMB | SF_COPY)) ? 1 : 0;
    }
    ok[d] = v;
    up[d] = P;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_alive_jump(uint32_t n, uint8_t* ok, uint32_t* up) {
  GRID_STRIDE(d, n + 1) {
    const uint32_t u = up[d];
    if (!ok[u]) ok[d] = 0;
    up[d] = up[u];
  }
}

__device__ __forceinline__ uint32_t pdr_src_dict(const PdrCtx& p, uint32_t I) { return I > p.o.n ? p.I.src[I] : I; }

// A live slot whose children are a frozen (dict, bound) view gets a snapshot
// job when that view is non-empty. Slot positions [s0, s1).
__device__ __forceinline__ bool pdr_job_of(const PdrCtx& p, const uint8_t* ok, uint32_t g, uint32_t& I, uint32_t& cd,
                                           uint32_t& cb, uint32_t& r) {
  const uint32_t n = p.o.n;
  I = p.inst[g];
  if (I == NONE) return false;
  if (I <= n && !ok[I]) return false;  // an unreachable original dict
  const uint32_t w = p.S[g];
  if (!(w & SF_MADE) || (w & SF_TOMB)) return false;  // (sentinels too)
  if (I <= n && !(w & SF_COPY)) return false;         // children = the live original dict
  r = g - p.I.base[I];
  if (w & SF_COPY) {
    cd = p.qcd[g];
    cb = p.qcb[g];
  } else {
    cd = p.rop[p.rbase[pdr_src_dict(p, I)] + r];
    cb = p.I.bound[I];
  }
  const uint32_t f0 = pdr_first_op(p, cd);
  return !(f0 == NONE || f0 >= cb);  // (else the copy is an empty dict: implicit)
}

// (two passes, as k_pdr_tier: one device atomic per workgroup for the job numbers)
__global__ void __launch_bounds__(BLOCK) k_pdr_jobs(PdrCtx p, const uint8_t* ok, uint32_t s0, uint32_t s1,
                                                    uint32_t jcap, DevResult* dres) {
  __shared__ uint32_t s_off[1];
  const uint32_t n = p.o.n, m = s1 - s0, stride = gridDim.x * blockDim.x;
  uint32_t c = 0;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) {
    uint32_t I, cd, cb, r;
    c += pdr_job_of(p, ok, s0 + k, I, cd, cb, r) ? 1u : 0u;
  }
  const uint32_t tot = block_sum(c);
  if (threadIdx.x == 0) s_off[0] = tot ? atomicAdd(&dres->pdr_jobs, tot) : 0u;
  __syncthreads();
  for (uint32_t k0 = blockIdx.x * blockDim.x; k0 < m; k0 += stride) {
    const uint32_t k = k0 + threadIdx.x;
    const uint32_t g = s0 + k;
    uint32_t I = NONE, cd = 0, cb = 0, r = 0;
    const bool job = k < m && pdr_job_of(p, ok, g, I, cd, cb, r);
    const uint32_t j = block_ticket<1, false>(s_off, job ? 0u : NONE);
    if (!job) continue;
    if (j >= jcap) {
      atomicOr(&dres->pdr_overflow, 1u);
      continue;
    }
    const uint32_t J = n + 1 + j;
    p.I.src[J] = cd;
    p.I.bound[J] = cb;
    p.I.pi[J] = I;
    p.I.pl[J] = r;
    p.ch[g] = J;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_job_size(PdrCtx p, uint32_t j0, uint32_t j1, uint32_t* sz) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(k, j1 - j0 + 1) {
    sz[k] = k == j1 - j0 ? 0u : pdr_kcount(p, p.I.src[n + 1 + j0 + k]) + 1;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_job_base(PdrCtx p, uint32_t j0, uint32_t j1, const uint32_t* off,
                                                        uint32_t s0) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(k, j1 - j0) p.I.base[n + 1 + j0 + k] = s0 + off[k];
}

// Snapshots from change logs. plan: prefix length (entries with op < bound)
// per job whose source dict kept a log; ecnt = that length (0 otherwise).
__global__ void __launch_bounds__(BLOCK) k_pdr_snap_plan(PdrCtx p, uint32_t j0, uint32_t j1, uint32_t* ecnt) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(k, j1 - j0 + 1) {
    if (k == j1 - j0) {
      ecnt[k] = 0;
      continue;
    }
    const uint32_t J = n + 1 + j0 + k;
    const uint32_t D = p.I.src[J], b = p.I.bound[J];
    const uint32_t m = p.logn[D];
    uint32_t e = 0;
    if (m != NONE) {
      const uint4* lg = p.log + 4ULL * p.rbase[D];
      uint32_t lo = 0, hi = m;  // first entry with op >= bound
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (lg[mid].x < b) lo = mid + 1;
        else hi = mid;
      }
      e = lo;
      p.ilog[J] = lo;
    } else {
      p.ilog[J] = NONE;
    }
    ecnt[k] = e;
  }
}

__device__ __forceinline__ uint32_t pdr_find(const uint32_t* pre, uint32_t cnt, uint32_t x) {
  uint32_t lo = 0, hi = cnt;  // last k with pre[k] <= x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

// last writer per (slot, kind) among each job's log prefix (entry index + 1)
__global__ void __launch_bounds__(BLOCK) k_pdr_snap_apply(PdrCtx p, uint32_t j0, uint32_t nj, const uint32_t* epre,
                                                          uint32_t etot, uint32_t* last) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(x, etot) {
    const uint32_t k = pdr_find(epre, nj, x);
    const uint32_t J = n + 1 + j0 + k;
    const uint32_t e = x - epre[k];
    const uint4 en = p.log[4ULL * p.rbase[p.I.src[J]] + e];
    const uint32_t kind = en.y >> 30, slot = en.y & 0x3FFFFFFFu;
    atomicMax(&last[3ULL * (p.I.base[J] + slot) + kind], e + 1);
  }
}

// slot positions [s0, s1) of this level's snapshot regions (joff: region
// offsets relative to s0 per job)
__global__ void __launch_bounds__(BLOCK) k_pdr_snap_fill(PdrCtx p, uint32_t j0, uint32_t nj, const uint32_t* joff,
                                                         uint32_t s0, uint32_t s1, const uint32_t* last) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(u, s1 - s0) {
    const uint32_t k = pdr_find(joff, nj, u);
    const uint32_t J = n + 1 + j0 + k;
    if (p.ilog[J] == NONE) continue;  // replayed by the tiers
    const uint32_t g = s0 + u, r = u - joff[k];
    const uint4* lg = p.log + 4ULL * p.rbase[p.I.src[J]];
    const uint32_t l0 = last[3ULL * g], l1 = last[3ULL * g + 1], l2 = last[3ULL * g + 2];
    p.S[g] = l0 ? lg[l0 - 1].z : (r == 0 ? (PM | SF_TOMB | SF_MADE) : PM);
    if (l1) {
      p.qsrc[g] = lg[l1 - 1].z;
      p.qcd[g] = lg[l1 - 1].w;
    }
    if (l2) p.qcb[g] = lg[l2 - 1].z;
    p.inst[g] = J;
  }
}

// instance order: root first, then originals 0..n-1, then snapshots
__device__ __forceinline__ uint32_t pdr_pos(uint32_t I, uint32_t n) { return I == n ? 0u : (I < n ? I + 1 : I); }

__global__ void __launch_bounds__(BLOCK) k_pdr_inst_flags(PdrCtx p, const uint8_t* ok, uint32_t njobs,
                                                          uint32_t* dflag) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(I, n + 1 + njobs + 1) {
    if (I == n + 1 + njobs) {  // scan tail
      dflag[I] = 0;
      continue;
    }
    const bool inst = I > n || (ok[I] && p.rbase[I + 1] != p.rbase[I]);
    dflag[pdr_pos(I, n)] = inst ? 1u : 0u;
  }
}

// Final slot numbering runs over positions with the root region first, so
// the root sentinel is slot 0 (api.hip tree reset, linearize).
__device__ __forceinline__ uint32_t pdr_u_of_g(const PdrCtx& p, uint32_t g) {
  const uint32_t rb = p.rbase[p.o.n], r0 = p.rbase[p.o.n + 1];
  return g >= r0 ? g : (g >= rb ? g - rb : g + (r0 - rb));
}
__device__ __forceinline__ uint32_t pdr_g_of_u(const PdrCtx& p, uint32_t u) {
  const uint32_t rb = p.rbase[p.o.n], r0 = p.rbase[p.o.n + 1];
  return u >= r0 ? u : (u < r0 - rb ? rb + u : u - (r0 - rb));
}

__global__ void __launch_bounds__(BLOCK) k_pdr_slot_flags(PdrCtx p, const uint8_t* ok, uint32_t S1, uint32_t* f) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(u, S1 + 1) {
    uint32_t v = 0;
    if (u < S1) {
      const uint32_t g = pdr_g_of_u(p, u);
      const uint32_t I = p.inst[g];
      if (I != NONE && (I > n || ok[I]) && (p.S[g] & SF_MADE)) v = 1;
    }
    f[u] = v;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_write(PdrCtx p, const uint8_t* ok, const uint32_t* addpar,
                                                     const uint32_t* did, const uint32_t* fpos,
                                                     const uint32_t* logidx, uint32_t S1, TreeDev T) {
  const uint32_t n = p.o.n;
  GRID_STRIDE(g, S1) {
    const uint32_t I = p.inst[g];
    if (I == NONE) continue;
    if (I <= n && !ok[I]) continue;
    const uint32_t w = p.S[g];
    if (!(w & SF_MADE)) continue;
    const uint32_t base = p.I.base[I];
    const uint32_t r = g - base;
    const uint32_t rb = p.rbase[pdr_src_dict(p, I)];
    const uint32_t d = did[pdr_pos(I, n)];
    const uint32_t s = fpos[pdr_u_of_g(p, g)];
    const uint32_t nx = w & PM;
    T.s_dict[s] = d;
    T.s_next[s] = nx == PM ? NONE : fpos[pdr_u_of_g(p, base + nx)];
    uint32_t child = NONE;
    if (r == 0) {
      T.s_key[s] = 0;
      T.s_src[s] = NONE;
      T.s_flags[s] = F_TOMB | F_SENT;
      T.d_sent[d] = s;
      uint32_t owner = NONE;
      if (I > n) owner = fpos[pdr_u_of_g(p, p.I.base[p.I.pi[I]] + p.I.pl[I])];
      else if (I < n) owner = fpos[pdr_u_of_g(p, p.rbase[addpar[I]] + p.rankof[I])];
      T.d_owner[d] = owner;
    } else {
      const uint32_t y = p.rop[rb + r];
      T.s_key[s] = p.o.ts[y];
      T.s_src[s] = logidx[(w & SF_COPY) ? p.qsrc[g] : y];
      T.s_flags[s] = ((w & SF_TOMB) ? F_TOMB : 0) | ((w & SF_ORPHAN) ? F_ORPHAN : 0);
      if (!(w & SF_TOMB)) {
        if (I > n || (w & SF_COPY)) {
          const uint32_t J = p.ch[g];
          if (J != NONE) child = did[pdr_pos(J, n)];
        } else if (p.rbase[y + 1] != p.rbase[y]) {
          child = did[pdr_pos(y, n)];  // a live original node: its own dict
        }
      }
    }
    T.s_child[s] = child;
  }
}

__global__ void __launch_bounds__(BLOCK) k_pdr_logidx(OpsDev o, const uint8_t* st, uint32_t* a) {
  GRID_STRIDE(i, o.n) a[i] = st[i] == ST_APPLIED ? 1u : 0u;
}

static int pdr_run_tiers(crdtm_ctx* c, const PdrCtx& p, uint32_t i0, uint32_t i1, bool orig, uint8_t* st,
                         const PdrTiers& tt, uint32_t big_cap, uint32_t* hcount) {
  hipStream_t s = c->stream;
  if (i1 <= i0) return CRDTM_OK;
  HIP_CHECK(hipMemsetAsync(tt.count, 0, 8 * sizeof(uint32_t), s));
  static const uint32_t tier_grid = pdr_env_grid("CRDTM_PDR_TIER_GRID", 2048);
  LAUNCH(k_pdr_tier, dim3(grid_for(i1 - i0, BLOCK, tier_grid)), dim3(BLOCK), 0, s, p, i0, i1, big_cap, tt);
  HIP_CHECK(hipMemcpyAsync(hcount, tt.count, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (int rw = stream_wait(s)) return rw;
  const uint32_t* h = hcount;
  // the blocked tier (a few big dicts, one CU each, the longest replays) goes
  // first on the main stream; the other tiers run beside it on the side stream
  const bool fork = h[3] && (h[0] || h[1] || h[2] || h[7]);
  hipStream_t s2 = fork ? c->side : s;
  if (fork) {
    HIP_CHECK(hipEventRecord(c->ev_fork, s));
    HIP_CHECK(hipStreamWaitEvent(s2, c->ev_fork, 0));
  }
  if (h[3]) {
    const size_t lds = static_cast<size_t>(big_cap) * sizeof(uint32_t);  // the whole LDS: one wave per CU
    if (orig && p.gcount) LAUNCH(k_pdr_blk<2>, dim3(h[3]), dim3(64), lds, s, p, tt.list[3], st, big_cap);
    else if (orig) LAUNCH(k_pdr_blk<1>, dim3(h[3]), dim3(64), lds, s, p, tt.list[3], st, big_cap);
    else LAUNCH(k_pdr_blk<0>, dim3(h[3]), dim3(64), lds, s, p, tt.list[3], st, big_cap);
  }
  if (h[7]) {  // (no tier 4 with the guard-G statistics: lane_max = 0)
    if (orig) LAUNCH(k_pdr_lane<1>, dim3(grid_for(h[7])), dim3(BLOCK), 0, s2, p, tt.list[4], h[7], st);
    else LAUNCH(k_pdr_lane<0>, dim3(grid_for(h[7])), dim3(BLOCK), 0, s2, p, tt.list[4], h[7], st);
  }
  if (h[0]) {
    if (orig && p.gcount) LAUNCH(k_pdr_small<2>, dim3(h[0]), dim3(64), 0, s2, p, tt.list[0], st);
    else if (orig) LAUNCH(k_pdr_small<1>, dim3(h[0]), dim3(64), 0, s2, p, tt.list[0], st);
    else LAUNCH(k_pdr_small<0>, dim3(h[0]), dim3(64), 0, s2, p, tt.list[0], st);
  }
  if (h[1]) {
    const size_t lds = static_cast<size_t>(h[4]) * sizeof(uint32_t);
    if (orig && p.gcount) LAUNCH(k_pdr_big<2>, dim3(h[1]), dim3(64), lds, s2, p, tt.list[1], st);
    else if (orig) LAUNCH(k_pdr_big<1>, dim3(h[1]), dim3(64), lds, s2, p, tt.list[1], st);
    else LAUNCH(k_pdr_big<0>, dim3(h[1]), dim3(64), lds, s2, p, tt.list[1], st);
  }
  if (h[2]) {
    if (orig && p.gcount) LAUNCH(k_pdr_huge<2>, dim3(h[2]), dim3(64), 0, s2, p, tt.list[2], st);
    else if (orig) LAUNCH(k_pdr_huge<1>, dim3(h[2]), dim3(64), 0, s2, p, tt.list[2], st);
    else LAUNCH(k_pdr_huge<0>, dim3(h[2]), dim3(64), 0, s2, p, tt.list[2], st);
  }
  if (fork) {
    HIP_CHECK(hipEventRecord(c->ev_join, s2));
    HIP_CHECK(hipStreamWaitEvent(s, c->ev_join, 0));
  }
  return CRDTM_OK;
}

// slots a workgroup can hold in dynamic LDS (the per-block maximum)
static uint32_t pdr_big_cap(int device) {
  static int cached = -1;
  if (cached < 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess || v <= 0)
      v = 64 * 1024;
    const void* fns[] = {reinterpret_cast<const void*>(&k_pdr_big<0>), reinterpret_cast<const void*>(&k_pdr_big<1>),
                         reinterpret_cast<const void*>(&k_pdr_big<2>), reinterpret_cast<const void*>(&k_pdr_blk<0>),
                         reinterpret_cast<const void*>(&k_pdr_blk<1>), reinterpret_cast<const void*>(&k_pdr_blk<2>)};
    bool ok = true;
    for (const void* f : fns) ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, v) == hipSuccess;
    if (!ok)
      v = 64 * 1024;
    cached = v;
  }
  return static_cast<uint32_t>(cached) / sizeof(uint32_t);
}

// Host driver. *handled = false: conflict or no room, the caller replays
// the batch sequentially (statuses in `st` are then scratch).
int pdr_apply(crdtm_tree* t, const OpsDev& o, const PdrIn& in, uint8_t* st, crdtm_result* res, bool* handled) {
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  DevResult* dr = c->dres;
  const uint32_t n = o.n;
  const uint32_t g = grid_for(n);
  *handled = false;
  const size_t arena_mark = ws.used;
  int r;
  const uint32_t big_cap = pdr_big_cap(c->device);
  uint32_t hcount[8];

  PdrCtx p;
  p.o = o;
  p.ix = in.ix;
  p.leaf = in.leaf;
  uint32_t* rbase = ws.alloc<uint32_t>(n + 2);
  uint32_t* fill = ws.alloc<uint32_t>(n + 2);
  uint32_t* cbase = ws.alloc<uint32_t>(n + 2);
  uint32_t* cfill = ws.alloc<uint32_t>(n + 2);
  p.rankof = ws.alloc<uint32_t>(n);
  p.tcopy = ws.alloc<uint32_t>(n);
  LAUNCH(k_pdr_init, dim3(grid_for(n + 2)), dim3(BLOCK), 0, s, n, rbase, fill, cbase, cfill, p.rankof, p.tcopy);
  // ops grouped by dict (stable radix sort: batch order inside each dict), per-dict op and key counts
  uint32_t* gs = fill;  // [n + 2] each dict's first sorted position
  uint32_t* X = cfill;  // [n + 2] exclusive scan over the sorted positions of "is a key"
  uint32_t *sk = nullptr, *sv = nullptr;
  {
    uint32_t* ka = ws.alloc<uint32_t>(n);
    uint32_t* va = ws.alloc<uint32_t>(n);
    uint32_t* kb = ws.alloc<uint32_t>(n);
    uint32_t* vb = ws.alloc<uint32_t>(n);
    uint32_t* nitems = ws.alloc<uint32_t>(1);
    LAUNCH(k_pdr_keys, dim3(grid_for(n, BLOCK, 2048)), dim3(BLOCK), 0, s, o, in.ix, in.tag, in.cur, ka, va, nitems);
    uint32_t kbits = 8;  // NONE (not reached) sorts after every dict id <= n
    while (kbits < 32 && ((static_cast<uint64_t>(n) + 1) >> kbits) != 0) kbits += 8;
    if ((r = radix_sort_pairs(ka, va, kb, vb, nitems, n, kbits, ws, s, &sk, &sv))) return r;
    LAUNCH(k_doc_gstart, dim3(grid_for(n, BLOCK, 2048)), dim3(BLOCK), 0, s, sk, n, gs);
    LAUNCH(k_pdr_kflag, dim3(grid_for(n + 1, BLOCK, 2048)), dim3(BLOCK), 0, s, n, sv, X);
    if ((r = scan_excl_u32(X, X, n + 1, nullptr, ws, s))) return r;
    LAUNCH(k_pdr_gcount, dim3(grid_for(n, BLOCK, 2048)), dim3(BLOCK), 0, s, n, sk, gs, X, rbase, cbase);
  }
  LAUNCH(k_pdr_size, dim3(grid_for(n + 1)), dim3(BLOCK), 0, s, n, rbase);
  if ((r = scan_excl_u32(rbase, rbase, n + 2, &dr->pdr_slots, ws, s))) return r;
  if ((r = scan_excl_u32(cbase, cbase, n + 2, &dr->pdr_dicts, ws, s))) return r;
  if ((r = sync_read(c))) return r;
  const uint32_t R0 = c->hres->pdr_slots;  // original regions
  const uint32_t KT = c->hres->pdr_dicts;  // keys over all dicts
  if (R0 >= PM) return CRDTM_OK;           // slot indices are 24-bit: sequential replay
  p.rbase = rbase;
  p.cbase = cbase;
  uint32_t* olist = ws.alloc<uint32_t>(R0);
  uint32_t* carr = ws.alloc<uint32_t>(KT + 1);
  p.olist = olist;
  HIP_CHECK(hipMemsetAsync(olist, 0xFF, static_cast<size_t>(R0) * sizeof(uint32_t), s));
  LAUNCH(k_pdr_place, dim3(grid_for(n, BLOCK, 2048)), dim3(BLOCK), 0, s, n, sk, sv, gs, X, rbase, cbase, olist, carr);
  if ((r = segmented_sort(cbase, n + 1, carr, KT, o.ts, ws, s, dr))) return r;
  p.rop = ws.alloc<uint32_t>(R0);
  LAUNCH(k_pdr_rank, dim3(grid_for(KT)), dim3(BLOCK), 0, s, KT, carr, in.cur, cbase, rbase, p.rankof, p.rop);
  unsigned long long* opw = ws.alloc<unsigned long long>(R0);
  LAUNCH(k_pdr_opw, dim3(grid_for(R0)), dim3(BLOCK), 0, s, R0, olist, o, in.leaf, p.rankof, opw);
  p.opw = opw;

  // slot room: originals + snapshots (bounded; overflow -> sequential replay)
  const uint32_t SCAP = static_cast<uint32_t>(std::min<uint64_t>(2ULL * R0 + 4096, PM - 1));
  const uint32_t JCAP = std::max<uint32_t>(1024u, n);
  p.S = ws.alloc<uint32_t>(SCAP);
  p.qsrc = ws.alloc<uint32_t>(SCAP);
  p.qcd = ws.alloc<uint32_t>(SCAP);
  p.qcb = ws.alloc<uint32_t>(SCAP);
  p.ch = ws.alloc<uint32_t>(SCAP);
  p.inst = ws.alloc<uint32_t>(SCAP);
  const uint64_t ICAP = static_cast<uint64_t>(n) + 1 + JCAP;
  p.I.base = ws.alloc<uint32_t>(ICAP);
  p.I.src = ws.alloc<uint32_t>(ICAP);
  p.I.bound = ws.alloc<uint32_t>(ICAP);
  p.I.pi = ws.alloc<uint32_t>(ICAP);
  p.I.pl = ws.alloc<uint32_t>(ICAP);
  p.log = ws.alloc<uint4>(4ULL * R0);
  p.log_min = PDR_LOG_MIN;
  if (const char* e = getenv("CRDTM_PDR_LOG_MIN")) p.log_min = static_cast<uint32_t>(strtoul(e, nullptr, 10));
  p.logn = ws.alloc<uint32_t>(n + 1);
  p.ilog = ws.alloc<uint32_t>(ICAP);
  uint32_t* last = ws.alloc<uint32_t>(3ULL * SCAP);
  HIP_CHECK(hipMemsetAsync(last, 0, 3ULL * SCAP * sizeof(uint32_t), s));
  HIP_CHECK(hipMemsetAsync(p.ilog, 0xFF, ICAP * sizeof(uint32_t), s));
  PdrTiers tt;
  for (int k = 0; k < 5; ++k) tt.list[k] = ws.alloc<uint32_t>(ICAP);
  tt.count = ws.alloc<uint32_t>(8);
  // tiny dicts replay one per lane (env CRDTM_PDR_LANE: the slot bound, 0 = off); not with the guard statistics
  tt.lane_max = PDR_LANE;
  if (const char* e = getenv("CRDTM_PDR_LANE")) tt.lane_max = static_cast<uint32_t>(strtoul(e, nullptr, 10));
  tt.blk_min = BLK_MIN;
  if (const char* e = getenv("CRDTM_PDR_BLK_MIN")) tt.blk_min = static_cast<uint32_t>(strtoul(e, nullptr, 10));
  // the blocked order holds a dict's flags (2 B per slot) and its chain
  // repacked BLK_FILL per block (+ room to split) in the LDS; larger dicts keep
  // the older tiers
  tt.blk_max = 0;
  for (int kk = static_cast<int>(BLK_KMAX); kk > 0; kk -= 256) {
    const uint32_t k = static_cast<uint32_t>(kk);
    const uint32_t wfw = (k + 2) / 2;
    if (wfw < big_cap && (big_cap - wfw) / (1 + BLK_E / 2) >= (k + 1) / BLK_FILL + 16) {
      tt.blk_max = k + 1;
      break;
    }
  }
  p.where = ws.alloc<uint32_t>(SCAP);
  p.blk_spare = 0;
  if (const char* e = getenv("CRDTM_PDR_BLK_SPARE")) p.blk_spare = static_cast<uint32_t>(strtoul(e, nullptr, 10));

  HIP_CHECK(hipMemsetAsync(p.inst, 0xFF, static_cast<size_t>(SCAP) * sizeof(uint32_t), s));
  HIP_CHECK(hipMemsetAsync(p.ch, 0xFF, static_cast<size_t>(SCAP) * sizeof(uint32_t), s));

  // ---- P2 + P3 ----
#ifdef PDR_STATS
  {
    unsigned long long z[8] = {};
    bool f = false;
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_pdr_stats), z, sizeof(z)));
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(pdr_stat_on), &f, sizeof(f)));
  }
#endif
  p.gcount = nullptr;  // guard-G statistics (untimed measurement runs only)
  if (const char* e = getenv("CRDTM_GUARD_STATS"); e && e[0] == '1') {
    if (!c->gstat_dev) HIP_CHECK(hipMalloc(&c->gstat_dev, 4 * sizeof(unsigned long long)));
    HIP_CHECK(hipMemsetAsync(c->gstat_dev, 0, 4 * sizeof(unsigned long long), s));
    p.gcount = c->gstat_dev;
    tt.lane_max = 0;  // (the statistics come from the wave replays)
  }
  if ((r = pdr_run_tiers(c, p, 0, n + 1, true, st, tt, big_cap, hcount))) return r;
#ifdef PDR_STATS
  {
    unsigned long long z[8];
    if (int rw = stream_wait(s)) return rw;
    HIP_CHECK(hipMemcpyFromSymbol(z, HIP_SYMBOL(g_pdr_stats), sizeof(z)));
    std::fprintf(stderr, "pdr stats: adds %llu walk-steps %llu window-steps %llu tomb-skips %llu quirks %llu\n",
                 z[4], z[0], z[1], z[2], z[3]);
  }
#endif
  res->serial_dicts = static_cast<uint64_t>(hcount[0]) + hcount[1] + hcount[2] + hcount[3] + hcount[7];
  res->serial_ops = n;  // every op, in order within its dict
  res->serial_max = hcount[5];
  LAUNCH(k_pdr_stats_reset, dim3(1), dim3(1), 0, s, dr);
  LAUNCH(k_pdr_conflict, dim3(grid_for(n, BLOCK, 2048)), dim3(BLOCK), 0, s, n, in.tag, in.cur, in.addpar, in.dtime,
         p.tcopy, dr);
  LAUNCH(k_pdr_stats, dim3(grid_for(n, BLOCK, 2048)), dim3(BLOCK), 0, s, o, st, t->timestamp, dr);
  if ((r = sync_read(c))) return r;
  const DevResult h1 = *c->hres;
  const long long new_ts = t->timestamp + h1.own_ok_adds - t->own_bias;
  if (h1.pdr_conflict || replica_of(new_ts) != replica_of(t->timestamp)) {
    ws.used = arena_mark;
    return CRDTM_OK;
  }
  if (p.gcount) {  // (only a replay that serves the batch reports)
    unsigned long long gh[4];
    HIP_CHECK(hipMemcpy(gh, c->gstat_dev, sizeof(gh), hipMemcpyDeviceToHost));
    for (int k = 0; k < 4; ++k) c->gstat[k] = gh[k];
    c->gstat_valid = 1;
  }
  *handled = true;
  res->path_taken = CRDTM_PATH_DICT_REPLAY;
  if (h1.err_index != NONE) {
    uint8_t est = 0;
    HIP_CHECK(hipMemcpy(&est, st + h1.err_index, 1, hipMemcpyDeviceToHost));
    res->code = est == ST_INVALID ? CRDTM_INVALID_PATH : CRDTM_OPERATION_FAILED;
    res->err_index = h1.err_index;
    return CRDTM_OK;
  }
  res->n_applied = h1.n_applied;
  res->n_already = h1.n_already;

  // ---- P5: reachable originals, snapshot jobs level by level ----
  uint8_t* ok = ws.alloc<uint8_t>(n + 1);
  uint32_t* up = ws.alloc<uint32_t>(n + 1);
  LAUNCH(k_pdr_alive_init, dim3(grid_for(n + 1)), dim3(BLOCK), 0, s, p, in.addpar, ok, up);
  for (uint32_t span = 1; span < in.maxlen + 1; span <<= 1)
    LAUNCH(k_pdr_alive_jump, dim3(grid_for(n + 1)), dim3(BLOCK), 0, s, n, ok, up);
  uint32_t s0 = 0, s1 = R0, j0 = 0;
  uint32_t* joff = ws.alloc<uint32_t>(JCAP + 1);
  uint32_t* epre = ws.alloc<uint32_t>(JCAP + 1);
  for (uint32_t level = 0;; ++level) {
    static const uint32_t jobs_grid = pdr_env_grid("CRDTM_PDR_JOBS_GRID", 2048);
    LAUNCH(k_pdr_jobs, dim3(grid_for(s1 - s0, BLOCK, jobs_grid)), dim3(BLOCK), 0, s, p, ok, s0, s1, JCAP, dr);
    if ((r = sync_read(c))) return r;
    if (c->hres->pdr_overflow || level > in.maxlen + 1) {  // no room: sequential replay
      *handled = false;
      ws.used = arena_mark;
      return CRDTM_OK;
    }
    const uint32_t j1 = c->hres->pdr_jobs;
    if (j1 == j0) break;
    LAUNCH(k_pdr_job_size, dim3(grid_for(j1 - j0 + 1)), dim3(BLOCK), 0, s, p, j0, j1, joff);
    if ((r = scan_excl_u32(joff, joff, j1 - j0 + 1, &dr->pdr_slots, ws, s))) return r;
    if ((r = sync_read(c))) return r;
    const uint64_t need = static_cast<uint64_t>(s1) + c->hres->pdr_slots;
    if (need > SCAP) {
      *handled = false;
      ws.used = arena_mark;
      return CRDTM_OK;
    }
    LAUNCH(k_pdr_job_base, dim3(grid_for(j1 - j0)), dim3(BLOCK), 0, s, p, j0, j1, joff, s1);
    // snapshots of logged dicts: rebuilt in parallel; the rest re-replay
    LAUNCH(k_pdr_snap_plan, dim3(grid_for(j1 - j0 + 1)), dim3(BLOCK), 0, s, p, j0, j1, epre);
    if ((r = scan_excl_u32(epre, epre, j1 - j0 + 1, &dr->pdr_dicts, ws, s))) return r;
    if ((r = pdr_run_tiers(c, p, n + 1 + j0, n + 1 + j1, false, st, tt, big_cap, hcount))) return r;
    if ((r = sync_read(c))) return r;
    const uint32_t etot = c->hres->pdr_dicts;
    if (etot)
      LAUNCH(k_pdr_snap_apply, dim3(grid_for(etot)), dim3(BLOCK), 0, s, p, j0, j1 - j0, epre, etot, last);
    LAUNCH(k_pdr_snap_fill, dim3(grid_for(static_cast<uint32_t>(need - s1))), dim3(BLOCK), 0, s, p, j0, j1 - j0,
           joff, s1, static_cast<uint32_t>(need), last);
    s0 = s1;
    s1 = static_cast<uint32_t>(need);
    j0 = j1;
  }
  const uint32_t nj = j0;

  // ---- numbering ----
  const uint32_t NI = n + 1 + nj;
  uint32_t* did = ws.alloc<uint32_t>(NI + 1);
  uint32_t* fpos = ws.alloc<uint32_t>(static_cast<uint64_t>(s1) + 1);
  LAUNCH(k_pdr_inst_flags, dim3(grid_for(NI + 1)), dim3(BLOCK), 0, s, p, ok, nj, did);
  if ((r = scan_excl_u32(did, did, NI + 1, &dr->pdr_dicts, ws, s))) return r;
  LAUNCH(k_pdr_slot_flags, dim3(grid_for(s1 + 1)), dim3(BLOCK), 0, s, p, ok, s1, fpos);
  if ((r = scan_excl_u32(fpos, fpos, s1 + 1, &dr->pdr_slots, ws, s))) return r;
  uint32_t* logidx = ws.alloc<uint32_t>(n + 1);
  LAUNCH(k_pdr_logidx, dim3(g), dim3(BLOCK), 0, s, o, st, logidx);
  if ((r = scan_excl_u32(logidx, logidx, n, nullptr, ws, s))) return r;
  if ((r = sync_read(c))) return r;
  const uint32_t n_dicts = c->hres->pdr_dicts, n_slots = c->hres->pdr_slots;
  TreeCaps need = t->cap;
  need.slots = std::max<uint64_t>(need.slots, n_slots + 1ULL);
  need.dicts = std::max<uint64_t>(need.dicts, n_dicts + 1ULL);
  need.log = std::max<uint64_t>(need.log, t->log_n + h1.n_applied + 1);
  need.lpath = std::max<uint64_t>(need.lpath, t->log_npath + o.n_path + 1);
  if (need.slots > t->cap.slots || need.dicts > t->cap.dicts || need.log > t->cap.log || need.lpath > t->cap.lpath) {
    if ((r = grow_tree(t, need))) return r;
  }
  LAUNCH(k_pdr_write, dim3(grid_for(s1)), dim3(BLOCK), 0, s, p, ok, in.addpar, did, fpos, logidx, s1, t->d);
  if ((r = post_pass(t, o, st, ws))) return r;
  t->n_slots = n_slots;
  t->n_dicts = n_dicts;
  t->timestamp = new_ts;
  t->doc_valid = false;
  res->code = CRDTM_OK;
  return CRDTM_OK;
}

}  // namespace crdtm

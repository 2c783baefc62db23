// forest.hip — the forest's flat documents (many
// independent documents of at most FL_MAXOPS ops with one-key paths), one
// workgroup per document for the slot map and one wave per document for the
// exact sequential replay. The general documents take k_forest (merge.hip
// forest_apply).
//
// Like every kernel file, built with -structurizecfg-skip-uniform-regions
// (Makefile): the replay's branches are all wave-uniform (scalar conditions
// from readfirstlane), and the default structurizer turns them into flow
// blocks with exec-mask bookkeeping the replay does not need (measured on the
// 12.5k config-5 documents: 2.61-2.64 ms per step with the flag against 2.77
// without).
#include "engine.h"
#include "kernels.h"

namespace crdtm {

// ---------------------------------------------------------------------------
// Forest fast path for flat documents (every op's path has length <= 1) of
// at most FL_MAXOPS ops, in two kernels.
// k_forest_prep (one 256-thread workgroup per document): every Add key and
// the sentinel key 0 get a slot such that slot order is key order
// (findInsertion's `ts > key` becomes a slot comparison): the replicas'
// counter ranges laid end to end when they fit (one scan), else the keys
// sorted in LDS (bitonic) with a key's slot = its first sorted position.
// Result: one packed word per op in HBM.
// k_forest_wave (one wave per document): the literal sequential replay of
// addAfterHelp / findInsertion / deleteHelp (src/Internal/Node.elm:56-122) on
// one packed word per slot {next, present, tombstone, orphan}, including the
// copy quirk (a flat node's children are always the initial empty dict, so a
// copy is the slot's own fields); then the visible document is hashed like
// k_forest and the oracle. Documents that do not fit are left to k_forest
// (fb[d] = 1).
// ---------------------------------------------------------------------------
constexpr uint32_t FL_MAXOPS = FL_SLOTS - 1;  // + the sentinel key: FL_SLOTS sort slots
constexpr uint32_t FL_N = 0x7FF;  // 11-bit "none"
// per-op word: tslot | aslot << 11 | DEL << 22 | INVALID << 23 | OWN << 24
constexpr uint32_t FO_DEL = 1u << 22, FO_INV = 1u << 23, FO_OWN = 1u << 24;

__device__ __forceinline__ uint32_t fl_lower(const long long* k, long long x) {
  uint32_t lo = 0, hi = FL_SLOTS;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (k[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

constexpr uint32_t FPREP_THREADS = 256;  // one workgroup (4 waves) per document
constexpr uint32_t FPREP_PER = FL_SLOTS / FPREP_THREADS;  // ops (sort keys) per thread
constexpr uint32_t FPREP_REPS = 64;  // replica ids the dense slot map covers

// A document's slot map. Dense form: slot(key) = base[replica] + counter, the
// replicas' counter ranges laid end to end after the sentinel's slot 0 --
// order preserving and injective, so findInsertion's `ts > key` stays a slot
// comparison; unused counters just leave unused slots. It needs every Add key
// >= 0 with replica id < FPREP_REPS and the ranges to fit FL_SLOTS; otherwise
// the keys are sorted (bitonic) and a slot is a key's first sorted position.
__global__ void __launch_bounds__(FPREP_THREADS) k_forest_prep(OpsDev o, const uint32_t* doc_off, uint32_t n_docs, long long ts0,
                                                    uint32_t* opw, uint16_t* sent, uint8_t* fb, longlong2* vt) {
  __shared__ long long skey[FL_SLOTS];
  __shared__ uint32_t cre[FL_SLOTS];  // slot -> its first Add (the one that can create it)
  __shared__ uint32_t rlo[FPREP_REPS], rhi[FPREP_REPS], rbase[FPREP_REPS];
  __shared__ uint32_t pflags;  // bit0: a path longer than 1 (not flat); bit1: no dense map
  const uint32_t d = blockIdx.x;
  if (d >= n_docs) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t ob = doc_off[d], nops = doc_off[d + 1] - ob;
  if (nops > FL_MAXOPS) {
    if (lane == 0) fb[d] = 1;
    return;
  }
  constexpr long long INF = 0x7fffffffffffffffLL;
  const long long own = replica_of(ts0);
  for (uint32_t j = lane; j < FL_SLOTS; j += FPREP_THREADS) cre[j] = NONE;
  if (lane < FPREP_REPS) {
    rlo[lane] = 0xffffffffu;
    rhi[lane] = 0;
  }
  if (lane == 0) pflags = 0;
  __syncthreads();
  // op j = lane + u * FPREP_THREADS stays in registers: ts, first path key,
  // and {1: empty path, 2: Add, 4: Add with a one-key path (owns a sort key)}
  long long kt[FPREP_PER], ka[FPREP_PER];
  uint32_t ks[FPREP_PER];
  uint32_t flags = 0;
#pragma unroll
  for (uint32_t u = 0; u < FPREP_PER; ++u) {
    const uint32_t j = lane + u * FPREP_THREADS;
    kt[u] = ka[u] = 0;
    ks[u] = 0;
    if (j < nops) {
      const uint32_t i = ob + j;
      const uint32_t p0 = o.off[i], L = o.off[i + 1] - p0;
      const bool add = o.kind[i] == CRDTM_ADD;
      kt[u] = o.ts[i];
      if (L > 1) flags |= 1u;
      if (L >= 1) ka[u] = o.path[p0];
      ks[u] = (L == 0 ? 1u : 0u) | (add ? 2u : 0u) | (add && L == 1 ? 4u : 0u);
      if (add && L == 1) {
        const long long t = kt[u];
        const unsigned long long r = static_cast<unsigned long long>(t) >> 32;
        if (t < 0 || r >= FPREP_REPS) {
          flags |= 2u;
        } else if (t > 0) {
          atomicMin(&rlo[r], static_cast<uint32_t>(t));
          atomicMax(&rhi[r], static_cast<uint32_t>(t));
        }
      }
    }
  }
  if (flags) atomicOr(&pflags, flags);
  __syncthreads();
  const uint32_t pf = pflags;
  if (pf & 1u) {
    if (lane == 0) fb[d] = 1;
    return;
  }
  if (!(pf & 2u) && lane < FPREP_REPS) {  // wave 0: the replicas' slot bases (one scan)
    const uint32_t lo = rlo[lane], hi = rhi[lane];
    const uint32_t range = hi < lo ? 0u : (hi - lo < FL_SLOTS ? hi - lo + 1u : FL_SLOTS);
    uint32_t inc = range;
#pragma unroll
    for (uint32_t k = 1; k < FPREP_REPS; k <<= 1) {
      const uint32_t y = __shfl_up(inc, k, FPREP_REPS);
      if (lane >= k) inc += y;
    }
    rbase[lane] = 1u + (inc - range) - lo;
    if (lane == FPREP_REPS - 1 && inc >= FL_SLOTS) atomicOr(&pflags, 2u);
  }
  __syncthreads();
  const bool dense = !(pflags & 2u);
  uint32_t tsl[FPREP_PER];
  if (dense) {
#pragma unroll
    for (uint32_t u = 0; u < FPREP_PER; ++u) {
      const long long t = kt[u];  // (an owned key is in the map; other ops' ts are not looked up)
      tsl[u] = (ks[u] & 4u) && t != 0 ? rbase[static_cast<unsigned long long>(t) >> 32] + static_cast<uint32_t>(t) : 0u;
      if (ks[u] & 4u) atomicMin(&cre[tsl[u]], lane + u * FPREP_THREADS);
    }
  } else {
#pragma unroll
    for (uint32_t u = 0; u < FPREP_PER; ++u) {
      const uint32_t j = lane + u * FPREP_THREADS;
      skey[j] = j < nops ? ((ks[u] & 4u) ? kt[u] : INF) : (j == nops ? 0 : INF);  // 0: the root dict's sentinel
    }
    for (uint32_t k = 2; k <= FL_SLOTS; k <<= 1) {
      for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
        __syncthreads();
        for (uint32_t i = lane; i < FL_SLOTS; i += FPREP_THREADS) {
          const uint32_t ixj = i ^ jj;
          if (ixj > i) {
            const long long a = skey[i], b = skey[ixj];
            if ((a > b) == ((i & k) == 0)) {
              skey[i] = b;
              skey[ixj] = a;
            }
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < FPREP_PER; ++u) {
      tsl[u] = (ks[u] & 2u) ? fl_lower(skey, kt[u]) : 0u;
      if (ks[u] & 4u) atomicMin(&cre[tsl[u]], lane + u * FPREP_THREADS);
    }
  }
  __syncthreads();  // cre complete: a slot is present iff some Add owns its key
#pragma unroll
  for (uint32_t u = 0; u < FPREP_PER; ++u) {
    const uint32_t j = lane + u * FPREP_THREADS;
    if (j >= nops) continue;
    uint32_t w;
    if (ks[u] & 1u) {
      w = FO_INV | FL_N | (FL_N << 11);
    } else {
      const long long k0 = ka[u];
      uint32_t ps = FL_N;
      if (dense) {
        const unsigned long long r = static_cast<unsigned long long>(k0) >> 32;
        const uint32_t c = static_cast<uint32_t>(k0);
        if (k0 == 0) ps = 0;
        else if (k0 > 0 && r < FPREP_REPS && c >= rlo[r] && c <= rhi[r] && cre[rbase[r] + c] != NONE) ps = rbase[r] + c;
      } else {
        const uint32_t p = fl_lower(skey, k0);
        if (p < FL_SLOTS && skey[p] == k0) ps = p;
      }
      if (!(ks[u] & 2u)) w = FO_DEL | ps | (FL_N << 11);
      else w = tsl[u] | (ps << 11) | (replica_of(kt[u]) == own ? FO_OWN : 0u);
    }
    opw[ob + j] = w;
  }
  if (lane == 0) sent[d] = static_cast<uint16_t>(dense ? 0u : fl_lower(skey, 0));
  if (!vt) return;
  // hash inputs per slot: value and timestamp of the Add that creates it
  longlong2* v = vt + static_cast<uint64_t>(d) * FL_SLOTS;
  for (uint32_t j = lane; j < FL_SLOTS; j += FPREP_THREADS) {
    const uint32_t c = cre[j];
    if (c != NONE) v[j] = make_longlong2(static_cast<long long>(o.val[ob + c]), o.ts[ob + c]);
  }
}

// ---------------------------------------------------------------------------
// Wave-per-document replay (the literal addAfterHelp / findInsertion /
// deleteHelp, src/Internal/Node.elm:56-122, copy quirk included) on a 16-bit
// word per slot {next:11, present, tombstone, orphan} in LDS. What a slot
// carries for the hash (value, timestamp of its Add; a copy takes the copied
// node's) lives in `vt`, written by k_forest_prep and updated on the (rare)
// copy quirk.
// ---------------------------------------------------------------------------
constexpr uint16_t FW_PRESENT = 1u << 11, FW_TOMB = 1u << 12, FW_ORPHAN = 1u << 13;
// slot words cover indices [0, FL_N]: slot FL_N ("none") stays 0 (absent, not
// a tombstone), so lookups of "none" need no test and tombstone runs end there
constexpr uint32_t FLANE_REGION = FL_N + 1;

// One wave per document, every lane computing the same replay: the op word
// comes from a register holding 64 op words (readlane) and every slot word is
// read by all lanes at one address, so the data stays in vector registers
// (the 4 SIMDs' ALUs) while each decision takes its condition to a scalar
// register and branches on it -- no exec-mask bookkeeping around divergent
// code on the CU's one scalar unit.
__device__ __forceinline__ uint32_t wuni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
// a wave-uniform comparison of vector values as a branch condition: the
// compare's lane mask itself (every lane agrees), instead of a 0/1 select
// moved to a scalar register and tested again
__device__ __forceinline__ bool uany(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0ULL; }

// DPW documents per workgroup, one wave each (each wave only ever touches
// its own slot region: no workgroup barrier, so a wave may leave early).
// Round 6: in this form (lane = thread id & 63, the document from workgroup
// and wave) the compiler keeps the replay's arithmetic on the vector units
// instead of the CU's one scalar unit (642 -> 317 scalar instructions):
// k_forest_wave 1.94-2.06 -> 1.67-1.75 ms on 12.5k documents; 2 or 4
// documents per workgroup measured the same as 1)
template <uint32_t DPW>
__global__ void __launch_bounds__(64 * DPW) k_forest_wave(const uint32_t* doc_off, uint32_t n_docs, long long ts0,
                                                    const uint32_t* opw, const uint16_t* sent, const uint8_t* fb,
                                                    longlong2* vt, int32_t* code_out, uint32_t* err_out,
                                                    uint32_t* applied_out, unsigned long long* vhash,
                                                    unsigned long long* vwords, long long* tstamp, uint32_t* overflow) {
  __shared__ uint16_t sl_all[DPW][FLANE_REGION];
  const uint32_t d = blockIdx.x * DPW + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  uint16_t* sl = sl_all[threadIdx.x >> 6];
  if (d >= n_docs || fb[d]) return;
  for (uint32_t j = lane; j < FLANE_REGION / 8; j += 64) reinterpret_cast<uint4*>(sl)[j] = make_uint4(0, 0, 0, 0);
  const uint32_t ob = wuni(doc_off[d]), nops = wuni(doc_off[d + 1]) - ob;
  const uint32_t s0 = wuni(sent[d]);
  wave_sync();  // (the wave's own LDS stores before its loads)
  auto rd = [&](uint32_t j) { return static_cast<uint32_t>(sl[j]); };
  auto wr = [&](uint32_t j, uint32_t w) { sl[j] = static_cast<uint16_t>(w); };
  wr(s0, FL_N | FW_PRESENT | FW_TOMB);
  uint32_t own = 0, applied = 0, err = NONE;
  int32_t code = CRDTM_OK;
  uint32_t vw = lane < nops ? opw[ob + lane] : 0u;
  for (uint32_t c0 = 0; c0 < nops; c0 += 64) {
    const uint32_t nxt = c0 + 64 + lane < nops ? opw[ob + c0 + 64 + lane] : 0u;  // next 64 op words, in flight
    const uint32_t kend = wuni(min(64u, nops - c0));
    for (uint32_t k = 0; k < kend; ++k) {
      const uint32_t w = __builtin_amdgcn_readlane(vw, k);
      const uint32_t t = w & FL_N;
      const uint32_t st = rd(t);
      // (if/else instead of `continue`, errors leave by goto: the loop keeps
      // no exit-code dispatch between ops)
      if (wuni(w & (FO_DEL | FO_INV))) {
        if (wuni((w & FO_INV) | ((st & FW_PRESENT) ^ FW_PRESENT))) {  // InvalidPath / deleteHelp NotFound (:112-122)
          err = c0 + k;
          code = (w & FO_INV) ? CRDTM_INVALID_PATH : CRDTM_OPERATION_FAILED;
          goto replay_done;
        }
        if (!wuni(st & FW_TOMB)) {
          wr(t, st | FW_TOMB);
          ++applied;
        }
      } else if (wuni(st & FW_PRESENT)) {  // `child ts parent` exists: AlreadyApplied
        own += (w >> 24) & 1u;
      } else {
        const uint32_t a = (w >> 11) & FL_N;
        const uint32_t sa = rd(a);
        if (!wuni(sa & FW_PRESENT)) {  // anchor missing: NotFound
          err = c0 + k;
          code = CRDTM_OPERATION_FAILED;
          goto replay_done;
        }
        const uint32_t x = t;
        uint32_t nk = a, node = a, sn = sa;  // findInsertion (:93-104)
        for (;;) {
          const uint32_t rn = sn & FL_N;
          uint32_t live = rn, wl = rd(rn);
          while (wuni(wl & FW_TOMB)) {  // nextNode: the first live node after next
            live = wl & FL_N;
            wl = rd(live);
          }
          // (measured in round 5: deciding `x > rn` before rn's word is read,
          // as the per-dict replays do, 2.61 -> 3.02 ms here; the anchor's word
          // read beside the target's, no change)
          if (uany(live == FL_N || x > rn)) break;
          nk = rn;
          node = live;
          sn = wl;
        }
        const bool same = uany(nk == node);
        const uint32_t snk = same ? sn : rd(nk);
        wr(x, (sn & FL_N) | FW_PRESENT | (snk & FW_ORPHAN));
        if (same) {
          wr(node, (sn & ~FL_N) | x);
        } else {  // copy quirk: slot nk := copy of node with next = x
          if (!wuni(snk & FW_ORPHAN)) {
            for (uint32_t q = snk & FL_N; uany(q != FL_N);) {
              const uint32_t sq = rd(q);
              wr(q, sq | FW_ORPHAN);
              if (uany(q == node)) break;
              q = sq & FL_N;
            }
          }
          wr(nk, x | FW_PRESENT | (snk & FW_ORPHAN));
          if (lane == 0) {
            longlong2* v = vt + static_cast<uint64_t>(d) * FL_SLOTS;
            v[nk] = v[node];
          }
        }
        ++applied;
        own += (w >> 24) & 1u;  // incrementTimestamp (src/CRDTree.elm:337-343)
      }
    }
    vw = nxt;
  }
replay_done:
  if (lane == 0) {
    code_out[d] = code;
    err_out[d] = err;
    applied_out[d] = applied;
    tstamp[d] = ts0 + own;
    overflow[d] = 0;
  }
  // the visible document's hash (the oracle's dumpVisible words), its
  // (value, timestamp) loads issued 8 entries ahead of the hash chain
  Fnv h;
  if (code == CRDTM_OK) {
    __threadfence_block();  // the copy quirk's vt writes (lane 0) before every lane's reads
    const longlong2* v = vt + static_cast<uint64_t>(d) * FL_SLOTS;
    uint32_t wc = rd(s0);
    bool more = true;
    while (more) {
      uint32_t sv[8];
      uint32_t c = 0;
      for (; c < 8; ++c) {
        uint32_t nx = wc & FL_N, wn = rd(nx);
        while (wuni(wn & FW_TOMB)) {
          nx = wn & FL_N;
          wn = rd(nx);
        }
        if (uany(nx == FL_N)) {
          more = false;
          break;
        }
        sv[c] = nx;
        wc = wn;
      }
      longlong2 e[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k)
        if (k < c) e[k] = v[sv[k]];
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) {
        if (k < c) {
          h.put(0);
          h.put(e[k].x);
          h.put(1);
          h.put(e[k].y);
        }
      }
    }
  }
  if (lane == 0) {
    vhash[d] = h.h;
    vwords[d] = h.n;
  }
}


int forest_flat_launch(const OpsDev& o, const uint32_t* doff, uint32_t n_docs, long long ts0, uint32_t* opw,
                       uint16_t* sent, uint8_t* fb, longlong2* vt, int32_t* code, uint32_t* err, uint32_t* applied,
                       unsigned long long* vhash, unsigned long long* vwords, long long* tstamp,
                       uint32_t* overflow, hipStream_t s) {
  if (!n_docs) return CRDTM_OK;
  LAUNCH(k_forest_prep, dim3(n_docs), dim3(FPREP_THREADS), 0, s, o, doff, n_docs, ts0, opw, sent, fb, vt);
  // one wave per document, its replay's branches scalar and its data vector
  // (measured on 12.5k config-5 documents: 2.36 ms; one lane per document with
  // divergent vector control 2.65 ms at one document per wave and 2.95 / 3.80 /
  // 5.70 ms at 2 / 4 / 8; the replay wholly scalar 2.79 ms; a flattened step
  // machine at 4-16 documents per wave 6-8.6 ms; round 5: the same replay with
  // structured control flow and every slot word made uniform at its read,
  // ~2x fewer instructions per op, 2.96 ms -- the dependent LDS reads and
  // scalar waits, not the issue count, bound it)
  // (env CRDTM_FOREST_DPW: documents per workgroup, 1 / 2 / 4)
  static const uint32_t dpw = [] {
    const char* e = getenv("CRDTM_FOREST_DPW");
    const int v = e ? atoi(e) : 1;
    return (v == 2 || v == 4) ? static_cast<uint32_t>(v) : 1u;
  }();
  const uint32_t nb = static_cast<uint32_t>((n_docs + dpw - 1) / dpw);
  if (dpw == 4)
    LAUNCH(k_forest_wave<4>, dim3(nb), dim3(256), 0, s, doff, n_docs, ts0, opw, sent, fb, vt, code, err, applied,
           vhash, vwords, tstamp, overflow);
  else if (dpw == 2)
    LAUNCH(k_forest_wave<2>, dim3(nb), dim3(128), 0, s, doff, n_docs, ts0, opw, sent, fb, vt, code, err, applied,
           vhash, vwords, tstamp, overflow);
  else
    LAUNCH(k_forest_wave<1>, dim3(nb), dim3(64), 0, s, doff, n_docs, ts0, opw, sent, fb, vt, code, err, applied,
           vhash, vwords, tstamp, overflow);
  return CRDTM_OK;
}

}  // namespace crdtm

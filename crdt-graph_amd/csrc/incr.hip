// incr.hip — incremental closed form for a flat document (SURVEY.md Appendix B,
// "incremental merge into an existing list"): `apply (Batch adds) tree`
// (src/CRDTree.elm:265-269) on a tree that already holds a flat document with
// no tombstones, in O(document) streaming passes plus O(batch) work, instead of
// re-merging log ++ batch.
//
// With no tombstone anywhere, findInsertion (src/Internal/Node.elm:93-104) is
// plain RGA: x goes after its anchor, past every following node with a larger
// timestamp. Against the document before the batch (the "base", in document
// order, keys dk[0..K)), a new node x therefore lands in the gap before base
// rank
//     g(x) = NSR(start, t) = the first rank r >= start with dk[r] < t,
// where for an anchor in the base start = rank(anchor) + 1 (the sentinel: 0)
// and t = ts(x); for an anchor a that is itself new, x's walk starts in a's
// gap and continues past base nodes with larger keys, so g(x) = NSR(g(a),
// ts(x)); since NSR(NSR(s, t1), t2) = NSR(s, min(t1, t2)), a chain of new
// anchors composes to one query with the chain's smallest timestamp (pointer
// jumping). New nodes in a gap before the one x lands in all have keys above
// that base node's key, hence above ts(x): x's walk passes them, so the base
// alone decides the gap. Inside a gap, the new nodes are an RGA list of their
// own: x starts after its anchor when the anchor is in the same gap, else at
// the gap's head, and walks past larger keys (replayed per gap, in batch order).
// Every other case — a Delete, a nested path, a duplicate or existing key, an
// anchor that is missing or later in the batch, replica-id drift, a tree that
// is not a clean flat document — is left to the general paths (merge.hip).
#include <algorithm>
#include <cstring>

#include "engine.h"
#include "kernels.h"

namespace crdtm {

constexpr uint32_t FI_BLK = 64;             // ranks per block minimum (one wave)
constexpr uint32_t FI_SUP = 64;             // blocks per superblock
constexpr uint32_t FI_MAX_BATCH = 1u << 14; // larger batches re-merge (k_fi_jump holds 16 per thread)
constexpr uint32_t FI_GAP_STEPS = 1u << 22; // walk budget per gap (else re-merge)
constexpr long long FI_INF = 0x7fffffffffffffffLL;

// flags word bits (fi[0])
enum : uint32_t { FI_FAIL = 1u, FI_BUDGET = 2u };

KeyIndex::~KeyIndex() {
  for (void* q : {static_cast<void*>(keys), static_cast<void*>(vals), static_cast<void*>(dk[0]),
                  static_cast<void*>(dk[1]), static_cast<void*>(rank), static_cast<void*>(doc2)})
    if (q) hipFree(q);
}

// key -> slot over every node of a flat tree (slots 1..n_slots-1 of the root dict)
__global__ void __launch_bounds__(BLOCK) k_kx_build(const long long* s_key, uint32_t n_slots, TsHash h) {
  GRID_STRIDE(q, n_slots) {
    if (q == 0) continue;
    tshash_insert(h, s_key[q], q);
  }
}

__global__ void __launch_bounds__(BLOCK) k_kx_insert(OpsDev o, uint32_t slot0, TsHash h) {
  GRID_STRIDE(i, o.n) tshash_insert(h, o.ts[i], slot0 + i);
}

// dk[r] = key of doc[r], rank_of[slot] = r (when the index has no document order yet)
__global__ void __launch_bounds__(BLOCK) k_fi_prep(uint32_t K, const uint32_t* doc, const long long* s_key,
                                                   long long* dk, uint32_t* rank_of) {
  GRID_STRIDE(r, K) {
    const uint32_t sl = doc[r];
    dk[r] = s_key[sl];
    rank_of[sl] = r;
  }
}

// bmin[b] = the smallest of keys [64 b, 64 b + 64): a wave covers four
// blocks, four keys per lane (two 16-byte loads), 16 lanes per block
__global__ void __launch_bounds__(BLOCK) k_fi_bmin(uint32_t K, const long long* dk, long long* bmin) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nb = (K + FI_BLK - 1) / FI_BLK;
  const uint32_t nw = (nb + 3) / 4;
  for (uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) / 64; w < nw; w += gridDim.x * blockDim.x / 64) {
    const uint32_t r = w * 256 + 4 * lane;
    long long k = FI_INF;
    if (r + 4 <= K) {
      const longlong2 a = *reinterpret_cast<const longlong2*>(dk + r);
      const longlong2 c = *reinterpret_cast<const longlong2*>(dk + r + 2);
      k = min(min(a.x, a.y), min(c.x, c.y));
    } else {
      for (uint32_t j = r; j < K && j < r + 4; ++j) k = min(k, dk[j]);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const uint32_t lo = __shfl_xor(static_cast<uint32_t>(k), o, 64);
      const uint32_t hi = __shfl_xor(static_cast<uint32_t>(static_cast<unsigned long long>(k) >> 32), o, 64);
      const long long v = static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo);
      k = v < k ? v : k;
    }
    const uint32_t b = w * 4 + lane / 16;
    if ((lane & 15) == 0 && b < nb) bmin[b] = k;
  }
}

__global__ void __launch_bounds__(BLOCK) k_fi_sup(uint32_t nb, const long long* bmin, long long* smin) {
  const uint32_t ns = (nb + FI_SUP - 1) / FI_SUP;
  GRID_STRIDE(s, ns) {
    long long m = FI_INF;
    const uint32_t e = min(nb, (s + 1) * FI_SUP);
    for (uint32_t b = s * FI_SUP; b < e; ++b) m = min(m, bmin[b]);
    smin[s] = m;
  }
}

// batch keys -> op index; a key seen twice fails the batch
__global__ void __launch_bounds__(BLOCK) k_fi_bidx(OpsDev o, TsHash bh, uint32_t* fi) {
  GRID_STRIDE(i, o.n) {
    const unsigned long long k = static_cast<unsigned long long>(o.ts[i]) ^ 0x8000000000000000ULL;
    uint32_t p = static_cast<uint32_t>(mix64(k)) & bh.mask;
    for (;;) {
      const unsigned long long prev = atomicCAS(&bh.keys[p], 0ULL, k);
      if (prev == 0ULL) {
        bh.vals[p] = i;
        break;
      }
      if (prev == k) {
        atomicOr(&fi[0], FI_FAIL);
        break;
      }
      p = (p + 1) & bh.mask;
    }
  }
}

// Each op must be a fresh flat Add whose anchor is the sentinel, a base node or
// an earlier op of the batch (addAfterHelp, src/Internal/Node.elm:62-90):
// par = the anchor op (NONE: a base anchor / the sentinel, start = its rank + 1),
// thr = ts; fi[1] counts own-replica Adds (incrementTimestamp).
__global__ void __launch_bounds__(BLOCK) k_fi_resolve(OpsDev o, TsHash kx, TsHash bh, const uint32_t* rank_of,
                                                      long long id0, uint32_t* par, uint32_t* par0, uint32_t* start,
                                                      long long* thr, uint32_t* fi) {
  uint32_t own = 0, fail = 0;
  GRID_STRIDE(i, o.n) {
    const long long ts = o.ts[i];
    const uint32_t b = o.off[i];
    uint32_t p = NONE, s = 0;
    if (o.kind[i] != CRDTM_ADD || o.off[i + 1] != b + 1 || ts <= 0 || ts >= TWO53 || tshash_find(kx, ts) != NONE) {
      fail = 1;
    } else {
      const long long a = o.path[b];
      if (a != 0) {
        const uint32_t sl = (a > 0 && a < TWO53) ? tshash_find(kx, a) : NONE;
        if (sl != NONE) {
          s = rank_of[sl] + 1;
        } else {
          const uint32_t j = (a > 0 && a < TWO53) ? tshash_find(bh, a) : NONE;
          if (j == NONE || j >= i) fail = 1;  // NotFound (or not yet applied): the general paths decide
          else p = j;
        }
      }
      if (replica_of(ts) == id0) ++own;
    }
    par[i] = p;
    par0[i] = p;
    start[i] = s;
    thr[i] = ts;
  }
  own = block_sum(own);
  fail = block_max(fail);
  if (threadIdx.x == 0) {
    if (own) atomicAdd(&fi[1], own);
    if (fail) atomicOr(&fi[0], FI_FAIL);
  }
}

// Pointer jumping, all rounds in one workgroup: (start, min threshold)
// composed along the new anchors. Each round reads every element's jumped
// values into registers, then (after a barrier) writes them back in place:
// no second buffer, and chains are short (typing runs), so the rounds stop
// once no anchor is left. Up to FI_JUMP_PER elements per thread.
constexpr uint32_t FI_JUMP_THREADS = 1024, FI_JUMP_PER = 16;
__global__ void __launch_bounds__(FI_JUMP_THREADS) k_fi_jump(uint32_t m, uint32_t rounds, uint32_t* P, uint32_t* S,
                                                             long long* T) {
  __shared__ uint32_t live[32];  // one flag per round (rounds <= 16: m <= 2^16)
  if (threadIdx.x < 32) live[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t k = 0; k < rounds; ++k) {
    uint32_t np[FI_JUMP_PER], ns[FI_JUMP_PER];
    long long nt[FI_JUMP_PER];
    uint32_t any = 0;
#pragma unroll
    for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
      const uint32_t i = threadIdx.x + u * FI_JUMP_THREADS;
      np[u] = NONE;
      if (i < m) {
        const uint32_t p = P[i];
        ns[u] = S[i];
        nt[u] = T[i];
        if (p != NONE) {
          np[u] = P[p];
          ns[u] = S[p];
          nt[u] = min(nt[u], T[p]);
          any |= np[u] != NONE;
        }
      }
    }
    __syncthreads();  // every read of this round before any write
#pragma unroll
    for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
      const uint32_t i = threadIdx.x + u * FI_JUMP_THREADS;
      if (i < m) {
        P[i] = np[u];
        S[i] = ns[u];
        T[i] = nt[u];
      }
    }
    if (any) live[k] = 1;
    __syncthreads();  // writes visible to the workgroup, live[k] final
    if (!live[k]) break;
  }
}

// g = NSR(start, thr) over the base keys, one wave per query: 64 keys, 64
// block minima or 64 superblock minima per step (ballot), then down again
__global__ void __launch_bounds__(BLOCK) k_fi_gap(uint32_t m, uint32_t K, const long long* dk, const long long* bmin,
                                                  const long long* smin, const uint32_t* start, const long long* thr,
                                                  uint32_t* gkey, uint32_t* gval) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nb = (K + FI_BLK - 1) / FI_BLK, ns = (nb + FI_SUP - 1) / FI_SUP;
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  if (i >= m) return;  // (wave-uniform)
  const long long t = thr[i];
  const uint32_t r = start[i];
  // first index >= from in [lo, hi) (64 wide, starting at lo) whose value is < t
  auto first64 = [&](const long long* v, uint32_t lo, uint32_t from, uint32_t hi) -> uint32_t {
    const uint32_t q = lo + lane;
    const unsigned long long mk = __ballot(q >= from && q < hi && v[q] < t);
    return mk ? lo + static_cast<uint32_t>(__builtin_ctzll(mk)) : NONE;
  };
  uint32_t g = K;
  if (r < K) {
    const uint32_t b = r / FI_BLK;
    uint32_t q = first64(dk, b * FI_BLK, r, K);
    if (q == NONE && b + 1 < nb) {
      const uint32_t s0 = (b + 1) / FI_SUP;
      uint32_t bb = first64(bmin, s0 * FI_SUP, b + 1, nb);
      for (uint32_t ss = s0 + 1; bb == NONE && ss < ns; ss += 64) {
        const uint32_t sq = first64(smin, ss, ss, ns);
        if (sq != NONE) bb = first64(bmin, sq * FI_SUP, sq * FI_SUP, nb);
      }
      if (bb != NONE) q = first64(dk, bb * FI_BLK, bb * FI_BLK, K);
    }
    if (q != NONE) g = q;
  }
  if (lane == 0) {
    gkey[i] = g;
    gval[i] = i;
  }
}

__global__ void k_fi_setn(uint32_t* p, uint32_t v) { *p = v; }

__global__ void __launch_bounds__(BLOCK) k_fi_pos(uint32_t m, const uint32_t* gv, uint32_t* pos) {
  GRID_STRIDE(k, m) pos[gv[k]] = k;
}

// gap heads: the first sorted position of every gap, listed (any order)
__global__ void __launch_bounds__(BLOCK) k_fi_gstart(uint32_t m, const uint32_t* gk, uint32_t* list, uint32_t* cnt) {
  GRID_STRIDE(k, m) {
    if (k == 0 || gk[k - 1] != gk[k]) list[atomicAdd(cnt, 1u)] = k;
  }
}

// One wave per gap: the gap's new nodes, in batch order, are inserted into a
// list of their own (RGA with no tombstones: after the anchor when it is in
// this gap, else after the head; past every following node with a larger
// timestamp) by lane 0 on keys and links staged in LDS (a gap larger than
// the LDS stage walks global memory instead); then ord[] = the list order
// and first[] = the gap's first sorted position.
constexpr uint32_t FI_GAP_LDS = 1024;
__global__ void __launch_bounds__(64) k_fi_gaps(uint32_t m, const uint32_t* list, const uint32_t* cnt,
                                                const uint32_t* gk, const uint32_t* gv, const uint32_t* par0,
                                                const uint32_t* pos, const long long* ts, uint32_t* nxt,
                                                uint32_t* ord, uint32_t* first, uint32_t* fi) {
  __shared__ long long lk[FI_GAP_LDS];
  __shared__ uint32_t la[FI_GAP_LDS], ln[FI_GAP_LDS], lo[FI_GAP_LDS];
  const uint32_t w = blockIdx.x, lane = threadIdx.x;
  if (w >= *cnt) return;
  const uint32_t k = list[w], g = gk[k];
  uint32_t e = k + 1;  // the gap's end: 64 positions per step
  for (;;) {
    const uint32_t q = e + lane;
    const unsigned long long mk = __ballot(q >= m || gk[q] != g);
    if (mk) {
      e += static_cast<uint32_t>(__builtin_ctzll(mk));
      break;
    }
    e += 64;
  }
  const uint32_t n = e - k;
  if (n <= FI_GAP_LDS) {
    for (uint32_t j = lane; j < n; j += 64) {
      const uint32_t op = gv[k + j];
      lk[j] = ts[op];
      const uint32_t a = par0[op];
      uint32_t l = NONE;
      if (a != NONE) {
        const uint32_t pa = pos[a];
        if (pa >= k && pa < e) l = pa - k;
      }
      la[j] = l;
    }
    __syncthreads();
    if (lane == 0) {
      uint32_t head = NONE;
      for (uint32_t j = 0; j < n; ++j) {
        const long long x = lk[j];
        uint32_t cur = la[j];  // NONE = the head
        uint32_t nx = cur == NONE ? head : ln[cur];
        while (nx != NONE && lk[nx] > x) {
          cur = nx;
          nx = ln[cur];
        }
        ln[j] = nx;
        if (cur == NONE) head = j;
        else ln[cur] = j;
      }
      uint32_t o = 0;
      for (uint32_t j = head; j != NONE; j = ln[j]) lo[j] = o++;
    }
    __syncthreads();
    for (uint32_t j = lane; j < n; j += 64) {
      ord[k + j] = lo[j];
      first[k + j] = k;
    }
    return;
  }
  if (lane != 0) return;
  uint32_t head = NONE, steps = 0;
  bool over = false;
  for (uint32_t q = k; q < e && !over; ++q) {
    const uint32_t op = gv[q];
    const long long x = ts[op];
    const uint32_t a = par0[op];
    uint32_t cur = NONE;  // NONE = the gap's head
    if (a != NONE) {
      const uint32_t pa = pos[a];
      if (pa >= k && pa < e) cur = pa;
    }
    uint32_t nx = cur == NONE ? head : nxt[cur];
    while (nx != NONE && ts[gv[nx]] > x) {
      cur = nx;
      nx = nxt[cur];
      if (++steps > FI_GAP_STEPS) {
        over = true;
        break;
      }
    }
    nxt[q] = nx;
    if (cur == NONE) head = q;
    else nxt[cur] = q;
  }
  if (over) {
    atomicOr(&fi[0], FI_BUDGET);
    return;
  }
  uint32_t o = 0;
  for (uint32_t q = head; q != NONE; q = nxt[q]) {
    ord[q] = o++;
    first[q] = k;
  }
}

// new document ranks: base rank r -> r + (new nodes in gaps <= r); new node
// at sorted position k -> its gap + the new nodes of earlier gaps + its order.
// Each workgroup bounds its base ranks' searches by two searches of its own.
__device__ __forceinline__ uint32_t fi_count_le(const uint32_t* gk, uint32_t lo, uint32_t hi, uint32_t r) {
  while (lo < hi) {  // count of gk <= r in [lo, hi) (gk ascending)
    const uint32_t mid = (lo + hi) >> 1;
    if (gk[mid] <= r) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(BLOCK) k_fi_doc(uint32_t K, uint32_t m, const uint32_t* doc, const uint32_t* gk,
                                                  const uint32_t* gv, const uint32_t* ord, const uint32_t* first,
                                                  uint32_t slot0, const long long* ts, const long long* dk,
                                                  uint32_t* newdoc, uint32_t* newrank, long long* newdk,
                                                  uint32_t* rank_of) {
  __shared__ uint32_t bnd[2];
  const uint32_t r0 = blockIdx.x * blockDim.x, r = r0 + threadIdx.x;
  if (r0 < K && threadIdx.x < 2) {
    const uint32_t rr = threadIdx.x == 0 ? r0 : min(K - 1, r0 + blockDim.x - 1);
    bnd[threadIdx.x] = threadIdx.x == 0 ? (r0 ? fi_count_le(gk, 0, m, r0 - 1) : 0u) : fi_count_le(gk, 0, m, rr);
  }
  __syncthreads();
  if (r < K) {
    const uint32_t p = r + fi_count_le(gk, bnd[0], bnd[1], r), sl = doc[r];
    newdoc[p] = sl;
    newdk[p] = dk[r];
    rank_of[sl] = p;
  } else if (r < K + m) {
    const uint32_t k = r - K;
    const uint32_t p = gk[k] + first[k] + ord[k], op = gv[k];
    newrank[k] = p;
    newdoc[p] = slot0 + op;
    newdk[p] = ts[op];
    rank_of[slot0 + op] = p;
  }
}

// next pointers: every new node, and the node before each gap's first one
__global__ void __launch_bounds__(BLOCK) k_fi_next(uint32_t K, uint32_t m, const uint32_t* gv, const uint32_t* ord,
                                                   const uint32_t* newrank, const uint32_t* newdoc, uint32_t slot0,
                                                   uint32_t* s_next) {
  const uint32_t n = K + m;
  GRID_STRIDE(k, m) {
    const uint32_t p = newrank[k], sl = slot0 + gv[k];
    s_next[sl] = p + 1 < n ? newdoc[p + 1] : NONE;
    if (ord[k] == 0) s_next[p == 0 ? 0u : newdoc[p - 1]] = sl;
  }
}

// node records of the new slots and the log append (every op applied, |path| = 1)
__global__ void __launch_bounds__(BLOCK) k_fi_commit(OpsDev o, uint32_t slot0, uint32_t log0, uint32_t lpath0,
                                                     TreeDev T) {
  GRID_STRIDE(i, o.n) {
    const uint32_t sl = slot0 + i;
    T.s_key[sl] = o.ts[i];
    T.s_src[sl] = log0 + i;
    T.s_flags[sl] = 0;
    T.s_child[sl] = NONE;
    T.s_dict[sl] = 0;
    T.l_kind[log0 + i] = o.kind[i];
    T.l_ts[log0 + i] = o.ts[i];
    T.l_val[log0 + i] = o.val[i];
    T.l_off[log0 + i] = lpath0 + i;
    T.l_path[lpath0 + i] = o.path[o.off[i]];
    if (i + 1 == o.n) T.l_off[log0 + o.n] = lpath0 + o.n;
  }
}

static uint32_t pow2_ge(uint64_t x) {
  uint64_t p = 1024;
  while (p < x) p <<= 1;
  return static_cast<uint32_t>(p);
}

static bool finc_allowed() {
  const char* e = getenv("CRDTM_INCREMENTAL");
  return !(e && (!strcmp(e, "replay") || !strcmp(e, "remerge")));
}

// (Re)builds the tree's key index when it does not describe the state; the
// document-order arrays get room for the batch and are rebuilt (ord_ready)
// when they are new or the index was stale.
static int kx_ensure(crdtm_tree* t, uint64_t extra) {
  crdtm_ctx* c = t->ctx;
  const uint64_t need_h = 2 * (t->n_slots + extra) + 1024, need_o = t->n_slots + extra + 1;
  if (!t->kidx) t->kidx = std::make_unique<KeyIndex>();
  KeyIndex& x = *t->kidx;
  if (x.ocap < need_o) {
    for (long long*& q : x.dk) {
      if (q) hipFree(q);
      q = nullptr;
    }
    if (x.rank) hipFree(x.rank);
    x.rank = nullptr;
    const uint64_t oc = 2 * need_o + 4096;
    HIP_CHECK(hipMalloc(&x.dk[0], oc * sizeof(long long)));
    HIP_CHECK(hipMalloc(&x.dk[1], oc * sizeof(long long)));
    HIP_CHECK(hipMalloc(&x.rank, oc * sizeof(uint32_t)));
    x.ocap = oc;
    x.ord_ready = false;
  }
  if (t->kidx_valid && static_cast<uint64_t>(x.mask) + 1 >= need_h) return CRDTM_OK;
  if (static_cast<uint64_t>(x.mask) + 1 < need_h) {
    if (x.keys) hipFree(x.keys);
    if (x.vals) hipFree(x.vals);
    x.keys = nullptr;
    x.vals = nullptr;
    const uint32_t cap = pow2_ge(2 * need_h);  // room for later batches before a rebuild
    HIP_CHECK(hipMalloc(&x.keys, static_cast<size_t>(cap) * sizeof(unsigned long long)));
    HIP_CHECK(hipMalloc(&x.vals, static_cast<size_t>(cap) * sizeof(uint32_t)));
    x.mask = cap - 1;
  }
  const uint32_t cap = x.mask + 1;
  HIP_CHECK(hipMemsetAsync(x.keys, 0, static_cast<size_t>(cap) * sizeof(unsigned long long), c->stream));
  HIP_CHECK(hipMemsetAsync(x.vals, 0xFF, static_cast<size_t>(cap) * sizeof(uint32_t), c->stream));
  LAUNCH(k_kx_build, dim3(grid_for(t->n_slots)), dim3(BLOCK), 0, c->stream, t->d.s_key,
         static_cast<uint32_t>(t->n_slots), TsHash{x.keys, x.vals, x.mask});
  t->kidx_valid = true;
  x.ord_ready = false;
  return CRDTM_OK;
}

int finc_apply(crdtm_tree* t, const OpsDev& o, uint8_t* st_out, crdtm_result* res, bool* handled) {
  *handled = false;
  const uint32_t m = o.n;
  const uint64_t K64 = t->n_slots - 1;
  if (!finc_allowed() || m == 0 || m > FI_MAX_BATCH || !t->flat_clean || !t->doc_valid || t->n_dicts != 1 ||
      t->doc_n != K64 || K64 == 0 || o.n_path != m || K64 + m >= 0x7FFFFFF0ULL)
    return CRDTM_OK;
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  const uint32_t K = static_cast<uint32_t>(K64);
  const size_t mark0 = ws.used;
  // every workspace buffer first: nothing is written to the state before the last check
  const uint32_t nb = (K + FI_BLK - 1) / FI_BLK, ns = (nb + FI_SUP - 1) / FI_SUP;
  long long* bmin = ws.alloc<long long>(nb);
  long long* smin = ws.alloc<long long>(ns);
  const uint32_t bcap = pow2_ge(2ULL * m);
  TsHash bh{ws.alloc<unsigned long long>(bcap), ws.alloc<uint32_t>(bcap), bcap - 1};
  uint32_t* fi = ws.alloc<uint32_t>(4);
  uint32_t* par[1] = {ws.alloc<uint32_t>(m)};
  uint32_t* sta[1] = {ws.alloc<uint32_t>(m)};
  long long* thr[1] = {ws.alloc<long long>(m)};
  uint32_t* par0 = ws.alloc<uint32_t>(m);
  uint32_t* gk[2] = {ws.alloc<uint32_t>(m), ws.alloc<uint32_t>(m)};
  uint32_t* gv[2] = {ws.alloc<uint32_t>(m), ws.alloc<uint32_t>(m)};
  uint32_t* nm = ws.alloc<uint32_t>(1);
  uint32_t* pos = ws.alloc<uint32_t>(m);
  uint32_t* nxt = ws.alloc<uint32_t>(m);
  uint32_t* glist = ws.alloc<uint32_t>(m);
  uint32_t* ord = ws.alloc<uint32_t>(m);
  uint32_t* first = ws.alloc<uint32_t>(m);
  uint32_t* newrank = ws.alloc<uint32_t>(m);
  uint8_t* st = ws.alloc<uint8_t>(m);
  long long* rep = ws.alloc<long long>(2ULL * m + 2);
  int r;
  if ((r = kx_ensure(t, m))) return r;
  KeyIndex& X = *t->kidx;
  const TsHash kx{X.keys, X.vals, X.mask};
  long long* dk = X.dk[X.cur];
  uint32_t* rank_of = X.rank;
  // ---- phase A: base order, anchors, validity ----
  HIP_CHECK(hipMemsetAsync(fi, 0, 4 * sizeof(uint32_t), s));
  HIP_CHECK(hipMemsetAsync(bh.keys, 0, static_cast<size_t>(bcap) * sizeof(unsigned long long), s));
  if (!X.ord_ready) {  // (kept up to date by every incremental merge after this one)
    LAUNCH(k_fi_prep, dim3(grid_for(K)), dim3(BLOCK), 0, s, K, t->d.doc, t->d.s_key, dk, rank_of);
    X.ord_ready = true;
  }
  LAUNCH(k_fi_bmin, dim3(grid_for(static_cast<uint64_t>(nb + 3) / 4 * 64)), dim3(BLOCK), 0, s, K, dk, bmin);
  LAUNCH(k_fi_sup, dim3(grid_for(ns)), dim3(BLOCK), 0, s, nb, bmin, smin);
  LAUNCH(k_fi_bidx, dim3(grid_for(m)), dim3(BLOCK), 0, s, o, bh, fi);
  LAUNCH(k_fi_resolve, dim3(grid_for(m)), dim3(BLOCK), 0, s, o, kx, bh, rank_of, replica_of(t->timestamp), par[0],
         par0, sta[0], thr[0], fi);
  // ---- phase B: gaps (pointer jumping over new anchors, one NSR query each) ----
  uint32_t rounds = 0;
  for (uint32_t span = 1; span < m; span <<= 1) ++rounds;
  if (rounds) LAUNCH(k_fi_jump, dim3(1), dim3(FI_JUMP_THREADS), 0, s, m, rounds, par[0], sta[0], thr[0]);
  const int cur = 0;
  LAUNCH(k_fi_gap, dim3(grid_for(64ULL * m)), dim3(BLOCK), 0, s, m, K, dk, bmin, smin, sta[cur], thr[cur], gk[0],
         gv[0]);
  LAUNCH(k_fi_setn, dim3(1), dim3(1), 0, s, nm, m);
  uint32_t bits = 8;
  while (bits < 32 && (static_cast<uint64_t>(K) >> bits) != 0) bits += 8;
  uint32_t *sk = nullptr, *sv = nullptr;
  if ((r = radix_sort_pairs(gk[0], gv[0], gk[1], gv[1], nm, m, bits, ws, s, &sk, &sv))) return r;
  LAUNCH(k_fi_pos, dim3(grid_for(m)), dim3(BLOCK), 0, s, m, sv, pos);
  LAUNCH(k_fi_gstart, dim3(grid_for(m)), dim3(BLOCK), 0, s, m, sk, glist, fi + 2);
  LAUNCH(k_fi_gaps, dim3(m), dim3(64), 0, s, m, glist, fi + 2, sk, sv, par0, pos, o.ts, nxt, ord, first, fi);
  uint32_t hf[4];
  HIP_CHECK(hipMemcpyAsync(hf, fi, sizeof(hf), hipMemcpyDeviceToHost, s));
  if (int rw = stream_wait(s)) return rw;
  const long long new_ts = t->timestamp + hf[1];
  if (hf[0] || replica_of(new_ts) != replica_of(t->timestamp)) {
    ws.used = mark0;  // the general paths decide (the key index stays valid: the state is untouched)
    return CRDTM_OK;
  }
  // ---- phase C: commit ----
  TreeCaps need = t->cap;
  need.slots = std::max<uint64_t>(need.slots, t->n_slots + m + 1);
  need.log = std::max<uint64_t>(need.log, t->log_n + m + 1);
  need.lpath = std::max<uint64_t>(need.lpath, t->log_npath + m + 1);
  need.doc = std::max<uint64_t>(need.doc, K64 + m + 1);
  if (need.slots > t->cap.slots || need.log > t->cap.log || need.lpath > t->cap.lpath || need.doc > t->cap.doc)
    if ((r = grow_tree(t, need))) return r;
  if (X.doc2_cap < t->cap.doc) {  // the next order's buffer matches the tree's doc capacity
    if (X.doc2) hipFree(X.doc2);
    X.doc2 = nullptr;
    HIP_CHECK(hipMalloc(&X.doc2, t->cap.doc * sizeof(uint32_t)));
    X.doc2_cap = t->cap.doc;
  }
  uint32_t* newdoc = X.doc2;
  const uint32_t slot0 = static_cast<uint32_t>(t->n_slots);
  LAUNCH(k_fi_doc, dim3(grid_for(K64 + m)), dim3(BLOCK), 0, s, K, m, t->d.doc, sk, sv, ord, first, slot0, o.ts,
         dk, newdoc, newrank, X.dk[X.cur ^ 1], rank_of);
  X.cur ^= 1;
  LAUNCH(k_fi_next, dim3(grid_for(m)), dim3(BLOCK), 0, s, K, m, sv, ord, newrank, newdoc, slot0, t->d.s_next);
  // the new order becomes the tree's (the store owns whichever buffer `doc` holds)
  std::swap(t->d.doc, X.doc2);
  std::swap(t->cap.doc, X.doc2_cap);
  t->store->d.doc = t->d.doc;
  LAUNCH(k_fi_commit, dim3(grid_for(m)), dim3(BLOCK), 0, s, o, slot0, static_cast<uint32_t>(t->log_n),
         static_cast<uint32_t>(t->log_npath), t->d);
  LAUNCH(k_kx_insert, dim3(grid_for(m)), dim3(BLOCK), 0, s, o, slot0, kx);
  HIP_CHECK(hipMemsetAsync(st, ST_APPLIED, m, s));
  if ((r = replica_fold(c, o, st, rep, ws, s))) return r;
  if (st_out) HIP_CHECK(hipMemsetAsync(st_out, CRDTM_ST_APPLIED, m, s));
  if ((r = sync_read(c))) return r;
  if ((r = take_replicas(t, rep))) return r;
  t->n_slots += m;
  t->doc_n += m;
  t->last_begin = t->log_n;
  t->log_n += m;
  t->log_npath += m;
  t->last_end = t->log_n;
  t->timestamp = new_ts;
  t->flat_clean = true;
  res->path_taken = CRDTM_PATH_CLOSED_FORM;
  res->flags |= CRDTM_FLAG_INCREMENTAL;
  res->n_applied = m;
  res->n_already = 0;
  *handled = true;
  return CRDTM_OK;
}

}  // namespace crdtm

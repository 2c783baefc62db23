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
//
// The base order lives in a gapped array (KeyIndex, engine.h): blocks of
// FI_CAP positions, built a quarter full, padding keyed +inf so the NSR searches
// run over it unchanged. A batch rewrites only the blocks its gaps fall in
// (O(batch) positions, not O(document)); a block that would overflow makes
// that batch merge densely (O(document)) and rebuild the blocks with fresh
// slack. The tree's dense `doc` is written from the blocks when read
// (linearize -> fi_materialize).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "engine.h"
#include "kernels.h"

namespace crdtm {

constexpr uint32_t FI_BLK = 64;             // positions per minimum (one wave)
constexpr uint32_t FI_SUP = 64;             // minima per superblock minimum
constexpr uint32_t FI_CAP = 256;            // positions per block of the gapped order
constexpr uint32_t FI_FILL = 64;            // entries per block when (re)built
constexpr uint32_t FI_MAX_BATCH = 1u << 14; // larger batches re-merge (k_fi_jump holds 16 per thread)
constexpr uint32_t FI_GAP_STEPS = 1u << 22; // walk budget per gap (else re-merge)
constexpr long long FI_INF = 0x7fffffffffffffffLL;
constexpr uint32_t FI_BPB = FI_CAP / FI_BLK;  // minima per block (one per wave of k_fi_rewrite)
static_assert(FI_CAP % FI_BLK == 0 && FI_CAP <= 1024, "whole waves per block");

constexpr uint32_t FI_WIN_MAX = 6;          // rebalance windows of up to 2^6 blocks
constexpr uint32_t FI_WIN_ENT = (FI_CAP << FI_WIN_MAX) / 2;  // entries of the largest window (half full)
constexpr uint32_t FI_WIN_THREADS = 1024;

// flags word bits (fi[0]); FI_OVER alone: no window takes a block's batch,
// merge densely. fi[1] own-replica Adds, fi[2] gaps, fi[3] blocks landed in,
// fi[4] overflowing blocks, fi[5] rebalance windows, fi[6] the commit gate
// (fi_gate, run by k_fi_win_list's last workgroup: FG_NONE = the general
// paths decide, nothing is written;
// FG_SPARSE = the blocks the batch lands in are rewritten; FG_DENSE = the
// batch's nodes and log are committed, the order is merged densely by the
// host after the result read), fi[7] k_fi_win_list's workgroups done
// (FI_TOUR: some gap was ordered by its Euler tour -- reported, decides nothing)
enum : uint32_t { FI_FAIL = 1u, FI_BUDGET = 2u, FI_OVER = 4u, FI_REPLICA = 8u, FI_TOUR = 16u };
enum : uint32_t { FG_NONE = 0u, FG_SPARSE = 1u, FG_DENSE = 2u };
constexpr uint32_t FI_COMMIT_GRID = 1024;  // (grid-stride commit kernels: sized before the counts are known)
constexpr uint32_t FI_WORDS = 8;

KeyIndex::~KeyIndex() {
  for (void* q : {static_cast<void*>(keys), static_cast<void*>(vals), static_cast<void*>(bent),
                  static_cast<void*>(bdk), static_cast<void*>(bcnt), static_cast<void*>(bend),
                  static_cast<void*>(bfirst), static_cast<void*>(bwin), static_cast<void*>(bmin),
                  static_cast<void*>(smin), static_cast<void*>(tmin), static_cast<void*>(rank),
                  static_cast<void*>(doc2)})
    if (q) hipFree(q);
}

// key -> slot over every node of a flat tree (slots 1..n_slots-1 of the root dict)
__global__ void __launch_bounds__(BLOCK) k_kx_build(const long long* s_key, uint32_t n_slots, TsHash h) {
  GRID_STRIDE(q, n_slots) {
    if (q == 0) continue;
    tshash_insert(h, s_key[q], q);
  }
}


// the gapped order from a dense one: block b holds ranks [FI_FILL b, FI_FILL b + FI_FILL)
__global__ void __launch_bounds__(BLOCK) k_fi_build(uint32_t K, uint32_t nbk, const uint32_t* doc,
                                                    const long long* s_key, uint32_t* bent, long long* bdk,
                                                    uint32_t* bcnt, uint32_t* bfirst, uint32_t* bend,
                                                    uint32_t* bwin, uint32_t* rank_of) {
  GRID_STRIDE(p, nbk * FI_CAP) {
    const uint32_t b = p / FI_CAP, j = p % FI_CAP, r = b * FI_FILL + j;
    if (j < FI_FILL && r < K) {
      const uint32_t sl = doc[r];
      bent[p] = sl;
      bdk[p] = s_key[sl];
      rank_of[sl] = p;
    } else {
      bent[p] = NONE;
      bdk[p] = FI_INF;
    }
    if (j == 0) {
      bcnt[b] = min(FI_FILL, K - b * FI_FILL);
      bfirst[b] = 0;
      bend[b] = 0;
      bwin[b] = 0;
    }
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

// the top level: the smallest key per FI_SUP superblocks (262,144 positions),
// so a search that runs far (a small threshold) crosses the document in a
// few steps instead of one superblock row of 64 per step
__global__ void __launch_bounds__(BLOCK) k_fi_top(uint32_t ns, const long long* smin, long long* tmin) {
  const uint32_t nt = (ns + FI_SUP - 1) / FI_SUP;
  GRID_STRIDE(t, nt) {
    long long m = FI_INF;
    const uint32_t e = min(ns, (t + 1) * FI_SUP);
    for (uint32_t q = t * FI_SUP; q < e; ++q) m = min(m, smin[q]);
    tmin[t] = m;
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

__device__ __forceinline__ long long wave_min64(long long k) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor(static_cast<uint32_t>(k), o, 64);
    const uint32_t hi = __shfl_xor(static_cast<uint32_t>(static_cast<unsigned long long>(k) >> 32), o, 64);
    const long long v = static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo);
    k = v < k ? v : k;
  }
  return k;
}

// the batch key table, the statuses (not applied: a gated commit that does
// not run leaves nothing for the replicas fold) and the flags words cleared
// (one launch)
__global__ void __launch_bounds__(BLOCK) k_fi_clear(unsigned long long* keys, uint32_t cap, uint32_t* fi, uint8_t* st,
                                                    uint32_t m, DevResult* dres) {
  GRID_STRIDE(q, cap) {
    keys[q] = 0;
    if (q < m) st[q] = ST_PENDING;
  }
  if (blockIdx.x == 0 && threadIdx.x < FI_WORDS) fi[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // (the replicas fold's counters, for the commit's fold)
    dres->n_replica_out = 0;
    dres->n_rep_list = 0;
  }
}

// The commit gate, decided on the device so that the commit is queued
// without a host round trip: the batch falls to the general paths when an
// op does not take the closed form, a gap's walk ran out of budget, or the
// own-replica Adds would carry the timestamp into the next replica id
// (incrementTimestamp, src/CRDTree.elm:337-343); it merges densely when a
// block overflows with no window to take it (or no LDS for the windows).
// The flags words go to the result block, read back once at the end.
// (run by the workgroup of k_fi_win_list that finishes last: the flags words
// are read at agent scope, every other workgroup's atomics being done)
__device__ void fi_gate(uint32_t* fi, long long ts0, uint32_t win_lds, DevResult* dres) {
  uint32_t v[FI_WORDS];
#pragma unroll
  for (uint32_t k = 0; k < FI_WORDS; ++k) v[k] = __hip_atomic_load(&fi[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t f = v[0];
  if (replica_of(ts0 + v[1]) != replica_of(ts0)) f |= FI_REPLICA;
  if (v[5] && !win_lds) f |= FI_OVER;
  v[0] = f;
  v[6] = (f & (FI_FAIL | FI_BUDGET | FI_REPLICA)) ? FG_NONE : (f & FI_OVER) ? FG_DENSE : FG_SPARSE;
  fi[0] = v[0];
  fi[6] = v[6];
#pragma unroll
  for (uint32_t k = 0; k < FI_WORDS; ++k) dres->fincr[k] = v[k];
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
    // (the three probes' first slots load together: the key's in the base,
    // the anchor's in the base and in the batch)
    const long long a = o.path[b];
    const bool ka = a > 0 && a < TWO53;
    const unsigned long long hk = static_cast<unsigned long long>(ts) ^ 0x8000000000000000ULL;
    const unsigned long long ha = static_cast<unsigned long long>(a) ^ 0x8000000000000000ULL;
    const uint32_t p1 = static_cast<uint32_t>(mix64(hk)) & kx.mask;
    const uint32_t p2 = static_cast<uint32_t>(mix64(ha)) & kx.mask;
    const uint32_t p3 = static_cast<uint32_t>(mix64(ha)) & bh.mask;
    const unsigned long long f1 = kx.keys[p1], f2 = ka ? kx.keys[p2] : 0ULL, f3 = ka ? bh.keys[p3] : 0ULL;
    if (o.kind[i] != CRDTM_ADD || o.off[i + 1] != b + 1 || ts <= 0 || ts >= TWO53 ||
        tshash_find_from(kx, hk, p1, f1) != NONE) {
      fail = 1;
    } else {
      if (a != 0) {
        const uint32_t sl = ka ? tshash_find_from(kx, ha, p2, f2) : NONE;
        if (sl != NONE) {
          s = rank_of[sl] + 1;
        } else {
          const uint32_t j = ka ? tshash_find_from(bh, ha, p3, f3) : NONE;
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

// Pointer jumping, all rounds in one workgroup, in LDS: each op's pointer
// to its farthest known new ancestor (u16) and the op of the smallest
// timestamp on the chain up to it (u16, the timestamp itself kept in
// registers for the thread's own ops). A pointer stops at the chain's root
// (the op whose anchor is a base node); the rounds stop once none moved.
// Then (start, threshold) = (the root's start, min(chain min, root's ts)).
constexpr uint32_t FI_JUMP_THREADS = 1024, FI_JUMP_PER = 16;
constexpr uint16_t FI_J_NONE = 0xFFFFu;
static_assert(FI_JUMP_THREADS * FI_JUMP_PER >= FI_MAX_BATCH && FI_MAX_BATCH <= FI_J_NONE, "u16 op indices");
__global__ void __launch_bounds__(FI_JUMP_THREADS) k_fi_jump(uint32_t m, uint32_t rounds, const uint32_t* P,
                                                             uint32_t* S, long long* T, const long long* ts) {
  __shared__ uint16_t lp[FI_JUMP_THREADS * FI_JUMP_PER], lt[FI_JUMP_THREADS * FI_JUMP_PER];
  uint16_t mp[FI_JUMP_PER], mt[FI_JUMP_PER];
  long long mv[FI_JUMP_PER];
#pragma unroll
  for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
    const uint32_t i = threadIdx.x + u * FI_JUMP_THREADS;
    const uint32_t p = i < m ? P[i] : NONE;
    mp[u] = p == NONE ? FI_J_NONE : static_cast<uint16_t>(p);
    mt[u] = static_cast<uint16_t>(i);
    mv[u] = i < m ? T[i] : 0;
    lp[i] = mp[u];
    lt[i] = mt[u];
  }
  __syncthreads();
  for (uint32_t k = 0; k < rounds; ++k) {
    int moved = 0;
#pragma unroll
    for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
      const uint16_t p = mp[u];
      if (p != FI_J_NONE) {
        const uint16_t pp = lp[p];
        if (pp != FI_J_NONE) {  // T over [i, p) composed with T over [p, pp)
          const uint16_t tq = lt[p];
          const long long tv = ts[tq];
          if (tv < mv[u]) {
            mv[u] = tv;
            mt[u] = tq;
          }
          mp[u] = pp;
          moved = 1;
        }
      }
    }
    __syncthreads();  // every read of this round before any write
#pragma unroll
    for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
      const uint32_t i = threadIdx.x + u * FI_JUMP_THREADS;
      lp[i] = mp[u];
      lt[i] = mt[u];
    }
    if (!__syncthreads_or(moved)) break;
  }
#pragma unroll
  for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
    const uint32_t i = threadIdx.x + u * FI_JUMP_THREADS;
    const uint16_t r = mp[u];
    if (i < m && r != FI_J_NONE) {
      S[i] = S[r];  // (a root's own start: roots are not written)
      T[i] = min(mv[u], ts[r]);
    }
  }
}

// The same with the thresholds themselves in LDS (8 + 2 bytes per op: m <=
// FI_JUMP_LDS_MAX): no global gather in the rounds.
constexpr uint32_t FI_JUMP_LDS_MAX = 16000;
__global__ void __launch_bounds__(FI_JUMP_THREADS) k_fi_jump_lds(uint32_t m, uint32_t rounds, const uint32_t* P,
                                                                 uint32_t* S, long long* T) {
  extern __shared__ unsigned long long fi_jump_lds[];
  long long* lt = reinterpret_cast<long long*>(fi_jump_lds);  // [m] threshold over [i, pointer)
  uint16_t* lp = reinterpret_cast<uint16_t*>(lt + m);         // [m] pointer
  uint16_t mp[FI_JUMP_PER];
  long long mv[FI_JUMP_PER];
#pragma unroll
  for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
    const uint32_t i = threadIdx.x + u * FI_JUMP_THREADS;
    const uint32_t p = i < m ? P[i] : NONE;
    mp[u] = p == NONE ? FI_J_NONE : static_cast<uint16_t>(p);
    mv[u] = i < m ? T[i] : 0;
    if (i < m) {
      lp[i] = mp[u];
      lt[i] = mv[u];
    }
  }
  __syncthreads();
  for (uint32_t k = 0; k < rounds; ++k) {
    int moved = 0;
#pragma unroll
    for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
      const uint16_t p = mp[u];
      if (p != FI_J_NONE) {
        const uint16_t pp = lp[p];
        if (pp != FI_J_NONE) {
          mv[u] = min(mv[u], lt[p]);
          mp[u] = pp;
          moved = 1;
        }
      }
    }
    __syncthreads();  // every read of this round before any write
#pragma unroll
    for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
      const uint32_t i = threadIdx.x + u * FI_JUMP_THREADS;
      if (i < m) {
        lp[i] = mp[u];
        lt[i] = mv[u];
      }
    }
    if (!__syncthreads_or(moved)) break;
  }
#pragma unroll
  for (uint32_t u = 0; u < FI_JUMP_PER; ++u) {
    const uint32_t i = threadIdx.x + u * FI_JUMP_THREADS;
    const uint16_t r = mp[u];
    if (i < m && r != FI_J_NONE) {
      S[i] = S[r];  // (a root's own start: roots are not written)
      T[i] = min(mv[u], lt[r]);  // (a root's threshold is its own timestamp)
    }
  }
}

// The same over many workgroups (anchors are earlier ops:
// par[i] < i). Each chunk of FI_JC ops jumps in LDS along the pointers that
// stay inside it; an op whose chain ends at a root of its chunk is final
// there, one whose chain leaves the chunk (at e, whose anchor is an earlier
// chunk's op) keeps jx = par[e] and jm = the chain's minimum up to e. Then
// each such op follows jx from chunk to chunk (at most one hop per earlier
// chunk) to a final op: its start, and the minimum over the hops — done by
// k_fi_gap's wave for the op before its search.
constexpr uint32_t FI_JC = 1024;
__global__ void __launch_bounds__(FI_JC) k_fi_jump_chunk(uint32_t m, const uint32_t* P, uint32_t* S, long long* T,
                                                         uint32_t* jx, long long* jm) {
  __shared__ long long lt[FI_JC];
  __shared__ uint16_t lp[FI_JC];
  const uint32_t c0 = blockIdx.x * FI_JC, j = threadIdx.x, i = c0 + j;
  const uint32_t n = min(FI_JC, m - c0);
  const uint32_t p = i < m ? P[i] : NONE;
  // local pointer: the anchor inside the chunk, else a stop (root or exit)
  uint16_t mp = (p != NONE && p >= c0) ? static_cast<uint16_t>(p - c0) : FI_J_NONE;
  long long mv = i < m ? T[i] : 0;
  if (j < n) {
    lp[j] = mp;
    lt[j] = mv;
  }
  const uint16_t first = mp;
  __syncthreads();
  for (;;) {
    int moved = 0;
    uint16_t np = mp;
    long long nv = mv;
    if (j < n && mp != FI_J_NONE) {
      const uint16_t pp = lp[mp];
      if (pp != FI_J_NONE) {
        nv = min(mv, lt[mp]);
        np = pp;
        moved = 1;
      }
    }
    __syncthreads();  // every read of this round before any write
    mp = np;
    mv = nv;
    if (j < n) {
      lp[j] = mp;
      lt[j] = mv;
    }
    if (!__syncthreads_or(moved)) break;
  }
  if (j >= n) return;
  if (first == FI_J_NONE) {  // a root, or an op whose anchor is an earlier chunk's
    jx[i] = p;
    jm[i] = mv;
    return;
  }
  const uint32_t e = c0 + mp;                  // the chain's last op in the chunk
  const long long mm = min(mv, lt[mp]);        // (e never moved: lt = its own threshold)
  const uint32_t pe = P[e];
  if (pe == NONE) {  // final here
    S[i] = S[e];
    T[i] = mm;
    jx[i] = NONE;
  } else {
    jx[i] = pe;
  }
  jm[i] = mm;
}

// (jx: the chunked pointer jumping's hops first, k_fi_jump_fix's work for
// this op, so it needs no launch of its own)
__global__ void __launch_bounds__(BLOCK) k_fi_gap(uint32_t m, uint32_t K, const long long* dk, const long long* bmin,
                                                  const long long* smin, const long long* tmin, uint32_t* start,
                                                  long long* thr, uint32_t* gkey, uint32_t* gval, const uint32_t* jx,
                                                  const long long* jm) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nb = (K + FI_BLK - 1) / FI_BLK, ns = (nb + FI_SUP - 1) / FI_SUP, nt = (ns + FI_SUP - 1) / FI_SUP;
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  if (i >= m) return;  // (wave-uniform)
  long long t;
  uint32_t r;
  uint32_t x = jx ? jx[i] : NONE;
  if (x != NONE) {  // (hops to a final op: an earlier chunk's per hop)
    t = jm[i];
    for (;;) {
      t = min(t, jm[x]);
      const uint32_t y = jx[x];
      if (y == NONE) break;
      x = y;
    }
    r = start[x];
    if (lane == 0) {
      start[i] = r;
      thr[i] = t;
    }
  } else {
    t = thr[i];
    r = start[i];
  }
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
      if (bb == NONE && s0 + 1 < ns) {
        // the rest of the top entry that holds superblock s0 + 1, then the
        // top level 64 entries per step, then down one superblock row
        const uint32_t t0 = (s0 + 1) / FI_SUP;
        uint32_t sq = first64(smin, t0 * FI_SUP, s0 + 1, ns);
        for (uint32_t tt = t0 + 1; sq == NONE && tt < nt; tt += 64) {
          const uint32_t tq = first64(tmin, tt, tt, nt);
          if (tq != NONE) sq = first64(smin, tq * FI_SUP, tq * FI_SUP, ns);
        }
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


// block of a gap position (Kp = past the end: the last block)
__device__ __forceinline__ uint32_t fi_blk(uint32_t g, uint32_t Kp) { return (g < Kp ? g : Kp - 1) / FI_CAP; }

// blocks the batch lands in: the first sorted position of each, listed (any
// order) in tl / fi[3], with their sorted range [bfirst, bend) per block; and
// the entry before each gap's first new node, from the layout before the
// batch (gpred: a base entry, since gaps are separated by their base nodes)
__global__ void __launch_bounds__(BLOCK) k_fi_tblk(uint32_t m, uint32_t nbk, const uint32_t* sk, const uint32_t* ord,
                                                   const uint32_t* bent, const uint32_t* bcnt, uint32_t* bfirst,
                                                   uint32_t* bend, uint32_t* tl, uint32_t* gpred, uint32_t* fi) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x, Kp = nbk * FI_CAP;
  uint32_t b = 0;
  bool head = false;
  if (k < m) {
    const uint32_t g = sk[k];
    b = fi_blk(g, Kp);
    head = k == 0 || fi_blk(sk[k - 1], Kp) != b;
    if (head) bfirst[b] = k;
    if (k + 1 == m || fi_blk(sk[k + 1], Kp) != b) bend[b] = k + 1;
    if (ord[k] == 0) {
      uint32_t pr;
      if (g >= Kp) pr = bent[(nbk - 1) * FI_CAP + bcnt[nbk - 1] - 1];
      else if (g % FI_CAP) pr = bent[g - 1];
      else pr = b ? bent[(b - 1) * FI_CAP + bcnt[b - 1] - 1] : 0u;
      gpred[k] = pr;
    }
  }
  const uint32_t t = wave_ticket(&fi[3], head);
  if (head) tl[t] = k;
}

// Rebalance windows (packed-memory array): for each block the batch would
// overflow (one wave per block it lands in), the smallest aligned window of
// 2^l blocks (l = 1..FI_WIN_MAX, clipped at the end) whose entries + new nodes
// fill at most half of it; every block of the window takes level l + 1 (the
// largest over windows: aligned windows nest), the block goes to ovl / fi[4].
// None: FI_OVER (the batch merges densely).
__global__ void __launch_bounds__(BLOCK) k_fi_win_pick(uint32_t nbk, const uint32_t* sk, const uint32_t* tl,
                                                       const uint32_t* bcnt, const uint32_t* bfirst,
                                                       const uint32_t* bend, uint32_t* bwin, uint32_t* ovl,
                                                       uint32_t* fi) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
  if (w >= fi[3]) return;  // (wave-uniform)
  const uint32_t b = fi_blk(sk[tl[w]], nbk * FI_CAP);
  if (bcnt[b] + bend[b] - bfirst[b] <= FI_CAP) return;
  if (lane == 0) ovl[atomicAdd(&fi[4], 1u)] = b;
  for (uint32_t l = 1; l <= FI_WIN_MAX; ++l) {
    const uint32_t n = 1u << l, w0 = b & ~(n - 1), ne = min(n, nbk - w0);
    uint32_t v = lane < ne ? bcnt[w0 + lane] + bend[w0 + lane] - bfirst[w0 + lane] : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (2 * v <= ne * FI_CAP) {
      if (lane < ne) atomicMax(&bwin[w0 + lane], l + 1);
      return;
    }
  }
  if (lane == 0) atomicOr(&fi[0], FI_OVER);
}

// the windows that act (one per maximal window: the first overflowing block
// of it to flag its leader lists it) in wl / fi[5]
constexpr uint32_t FI_WIN_LISTED = 0x80u;
__global__ void __launch_bounds__(BLOCK) k_fi_win_list(const uint32_t* ovl, uint32_t* fi, uint32_t* bwin,
                                                       uint32_t* wl, uint32_t* wlev, long long ts0, uint32_t win_lds,
                                                       DevResult* dres) {
  __shared__ bool last;
  GRID_STRIDE(w, fi[4]) {
    const uint32_t b = ovl[w], L = bwin[b] & ~FI_WIN_LISTED;
    const uint32_t w0 = b & ~((1u << (L - 1)) - 1u);
    if (atomicCAS(&bwin[w0], L, L | FI_WIN_LISTED) == L) {
      const uint32_t u = atomicAdd(&fi[5], 1u);
      wl[u] = w0;
      wlev[u] = L;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(&fi[7], 1u) == gridDim.x - 1;  // (fi[7]: workgroups done)
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {  // the commit gate
    __threadfence();
    fi_gate(fi, ts0, win_lds, dres);
  }
}

// One workgroup per block the batch lands in, outside every window: the
// block's entries and its new nodes merged in LDS, then written back in
// place. A base entry moves right by the new nodes whose gap is at or before
// it; a new node sits at its gap + the new nodes of earlier gaps in the block
// + its order in its gap. Moved and new entries get their position in
// rank_of, the new nodes their next links (and the entry before each gap
// its new first); the block's minima are recomputed.
__device__ __forceinline__ void fi_rewrite_one(uint32_t nbk, uint32_t k, const uint32_t* sk, const uint32_t* sv,
                                               const uint32_t* ord, const uint32_t* first, const uint32_t* gpred,
                                               uint32_t slot0, const long long* ts, uint32_t* bent, long long* bdk,
                                               uint32_t* bcnt, uint32_t* bfirst, uint32_t* bend, const uint32_t* bwin,
                                               long long* bmin, uint32_t* rank_of, uint32_t* s_next, uint32_t* se,
                                               long long* sd) {
  const uint32_t Kp = nbk * FI_CAP, j = threadIdx.x;
  const uint32_t b = fi_blk(sk[k], Kp), base = b * FI_CAP;
  if (bwin[b]) return;  // a window rebalances it
  const uint32_t e = bend[b], cnt = bcnt[b];
  if (j < cnt) {
    const uint32_t pos = base + j;
    uint32_t lo = k, hi = e;  // new nodes with gap <= pos
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (sk[mid] <= pos) lo = mid + 1;
      else hi = mid;
    }
    const uint32_t nj = j + (lo - k), sl = bent[pos];
    se[nj] = sl;
    sd[nj] = bdk[pos];
    if (nj != j) rank_of[sl] = base + nj;
  }
  for (uint32_t q = k + j; q < e; q += FI_CAP) {
    const uint32_t g = sk[q];
    const uint32_t nj = (g >= Kp ? cnt : g - base) + (first[q] - k) + ord[q];
    const uint32_t op = sv[q];
    se[nj] = slot0 + op;
    sd[nj] = ts[op];
    rank_of[slot0 + op] = base + nj;
  }
  __syncthreads();
  const uint32_t c2 = cnt + (e - k);
  // next links: a new node's successor is the next entry of its block (its
  // gap's base node follows it; past the end only at the document's end)
  for (uint32_t q = k + j; q < e; q += FI_CAP) {
    const uint32_t g = sk[q];
    const uint32_t nj = (g >= Kp ? cnt : g - base) + (first[q] - k) + ord[q], sl = slot0 + sv[q];
    s_next[sl] = nj + 1 < c2 ? se[nj + 1] : NONE;
    if (ord[q] == 0) s_next[gpred[q]] = sl;
  }
  long long v = FI_INF;
  if (j < c2) {
    bent[base + j] = se[j];
    v = sd[j];
    bdk[base + j] = v;
  }
  v = wave_min64(v);
  if ((j & 63) == 0) bmin[FI_BPB * b + (j >> 6)] = v;
  if (j == 0) {
    bcnt[b] = c2;
    bfirst[b] = 0;
    bend[b] = 0;
  }
}

__global__ void __launch_bounds__(FI_CAP) k_fi_rewrite(uint32_t nbk, const uint32_t* tl, const uint32_t* fi,
                                                       const uint32_t* sk, const uint32_t* sv, const uint32_t* ord,
                                                       const uint32_t* first, const uint32_t* gpred, uint32_t slot0,
                                                       const long long* ts, uint32_t* bent, long long* bdk,
                                                       uint32_t* bcnt, uint32_t* bfirst, uint32_t* bend,
                                                       const uint32_t* bwin, long long* bmin, uint32_t* rank_of,
                                                       uint32_t* s_next) {
  __shared__ uint32_t se[FI_CAP];
  __shared__ long long sd[FI_CAP];
  if (fi[6] != FG_SPARSE) return;  // (grid-uniform: the gate)
  for (uint32_t wb = blockIdx.x; wb < fi[3]; wb += gridDim.x) {  // (workgroup-uniform)
    fi_rewrite_one(nbk, tl[wb], sk, sv, ord, first, gpred, slot0, ts, bent, bdk, bcnt, bfirst, bend, bwin, bmin,
                   rank_of, s_next, se, sd);
    __syncthreads();  // (the next block reuses the LDS)
  }
}

// One workgroup per rebalance window [w0, w0 + ne): every block's merged
// content (as in k_fi_rewrite) staged in LDS in window order, then spread
// evenly over the window's blocks (each keeps >= 1 entry: every block had
// one), padding cleared, minima recomputed, next links of the new nodes set,
// the window's marks cleared.
__global__ void __launch_bounds__(FI_WIN_THREADS) k_fi_win(uint32_t nbk, const uint32_t* wl, const uint32_t* wlev,
                                                           const uint32_t* fi, const uint32_t* sk, const uint32_t* sv,
                                                           const uint32_t* ord, const uint32_t* first,
                                                           const uint32_t* gpred, uint32_t slot0, const long long* ts,
                                                           uint32_t* bent, long long* bdk, uint32_t* bcnt,
                                                           uint32_t* bfirst, uint32_t* bend, uint32_t* bwin,
                                                           long long* bmin, uint32_t* rank_of, uint32_t* s_next) {
  extern __shared__ unsigned long long fi_win_lds[];
  long long* sd = reinterpret_cast<long long*>(fi_win_lds);     // [FI_WIN_ENT]
  uint32_t* se = reinterpret_cast<uint32_t*>(sd + FI_WIN_ENT);  // [FI_WIN_ENT]
  __shared__ uint32_t vp[(1u << FI_WIN_MAX) + 1];  // window-order start of each block's content
  if (fi[6] != FG_SPARSE) return;  // (grid-uniform: the gate)
  for (uint32_t wi = blockIdx.x; wi < fi[5]; wi += gridDim.x) {  // (workgroup-uniform)
  const uint32_t Kp = nbk * FI_CAP, w0 = wl[wi], L = wlev[wi];
  const uint32_t ne = min(1u << (L - 1), nbk - w0);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = FI_WIN_THREADS / 64;
  if (tid < 64) {
    const uint32_t v = tid < ne ? bcnt[w0 + tid] + bend[w0 + tid] - bfirst[w0 + tid] : 0u;
    const uint32_t inc = wave_incl_scan(v);
    vp[tid] = inc - v;
    if (tid == 63) vp[64] = inc;
  }
  __syncthreads();
  const uint32_t T = vp[64];
  // stage: one wave per block of the window
  for (uint32_t i = wv; i < ne; i += nw) {
    const uint32_t b = w0 + i, base = b * FI_CAP, cnt = bcnt[b], k = bfirst[b], e = bend[b], v0 = vp[i];
    for (uint32_t j = lane; j < cnt; j += 64) {
      const uint32_t p = base + j;
      uint32_t lo = k, hi = e;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sk[mid] <= p) lo = mid + 1;
        else hi = mid;
      }
      se[v0 + j + (lo - k)] = bent[p];
      sd[v0 + j + (lo - k)] = bdk[p];
    }
    for (uint32_t q = k + lane; q < e; q += 64) {
      const uint32_t g = sk[q];
      const uint32_t nj = (g >= Kp ? cnt : g - base) + (first[q] - k) + ord[q];
      const uint32_t op = sv[q];
      se[v0 + nj] = slot0 + op;
      sd[v0 + nj] = ts[op];
    }
  }
  __syncthreads();
  // next links of the new nodes (their successor is in the window: see k_fi_rewrite)
  for (uint32_t i = wv; i < ne; i += nw) {
    const uint32_t b = w0 + i, base = b * FI_CAP, cnt = bcnt[b], k = bfirst[b], e = bend[b], v0 = vp[i];
    for (uint32_t q = k + lane; q < e; q += 64) {
      const uint32_t g = sk[q];
      const uint32_t v = v0 + (g >= Kp ? cnt : g - base) + (first[q] - k) + ord[q], sl = slot0 + sv[q];
      s_next[sl] = v + 1 < T ? se[v + 1] : NONE;
      if (ord[q] == 0) s_next[gpred[q]] = sl;
    }
  }
  // spread: block i of the window takes qn (+1 for the first rm) entries
  const uint32_t qn = T / ne, rm = T % ne;
  auto vstart = [&](uint32_t i) -> uint32_t { return i * qn + min(i, rm); };
  for (uint32_t x = tid; x < ne * FI_CAP; x += FI_WIN_THREADS) {
    const uint32_t i = x / FI_CAP, j = x % FI_CAP, c = qn + (i < rm ? 1u : 0u), p = (w0 + i) * FI_CAP + j;
    if (j < c) {
      const uint32_t v = vstart(i) + j, sl = se[v];
      bent[p] = sl;
      bdk[p] = sd[v];
      rank_of[sl] = p;
    } else {
      bent[p] = NONE;
      bdk[p] = FI_INF;
    }
  }
  // minima per 64 positions (one wave each, from the stage)
  for (uint32_t gq = wv; gq < ne * FI_BPB; gq += nw) {
    const uint32_t i = gq / FI_BPB, c = qn + (i < rm ? 1u : 0u), j = (gq % FI_BPB) * 64 + lane;
    const long long v = wave_min64(j < c ? sd[vstart(i) + j] : FI_INF);
    if (lane == 0) bmin[FI_BPB * w0 + gq] = v;
  }
  __syncthreads();  // (every wave has read bfirst / bend)
  for (uint32_t i = tid; i < ne; i += FI_WIN_THREADS) {
    bcnt[w0 + i] = qn + (i < rm ? 1u : 0u);
    bfirst[w0 + i] = 0;
    bend[w0 + i] = 0;
    bwin[w0 + i] = 0;
  }
  __syncthreads();  // (the next window reuses the LDS)
  }
}

// superblock minima over the rewritten blocks' superblocks (one wave each;
// blocks of one superblock write the same value)
__device__ __forceinline__ void fi_sup_one(uint32_t sp, uint32_t nb, const long long* bmin, long long* smin) {
  const uint32_t lane = threadIdx.x & 63, q = sp * FI_SUP + lane;
  const long long v = wave_min64(q < nb ? bmin[q] : FI_INF);
  if (lane == 0) smin[sp] = v;
}
// (one wave per block landed in, then one per window; a superblock both
// touch is recomputed twice from the same final minima)
__global__ void __launch_bounds__(BLOCK) k_fi_sup_fix(uint32_t nbk, const uint32_t* tl, const uint32_t* sk,
                                                      const uint32_t* wl, const uint32_t* wlev, const uint32_t* fi,
                                                      const long long* bmin, long long* smin) {
  if (fi[6] != FG_SPARSE) return;  // (grid-uniform: the gate)
  const uint32_t Kp = nbk * FI_CAP, nw = gridDim.x * blockDim.x / 64, nblk = fi[3], nwin = fi[5];
  for (uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) / 64; w < nblk + nwin; w += nw) {  // (wave-uniform)
    if (w < nblk) {
      fi_sup_one(FI_BPB * fi_blk(sk[tl[w]], Kp) / FI_SUP, Kp / FI_BLK, bmin, smin);
    } else {
      const uint32_t w0 = wl[w - nblk], ne = min(1u << (wlev[w - nblk] - 1), nbk - w0);
      for (uint32_t sp = FI_BPB * w0 / FI_SUP; sp <= (FI_BPB * (w0 + ne) - 1) / FI_SUP; ++sp)
        fi_sup_one(sp, FI_BPB * nbk, bmin, smin);
    }
  }
}

// ... then the top entries over every superblock the blocks and windows
// touched (one wave per block or window; after k_fi_sup_fix)
__device__ __forceinline__ void fi_top_one(uint32_t tp, uint32_t ns, const long long* smin, long long* tmin) {
  const uint32_t lane = threadIdx.x & 63, q = tp * FI_SUP + lane;
  const long long v = wave_min64(q < ns ? smin[q] : FI_INF);
  if (lane == 0) tmin[tp] = v;
}
__global__ void __launch_bounds__(BLOCK) k_fi_top_fix(uint32_t nbk, const uint32_t* tl, const uint32_t* sk,
                                                      const uint32_t* wl, const uint32_t* wlev, const uint32_t* fi,
                                                      const long long* smin, long long* tmin) {
  if (fi[6] != FG_SPARSE) return;  // (grid-uniform: the gate)
  const uint32_t Kp = nbk * FI_CAP, ns = (FI_BPB * nbk + FI_SUP - 1) / FI_SUP;
  const uint32_t nw = gridDim.x * blockDim.x / 64, nblk = fi[3], nwin = fi[5];
  for (uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) / 64; w < nblk + nwin; w += nw) {  // (wave-uniform)
    if (w < nblk) {
      fi_top_one(FI_BPB * fi_blk(sk[tl[w]], Kp) / FI_SUP / FI_SUP, ns, smin, tmin);
    } else {
      const uint32_t w0 = wl[w - nblk], ne = min(1u << (wlev[w - nblk] - 1), nbk - w0);
      for (uint32_t tp = FI_BPB * w0 / FI_SUP / FI_SUP; tp <= (FI_BPB * (w0 + ne) - 1) / FI_SUP / FI_SUP; ++tp)
        fi_top_one(tp, ns, smin, tmin);
    }
  }
}

// the dense order from the gapped one (off = exclusive scan of bcnt)
__global__ void __launch_bounds__(BLOCK) k_fi_compact(uint32_t nbk, const uint32_t* off, const uint32_t* bent,
                                                      const uint32_t* bcnt, uint32_t* doc) {
  GRID_STRIDE(p, nbk * FI_CAP) {
    const uint32_t b = p / FI_CAP, j = p % FI_CAP;
    if (j < bcnt[b]) doc[off[b] + j] = bent[p];
  }
}

// gap positions (sorted) -> dense ranks, for a dense merge (monotone: the
// order stays sorted)
__global__ void __launch_bounds__(BLOCK) k_fi_dense_gaps(uint32_t m, uint32_t Kp, uint32_t K, const uint32_t* off,
                                                         uint32_t* sk) {
  GRID_STRIDE(k, m) {
    const uint32_t g = sk[k];
    sk[k] = g >= Kp ? K : off[g / FI_CAP] + g % FI_CAP;
  }
}

// One wave per gap: the gap's new nodes, in batch order, are inserted into a
// list of their own (RGA with no tombstones: after the anchor when it is in
// this gap, else after the head; past every following node with a larger
// timestamp) by lane 0 on keys and links staged in LDS (a gap larger than
// the LDS stage walks global memory instead); then ord[] = the list order
// and first[] = the gap's first sorted position.
constexpr uint32_t FI_GAP_LDS = 1024;
// (le[j]: j's successor in the gap's list and that successor's key in one
// word, key << 11 | index: a walk step is one LDS read; keys are positive
// timestamps below 2^53)
constexpr uint32_t FI_LE_NONE = 0x7FF;
static_assert(FI_GAP_LDS < FI_LE_NONE, "11-bit list indices");
struct FiGapLds {
  long long lk[FI_GAP_LDS];
  unsigned long long le[FI_GAP_LDS];
  uint32_t la[FI_GAP_LDS], lo[FI_GAP_LDS];
  uint16_t fc[FI_GAP_LDS + 2];  // (the tour: first child per op, the gap's head list at [n])
};
// (an anchor op is in the gap iff its own gap key is the gap's; its place
// there is its rank among the gap's ops, which are in batch order)
__device__ __forceinline__ uint32_t fi_rank_of(const uint32_t* v, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (v[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// A gap whose every anchor inside it has a smaller key than its op (keys
// grow along the anchors, as Lamport timestamps do) is its ops' tree in DFS
// order, children by descending key: the replay's walk from an anchor passes
// exactly the subtrees of the anchor's children with larger keys (their
// descendants' keys are larger still) and stops at the first smaller key,
// which is the next child, or an uncle's, whose key is below the anchor's. So
// the order comes without the serial replay: the children grouped by anchor
// and sorted by key (a bitonic network over (anchor << 53 | ~key) words), an
// Euler tour through them, and the tour ranked by pointer jumping; the rank of
// op v is n - (the enters from v's on). One wave, in LDS (the workgroup is
// the wave: its LDS accesses are in program order). Returns false, having
// written nothing, when some anchor's key is not below its op's.
constexpr uint32_t FI_TOUR_MIN = 24;  // (smaller gaps: the serial replay)
constexpr uint16_t FI_T_NONE = 0xFFFFu;
__device__ bool fi_gap_tour(uint32_t n, FiGapLds& L) {
  const uint32_t lane = threadIdx.x;
  long long* lk = L.lk;
  uint32_t* la = L.la;
  constexpr unsigned long long KM = (1ULL << 53) - 1ULL;
  bool bad = false;
  for (uint32_t j = lane; j < n; j += 64) {
    const uint32_t a = la[j];
    const long long x = lk[j];
    if (x <= 0 || x > static_cast<long long>(KM) || (a != NONE && !(x > lk[a]))) bad = true;
  }
  if (__ballot(bad)) return false;
  // children sorted: (anchor, descending key) words, the op alongside
  unsigned long long* c = L.le;
  uint16_t* sp = reinterpret_cast<uint16_t*>(L.lo);  // [FI_GAP_LDS] sorted ops
  uint16_t* ns = sp + FI_GAP_LDS;                    // [FI_GAP_LDS] next sibling
  uint16_t* fc = L.fc;
  uint32_t N2 = 2;
  while (N2 < n) N2 <<= 1;
  for (uint32_t j = lane; j < N2; j += 64) {
    if (j < n) {
      const uint32_t a = la[j];
      c[j] = (static_cast<unsigned long long>(a == NONE ? 0x7FFu : a) << 53) | (KM - static_cast<unsigned long long>(lk[j]));
      sp[j] = static_cast<uint16_t>(j);
    } else {
      c[j] = ~0ULL;
      sp[j] = FI_T_NONE;
    }
  }
  for (uint32_t k = 2; k <= N2; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      __builtin_amdgcn_wave_barrier();
      for (uint32_t t = lane; t < N2 / 2; t += 64) {
        const uint32_t i = 2 * t - (t & (j - 1)), q = i + j;
        const unsigned long long x = c[i], y = c[q];
        if ((x > y) == !(i & k)) {
          c[i] = y;
          c[q] = x;
          const uint16_t u = sp[i];
          sp[i] = sp[q];
          sp[q] = u;
        }
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  // first child per anchor (the head list at n), next sibling per op
  for (uint32_t v = lane; v <= n; v += 64) fc[v] = FI_T_NONE;
  __builtin_amdgcn_wave_barrier();
  for (uint32_t p = lane; p < n; p += 64) {
    const uint32_t P = static_cast<uint32_t>(c[p] >> 53), u = sp[p];
    const uint32_t Pp = p ? static_cast<uint32_t>(c[p - 1] >> 53) : 0xFFFFFFFFu;
    const uint32_t Pn = p + 1 < n ? static_cast<uint32_t>(c[p + 1] >> 53) : 0xFFFFFFFFu;
    if (Pp != P) fc[P == 0x7FFu ? n : P] = static_cast<uint16_t>(u);
    ns[u] = Pn == P ? sp[p + 1] : FI_T_NONE;
  }
  __builtin_amdgcn_wave_barrier();
  // the tour: enter(v) = v (weight 1), exit(v) = n + v (weight 0)
  uint16_t* tn = reinterpret_cast<uint16_t*>(lk);  // [2 FI_GAP_LDS] successor
  uint16_t* tv = tn + 2 * FI_GAP_LDS;              // [2 FI_GAP_LDS] enters from here to the end
  for (uint32_t v = lane; v < n; v += 64) {
    const uint32_t f = fc[v], s = ns[v], a = la[v];
    tn[v] = static_cast<uint16_t>(f != FI_T_NONE ? f : n + v);
    tv[v] = 1;
    tn[n + v] = static_cast<uint16_t>(s != FI_T_NONE ? s : (a == NONE ? FI_T_NONE : n + a));
    tv[n + v] = 0;
  }
  for (;;) {  // (pointer jumping: every pair is read before any is written)
    bool moved = false;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t x0 = lane; x0 < 2 * n; x0 += 64 * 8) {
      uint32_t y[8], ny[8], vy[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        const uint32_t x = x0 + 64 * u;
        y[u] = x < 2 * n ? tn[x] : FI_T_NONE;
      }
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        ny[u] = y[u] != FI_T_NONE ? tn[y[u]] : FI_T_NONE;
        vy[u] = y[u] != FI_T_NONE ? tv[y[u]] : 0u;
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        const uint32_t x = x0 + 64 * u;
        if (y[u] != FI_T_NONE) {
          tv[x] = static_cast<uint16_t>(tv[x] + vy[u]);
          tn[x] = static_cast<uint16_t>(ny[u]);
          moved = true;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (!__ballot(moved)) break;
  }
  // the order: n - (the enters from v's enter on)
  for (uint32_t v = lane; v < n; v += 64) L.la[v] = n - tv[v];
  return true;
}

__device__ __forceinline__ void fi_gap_one(uint32_t k, uint32_t m, const uint32_t* gk, const uint32_t* gv,
                                           const uint32_t* gk0, const uint32_t* par0, const long long* ts,
                                           uint32_t* nxt, uint32_t* ord, uint32_t* first, uint32_t* fi,
                                           FiGapLds& L) {
  long long* lk = L.lk;
  unsigned long long* le = L.le;
  uint32_t *la = L.la, *lo = L.lo;
  const uint32_t lane = threadIdx.x;
  const uint32_t g = gk[k];
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
    // three dependent gathers (op, its key and anchor, the anchor's gap),
    // each issued for all of the lane's entries at once; the ops staged in
    // LDS (lo, free until the order) for the anchors' ranks
    constexpr uint32_t PER = FI_GAP_LDS / 64;
    uint32_t op[PER], av[PER];
    long long kv[PER];
#pragma unroll
    for (uint32_t u = 0; u < PER; ++u) {
      const uint32_t j = lane + 64 * u;
      op[u] = j < n ? gv[k + j] : 0u;
      if (j < n) lo[j] = op[u];
    }
#pragma unroll
    for (uint32_t u = 0; u < PER; ++u) {
      const bool in = lane + 64 * u < n;
      kv[u] = in ? ts[op[u]] : 0;
      av[u] = in ? par0[op[u]] : NONE;
    }
#pragma unroll
    for (uint32_t u = 0; u < PER; ++u) av[u] = (av[u] != NONE && gk0[av[u]] == g) ? av[u] : NONE;
    __syncthreads();  // (lo staged)
#pragma unroll
    for (uint32_t u = 0; u < PER; ++u) {
      const uint32_t j = lane + 64 * u;
      if (j < n) {
        lk[j] = kv[u];
        la[j] = av[u] != NONE ? fi_rank_of(lo, n, av[u]) : NONE;
      }
    }
    __syncthreads();
    if (n >= FI_TOUR_MIN && fi_gap_tour(n, L)) {
      if (lane == 0) atomicOr(&fi[0], FI_TOUR);
      __syncthreads();
      for (uint32_t j = lane; j < n; j += 64) {
        ord[k + j] = la[j];
        first[k + j] = k;
      }
      return;
    }
    if (lane == 0) {
      unsigned long long hd = FI_LE_NONE;  // the head's entry (its key << 11 | index)
      long long x = lk[0];
      uint32_t a = la[0];
      for (uint32_t j = 0; j < n; ++j) {
        const long long xn = j + 1 < n ? lk[j + 1] : 0;  // (the next op's, in flight)
        const uint32_t an = j + 1 < n ? la[j + 1] : NONE;
        uint32_t cur = a;  // NONE = the head
        unsigned long long e = cur == NONE ? hd : le[cur];
        while ((e & FI_LE_NONE) != FI_LE_NONE && static_cast<long long>(e >> 11) > x) {
          cur = static_cast<uint32_t>(e & FI_LE_NONE);
          e = le[cur];
        }
        le[j] = e;
        const unsigned long long me = (static_cast<unsigned long long>(x) << 11) | j;
        if (cur == NONE) hd = me;
        else le[cur] = me;
        x = xn;
        a = an;
      }
      uint32_t o = 0;
      for (uint32_t j = static_cast<uint32_t>(hd & FI_LE_NONE); j != FI_LE_NONE;
           j = static_cast<uint32_t>(le[j] & FI_LE_NONE))
        lo[j] = o++;
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
    if (a != NONE && gk0[a] == g) cur = k + fi_rank_of(gv + k, e - k, a);
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

// (a grid of at most FI_GAPS_GRID single-wave workgroups loops over the gaps:
// one per op would schedule thousands of LDS-holding workgroups that exit)
constexpr uint32_t FI_GAPS_GRID = 2048;
// (each workgroup takes the gaps that start in its chunk of sorted
// positions: a head is a position whose key differs from the one before)
__global__ void __launch_bounds__(64) k_fi_gaps(uint32_t m, const uint32_t* gk, const uint32_t* gv, const uint32_t* gk0,
                                                const uint32_t* par0, const long long* ts, uint32_t* nxt,
                                                uint32_t* ord, uint32_t* first, uint32_t* fi) {
  __shared__ FiGapLds L;
  const uint32_t lane = threadIdx.x;
  const uint32_t C = (m + gridDim.x - 1) / gridDim.x, c0 = blockIdx.x * C, c1 = min(m, c0 + C);
  for (uint32_t b = c0; b < c1; b += 64) {
    const uint32_t q = b + lane;
    unsigned long long hm = __ballot(q < c1 && (q == 0 || gk[q - 1] != gk[q]));
    while (hm) {
      const uint32_t k = b + static_cast<uint32_t>(__builtin_ctzll(hm));
      hm &= hm - 1;
      fi_gap_one(k, m, gk, gv, gk0, par0, ts, nxt, ord, first, fi, L);
      wave_sync();  // (the next gap reuses the LDS; one wave per workgroup)
    }
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
                                                  uint32_t slot0, uint32_t* newdoc, uint32_t* newrank) {
  __shared__ uint32_t bnd[2];
  const uint32_t r0 = blockIdx.x * blockDim.x, r = r0 + threadIdx.x;
  if (r0 < K && threadIdx.x < 2) {
    const uint32_t rr = threadIdx.x == 0 ? r0 : min(K - 1, r0 + blockDim.x - 1);
    bnd[threadIdx.x] = threadIdx.x == 0 ? (r0 ? fi_count_le(gk, 0, m, r0 - 1) : 0u) : fi_count_le(gk, 0, m, rr);
  }
  __syncthreads();
  if (r < K) {
    newdoc[r + fi_count_le(gk, bnd[0], bnd[1], r)] = doc[r];
  } else if (r < K + m) {
    const uint32_t k = r - K;
    const uint32_t p = gk[k] + first[k] + ord[k];
    newrank[k] = p;
    newdoc[p] = slot0 + gv[k];
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
                                                     TreeDev T, uint8_t* st, uint8_t* st_out, const uint32_t* fi,
                                                     TsHash kx) {
  if (fi[6] == FG_NONE) return;  // (grid-uniform: the gate)
  GRID_STRIDE(i, o.n) {
    tshash_insert(kx, o.ts[i], slot0 + i);  // (the key index: the batch's keys)
    const uint32_t sl = slot0 + i;
    st[i] = ST_APPLIED;
    if (st_out) st_out[i] = CRDTM_ST_APPLIED;
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

// The dense order from the gapped one, into the tree's `doc`.
static int fi_compact_doc(crdtm_tree* t, Arena& ws, hipStream_t s) {
  KeyIndex& X = *t->kidx;
  uint32_t* off = ws.alloc<uint32_t>(X.nbk + 1);
  int r = scan_excl_u32(X.bcnt, off, X.nbk, nullptr, ws, s);
  if (r) return r;
  LAUNCH(k_fi_compact, dim3(grid_for(static_cast<uint64_t>(X.nbk) * FI_CAP)), dim3(BLOCK), 0, s, X.nbk, off, X.bent,
         X.bcnt, t->d.doc);
  t->doc_gapped = false;
  return CRDTM_OK;
}

int fi_materialize(crdtm_tree* t) {
  if (!t->doc_gapped) return CRDTM_OK;
  if (!t->kidx || !t->kidx->ord_ready || !t->kidx_valid) {  // (cannot happen after a good merge)
    t->doc_gapped = false;
    t->doc_valid = false;
    return CRDTM_OK;
  }
  return fi_compact_doc(t, t->ctx->ws, t->ctx->stream);
}

// The gapped order from the tree's dense `doc` (K entries), a quarter full.
static int fi_build(crdtm_tree* t, uint32_t K, hipStream_t s) {
  KeyIndex& X = *t->kidx;
  const uint32_t nbk = (K + FI_FILL - 1) / FI_FILL;
  if (X.bcap < nbk) {
    for (void* q : {static_cast<void*>(X.bent), static_cast<void*>(X.bdk), static_cast<void*>(X.bcnt),
                    static_cast<void*>(X.bend), static_cast<void*>(X.bfirst), static_cast<void*>(X.bwin),
                    static_cast<void*>(X.bmin), static_cast<void*>(X.smin), static_cast<void*>(X.tmin)})
      if (q) hipFree(q);
    const uint64_t bc = 2ULL * nbk + 64;
    HIP_CHECK(hipMalloc(&X.bent, bc * FI_CAP * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.bdk, bc * FI_CAP * sizeof(long long)));
    HIP_CHECK(hipMalloc(&X.bcnt, bc * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.bend, bc * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.bfirst, bc * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.bwin, bc * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&X.bmin, FI_BPB * bc * sizeof(long long)));
    HIP_CHECK(hipMalloc(&X.smin, (FI_BPB * bc / FI_SUP + 1) * sizeof(long long)));
    HIP_CHECK(hipMalloc(&X.tmin, ((FI_BPB * bc / FI_SUP + 1) / FI_SUP + 2) * sizeof(long long)));
    X.bcap = bc;
  }
  X.nbk = nbk;
  const uint32_t Kp = nbk * FI_CAP;
  LAUNCH(k_fi_build, dim3(grid_for(Kp)), dim3(BLOCK), 0, s, K, nbk, t->d.doc, t->d.s_key, X.bent, X.bdk, X.bcnt,
         X.bfirst, X.bend, X.bwin, X.rank);
  LAUNCH(k_fi_bmin, dim3(grid_for(static_cast<uint64_t>(Kp / FI_BLK + 3) / 4 * 64)), dim3(BLOCK), 0, s, Kp, X.bdk,
         X.bmin);
  LAUNCH(k_fi_sup, dim3(grid_for(FI_BPB * nbk / FI_SUP + 1)), dim3(BLOCK), 0, s, FI_BPB * nbk, X.bmin, X.smin);
  LAUNCH(k_fi_top, dim3(grid_for(FI_BPB * nbk / FI_SUP / FI_SUP + 1)), dim3(BLOCK), 0, s,
         (FI_BPB * nbk + FI_SUP - 1) / FI_SUP, X.smin, X.tmin);
  X.ord_ready = true;
  return CRDTM_OK;
}

// (Re)builds the tree's key index when it does not describe the state, with
// room for `extra` more nodes; the gapped order is rebuilt (ord_ready) when
// its arrays are new or the index was stale (a gapped document is written
// back to `doc` first).
static int kx_ensure(crdtm_tree* t, uint64_t extra, Arena& ws) {
  crdtm_ctx* c = t->ctx;
  const uint64_t need_h = 2 * (t->n_slots + extra) + 1024, need_r = t->n_slots + extra + 1;
  if (!t->kidx) t->kidx = std::make_unique<KeyIndex>();
  KeyIndex& x = *t->kidx;
  const bool hash_ok = t->kidx_valid && static_cast<uint64_t>(x.mask) + 1 >= need_h;
  if (hash_ok && x.rcap >= need_r) return CRDTM_OK;
  if (t->doc_gapped) {
    int r = fi_compact_doc(t, ws, c->stream);
    if (r) return r;
  }
  x.ord_ready = false;
  if (x.rcap < need_r) {
    if (x.rank) hipFree(x.rank);
    x.rank = nullptr;
    const uint64_t rc = 2 * need_r + 4096;
    HIP_CHECK(hipMalloc(&x.rank, rc * sizeof(uint32_t)));
    x.rcap = rc;
  }
  if (hash_ok) return CRDTM_OK;
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
  return CRDTM_OK;
}

int finc_apply(crdtm_tree* t, const OpsDev& o, uint8_t* st_out, crdtm_result* res, bool* handled) {
  *handled = false;
  const uint32_t m = o.n;
  const uint64_t K64 = t->n_slots - 1;
  if (!finc_allowed() || m == 0 || m > FI_MAX_BATCH || !t->flat_clean || !t->doc_valid || t->n_dicts != 1 ||
      t->doc_n != K64 || K64 == 0 || o.n_path != m || K64 + m >= 0x7FFFFFF0ULL || 2 * (K64 + m) >= 0x7FFFFFF0ULL)
    return CRDTM_OK;
  if (t->doc_gapped && !(t->kidx && t->kidx->ord_ready && t->kidx_valid)) return CRDTM_OK;
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  const uint32_t K = static_cast<uint32_t>(K64);
  const size_t mark0 = ws.used;
  int r;
  if ((r = kx_ensure(t, m, ws))) return r;
  KeyIndex& X = *t->kidx;
  if (!X.ord_ready && (r = fi_build(t, K, s))) return r;
  const uint32_t nbk = X.nbk, Kp = nbk * FI_CAP;
  // every workspace buffer first: nothing is written to the state before the last check
  const uint32_t bcap = pow2_ge(2ULL * m);
  TsHash bh{ws.alloc<unsigned long long>(bcap), ws.alloc<uint32_t>(bcap), bcap - 1};
  uint32_t* fi = ws.alloc<uint32_t>(FI_WORDS);
  uint32_t* par[1] = {ws.alloc<uint32_t>(m)};
  uint32_t* sta[1] = {ws.alloc<uint32_t>(m)};
  long long* thr[1] = {ws.alloc<long long>(m)};
  uint32_t* par0 = ws.alloc<uint32_t>(m);
  uint32_t* gk[2] = {ws.alloc<uint32_t>(m), ws.alloc<uint32_t>(m)};
  uint32_t* gv[2] = {ws.alloc<uint32_t>(m), ws.alloc<uint32_t>(m)};
  uint32_t* nxt = ws.alloc<uint32_t>(m);
  uint32_t* tl = ws.alloc<uint32_t>(m);
  uint32_t* ovl = ws.alloc<uint32_t>(m);
  uint32_t* gpred = ws.alloc<uint32_t>(m);
  uint32_t* wl = ws.alloc<uint32_t>(m);
  uint32_t* wlev = ws.alloc<uint32_t>(m);
  uint32_t* ord = ws.alloc<uint32_t>(m);
  uint32_t* first = ws.alloc<uint32_t>(m);
  uint32_t* newrank = ws.alloc<uint32_t>(m);
  uint8_t* st = ws.alloc<uint8_t>(m);
  long long* rep = ws.alloc<long long>(2ULL * m + 2);
  unsigned long long* scw = ws.alloc<unsigned long long>((m + 1023) & ~1023u);  // (the gap sort's chunks)
  uint32_t* jx = ws.alloc<uint32_t>(m);  // (the chunked pointer jumping's exits and minima)
  long long* jm = ws.alloc<long long>(m);
  const TsHash kx{X.keys, X.vals, X.mask};
  uint32_t* rank_of = X.rank;
  // ---- phase A: anchors, validity ----
  LAUNCH(k_fi_clear, dim3(grid_for(bcap)), dim3(BLOCK), 0, s, bh.keys, bcap, fi, st, m, c->dres);
  LAUNCH(k_fi_bidx, dim3(grid_for(m)), dim3(BLOCK), 0, s, o, bh, fi);
  LAUNCH(k_fi_resolve, dim3(grid_for(m)), dim3(BLOCK), 0, s, o, kx, bh, rank_of, replica_of(t->timestamp), par[0],
         par0, sta[0], thr[0], fi);
  // ---- phase B: gaps (pointer jumping over new anchors, one NSR query each
  // over the gapped order), the blocks they land in ----
  uint32_t rounds = 0;
  for (uint32_t span = 1; span < m; span <<= 1) ++rounds;
  static const bool jump_lds = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fi_jump_lds),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   FI_JUMP_LDS_MAX * 10) == hipSuccess;
  static const bool jump_chunks = [] {  // (CRDTM_FI_JUMP=lds: the one-workgroup kernel, for A/B)
    const char* e = getenv("CRDTM_FI_JUMP");
    return !(e && !strcmp(e, "lds"));
  }();
  if (rounds && jump_chunks) {
    const uint32_t nch = (m + FI_JC - 1) / FI_JC;
    LAUNCH(k_fi_jump_chunk, dim3(nch), dim3(FI_JC), 0, s, m, par[0], sta[0], thr[0], jx, jm);
  } else if (rounds && jump_lds && m <= FI_JUMP_LDS_MAX)
    LAUNCH(k_fi_jump_lds, dim3(1), dim3(FI_JUMP_THREADS), static_cast<size_t>(m) * 10, s, m, rounds, par[0], sta[0],
           thr[0]);
  else if (rounds)
    LAUNCH(k_fi_jump, dim3(1), dim3(FI_JUMP_THREADS), 0, s, m, rounds, par[0], sta[0], thr[0], o.ts);
  // (measured and reverted in round 5: four queries per wave, 16 lanes
  // each -- 0.65 ms more per 100 batches: a query's long search held up the
  // wave's other three)
  LAUNCH(k_fi_gap, dim3(grid_for(64ULL * m)), dim3(BLOCK), 0, s, m, Kp, X.bdk, X.bmin, X.smin, X.tmin, sta[0],
         thr[0], gk[0], gv[0], (rounds && jump_chunks) ? jx : nullptr, jm);
  // (test hook: one batch's gap keys, for tools/xbench_sort.py)
  static const char* dump = test_hooks() ? getenv("CRDTM_FI_DUMP_KEYS") : nullptr;
  if (dump && *dump) {
    std::vector<uint32_t> hk(m);
    HIP_CHECK(hipMemcpyAsync(hk.data(), gk[0], m * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (FILE* fp = fopen(dump, "wb")) {
      fwrite(hk.data(), sizeof(uint32_t), m, fp);
      fclose(fp);
    }
  }
  uint32_t bits = 4;  // (gap positions run to Kp inclusive)
  while (bits < 32 && (static_cast<uint64_t>(Kp) >> bits) != 0) bits += 4;
  uint32_t *sk = gk[1], *sv = gv[1];
  // (measured and reverted in round 5: a bitonic network over (gap, op)
  // words in one workgroup's LDS, 0.47 ms per batch against 0.29)
  if ((r = radix_sort_small(gk[0], gv[0], m, bits, sk, sv, s, scw))) return r;
  const uint32_t gm = (m + BLOCK - 1) / BLOCK;  // one item per thread
  // (the gap heads and the anchors' places are found by k_fi_gaps itself:
  // one launch fewer than a separate pass listing them)
  static const uint32_t gaps_grid = [] {  // (env CRDTM_GAPS_GRID: A/B)
    const char* e = getenv("CRDTM_GAPS_GRID");
    return e ? std::max(1, atoi(e)) : static_cast<int>(FI_GAPS_GRID);
  }();
  LAUNCH(k_fi_gaps, dim3(std::min(m, static_cast<uint32_t>(gaps_grid))), dim3(64), 0, s, m, sk, sv, gk[0], par0, o.ts, nxt, ord, first,
         fi);
  LAUNCH(k_fi_tblk, dim3(gm), dim3(BLOCK), 0, s, m, nbk, sk, ord, X.bent, X.bcnt, X.bfirst, X.bend, tl, gpred, fi);
  LAUNCH(k_fi_win_pick, dim3(grid_for(64ULL * m)), dim3(BLOCK), 0, s, nbk, sk, tl, X.bcnt, X.bfirst, X.bend, X.bwin,
         ovl, fi);
  // (resolved before the commit is queued: nothing may fail once it is)
  static const bool win_lds = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fi_win),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  FI_WIN_ENT * 12) == hipSuccess;
  // (its last workgroup decides the commit gate)
  LAUNCH(k_fi_win_list, dim3(grid_for(m)), dim3(BLOCK), 0, s, ovl, fi, X.bwin, wl, wlev,
         static_cast<long long>(t->timestamp), win_lds ? 1u : 0u, c->dres);
  // ---- phase C: the commit, queued at once and gated on the device
  // (k_fi_gate): one host round trip per batch, at its end ----
  TreeCaps need = t->cap;
  need.slots = std::max<uint64_t>(need.slots, t->n_slots + m + 1);
  need.log = std::max<uint64_t>(need.log, t->log_n + m + 1);
  need.lpath = std::max<uint64_t>(need.lpath, t->log_npath + m + 1);
  need.doc = std::max<uint64_t>(need.doc, K64 + m + 1);
  if (need.slots > t->cap.slots || need.log > t->cap.log || need.lpath > t->cap.lpath || need.doc > t->cap.doc)
    if ((r = grow_tree(t, need))) return r;
  const uint32_t slot0 = static_cast<uint32_t>(t->n_slots);
  LAUNCH(k_fi_commit, dim3(grid_for(m)), dim3(BLOCK), 0, s, o, slot0, static_cast<uint32_t>(t->log_n),
         static_cast<uint32_t>(t->log_npath), t->d, st, st_out, fi, kx);
  // O(batch): the blocks the batch lands in (grid-stride over the device's
  // counts; blocks and windows are at most one per op)
  const uint32_t cg = std::min<uint32_t>(FI_COMMIT_GRID, std::min<uint32_t>(m, nbk));
  const uint32_t wg = std::min<uint32_t>(256u, cg);
  LAUNCH(k_fi_rewrite, dim3(cg), dim3(FI_CAP), 0, s, nbk, tl, fi, sk, sv, ord, first, gpred, slot0, o.ts, X.bent,
         X.bdk, X.bcnt, X.bfirst, X.bend, X.bwin, X.bmin, rank_of, t->d.s_next);
  if (win_lds)
    LAUNCH(k_fi_win, dim3(wg), dim3(FI_WIN_THREADS), FI_WIN_ENT * 12, s, nbk, wl, wlev, fi, sk, sv, ord, first, gpred,
           slot0, o.ts, X.bent, X.bdk, X.bcnt, X.bfirst, X.bend, X.bwin, X.bmin, rank_of, t->d.s_next);
  LAUNCH(k_fi_sup_fix, dim3(grid_for(64ULL * cg)), dim3(BLOCK), 0, s, nbk, tl, sk, wl, wlev, fi, X.bmin, X.smin);
  LAUNCH(k_fi_top_fix, dim3(grid_for(64ULL * cg)), dim3(BLOCK), 0, s, nbk, tl, sk, wl, wlev, fi, X.smin, X.tmin);
  // (statuses not applied fold nothing; k_fi_clear zeroed the fold's counters)
  if ((r = replica_fold(c, o, st, rep, ws, s, true))) return r;
  if ((r = sync_read(c))) return r;
  uint32_t hf[FI_WORDS];
  std::memcpy(hf, c->hres->fincr, sizeof(hf));
  if (hf[6] == FG_NONE) {
    // the general paths decide: the state is untouched (every commit kernel
    // read the gate), the key index stays valid; the blocks' per-batch marks
    // are not cleared, so they are rebuilt when next used
    if (t->doc_gapped && (r = fi_compact_doc(t, ws, s))) return r;
    X.ord_ready = false;
    ws.used = mark0;
    return CRDTM_OK;
  }
  const long long new_ts = t->timestamp + hf[1];
  const bool dense = hf[6] == FG_DENSE;
  if (!dense) {
    t->doc_gapped = true;
  } else {  // a block overflows: merge densely, then rebuild the blocks
    if ((r = fi_compact_doc(t, ws, s))) return r;
    uint32_t* off = ws.alloc<uint32_t>(nbk + 1);
    if ((r = scan_excl_u32(X.bcnt, off, nbk, nullptr, ws, s))) return r;
    LAUNCH(k_fi_dense_gaps, dim3(grid_for(m)), dim3(BLOCK), 0, s, m, Kp, K, off, sk);
    if (X.doc2_cap < t->cap.doc) {  // the next order's buffer matches the tree's doc capacity
      if (X.doc2) hipFree(X.doc2);
      X.doc2 = nullptr;
      HIP_CHECK(hipMalloc(&X.doc2, t->cap.doc * sizeof(uint32_t)));
      X.doc2_cap = t->cap.doc;
    }
    uint32_t* newdoc = X.doc2;
    LAUNCH(k_fi_doc, dim3(grid_for(K64 + m)), dim3(BLOCK), 0, s, K, m, t->d.doc, sk, sv, ord, first, slot0, newdoc,
           newrank);
    LAUNCH(k_fi_next, dim3(grid_for(m)), dim3(BLOCK), 0, s, K, m, sv, ord, newrank, newdoc, slot0, t->d.s_next);
    // the new order becomes the tree's (the store owns whichever buffer `doc` holds)
    std::swap(t->d.doc, X.doc2);
    std::swap(t->cap.doc, X.doc2_cap);
    t->store->d.doc = t->d.doc;
    if ((r = fi_build(t, K + m, s))) return r;
    t->doc_gapped = false;
  }
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
  res->flags |= CRDTM_FLAG_INCREMENTAL | (dense ? CRDTM_FLAG_INCR_DENSE : 0u) |
                (!dense && hf[5] ? CRDTM_FLAG_INCR_WINDOWS : 0u) | ((hf[0] & FI_TOUR) ? CRDTM_FLAG_INCR_TOUR : 0u);
  res->n_applied = m;
  res->n_already = 0;
  *handled = true;
  return CRDTM_OK;
}

}  // namespace crdtm

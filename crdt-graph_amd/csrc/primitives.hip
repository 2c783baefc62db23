// primitives.hip — device-wide scan, segmented child sort and list ranking
// for the crdtm engine (gfx950: wave64, 256 CUs, 160 KiB LDS per CU).
//
// These are the building blocks of north-star kernels (2) segmented sibling
// sort and (4) Euler-tour list ranking. Everything is integer, HBM-bound work.

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstring>

#include "engine.h"
#include "listrank.h"
#include "scan.h"

namespace crdtm {

// out[i] = sum(in[0..i)); *total (device) = sum(in). in may alias out.
int scan_excl_u32(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* total, Arena& ws, hipStream_t st) {
  return dscan<SumOp, false>(ArrGen{in}, out, n, total, ws, st, nullptr);  // errors: ws.scan_err
}

// ---------------------------------------------------------------------------
// Segmented sort of children by key (ascending, unique keys per segment).
// seg_start[u]..seg_start[u+1) of carr; key(v) from sort_key(v).
// Small segments: one lane each (insertion sort). Large: one workgroup each,
// bitonic in LDS up to LDS_SORT_MAX, else a workgroup merge sort in HBM.
// ---------------------------------------------------------------------------
constexpr uint32_t SMALL_SEG = 16;
constexpr uint32_t MID_SEG = 512;
constexpr uint32_t LDS_SORT_MAX = 4096;

// Sort keys: an explicit per-item array, or the item id itself descending
// (timestamp-slot numbering: slot order == timestamp order).
struct ArrKey {
  static constexpr bool kFromId = false;  // the key is a gather: k_sort_big keeps keys in LDS
  const long long* k;
  __device__ __forceinline__ long long operator()(uint32_t v) const { return k[v]; }
};
struct IdKey {
  static constexpr bool kFromId = true;  // the key is arithmetic on the id: k_sort_big keeps ids only
  __device__ __forceinline__ long long operator()(uint32_t v) const { return static_cast<long long>(v); }
};
struct NegIdKey {
  static constexpr bool kFromId = true;
  __device__ __forceinline__ long long operator()(uint32_t v) const { return -static_cast<long long>(v); }
};

// Segments of 2 swap in place; tiny ones (3..SMALL_SEG) sort in place too:
// the lane's items load together into registers and each item's rank
// (smaller keys, ties by position: stable) comes from static-index compares
// bounded by the wave's longest tiny segment (a scalar bound, so the steps
// beyond it are skipped) — no dependent loads and no list of tiny segments
// (a list append per tiny segment serialises on its counter: ~10^5 of them
// in a 10M-op flat merge). Mid and big segments go to their lists with
// wave-aggregated appends.
template <class KEY>
__global__ void __launch_bounds__(BLOCK) k_sort_small(const uint32_t* __restrict__ seg_start, uint32_t n_seg,
                                                      uint32_t* __restrict__ carr, KEY sort_key, uint32_t skip,
                                                      uint32_t* __restrict__ mid_list, uint32_t* __restrict__ n_mid,
                                                      uint32_t* __restrict__ big_list, uint32_t* __restrict__ n_big) {
  // the loop bound is uniform per workgroup, so every lane reaches the wave steps
  for (uint32_t u0 = blockIdx.x * blockDim.x; u0 < n_seg; u0 += gridDim.x * blockDim.x) {
    const uint32_t u = u0 + threadIdx.x;
    uint32_t len = 0, b = 0;
    if (u < n_seg && u != skip) {
      b = seg_start[u];
      len = seg_start[u + 1] - b;
      if (len == 2) {
        const uint32_t x = carr[b], y = carr[b + 1];
        if (sort_key(y) < sort_key(x)) {
          carr[b] = y;
          carr[b + 1] = x;
        }
      }
    }
    const uint32_t tl = len > 2 && len <= SMALL_SEG ? len : 0u;
    uint32_t wl = tl;
    for (int o = 32; o > 0; o >>= 1) wl = max(wl, static_cast<uint32_t>(__shfl_xor(static_cast<int>(wl), o, 64)));
    wl = __builtin_amdgcn_readfirstlane(wl);
    if (wl) {
      uint32_t v[SMALL_SEG];
      long long k[SMALL_SEG];
#pragma unroll
      for (uint32_t t = 0; t < SMALL_SEG; ++t) {
        v[t] = 0;
        k[t] = 0x7fffffffffffffffLL;
        if (t < wl && t < tl) {
          v[t] = carr[b + t];
          k[t] = sort_key(v[t]);
        }
      }
#pragma unroll
      for (uint32_t t = 0; t < SMALL_SEG; ++t) {
        if (t < wl) {
          uint32_t rk = 0;
#pragma unroll
          for (uint32_t j = 0; j < SMALL_SEG; ++j) {
            if (j < wl) {
              if (j < t) rk += k[j] <= k[t] ? 1u : 0u;
              else if (j > t) rk += k[j] < k[t] ? 1u : 0u;
            }
          }
          if (t < tl) carr[b + rk] = v[t];
        }
      }
    }
    // wave-aggregated appends: one atomic per wave and list
    const bool mi = len > SMALL_SEG && len <= MID_SEG, bi = len > MID_SEG;
    const uint32_t km = wave_ticket(n_mid, mi), kb = wave_ticket(n_big, bi);
    if (mi) mid_list[km] = u;
    if (bi) big_list[kb] = u;
  }
}

// One wave per mid-size segment (17..MID_SEG): copy the keys to LDS; every
// lane holds up to MID_SEG/64 items and counts the smaller keys (keys are
// unique) in one sweep of broadcast 16-byte LDS reads, then writes each item
// at its rank.
template <class KEY>
__global__ void __launch_bounds__(BLOCK) k_sort_mid(const uint32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ mid_list,
                                                    const uint32_t* __restrict__ n_mid, uint32_t* __restrict__ carr,
                                                    KEY sort_key) {
  constexpr uint32_t T = MID_SEG / 64;
  __shared__ __attribute__((aligned(16))) long long skey[BLOCK / 64][MID_SEG + 2];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t nm = *n_mid;
  const uint32_t waves = gridDim.x * (BLOCK / 64);
  for (uint32_t mi = blockIdx.x * (BLOCK / 64) + wv; mi < nm; mi += waves) {
    const uint32_t u = mid_list[mi];
    const uint32_t b = seg_start[u], len = seg_start[u + 1] - b;
    uint32_t id[T];
    long long kk[T];
    uint32_t rk[T];
#pragma unroll
    for (uint32_t t = 0; t < T; ++t) {
      const uint32_t j = lane + 64 * t;
      id[t] = j < len ? carr[b + j] : 0u;
      kk[t] = j < len ? sort_key(id[t]) : 0x7fffffffffffffffLL;
      rk[t] = 0;
      if (j < len) skey[wv][j] = kk[t];
    }
    if (lane == 0) skey[wv][len] = 0x7fffffffffffffffLL;  // pad to an even count
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const longlong2* k2 = reinterpret_cast<const longlong2*>(skey[wv]);
#pragma unroll 4
    for (uint32_t m = 0; m < (len + 1) / 2; ++m) {
      const longlong2 a = k2[m];
#pragma unroll
      for (uint32_t t = 0; t < T; ++t) rk[t] += (a.x < kk[t] ? 1u : 0u) + (a.y < kk[t] ? 1u : 0u);
    }
#pragma unroll
    for (uint32_t t = 0; t < T; ++t)
      if (lane + 64 * t < len) carr[b + rk[t]] = id[t];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// One workgroup per large segment (MID_SEG+1..LDS_SORT_MAX): bitonic sort
// over the next power of two in LDS (padding sorts last). Every step is one
// compare-exchange per pair, pairs spread over all threads (pair q works on
// i = q with a zero bit inserted at jj, and i | jj). The network is LDS
// bandwidth bound, so when the key is arithmetic on the id (IdKey /
// NegIdKey) only the 4-byte ids live in LDS and keys are recomputed.
template <class KEY>
__device__ __forceinline__ long long big_key(KEY sort_key, uint32_t v) {
  return v == NONE ? 0x7fffffffffffffffLL : sort_key(v);
}

template <class KEY>
__global__ void __launch_bounds__(1024) k_sort_big(const uint32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ big_list,
                                                    const uint32_t* __restrict__ n_big, uint32_t* __restrict__ carr,
                                                    KEY sort_key) {
  constexpr bool FROM_ID = KEY::kFromId;
  __shared__ long long skey[FROM_ID ? 1 : LDS_SORT_MAX];
  __shared__ uint32_t sid[LDS_SORT_MAX];
  const uint32_t nb = *n_big;
  for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
    const uint32_t u = big_list[bi];
    const uint32_t b = seg_start[u], len = seg_start[u + 1] - b;
    if (len > LDS_SORT_MAX) continue;  // huge: multi-workgroup path (segmented_sort)
    uint32_t p2 = 1;
    while (p2 < len) p2 <<= 1;
    for (uint32_t j = threadIdx.x; j < p2; j += blockDim.x) {
      const uint32_t v = j < len ? carr[b + j] : NONE;
      sid[j] = v;
      if constexpr (!FROM_ID) skey[j] = big_key(sort_key, v);
    }
    __syncthreads();
    for (uint32_t k = 2; k <= p2; k <<= 1) {
      for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
        for (uint32_t q = threadIdx.x; q < p2 / 2; q += blockDim.x) {
          const uint32_t i = ((q & ~(jj - 1)) << 1) | (q & (jj - 1)), ixj = i | jj;
          const bool up = (i & k) == 0;
          const uint32_t va = sid[i], vc = sid[ixj];
          long long a, c;
          if constexpr (FROM_ID) {
            a = big_key(sort_key, va);
            c = big_key(sort_key, vc);
          } else {
            a = skey[i];
            c = skey[ixj];
          }
          if ((a > c) == up) {
            sid[i] = vc;
            sid[ixj] = va;
            if constexpr (!FROM_ID) {
              skey[i] = c;
              skey[ixj] = a;
            }
          }
        }
        __syncthreads();
      }
    }
    for (uint32_t j = threadIdx.x; j < len; j += blockDim.x) carr[b + j] = sid[j];
    __syncthreads();
  }
}

// Huge segments (> LDS_SORT_MAX), all of them at once: a table of the huge
// segments {begin, length, first chunk, first merge tile}; chunk-sort in LDS,
// then merge passes with merge-path partitioning, one launch per width for
// every segment (a segment already merged at this width is copied through).
struct HugeTable {
  uint32_t* b;     // segment begin
  uint32_t* len;   // segment length
  uint32_t* cpre;  // [nh + 1] exclusive prefix of LDS chunks
  uint32_t* tpre;  // [nh + 1] exclusive prefix of merge tiles
  uint32_t nh;
};

__device__ __forceinline__ uint32_t huge_find(const uint32_t* pre, uint32_t nh, uint32_t x) {
  uint32_t lo = 0, hi = nh;  // last k with pre[k] <= x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

template <class KEY>
__global__ void __launch_bounds__(1024) k_sort_chunks(uint32_t* __restrict__ carr, HugeTable ht, KEY sort_key) {
  __shared__ long long skey[LDS_SORT_MAX];
  __shared__ uint32_t sid[LDS_SORT_MAX];
  const uint32_t seg = huge_find(ht.cpre, ht.nh, blockIdx.x);
  const uint32_t b = ht.b[seg], len = ht.len[seg];
  const uint32_t r0 = (blockIdx.x - ht.cpre[seg]) * LDS_SORT_MAX;
  const uint32_t rl = min(LDS_SORT_MAX, len - r0);
  for (uint32_t j = threadIdx.x; j < LDS_SORT_MAX; j += blockDim.x) {
    if (j < rl) {
      uint32_t v = carr[b + r0 + j];
      sid[j] = v;
      skey[j] = sort_key(v);
    } else {
      sid[j] = NONE;
      skey[j] = 0x7fffffffffffffffLL;
    }
  }
  __syncthreads();
  for (uint32_t k = 2; k <= LDS_SORT_MAX; k <<= 1) {
    for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
      for (uint32_t i = threadIdx.x; i < LDS_SORT_MAX; i += blockDim.x) {
        uint32_t ixj = i ^ jj;
        if (ixj > i) {
          bool up = (i & k) == 0;
          long long a = skey[i], c = skey[ixj];
          if ((a > c) == up) {
            skey[i] = c;
            skey[ixj] = a;
            uint32_t t = sid[i];
            sid[i] = sid[ixj];
            sid[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t j = threadIdx.x; j < rl; j += blockDim.x) carr[b + r0 + j] = sid[j];
}

constexpr uint32_t MERGE_PER_THREAD = 8;
constexpr uint32_t MERGE_TILE = BLOCK * MERGE_PER_THREAD;  // 2048 outputs per workgroup

template <class KEY>
__global__ void __launch_bounds__(BLOCK) k_merge_pass(const uint32_t* __restrict__ src_base,
                                                      uint32_t* __restrict__ dst_base, HugeTable ht, uint32_t width,
                                                      KEY sort_key) {
  const uint32_t seg = huge_find(ht.tpre, ht.nh, blockIdx.x);
  const uint32_t len = ht.len[seg];
  const uint32_t* __restrict__ src = src_base + ht.b[seg];
  uint32_t* __restrict__ dst = dst_base + ht.b[seg];
  const uint32_t d0 = (blockIdx.x - ht.tpre[seg]) * MERGE_TILE + threadIdx.x * MERGE_PER_THREAD;
  if (d0 >= len) return;
  const uint32_t pair = d0 / (2 * width);
  const uint32_t a0 = pair * 2 * width, a1 = min(a0 + width, len), b1 = min(a0 + 2 * width, len);
  const uint32_t na = a1 - a0, nb = b1 - a1;
  const uint32_t d = d0 - a0;  // output rank within the pair
  uint32_t lo = d > nb ? d - nb : 0, hi = min(d, na);
  while (lo < hi) {  // merge path: #taken from A among the first d outputs
    const uint32_t mid = (lo + hi) >> 1;
    if (sort_key(src[a0 + mid]) < sort_key(src[a1 + d - mid - 1])) lo = mid + 1;
    else hi = mid;
  }
  uint32_t i = lo, j = d - lo;
  const uint32_t dend = min(d + MERGE_PER_THREAD, na + nb);
  for (uint32_t q = d; q < dend; ++q) {
    bool takeA;
    if (i >= na) takeA = false;
    else if (j >= nb) takeA = true;
    else takeA = sort_key(src[a0 + i]) < sort_key(src[a1 + j]);
    dst[a0 + q] = takeA ? src[a0 + i++] : src[a1 + j++];
  }
}

__global__ void k_sort_big_filter(const uint32_t* __restrict__ seg_start, const uint32_t* __restrict__ big_list,
                                  const uint32_t* __restrict__ n_big, uint32_t* __restrict__ huge,
                                  uint32_t* __restrict__ n_huge) {
  const uint32_t nb = *n_big;
  for (uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x; bi < nb; bi += gridDim.x * blockDim.x) {
    const uint32_t u = big_list[bi];
    if (seg_start[u + 1] - seg_start[u] > LDS_SORT_MAX) huge[atomicAdd(n_huge, 1u)] = u;
  }
}

// One workgroup: fill the huge table from the huge segment list and publish
// {chunks, tiles, longest} for the host.
__global__ void __launch_bounds__(BLOCK) k_huge_meta(const uint32_t* __restrict__ seg_start,
                                                     const uint32_t* __restrict__ huge, HugeTable ht,
                                                     uint32_t* __restrict__ out) {
  __shared__ uint32_t sc[BLOCK / 64], stl[BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry_c = 0, carry_t = 0, mx = 0;
  for (uint32_t k0 = 0; k0 < ht.nh; k0 += BLOCK) {
    const uint32_t k = k0 + threadIdx.x;
    uint32_t c = 0, tl = 0;
    if (k < ht.nh) {
      const uint32_t u = huge[k];
      const uint32_t b = seg_start[u], len = seg_start[u + 1] - b;
      ht.b[k] = b;
      ht.len[k] = len;
      c = (len + LDS_SORT_MAX - 1) / LDS_SORT_MAX;
      tl = (len + MERGE_TILE - 1) / MERGE_TILE;
      mx = max(mx, len);
    }
    const uint32_t ic = wave_incl_scan(c), it = wave_incl_scan(tl);
    if (lane == 63) {
      sc[wave] = ic;
      stl[wave] = it;
    }
    __syncthreads();
    uint32_t pc = carry_c, pt = carry_t, tc = 0, tt = 0;
    for (int w = 0; w < BLOCK / 64; ++w) {
      if (w < wave) {
        pc += sc[w];
        pt += stl[w];
      }
      tc += sc[w];
      tt += stl[w];
    }
    if (k < ht.nh) {
      ht.cpre[k] = pc + ic - c;
      ht.tpre[k] = pt + it - tl;
    }
    carry_c += tc;
    carry_t += tt;
    __syncthreads();
  }
  mx = block_max(mx);
  if (threadIdx.x == 0) {
    ht.cpre[ht.nh] = carry_c;
    ht.tpre[ht.nh] = carry_t;
    out[0] = carry_c;
    out[1] = carry_t;
    out[2] = mx;
  }
}

__global__ void __launch_bounds__(BLOCK) k_huge_copy(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                     HugeTable ht) {
  const uint32_t seg = huge_find(ht.tpre, ht.nh, blockIdx.x);
  const uint32_t b = ht.b[seg], len = ht.len[seg];
  const uint32_t t0 = (blockIdx.x - ht.tpre[seg]) * MERGE_TILE;
  for (uint32_t q = t0 + threadIdx.x; q < min(t0 + MERGE_TILE, len); q += BLOCK) dst[b + q] = src[b + q];
}

template <class KEY>
static int segmented_sort_t(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items, KEY sort_key,
                            Arena& ws, hipStream_t st, DevResult* dres, uint32_t skip) {
  uint32_t* mid = ws.alloc<uint32_t>(n_seg + 1);
  uint32_t* big = ws.alloc<uint32_t>(n_seg + 1);
  uint32_t* huge = ws.alloc<uint32_t>(n_seg + 1);
  uint32_t* scratch = ws.alloc<uint32_t>(n_items + 1);
  uint32_t* nbig = &dres->big_segments;
  uint32_t* nhuge = &dres->huge_segments;
  uint32_t* nmid = &dres->mid_segments;
  // big / huge / mid segment counters are 0 on entry (k_dres_init; reset on exit)
  LAUNCH(k_sort_small<KEY>, dim3(grid_for(n_seg)), dim3(BLOCK), 0, st, seg_start, n_seg, carr, sort_key, skip, mid,
         nmid, big, nbig);
  LAUNCH(k_sort_mid<KEY>, dim3(1024), dim3(BLOCK), 0, st, seg_start, mid, nmid, carr, sort_key);
  // segments of MID_SEG+1..LDS_SORT_MAX: one workgroup each (huge ones are skipped there)
  LAUNCH(k_sort_big<KEY>, dim3(256), dim3(1024), 0, st, seg_start, big, nbig, carr, sort_key);
  LAUNCH(k_sort_big_filter, dim3(16), dim3(BLOCK), 0, st, seg_start, big, nbig, huge, nhuge);
  uint32_t cn[3] = {0, 0, 0};  // big, huge, mid
  HIP_CHECK(hipMemcpyAsync(cn, nbig, sizeof(cn), hipMemcpyDeviceToHost, st));
  if (int rw = stream_wait(st)) return rw;
  const uint32_t nh = cn[1];
  static const bool stats = getenv("CRDTM_SORT_STATS") != nullptr;
  if (stats)
    fprintf(stderr, "[crdtm] segmented sort: %u segments, %u mid (%u..%u), %u big (..%u), %u huge\n", n_seg, cn[2],
            SMALL_SEG + 1, MID_SEG, cn[0], LDS_SORT_MAX, cn[1]);
  // leave the three counters at 0 for the next sort of this merge
  static_assert(offsetof(DevResult, huge_segments) == offsetof(DevResult, big_segments) + 4 &&
                    offsetof(DevResult, mid_segments) == offsetof(DevResult, big_segments) + 8,
                "sort counters are contiguous");
  HIP_CHECK(hipMemsetAsync(nbig, 0, 3 * sizeof(uint32_t), st));
  if (nh == 0) return CRDTM_OK;
  HugeTable ht;
  ht.nh = nh;
  ht.b = ws.alloc<uint32_t>(nh);
  ht.len = ws.alloc<uint32_t>(nh);
  ht.cpre = ws.alloc<uint32_t>(nh + 1);
  ht.tpre = ws.alloc<uint32_t>(nh + 1);
  uint32_t* meta = ws.alloc<uint32_t>(4);
  LAUNCH(k_huge_meta, dim3(1), dim3(BLOCK), 0, st, seg_start, huge, ht, meta);
  uint32_t hm[3];
  HIP_CHECK(hipMemcpyAsync(hm, meta, sizeof(hm), hipMemcpyDeviceToHost, st));
  if (int rw = stream_wait(st)) return rw;
  LAUNCH(k_sort_chunks<KEY>, dim3(hm[0]), dim3(1024), 0, st, carr, ht, sort_key);
  uint32_t* src = carr;
  uint32_t* dst = scratch;
  for (uint32_t w = LDS_SORT_MAX; w < hm[2]; w <<= 1) {
    LAUNCH(k_merge_pass<KEY>, dim3(hm[1]), dim3(BLOCK), 0, st, src, dst, ht, w, sort_key);
    std::swap(src, dst);
  }
  if (src != carr) LAUNCH(k_huge_copy, dim3(hm[1]), dim3(BLOCK), 0, st, src, carr, ht);
  return CRDTM_OK;
}

int segmented_sort(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items,
                   const long long* sort_key, Arena& ws, hipStream_t st, DevResult* dres) {
  return segmented_sort_t(seg_start, n_seg, carr, n_items, ArrKey{sort_key}, ws, st, dres, NONE);
}

int segmented_sort_skip(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items,
                        const long long* sort_key, Arena& ws, hipStream_t st, DevResult* dres, uint32_t skip) {
  return segmented_sort_t(seg_start, n_seg, carr, n_items, ArrKey{sort_key}, ws, st, dres, skip);
}

int segmented_sort_desc_id(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items, Arena& ws,
                           hipStream_t st, DevResult* dres, uint32_t skip) {
  return segmented_sort_t(seg_start, n_seg, carr, n_items, NegIdKey{}, ws, st, dres, skip);
}

int segmented_sort_asc_id(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items, Arena& ws,
                          hipStream_t st, DevResult* dres) {
  return segmented_sort_t(seg_start, n_seg, carr, n_items, IdKey{}, ws, st, dres, NONE);
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort of (u32 key, u32 value) pairs, 8 bits per pass. The
// item count may live on the device (n_dev: read by every kernel); the host
// gives an upper bound for the grid. Per pass: per-tile digit histograms
// (digit-major, so one exclusive scan gives every (digit, tile) its output
// base), then every tile ranks its items stably — within a wave by digit
// match masks from 8 ballots, across the workgroup's waves and rounds by
// LDS digit counters — and scatters them. No global atomics: a digit shared
// by many items costs nothing extra (counting sorts by parent pay a
// serialised device-scope atomic per item on a hot parent, ~12 ns each).
// ---------------------------------------------------------------------------
constexpr uint32_t RS_ITEMS = 8;
constexpr uint32_t RS_TILE = BLOCK * RS_ITEMS;

// The tiles that hold items: the host launches for n_max, the device count
// decides (the histogram is digit-major over these tiles only, so its scan
// and the launches past the items cost nothing when n is far below n_max).
__device__ __forceinline__ uint32_t rs_tiles(uint32_t n) { return n ? (n + RS_TILE - 1) / RS_TILE : 1u; }

__global__ void __launch_bounds__(BLOCK) k_rs_hist(const uint32_t* __restrict__ keys, const uint32_t* n_dev,
                                                   uint32_t shift, uint32_t* __restrict__ hist,
                                                   uint32_t* __restrict__ hn) {
  __shared__ uint32_t h[256];
  const uint32_t n = *n_dev;
  const uint32_t nt = rs_tiles(n);
  if (blockIdx.x == 0 && threadIdx.x == 0) *hn = 256 * nt;  // (the scan's device-side length)
  if (blockIdx.x >= nt) return;
  for (uint32_t j = threadIdx.x; j < 256; j += BLOCK) h[j] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RS_TILE;
  uint32_t k[RS_ITEMS];  // every load in flight before the first LDS atomic
#pragma unroll
  for (uint32_t j = 0; j < RS_ITEMS; ++j) {
    const uint32_t i = base + j * BLOCK + threadIdx.x;
    k[j] = i < n ? keys[i] : 0u;
  }
#pragma unroll
  for (uint32_t j = 0; j < RS_ITEMS; ++j)
    if (base + j * BLOCK + threadIdx.x < n) atomicAdd(&h[(k[j] >> shift) & 255u], 1u);
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < 256; d += BLOCK) hist[d * nt + blockIdx.x] = h[d];
}

__global__ void __launch_bounds__(BLOCK) k_rs_scatter(const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ vals, const uint32_t* n_dev,
                                                      uint32_t shift, const uint32_t* __restrict__ off,
                                                      uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                      uint32_t* __restrict__ inv) {
  constexpr uint32_t NW = BLOCK / 64;
  static_assert(BLOCK == 256, "one digit per thread in the prefix step");
  // per (row, wave, digit): the count of the wave's items of that digit in
  // that row, then (in place) their first output position
  __shared__ uint32_t wc[RS_ITEMS][NW][256];
  const uint32_t n = *n_dev;
  const uint32_t nt = rs_tiles(n);
  const uint32_t base = blockIdx.x * RS_TILE;
  if (base >= n) return;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned long long lt = (1ULL << lane) - 1ULL;
  uint32_t ka[RS_ITEMS], va[RS_ITEMS];  // the tile's items, all loads in flight first
#pragma unroll
  for (uint32_t j = 0; j < RS_ITEMS; ++j) {
    const uint32_t i = base + j * BLOCK + threadIdx.x;
    ka[j] = i < n ? keys[i] : 0u;
    va[j] = i < n ? vals[i] : 0u;
  }
  const uint32_t run0 = off[threadIdx.x * nt + blockIdx.x];  // (digit threadIdx.x: its tile's output base)
#pragma unroll
  for (uint32_t j = 0; j < RS_ITEMS; ++j)
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) wc[j][w][threadIdx.x] = 0;
  __syncthreads();
  // every row ranked at once: within a wave by digit match masks (8 ballots),
  // the leader of each digit present stores the wave's count
  uint32_t lr[RS_ITEMS];
#pragma unroll
  for (uint32_t j = 0; j < RS_ITEMS; ++j) {
    const bool valid = base + j * BLOCK + threadIdx.x < n;
    const uint32_t d = (ka[j] >> shift) & 255u;
    unsigned long long m = __ballot(valid);
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
      const unsigned long long bb = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bb : ~bb;
    }
    lr[j] = static_cast<uint32_t>(__popcll(m & lt));
    if (valid && lr[j] == 0) wc[j][wv][d] = static_cast<uint32_t>(__popcll(m));
  }
  __syncthreads();
  {  // thread = digit: exclusive prefix over (row, wave) in item order (stable)
    uint32_t run = run0;
#pragma unroll
    for (uint32_t j = 0; j < RS_ITEMS; ++j)
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w) {
        const uint32_t c = wc[j][w][threadIdx.x];
        wc[j][w][threadIdx.x] = run;
        run += c;
      }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < RS_ITEMS; ++j) {
    if (base + j * BLOCK + threadIdx.x >= n) continue;
    const uint32_t pos = wc[j][wv][(ka[j] >> shift) & 255u] + lr[j];
    kout[pos] = ka[j];
    vout[pos] = va[j];
    if (inv) inv[va[j]] = pos;
  }
}

// Sorts n_dev (<= n_max) pairs by the low `bits` bits of the keys, stably.
// The result lands in (k0, v0) when the pass count is even, else in (k1, v1):
// *out_k / *out_v point to it. inv (optional, values < n_max): inv[v] = the
// sorted position of value v, written by the last pass.
int radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, const uint32_t* n_dev, uint32_t n_max,
                     uint32_t bits, Arena& ws, hipStream_t st, uint32_t** out_k, uint32_t** out_v, uint32_t* inv) {
  const uint32_t ntiles = std::max<uint32_t>(1, (n_max + RS_TILE - 1) / RS_TILE);
  uint32_t* hist = ws.alloc<uint32_t>(256ULL * ntiles + 2);
  uint32_t* hn = hist + 256ULL * ntiles + 1;  // 256 x the tiles that hold items (device)
  uint32_t *ki = k0, *vi = v0, *ko = k1, *vo = v1;
  for (uint32_t shift = 0; shift < bits; shift += 8) {
    LAUNCH(k_rs_hist, dim3(ntiles), dim3(BLOCK), 0, st, ki, n_dev, shift, hist, hn);
    int r = dscan<SumOp, false>(ArrGen{hist}, hist, 256ULL * ntiles, nullptr, ws, st, nullptr, hn);
    if (r) return r;
    LAUNCH(k_rs_scatter, dim3(ntiles), dim3(BLOCK), 0, st, ki, vi, n_dev, shift, hist, ko, vo,
           shift + 8 >= bits ? inv : nullptr);
    std::swap(ki, ko);
    std::swap(vi, vo);
  }
  *out_k = ki;
  *out_v = vi;
  return CRDTM_OK;
}

struct FillArgs {
  void* p[FillList::MAX];
  uint64_t bytes[FillList::MAX];
  uint32_t pat[FillList::MAX];
};
// region blockIdx.y: 16-byte stores over its aligned body, 4-byte stores
// for the unaligned head words, bytes for the tail
__global__ void __launch_bounds__(BLOCK) k_fill_batch(FillArgs a) {
  const uint32_t j = blockIdx.y;
  char* p = static_cast<char*>(a.p[j]);
  const uint64_t nb = a.bytes[j];
  const uint32_t v = a.pat[j];
  const uint64_t head = ((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) < nb
                            ? ((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) : (nb & ~3ULL);
  const uint64_t n16 = (nb - head) / 16;
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x, ts = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint4* b16 = reinterpret_cast<uint4*>(p + head);
  for (uint64_t i = t0; i < n16; i += ts) b16[i] = make_uint4(v, v, v, v);
  if (t0 < head / 4) reinterpret_cast<uint32_t*>(p)[t0] = v;
  const uint64_t done = head + 16 * n16;
  if (t0 < nb - done) {  // (< 16 tail bytes)
    const uint64_t q = done + t0;
    p[q] = static_cast<char>(v >> (8 * (q & 3)));
  }
}

int FillList::launch(hipStream_t s) {
  if (overflow || n > MAX) {
    n = 0;
    overflow = false;
    return CRDTM_E_ARG;
  }
  if (n == 0) return CRDTM_OK;
  FillArgs a;
  uint64_t mx = 0;
  for (int k = 0; k < n; ++k) {
    if (reinterpret_cast<uintptr_t>(p[k]) & 3) return CRDTM_E_ARG;
    a.p[k] = p[k];
    a.bytes[k] = bytes[k];
    a.pat[k] = pat[k];
    mx = std::max(mx, bytes[k]);
  }
  const uint32_t gx = std::max<uint32_t>(1, std::min<uint64_t>(512, (mx / 16 + BLOCK - 1) / BLOCK));
  LAUNCH(k_fill_batch, dim3(gx, static_cast<uint32_t>(n)), dim3(BLOCK), 0, s, a);
  n = 0;
  return CRDTM_OK;
}

// One-workgroup radix sort for small batches (n <= RS_SMALL_MAX): the pairs
// stay in LDS for every pass (4-bit digits, 512 threads x 32 consecutive
// items): per pass each thread counts its items' digits, one workgroup scan
// over the digit-major [16][512] counts gives every thread its runs, and the
// items scatter back into LDS, stably. One launch instead of three per 8-bit
// pass (the multi-workgroup sort above is latency-bound at this size).
constexpr uint32_t RS_SMALL_T = 512, RS_SMALL_IPT = RS_SMALL_MAX / RS_SMALL_T;
static_assert(RS_SMALL_IPT == 32, "one pad word per thread's 32 items");
// (item i at word i + i / 32: a thread's 32 consecutive items sit in 32 banks)
__device__ __forceinline__ uint32_t rs_pad(uint32_t i) { return i + (i >> 5); }
constexpr uint32_t RS_SMALL_WORDS = RS_SMALL_MAX + RS_SMALL_MAX / 32;
// counts [digit][thread] as u16, one pad word per 64 (the scan reads 16
// consecutive counts per thread: without the pad, 16 lanes share a bank)
__device__ __forceinline__ uint32_t rs_cpad(uint32_t x) { return x + 2 * (x >> 6); }
constexpr uint32_t RS_SMALL_CNT = 16 * RS_SMALL_T + 2 * (16 * RS_SMALL_T / 64);
constexpr size_t RS_SMALL_LDS = 2 * RS_SMALL_WORDS * sizeof(uint32_t) + RS_SMALL_CNT * sizeof(uint16_t);

__global__ void __launch_bounds__(RS_SMALL_T) k_rs_small(const uint32_t* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin, uint32_t n, uint32_t bits,
                                                         uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  extern __shared__ uint32_t rs_small_lds[];
  uint32_t* sk = rs_small_lds;
  uint32_t* sv = sk + RS_SMALL_WORDS;
  uint16_t* cnt = reinterpret_cast<uint16_t*>(sv + RS_SMALL_WORDS);  // [digit][thread]
  __shared__ uint32_t wsum[RS_SMALL_T / 64];
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  {  // every global load in flight before the first LDS store
    uint32_t k0[RS_SMALL_IPT], v0[RS_SMALL_IPT];
#pragma unroll
    for (uint32_t j = 0; j < RS_SMALL_IPT; ++j) {
      const uint32_t i = t + j * RS_SMALL_T;
      k0[j] = i < n ? kin[i] : 0xFFFFFFFFu;  // padding: digit 15 in every pass, after every item
      v0[j] = i < n ? vin[i] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < RS_SMALL_IPT; ++j) {
      sk[rs_pad(t + j * RS_SMALL_T)] = k0[j];
      sv[rs_pad(t + j * RS_SMALL_T)] = v0[j];
    }
  }
  __syncthreads();
  for (uint32_t shift = 0; shift < bits; shift += 4) {
    uint32_t k[RS_SMALL_IPT], v[RS_SMALL_IPT];
    unsigned long long c0 = 0, c1 = 0;  // 8-bit counters of digits 0-7 / 8-15
#pragma unroll
    for (uint32_t j = 0; j < RS_SMALL_IPT; ++j) {
      k[j] = sk[t * (RS_SMALL_IPT + 1) + j];
      v[j] = sv[t * (RS_SMALL_IPT + 1) + j];
      const uint32_t d = (k[j] >> shift) & 15u;
      if (d < 8) c0 += 1ULL << (8 * d);
      else c1 += 1ULL << (8 * (d - 8));
    }
#pragma unroll
    for (uint32_t d = 0; d < 16; ++d)
      cnt[rs_cpad(d * RS_SMALL_T + t)] = static_cast<uint16_t>(((d < 8 ? c0 : c1) >> (8 * (d & 7))) & 0xFFu);
    __syncthreads();
    // exclusive scan of cnt in digit-major order: thread t owns entries [16 t, 16 t + 16)
    uint32_t loc[16], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      loc[j] = sum;
      sum += cnt[rs_cpad(t * 16 + j)];
    }
    const uint32_t inc = wave_incl_scan(sum);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = inc - sum;
    for (uint32_t w = 0; w < wv; ++w) pre += wsum[w];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) cnt[rs_cpad(t * 16 + j)] = static_cast<uint16_t>(pre + loc[j]);
    __syncthreads();
    // scatter (every thread holds its items: the arrays are free); an item's
    // place = its digit's run start for this thread + the thread's earlier
    // items of that digit (packed 8-bit running counts)
    // (every run start read before the first store: the stores would order the loads)
    uint32_t q[RS_SMALL_IPT];
#pragma unroll
    for (uint32_t j = 0; j < RS_SMALL_IPT; ++j) q[j] = cnt[rs_cpad(((k[j] >> shift) & 15u) * RS_SMALL_T + t)];
    unsigned long long r0 = 0, r1 = 0;
#pragma unroll
    for (uint32_t j = 0; j < RS_SMALL_IPT; ++j) {
      const uint32_t d = (k[j] >> shift) & 15u;
      const uint32_t sh = 8 * (d & 7);
      const uint32_t before = static_cast<uint32_t>(((d < 8 ? r0 : r1) >> sh) & 0xFFu);
      if (d < 8) r0 += 1ULL << sh;
      else r1 += 1ULL << sh;
      q[j] = rs_pad(q[j] + before);
    }
#pragma unroll
    for (uint32_t j = 0; j < RS_SMALL_IPT; ++j) {
      sk[q[j]] = k[j];
      sv[q[j]] = v[j];
    }
    __syncthreads();
  }
  for (uint32_t i = t; i < n; i += RS_SMALL_T) {
    kout[i] = sk[rs_pad(i)];
    vout[i] = sv[rs_pad(i)];
  }
}

// The same sort with 1024 threads x 16 items (four waves per SIMD to cover
// the LDS latency, half the items per thread and pass) for values below
// 2^16 (op indices of a batch of at most RS_SMALL_MAX): the values ride in
// LDS as u16, so keys, values and the [16][1024] counts fit the 160 KB.
constexpr uint32_t RS_W_T = 1024, RS_W_IPT = RS_SMALL_MAX / RS_W_T;
static_assert(RS_W_IPT == 16, "one pad word per thread's 16 items");
__device__ __forceinline__ uint32_t rs_wpad(uint32_t i) { return i + (i >> 4); }
constexpr uint32_t RS_W_WORDS = RS_SMALL_MAX + RS_SMALL_MAX / 16;
constexpr uint32_t RS_W_CNT = 16 * RS_W_T + 2 * (16 * RS_W_T / 64);
constexpr size_t RS_W_LDS = RS_W_WORDS * sizeof(uint32_t) + RS_W_WORDS * sizeof(uint16_t) + RS_W_CNT * sizeof(uint16_t);
static_assert(RS_W_LDS <= 160 * 1024, "fits the LDS");

__global__ void __launch_bounds__(RS_W_T) k_rs_small_w(const uint32_t* __restrict__ kin,
                                                       const uint32_t* __restrict__ vin, uint32_t n, uint32_t bits,
                                                       uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  extern __shared__ uint32_t rs_small_lds[];
  uint32_t* sk = rs_small_lds;
  uint16_t* sv = reinterpret_cast<uint16_t*>(sk + RS_W_WORDS);
  uint16_t* cnt = sv + RS_W_WORDS + (RS_W_WORDS & 1u);  // [digit][thread]
  __shared__ uint32_t wsum[RS_W_T / 64], wor[RS_W_T / 64], wand[RS_W_T / 64];
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t kor = 0, kand = 0xFFFFFFFFu;
  {
    uint32_t k0[RS_W_IPT], v0[RS_W_IPT];
#pragma unroll
    for (uint32_t j = 0; j < RS_W_IPT; ++j) {
      const uint32_t i = t + j * RS_W_T;
      k0[j] = i < n ? kin[i] : 0u;
      v0[j] = i < n ? vin[i] : 0u;
      if (i < n) {
        kor |= k0[j];
        kand &= k0[j];
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < RS_W_IPT; ++j) {
      if (t + j * RS_W_T < n) {
        sk[rs_wpad(t + j * RS_W_T)] = k0[j];
        sv[rs_wpad(t + j * RS_W_T)] = static_cast<uint16_t>(v0[j]);
      }
    }
  }
  // the bits where the keys differ (OR ^ AND): a digit every key shares
  // needs no pass (a batch typed into one gap: none at all)
  for (uint32_t d = 32; d > 0; d >>= 1) {
    kor |= __shfl_xor(kor, d);
    kand &= __shfl_xor(kand, d);
  }
  if (lane == 0) {
    wor[wv] = kor;
    wand[wv] = kand;
  }
  __syncthreads();
  kor = 0;
  kand = 0xFFFFFFFFu;
#pragma unroll
  for (uint32_t w = 0; w < RS_W_T / 64; ++w) {
    kor |= wor[w];
    kand &= wand[w];
  }
  const uint32_t diff = kor ^ kand;
  // (the items fill positions [0, n) before and after every pass: a thread's
  // blocked positions past n hold nothing and count nothing)
  const uint32_t nj = n > t * RS_W_IPT ? min(RS_W_IPT, n - t * RS_W_IPT) : 0u;
  for (uint32_t shift = 0; shift < bits; shift += 4) {
    if (!((diff >> shift) & 15u)) continue;  // (block-uniform; the padding stays last)
    uint32_t k[RS_W_IPT], v[RS_W_IPT];
    unsigned long long c0 = 0, c1 = 0;  // 8-bit counters of digits 0-7 / 8-15
#pragma unroll
    for (uint32_t j = 0; j < RS_W_IPT; ++j) {
      k[j] = j < nj ? sk[t * (RS_W_IPT + 1) + j] : 0u;
      v[j] = j < nj ? sv[t * (RS_W_IPT + 1) + j] : 0u;
      const uint32_t d = (k[j] >> shift) & 15u;
      if (j >= nj) continue;
      if (d < 8) c0 += 1ULL << (8 * d);
      else c1 += 1ULL << (8 * (d - 8));
    }
#pragma unroll
    for (uint32_t d = 0; d < 16; ++d)
      cnt[rs_cpad(d * RS_W_T + t)] = static_cast<uint16_t>(((d < 8 ? c0 : c1) >> (8 * (d & 7))) & 0xFFu);
    __syncthreads();
    uint32_t loc[16], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      loc[j] = sum;
      sum += cnt[rs_cpad(t * 16 + j)];
    }
    const uint32_t inc = wave_incl_scan(sum);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = inc - sum;
    for (uint32_t w = 0; w < wv; ++w) pre += wsum[w];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) cnt[rs_cpad(t * 16 + j)] = static_cast<uint16_t>(pre + loc[j]);
    __syncthreads();
    uint32_t q[RS_W_IPT];
#pragma unroll
    for (uint32_t j = 0; j < RS_W_IPT; ++j) q[j] = cnt[rs_cpad(((k[j] >> shift) & 15u) * RS_W_T + t)];
    unsigned long long r0 = 0, r1 = 0;
#pragma unroll
    for (uint32_t j = 0; j < RS_W_IPT; ++j) {
      const uint32_t d = (k[j] >> shift) & 15u;
      const uint32_t sh = 8 * (d & 7);
      const uint32_t before = static_cast<uint32_t>(((d < 8 ? r0 : r1) >> sh) & 0xFFu);
      if (d < 8) r0 += 1ULL << sh;
      else r1 += 1ULL << sh;
      q[j] = rs_wpad(q[j] + before);
    }
#pragma unroll
    for (uint32_t j = 0; j < RS_W_IPT; ++j) {
      if (j < nj) {
        sk[q[j]] = k[j];
        sv[q[j]] = static_cast<uint16_t>(v[j]);
      }
    }
    __syncthreads();
  }
  for (uint32_t i = t; i < n; i += RS_W_T) {
    kout[i] = sk[rs_wpad(i)];
    vout[i] = sv[rs_wpad(i)];
  }
}

// The same sort over many workgroups in two launches: each chunk of 1,024
// pairs sorts its (key << 16 | value) words in LDS (a bitonic network: the
// words are distinct, so the order is total), then every pair's place is its
// place in its chunk plus, per other chunk, the words below its own (16
// lanes per pair, one binary search each over L2-resident chunks). Ties of
// key go by value: the stable order when the values are the input positions
// (the caller's op indices).
constexpr uint32_t RS_C_CHUNK = 1024, RS_C_T = RS_C_CHUNK / 2, RS_C_MAXCH = RS_SMALL_MAX / RS_C_CHUNK;
static_assert(RS_C_MAXCH == 16, "one lane of a 16-lane group per chunk");

__global__ void __launch_bounds__(RS_C_T) k_rs_chunk(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                     uint32_t n, unsigned long long* __restrict__ cw) {
  __shared__ unsigned long long w[RS_C_CHUNK];
  const uint32_t t = threadIdx.x, c0 = blockIdx.x * RS_C_CHUNK;
#pragma unroll
  for (uint32_t u = 0; u < 2; ++u) {
    const uint32_t i = c0 + t + u * RS_C_T;
    w[t + u * RS_C_T] = i < n ? (static_cast<unsigned long long>(kin[i]) << 16) | (vin[i] & 0xFFFFu) : ~0ULL;
  }
  // (a stage of distance j <= 64 keeps word e with the wave e / 128: between
  // two such stages the wave's own in-order LDS accesses suffice; a stage of
  // distance >= 128 crosses waves and takes the workgroup barrier around it)
  bool cross = true;  // (the load above)
  for (uint32_t k = 2; k <= RS_C_CHUNK; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      const bool cj = j >= 128;
      if (cross || cj) __syncthreads();
      else __builtin_amdgcn_wave_barrier();
      cross = cj;
      const uint32_t i = 2 * t - (t & (j - 1)), q = i + j;  // (bit j of i clear)
      const unsigned long long a = w[i], b = w[q];
      if ((a > b) == !(i & k)) {  // ascending where bit k of i is clear
        w[i] = b;
        w[q] = a;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t u = 0; u < 2; ++u) cw[c0 + t + u * RS_C_T] = w[t + u * RS_C_T];
}

__global__ void __launch_bounds__(BLOCK) k_rs_merge(const unsigned long long* __restrict__ cw, uint32_t n,
                                                     uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 4, m = threadIdx.x & 15;
  const uint32_t nch = (n + RS_C_CHUNK - 1) / RS_C_CHUNK;
  if (g >= nch * RS_C_CHUNK) return;  // (whole 16-lane groups)
  const unsigned long long c = cw[g];
  const uint32_t own = g / RS_C_CHUNK;
  uint32_t below = 0;
  if (m == own) {
    below = g % RS_C_CHUNK;
  } else if (m < nch) {
    const unsigned long long* v = cw + m * RS_C_CHUNK;
    uint32_t lo = 0, hi = RS_C_CHUNK;  // (the words < c: padding words are above every pair's)
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (v[mid] < c) lo = mid + 1;
      else hi = mid;
    }
    below = lo;
  }
#pragma unroll
  for (uint32_t o = 8; o > 0; o >>= 1) below += __shfl_xor(below, o, 16);
  if (m == 0 && c != ~0ULL) {
    kout[below] = static_cast<uint32_t>(c >> 16);
    vout[below] = static_cast<uint32_t>(c & 0xFFFFu);
  }
}

int radix_sort_small(const uint32_t* kin, const uint32_t* vin, uint32_t n, uint32_t bits, uint32_t* kout,
                     uint32_t* vout, hipStream_t st, unsigned long long* cw) {
  static const bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rs_small),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 static_cast<int>(RS_SMALL_LDS)) == hipSuccess;
  static const bool w_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rs_small_w),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               static_cast<int>(RS_W_LDS)) == hipSuccess;
  // CRDTM_RS_SMALL: "w" / "512" select the one-workgroup kernels (A/B)
  static const char* sel = getenv("CRDTM_RS_SMALL");
  static const bool wide = !(sel && !strcmp(sel, "512"));
  static const bool chunked = !sel || !*sel;
  if (n > RS_SMALL_MAX) return CRDTM_E_HIP;
  if (!n) return CRDTM_OK;
  if (chunked && cw) {
    const uint32_t nch = (n + RS_C_CHUNK - 1) / RS_C_CHUNK;
    LAUNCH(k_rs_chunk, dim3(nch), dim3(RS_C_T), 0, st, kin, vin, n, cw);
    LAUNCH(k_rs_merge, dim3((nch * RS_C_CHUNK * 16 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, cw, n, kout, vout);
    return CRDTM_OK;
  }
  if (wide && w_ok) {  // (the caller's values are op indices of the batch: below n <= 2^14)
    LAUNCH(k_rs_small_w, dim3(1), dim3(RS_W_T), RS_W_LDS, st, kin, vin, n, bits, kout, vout);
    return CRDTM_OK;
  }
  if (!lds_ok) return CRDTM_E_HIP;
  LAUNCH(k_rs_small, dim3(1), dim3(RS_SMALL_T), RS_SMALL_LDS, st, kin, vin, n, bits, kout, vout);
  return CRDTM_OK;
}

// ---------------------------------------------------------------------------
// List ranking (north-star kernel 4). Level 0 input: ent[e] = {succ, wbits}
// (succ: NONE = end of list, ABSENT = not in any list; wbits bit1 -> high
// word +1, bit0 -> low word +1). Output: excl[e] = sum of the weights of the
// entries before e along the list from `head` (~0 for entries not on it).
//
// Sublist method with deterministic splitters: index block b (2^kbits
// entries) nominates one hashed candidate; present candidates (plus the head)
// walk their sublist, each step one 8-byte load. The reduced list (one entry
// per block, + the head) is ranked recursively, serially once it is short,
// and a last pass adds each splitter's prefix to its sublist. No atomics.
// ---------------------------------------------------------------------------
constexpr uint64_t LR_SERIAL = 64;

__host__ __device__ __forceinline__ uint64_t lr_cand(uint64_t b, uint32_t kbits) {
  return (b << kbits) + (mix64(b * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL) & ((1ULL << kbits) - 1));
}


template <bool PACKED>
__global__ void __launch_bounds__(BLOCK) k_lr_walk(const uint2* __restrict__ ent, const uint32_t* __restrict__ succ,
                                                   const unsigned long long* __restrict__ w, uint64_t n,
                                                   uint32_t kbits, uint32_t head, uint64_t head_id, uint64_t nb,
                                                   uint4* __restrict__ ol, uint32_t* __restrict__ red_succ,
                                                   unsigned long long* __restrict__ red_w) {
  for (uint64_t id = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; id <= nb;
       id += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    uint64_t e;
    if (id == nb) {
      if (head_id != nb) { red_succ[id] = ABSENT; continue; }
      e = head;
    } else {
      e = lr_cand(id, kbits);
      const uint32_t s0 = e < n ? (PACKED ? ent[e].x : succ[e]) : ABSENT;
      if (s0 == ABSENT) { red_succ[id] = ABSENT; continue; }
    }
    uint32_t cur = static_cast<uint32_t>(e);
    unsigned long long acc = 0;
    uint32_t nxt;
    for (uint64_t steps = 0;; ++steps) {
      unsigned long long wc;
      if (PACKED) {
        const uint2 x = ent[cur];
        nxt = x.x;
        wc = lr_weight(x.y);
      } else {
        nxt = succ[cur];
        wc = w[cur];
      }
      // owner and local prefix as one 16-byte record: one line per visited
      // entry instead of one in each of two arrays
      ol[cur] = make_uint4(static_cast<uint32_t>(id), static_cast<uint32_t>(acc), static_cast<uint32_t>(acc >> 32), 0u);
      acc += wc;
      if (nxt >= n || steps > n) { nxt = NONE; break; }  // end (cycle guard never taken on a valid list)
      if (nxt == lr_cand(nxt >> kbits, kbits)) break;      // next splitter
      cur = nxt;
    }
    red_w[id] = acc;
    red_succ[id] = nxt == NONE ? NONE : (nxt >> kbits);
  }
}

// Serial ranking of a short list by one lane.
__global__ void k_lr_serial(const uint32_t* __restrict__ succ, const unsigned long long* __restrict__ w,
                            uint64_t head, unsigned long long* __restrict__ excl, uint64_t n_entries) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t cur = head;
  unsigned long long acc = 0;
  for (uint64_t steps = 0; cur < n_entries && steps <= n_entries; ++steps) {
    excl[cur] = acc;
    acc += w[cur];
    cur = succ[cur];
  }
}

// An entry marked ABSENT is on no list (~0); every other entry lies on the
// one list from the head (an Euler tour of a tree; a reduced list of its
// sublists), so its walk record was written.
__global__ void __launch_bounds__(BLOCK) k_lr_apply(uint64_t n, const uint2* __restrict__ ent,
                                                    const uint32_t* __restrict__ succ, const uint4* __restrict__ ol,
                                                    uint64_t nb, const unsigned long long* __restrict__ red_excl,
                                                    unsigned long long* __restrict__ excl) {
  for (uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; e < n;
       e += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t s = ent ? ent[e].x : succ[e];
    if (s == ABSENT) {
      excl[e] = ~0ULL;
      continue;
    }
    const uint4 r = ol[e];
    excl[e] = r.x <= nb ? red_excl[r.x] + (static_cast<unsigned long long>(r.z) << 32 | r.y) : ~0ULL;
  }
}

static int list_rank_level(const uint2* ent, const uint32_t* succ, const unsigned long long* w, uint64_t n,
                           uint32_t head, unsigned long long* excl, Arena& ws, hipStream_t st, int level) {
  const uint32_t kbits = level == 0 ? 4u : 3u;
  const uint64_t nb = (n + (1ULL << kbits) - 1) >> kbits;
  const uint64_t head_id = (lr_cand(head >> kbits, kbits) == head) ? (head >> kbits) : nb;
  uint4* ol = ws.alloc<uint4>(n);
  uint32_t* red_succ = ws.alloc<uint32_t>(nb + 1);
  unsigned long long* red_w = ws.alloc<unsigned long long>(nb + 1);
  unsigned long long* red_excl = ws.alloc<unsigned long long>(nb + 1);
  if (ent) {
    LAUNCH(k_lr_walk<true>, dim3(grid_for(nb + 1)), dim3(BLOCK), 0, st, ent, nullptr, nullptr, n, kbits, head,
           head_id, nb, ol, red_succ, red_w);
  } else {
    LAUNCH(k_lr_walk<false>, dim3(grid_for(nb + 1)), dim3(BLOCK), 0, st, nullptr, succ, w, n, kbits, head, head_id,
           nb, ol, red_succ, red_w);
  }
  if (nb + 1 <= LR_SERIAL || level >= 7) {
    LAUNCH(k_lr_serial, dim3(1), dim3(64), 0, st, red_succ, red_w, head_id, red_excl, nb + 1);
  } else {
    int r = list_rank_level(nullptr, red_succ, red_w, nb + 1, static_cast<uint32_t>(head_id), red_excl, ws, st,
                            level + 1);
    if (r) return r;
  }
  LAUNCH(k_lr_apply, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, ent, succ, ol, nb, red_excl, excl);
  return CRDTM_OK;
}

int list_rank_unpacked(const uint32_t* succ, const unsigned long long* w, uint64_t n, uint32_t head,
                       unsigned long long* excl, Arena& ws, hipStream_t st) {
  return list_rank_level(nullptr, succ, w, n, head, excl, ws, st, 1);
}

int list_rank_packed(const uint2* ent, uint64_t n, uint32_t head, unsigned long long* excl, Arena& ws,
                     hipStream_t st) {
  return list_rank_level(ent, nullptr, nullptr, n, head, excl, ws, st, 0);
}

int list_rank(const uint2* ent, uint64_t n, uint32_t head, unsigned long long* excl, Arena& ws, hipStream_t st) {
  return list_rank_fused(PackedSrc{ent}, n, head, ExclSink{excl}, ws, st);
}

}  // namespace crdtm

// Kernel microbenchmark hook (not part of the drop-in ABI, include/crdtm.h):
// the batch sort of radix_sort_small on caller device buffers, on a caller
// stream. which: 0 or 1 = 1024 threads, 2 = 512 threads, 3 = chunks + merge (the default; cw: n rounded up to
// 1,024 words of scratch).
extern "C" __attribute__((visibility("default"))) int crdtm_xbench_sort_small(const uint32_t* kin, const uint32_t* vin,
                                                                             uint32_t n, uint32_t bits, uint32_t* kout,
                                                                             uint32_t* vout, void* stream, int which,
                                                                             unsigned long long* cw) {
  static const bool set = [] {
    bool ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&crdtm::k_rs_small),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(crdtm::RS_SMALL_LDS)) == hipSuccess;
    ok &= hipFuncSetAttribute(reinterpret_cast<const void*>(&crdtm::k_rs_small_w),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(crdtm::RS_W_LDS)) == hipSuccess;
    return ok;
  }();
  if (!set || n > crdtm::RS_SMALL_MAX || !n) return CRDTM_E_HIP;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (which == 3) {
    const uint32_t nch = (n + crdtm::RS_C_CHUNK - 1) / crdtm::RS_C_CHUNK;
    hipLaunchKernelGGL(crdtm::k_rs_chunk, dim3(nch), dim3(crdtm::RS_C_T), 0, s, kin, vin, n, cw);
    hipLaunchKernelGGL(crdtm::k_rs_merge, dim3((nch * crdtm::RS_C_CHUNK * 16 + crdtm::BLOCK - 1) / crdtm::BLOCK),
                       dim3(crdtm::BLOCK), 0, s, cw, n, kout, vout);
  } else if (which <= 1)
    hipLaunchKernelGGL(crdtm::k_rs_small_w, dim3(1), dim3(crdtm::RS_W_T), crdtm::RS_W_LDS, s, kin, vin, n, bits,
                       kout, vout);
  else
    hipLaunchKernelGGL(crdtm::k_rs_small, dim3(1), dim3(crdtm::RS_SMALL_T), crdtm::RS_SMALL_LDS, s, kin, vin, n,
                       bits, kout, vout);
  return hipGetLastError() == hipSuccess ? CRDTM_OK : CRDTM_E_HIP;
}

// Kernel microbenchmark hook: host microseconds per launch of an empty
// kernel on `stream` (nullptr: a stream of its own), n launches after 100
// warm-up ones.
namespace crdtm {
__global__ void k_xbench_null(uint32_t x, uint32_t* out) {
  if (x == 0xFFFFFFFFu && threadIdx.x == 0) *out = x;
}
}  // namespace crdtm
extern "C" __attribute__((visibility("default"))) double crdtm_xbench_launch(void* stream, int n) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  bool own = false;
  if (!s) {
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -1.0;
    own = true;
  }
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(crdtm::k_xbench_null, dim3(64), dim3(256), 0, s, 0u, nullptr);
  if (hipStreamSynchronize(s) != hipSuccess) return -1.0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(crdtm::k_xbench_null, dim3(64), dim3(256), 0, s, 0u, nullptr);
  const auto t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(s);
  if (own) hipStreamDestroy(s);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

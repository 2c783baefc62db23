// primitives.hip — device-wide scan, segmented child sort and list ranking
// for the crdtm engine (gfx950: wave64, 256 CUs, 160 KiB LDS per CU).
//
// These are the building blocks of north-star kernels (2) segmented sibling
// sort and (4) Euler-tour list ranking. Everything is integer, HBM-bound work.

#include "engine.h"

namespace crdtm {

// ---------------------------------------------------------------------------
// Exclusive scan (u32), three-phase: per-block scan with block totals,
// recursive scan of totals, uniform add. 256 threads x 8 items per block.
// ---------------------------------------------------------------------------
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds_waves, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan(v);
  if (lane == 63) lds_waves[wave] = inc;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / 64; ++w) {
    uint32_t s = lds_waves[w];
    if (w < wave) wbase += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wbase + inc - v;
}

__global__ void __launch_bounds__(BLOCK) k_scan_tiles(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      uint32_t* __restrict__ tile_sums, uint64_t n) {
  __shared__ uint32_t lw[BLOCK / 64];
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    v[j] = (base + j < n) ? in[base + j] : 0u;
    s += v[j];
  }
  uint32_t tot;
  uint32_t ex = block_excl_scan(s, lw, &tot);
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    if (base + j < n) out[base + j] = ex;
    ex += v[j];
  }
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK) k_scan_add(uint32_t* __restrict__ out, const uint32_t* __restrict__ tile_off,
                                                    uint64_t n) {
  const uint32_t add = tile_off[blockIdx.x];
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j)
    if (base + j < n) out[base + j] += add;
}

__global__ void k_store_total(const uint32_t* in_last, const uint32_t* out_last, uint32_t* total) {
  *total = *in_last + *out_last;
}

// out[i] = sum(in[0..i)); *total (device) = sum(in). in may alias out.
int scan_excl_u32(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* total, Arena& ws, hipStream_t st) {
  if (n == 0) {
    if (total) HIP_CHECK(hipMemsetAsync(total, 0, sizeof(uint32_t), st));
    return CRDTM_OK;
  }
  const uint64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  uint32_t* sums = ws.alloc<uint32_t>(tiles + 1);
  // keep the last input element: `in` may alias `out`
  uint32_t* last_in = ws.alloc<uint32_t>(1);
  HIP_CHECK(hipMemcpyAsync(last_in, in + n - 1, sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
  LAUNCH(k_scan_tiles, dim3(static_cast<uint32_t>(tiles)), dim3(BLOCK), 0, st, in, out, sums, n);
  if (tiles > 1) {
    int r = scan_excl_u32(sums, sums, tiles, nullptr, ws, st);
    if (r) return r;
    LAUNCH(k_scan_add, dim3(static_cast<uint32_t>(tiles)), dim3(BLOCK), 0, st, out, sums, n);
  }
  if (total) LAUNCH(k_store_total, dim3(1), dim3(1), 0, st, last_in, out + n - 1, total);
  return CRDTM_OK;
}

// ---------------------------------------------------------------------------
// Segmented sort of children by key (ascending, unique keys per segment).
// seg_start[u]..seg_start[u+1) of carr; key(v) from sort_key[v].
// Small segments: one lane each (insertion sort). Large: one workgroup each,
// bitonic in LDS up to LDS_SORT_MAX, else a workgroup merge sort in HBM.
// ---------------------------------------------------------------------------
constexpr uint32_t SMALL_SEG = 16;
constexpr uint32_t LDS_SORT_MAX = 4096;

__global__ void __launch_bounds__(BLOCK) k_sort_small(const uint32_t* __restrict__ seg_start, uint32_t n_seg,
                                                      uint32_t* __restrict__ carr,
                                                      const long long* __restrict__ sort_key,
                                                      uint32_t* __restrict__ big_list, uint32_t* __restrict__ n_big) {
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < n_seg; u += gridDim.x * blockDim.x) {
    const uint32_t b = seg_start[u], e = seg_start[u + 1];
    const uint32_t len = e - b;
    if (len < 2) continue;
    if (len > SMALL_SEG) {
      big_list[atomicAdd(n_big, 1u)] = u;
      continue;
    }
    uint32_t ids[SMALL_SEG];
    long long keys[SMALL_SEG];
    for (uint32_t j = 0; j < len; ++j) {
      uint32_t v = carr[b + j];
      long long k = sort_key[v];
      uint32_t p = j;
      while (p > 0 && keys[p - 1] > k) {
        keys[p] = keys[p - 1];
        ids[p] = ids[p - 1];
        --p;
      }
      keys[p] = k;
      ids[p] = v;
    }
    for (uint32_t j = 0; j < len; ++j) carr[b + j] = ids[j];
  }
}

// One workgroup per large segment. Bitonic sort over the next power of two
// in LDS (keys padded with +inf) when it fits; otherwise an in-HBM merge sort
// with ping-pong through `scratch` (same offsets as carr).
__global__ void __launch_bounds__(1024) k_sort_big(const uint32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ big_list,
                                                    const uint32_t* __restrict__ n_big, uint32_t* __restrict__ carr,
                                                    uint32_t* __restrict__ scratch,
                                                    const long long* __restrict__ sort_key) {
  __shared__ long long skey[LDS_SORT_MAX];
  __shared__ uint32_t sid[LDS_SORT_MAX];
  const uint32_t nb = *n_big;
  for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
    const uint32_t u = big_list[bi];
    const uint32_t b = seg_start[u], len = seg_start[u + 1] - b;
    if (len <= LDS_SORT_MAX) {
      uint32_t p2 = 1;
      while (p2 < len) p2 <<= 1;
      for (uint32_t j = threadIdx.x; j < p2; j += blockDim.x) {
        if (j < len) {
          uint32_t v = carr[b + j];
          sid[j] = v;
          skey[j] = sort_key[v];
        } else {
          sid[j] = NONE;
          skey[j] = 0x7fffffffffffffffLL;
        }
      }
      __syncthreads();
      for (uint32_t k = 2; k <= p2; k <<= 1) {
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
          for (uint32_t i = threadIdx.x; i < p2; i += blockDim.x) {
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
      for (uint32_t j = threadIdx.x; j < len; j += blockDim.x) carr[b + j] = sid[j];
      __syncthreads();
    } else {
      // 1) sort runs of LDS_SORT_MAX in LDS
      for (uint32_t r0 = 0; r0 < len; r0 += LDS_SORT_MAX) {
        const uint32_t rl = min(LDS_SORT_MAX, len - r0);
        for (uint32_t j = threadIdx.x; j < LDS_SORT_MAX; j += blockDim.x) {
          if (j < rl) {
            uint32_t v = carr[b + r0 + j];
            sid[j] = v;
            skey[j] = sort_key[v];
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
        __syncthreads();
      }
      // 2) merge passes (merge-path partition per thread)
      uint32_t* src = carr + b;
      uint32_t* dst = scratch + b;
      for (uint32_t width = LDS_SORT_MAX; width < len; width <<= 1) {
        for (uint32_t m0 = 0; m0 < len; m0 += 2 * width) {
          const uint32_t a0 = m0, a1 = min(m0 + width, len), b1 = min(m0 + 2 * width, len);
          const uint32_t na = a1 - a0, nbb = b1 - a1, tot = na + nbb;
          const uint32_t per = (tot + blockDim.x - 1) / blockDim.x;
          const uint32_t d0 = min(threadIdx.x * per, tot), d1 = min(d0 + per, tot);
          // merge path: find i in A, j in B with i + j = d0
          uint32_t lo = d0 > nbb ? d0 - nbb : 0, hi = min(d0, na);
          while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (sort_key[src[a0 + mid]] < sort_key[src[a1 + d0 - mid - 1]]) lo = mid + 1;
            else hi = mid;
          }
          uint32_t i = lo, j = d0 - lo;
          for (uint32_t d = d0; d < d1; ++d) {
            bool takeA;
            if (i >= na) takeA = false;
            else if (j >= nbb) takeA = true;
            else takeA = sort_key[src[a0 + i]] < sort_key[src[a1 + j]];
            dst[m0 + d] = takeA ? src[a0 + i++] : src[a1 + j++];
          }
        }
        __syncthreads();
        uint32_t* t = src;
        src = dst;
        dst = t;
      }
      if (src != carr + b)
        for (uint32_t j = threadIdx.x; j < len; j += blockDim.x) carr[b + j] = src[j];
      __syncthreads();
    }
  }
}

int segmented_sort(const uint32_t* seg_start, uint32_t n_seg, uint32_t* carr, uint32_t n_items,
                   const long long* sort_key, Arena& ws, hipStream_t st, DevResult* dres) {
  uint32_t* big = ws.alloc<uint32_t>(n_seg + 1);
  uint32_t* nbig = &dres->big_segments;
  HIP_CHECK(hipMemsetAsync(nbig, 0, sizeof(uint32_t), st));
  LAUNCH(k_sort_small, dim3(grid_for(n_seg)), dim3(BLOCK), 0, st, seg_start, n_seg, carr, sort_key, big,
                     nbig);
  uint32_t* scratch = ws.alloc<uint32_t>(n_items + 1);
  LAUNCH(k_sort_big, dim3(512), dim3(1024), 0, st, seg_start, big, nbig, carr, scratch, sort_key);
  return CRDTM_OK;
}

// ---------------------------------------------------------------------------
// List ranking (north-star kernel 4). Input: succ[e] (NONE = end of list,
// ABSENT = not in any list), weight[e] (u64), head. Output: excl[e] = sum of
// weights of the entries before e along the list from head.
// Sublist method: the head (id 0) plus hashed splitters (~1/K of the entries)
// each walk their sublist; the reduced list of splitters (head id 0) is ranked
// recursively, serially once it is short; a last pass adds each splitter's
// prefix to the entries of its sublist.
// ---------------------------------------------------------------------------
constexpr uint64_t LR_SERIAL = 2048;

__global__ void k_lr_head(uint32_t head, uint32_t* split_entry, uint32_t* n_split) {
  split_entry[0] = head;
  *n_split = 1;
}

__global__ void __launch_bounds__(BLOCK) k_lr_pick(const uint32_t* __restrict__ succ, uint64_t n, uint32_t head,
                                                   uint32_t kmask, uint64_t cap, uint32_t* __restrict__ split_id,
                                                   uint32_t* __restrict__ split_entry, uint32_t* __restrict__ n_split) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t trips = (n + stride - 1) / stride;  // uniform trip count: wave_ticket needs every lane
  for (uint64_t t = 0; t < trips; ++t) {
    const uint64_t e = t * stride + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
    const bool in = e < n;
    const bool pick = in && e != head && succ[e] != ABSENT &&
                      (static_cast<uint32_t>(mix64(e * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL)) & kmask) == 0;
    const uint32_t tk = wave_ticket(n_split, pick);
    if (!in) continue;
    uint32_t id = NONE;
    if (e == head) {
      id = 0;
    } else if (pick && tk < cap) {
      id = tk;
      split_entry[tk] = static_cast<uint32_t>(e);
    }
    split_id[e] = id;
  }
}

__global__ void __launch_bounds__(BLOCK) k_lr_walk(const uint32_t* __restrict__ succ,
                                                   const unsigned long long* __restrict__ w,
                                                   const uint32_t* __restrict__ split_id,
                                                   const uint32_t* __restrict__ split_entry,
                                                   const uint32_t* __restrict__ n_split, uint64_t cap,
                                                   uint64_t n_entries, unsigned long long* __restrict__ local,
                                                   uint32_t* __restrict__ owner, uint32_t* __restrict__ red_succ,
                                                   unsigned long long* __restrict__ red_w) {
  const uint64_t ns = min(static_cast<uint64_t>(*n_split), cap);
  for (uint64_t id = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; id < cap;
       id += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    if (id >= ns) {
      red_succ[id] = ABSENT;
      continue;
    }
    uint32_t cur = split_entry[id];
    unsigned long long acc = 0;
    uint32_t nxt;
    for (uint64_t steps = 0;; ++steps) {
      if (steps > n_entries) { nxt = NONE; break; }  // cycle guard (never taken on a valid list)
      local[cur] = acc;
      owner[cur] = static_cast<uint32_t>(id);
      acc += w[cur];
      nxt = succ[cur];
      if (nxt >= n_entries) { nxt = NONE; break; }  // end (or a malformed link)
      if (split_id[nxt] != NONE) break;
      cur = nxt;
    }
    red_w[id] = acc;
    red_succ[id] = (nxt == NONE) ? NONE : split_id[nxt];
  }
}

// Serial ranking of a short list by one lane (head id 0).
__global__ void k_lr_serial(const uint32_t* __restrict__ succ, const unsigned long long* __restrict__ w,
                            unsigned long long* __restrict__ excl, uint64_t n_entries) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t cur = 0;
  unsigned long long acc = 0;
  for (uint64_t steps = 0; cur < n_entries && steps <= n_entries; ++steps) {
    excl[cur] = acc;
    acc += w[cur];
    cur = succ[cur];
  }
}

__global__ void __launch_bounds__(BLOCK) k_lr_apply(uint64_t n, const uint32_t* __restrict__ owner,
                                                    const unsigned long long* __restrict__ local,
                                                    const unsigned long long* __restrict__ red_excl,
                                                    unsigned long long* __restrict__ excl) {
  for (uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; e < n;
       e += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t o = owner[e];
    excl[e] = (o == NONE) ? ~0ULL : red_excl[o] + local[e];  // ~0: not on the list
  }
}

int list_rank(const uint32_t* succ, const unsigned long long* w, uint64_t n, uint32_t head,
              unsigned long long* excl, Arena& ws, hipStream_t st, DevResult* dres, int level) {
  const uint32_t kmask = level == 0 ? 31u : 15u;
  uint64_t cap = n / (kmask + 1) * 2 + 1024;
  if (cap > n) cap = n;
  uint32_t* split_id = ws.alloc<uint32_t>(n);
  uint32_t* split_entry = ws.alloc<uint32_t>(cap);
  uint32_t* owner = ws.alloc<uint32_t>(n);
  unsigned long long* local = ws.alloc<unsigned long long>(n);
  uint32_t* red_succ = ws.alloc<uint32_t>(cap);
  unsigned long long* red_w = ws.alloc<unsigned long long>(cap);
  unsigned long long* red_excl = ws.alloc<unsigned long long>(cap);
  uint32_t* nsp = &dres->n_split[level < 8 ? level : 7];
  HIP_CHECK(hipMemsetAsync(owner, 0xFF, n * sizeof(uint32_t), st));
  LAUNCH(k_lr_head, dim3(1), dim3(1), 0, st, head, split_entry, nsp);
  LAUNCH(k_lr_pick, dim3(grid_for(n, BLOCK, 4096)), dim3(BLOCK), 0, st, succ, n, head, kmask, cap, split_id,
                     split_entry, nsp);
  LAUNCH(k_lr_walk, dim3(grid_for(cap)), dim3(BLOCK), 0, st, succ, w, split_id, split_entry, nsp, cap,
                     n, local, owner, red_succ, red_w);
  if (cap <= LR_SERIAL || level >= 7) {
    LAUNCH(k_lr_serial, dim3(1), dim3(64), 0, st, red_succ, red_w, red_excl, cap);
  } else {
    int r = list_rank(red_succ, red_w, cap, 0u, red_excl, ws, st, dres, level + 1);
    if (r) return r;
  }
  LAUNCH(k_lr_apply, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, owner, local, red_excl, excl);
  return CRDTM_OK;
}

}  // namespace crdtm

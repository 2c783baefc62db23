// listrank.h — list ranking front end with local contraction, templated on
// where the list entries come from (SRC) and where the ranks go (SINK), so a
// caller can build its list on the fly and consume ranks without
// materialising either array.
//
// SRC:  __device__ uint2 operator()(uint64_t e) const -> {succ, wbits}
//       (succ: NONE = end of list, ABSENT = entry not in any list;
//        wbits bit1 -> high word +1, bit0 -> low word +1)
// SINK: __device__ void operator()(uint64_t e, unsigned long long rank) const,
//       called once for every entry on the list (rank = exclusive prefix of
//       the weights along the list from `head`). ExclSink also writes ~0 for
//       entries off the list.
#pragma once

#include <cstdio>
#include <cstdlib>

#include "engine.h"

namespace crdtm {

__device__ __forceinline__ unsigned long long lr_weight(uint32_t wbits) {
  return (static_cast<unsigned long long>((wbits >> 1) & 1u) << 32) | (wbits & 1u);
}

struct PackedSrc {
  const uint2* ent;
  __device__ __forceinline__ uint2 operator()(uint64_t e) const { return ent[e]; }
};

struct ExclSink {
  unsigned long long* excl;
  static constexpr bool kOffList = true;  // also told about entries off the list
  __device__ __forceinline__ void operator()(uint64_t e, unsigned long long r) const { excl[e] = r; }
};

// ---------------------------------------------------------------------------
// Local contraction. Lists built over slot numbering have strong memory
// locality: a typing run's Euler entries are consecutive. A workgroup takes
// a tile of LC_T consecutive entries, finds the pieces of the list that stay
// inside the tile (local chains) by pointer jumping in LDS, and emits one
// contracted node per local chain (weight = chain total, successor = the
// chain that follows its tail). The contracted list is ranked by the
// sublist method; each entry's rank = its chain's rank + its prefix inside
// the chain. A cycle inside a tile (never on a valid list) leaves its
// entries unranked, like entries off the list.
// ---------------------------------------------------------------------------
constexpr uint32_t LC_LOG = 10;
constexpr uint32_t LC_T = 1u << LC_LOG;
static_assert(LC_T < 0xFFFFu, "tile-local chain ids and prefixes are 16-bit");
constexpr uint32_t LC_PER = LC_T / BLOCK;
constexpr uint64_t LC_MIN = 1ULL << 16;  // shorter lists: sublist method on a materialised list

// Inside a tile both weight counters stay below 2^16, so a weight travels as
// one 32-bit word {tour nodes:16 | visible:16} (the halves never carry).
__device__ __forceinline__ uint32_t lc_pw(uint32_t wbits) { return (((wbits >> 1) & 1u) << 16) | (wbits & 1u); }
__device__ __forceinline__ unsigned long long lc_unpack(uint32_t pw) {
  return (static_cast<unsigned long long>(pw >> 16) << 32) | (pw & 0xFFFFu);
}
constexpr uint16_t LC_NONE = 0xFFFFu;

// Contraction of one tile. Outputs: hidx[e] = the tile-local index of e's
// chain (LC_NONE: off every list), pre[e] = e's packed prefix inside its chain,
// tcnt[tile] = chains in the tile; per chain, at sparse position
// tile * LC_T + local: the successor entry of its tail (sp_succ) and its
// total weight (sp_w). No global atomics: chain ids become dense after a
// scan of tcnt (k_lc_link).
template <class SRC>
__global__ void __launch_bounds__(BLOCK) k_lc_contract(SRC srcf, uint64_t n, uint16_t* __restrict__ hidx,
                                                       uint32_t* __restrict__ pre,
                                                       uint32_t* __restrict__ tcnt, uint32_t* __restrict__ sp_succ,
                                                       unsigned long long* __restrict__ sp_w) {
  __shared__ uint32_t P[LC_T];
  __shared__ uint32_t V[LC_T];
  __shared__ uint32_t W[LC_T];
  __shared__ uint32_t sw[BLOCK / 64];
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * LC_T;
#pragma unroll
  for (uint32_t k = 0; k < LC_PER; ++k) P[threadIdx.x + k * BLOCK] = NONE;
  __syncthreads();
  uint32_t sc[LC_PER];
#pragma unroll
  for (uint32_t k = 0; k < LC_PER; ++k) {
    const uint32_t l = threadIdx.x + k * BLOCK;
    const uint64_t e = base + l;
    const uint2 x = e < n ? srcf(e) : make_uint2(ABSENT, 0u);
    sc[k] = x.x;
    W[l] = x.y;
    if (x.x < n && x.x >= base && x.x < base + LC_T) P[x.x - base] = l;  // my successor's local predecessor
  }
  __syncthreads();
  uint32_t p[LC_PER];
  uint32_t v[LC_PER];
#pragma unroll
  for (uint32_t k = 0; k < LC_PER; ++k) {
    const uint32_t l = threadIdx.x + k * BLOCK;
    p[k] = P[l];
    v[k] = p[k] != NONE ? lc_pw(W[p[k]]) : 0u;
    V[l] = v[k];
  }
  __syncthreads();
  // Wyllie pointer jumping toward the chain head (<= log2(LC_T) rounds)
  for (uint32_t round = 0; round <= LC_LOG; ++round) {
    bool ch = false;
#pragma unroll
    for (uint32_t k = 0; k < LC_PER; ++k) {
      if (p[k] == NONE) continue;
      const uint32_t pp = P[p[k]];
      if (pp != NONE) {
        v[k] += V[p[k]];
        p[k] = pp;
        ch = true;
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < LC_PER; ++k) {
      const uint32_t l = threadIdx.x + k * BLOCK;
      P[l] = p[k];
      V[l] = v[k];
    }
    if (!__syncthreads_or(ch)) break;
  }
  // heads: present entries without a local predecessor, numbered in the tile
  uint32_t nh = 0;
  bool head[LC_PER], cyc[LC_PER];
#pragma unroll
  for (uint32_t k = 0; k < LC_PER; ++k) {
    const bool present = sc[k] != ABSENT;
    cyc[k] = present && p[k] != NONE && P[p[k]] != NONE;  // still jumping: a cycle
    head[k] = present && p[k] == NONE;
    nh += head[k] ? 1u : 0u;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(nh);
  if (lane == 63) sw[wave] = inc;
  __syncthreads();
  uint32_t off = inc - nh, tot = 0;
  for (int w = 0; w < BLOCK / 64; ++w) {
    if (w < wave) off += sw[w];
    tot += sw[w];
  }
  if (threadIdx.x == 0) tcnt[blockIdx.x] = tot;
#pragma unroll
  for (uint32_t k = 0; k < LC_PER; ++k) {
    if (head[k]) P[threadIdx.x + k * BLOCK] = off++;  // P[head] := its tile-local chain id
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < LC_PER; ++k) {
    const uint32_t l = threadIdx.x + k * BLOCK;
    const uint64_t e = base + l;
    if (e >= n) continue;
    if (sc[k] == ABSENT || cyc[k]) {
      hidx[e] = LC_NONE;
      continue;
    }
    const uint32_t h = P[head[k] ? l : p[k]];
    hidx[e] = static_cast<uint16_t>(h);
    pre[e] = v[k];
    const uint32_t s = sc[k];
    if (!(s < n && s >= base && s < base + LC_T)) {  // tail of its local chain
      sp_w[base + h] = lc_unpack(v[k] + lc_pw(W[l]));
      sp_succ[base + h] = s;  // entry id of the next chain's head (or NONE)
    }
  }
}

// Dense contracted list: chain (tile t, local h) -> toff[t] + h; its
// successor is the chain headed by entry s, i.e. toff[s / LC_T] + hidx[s].
static __global__ void __launch_bounds__(BLOCK) k_lc_link(const uint32_t* __restrict__ toff,
                                                          const uint16_t* __restrict__ hidx,
                                                          const uint32_t* __restrict__ sp_succ,
                                                          const unsigned long long* __restrict__ sp_w,
                                                          uint32_t* __restrict__ rsucc,
                                                          unsigned long long* __restrict__ rw) {
  const uint32_t t = blockIdx.x;
  const uint32_t b = toff[t], cnt = toff[t + 1] - b;
  const uint64_t base = static_cast<uint64_t>(t) * LC_T;
  for (uint32_t h = threadIdx.x; h < cnt; h += blockDim.x) {
    const uint32_t s = sp_succ[base + h];
    rsucc[b + h] = s == NONE ? NONE : toff[s / LC_T] + hidx[s];
    rw[b + h] = sp_w[base + h];
  }
}

// {contracted list length, contracted id of the list head} in one word pair
static __global__ void k_lc_meta(const uint32_t* toff, uint32_t tiles, const uint16_t* hidx, uint32_t head,
                                 uint32_t* meta) {
  meta[0] = toff[tiles];
  const uint32_t h = hidx[head];
  meta[1] = h == LC_NONE ? NONE : toff[head / LC_T] + h;
}

template <class SINK>
__global__ void __launch_bounds__(BLOCK) k_lc_expand(uint64_t n, const uint32_t* __restrict__ toff,
                                                     const uint16_t* __restrict__ hidx,
                                                     const uint32_t* __restrict__ pre,
                                                     const unsigned long long* __restrict__ rexcl, SINK sink) {
  for (uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; e < n;
       e += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t h = hidx[e];
    const unsigned long long b = h != LC_NONE ? rexcl[toff[e / LC_T] + h] : ~0ULL;
    if (b != ~0ULL) sink(e, b + lc_unpack(pre[e]));
    else if (SINK::kOffList) sink(e, ~0ULL);
  }
}

template <class SRC>
__global__ void __launch_bounds__(BLOCK) k_lr_materialise(SRC srcf, uint64_t n, uint2* ent) {
  for (uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; e < n;
       e += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    ent[e] = srcf(e);
}

template <class SINK>
__global__ void __launch_bounds__(BLOCK) k_lr_sink(uint64_t n, const unsigned long long* __restrict__ excl,
                                                   SINK sink) {
  for (uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; e < n;
       e += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const unsigned long long r = excl[e];
    if (r != ~0ULL || SINK::kOffList) sink(e, r);
  }
}

template <class SRC, class SINK>
int list_rank_fused(SRC srcf, uint64_t n, uint32_t head, SINK sink, Arena& ws, hipStream_t st) {
  if (n < LC_MIN || n >= 0xFFFFFFF0ULL) {
    uint2* ent = ws.alloc<uint2>(n);
    unsigned long long* excl = ws.alloc<unsigned long long>(n);
    LAUNCH(k_lr_materialise<SRC>, dim3(grid_for(n)), dim3(BLOCK), 0, st, srcf, n, ent);
    int r = list_rank_packed(ent, n, head, excl, ws, st);
    if (r) return r;
    LAUNCH(k_lr_sink<SINK>, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, excl, sink);
    return CRDTM_OK;
  }
  const uint64_t tiles = (n + LC_T - 1) / LC_T;
  uint16_t* hidx = ws.alloc<uint16_t>(n);
  uint32_t* pre = ws.alloc<uint32_t>(n);
  uint32_t* sp_succ = ws.alloc<uint32_t>(tiles * LC_T);
  unsigned long long* sp_w = ws.alloc<unsigned long long>(tiles * LC_T);
  uint32_t* toff = ws.alloc<uint32_t>(tiles + 1);
  LAUNCH(k_lc_contract<SRC>, dim3(static_cast<uint32_t>(tiles)), dim3(BLOCK), 0, st, srcf, n, hidx, pre, toff,
         sp_succ, sp_w);
  HIP_CHECK(hipMemsetAsync(toff + tiles, 0, sizeof(uint32_t), st));
  int r = scan_excl_u32(toff, toff, tiles + 1, nullptr, ws, st);
  if (r) return r;
  uint32_t* meta = ws.alloc<uint32_t>(2);
  LAUNCH(k_lc_meta, dim3(1), dim3(1), 0, st, toff, static_cast<uint32_t>(tiles), hidx, head, meta);
  uint32_t hv[2] = {0, NONE};
  HIP_CHECK(hipMemcpyAsync(hv, meta, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  uint32_t* rsucc = ws.alloc<uint32_t>(tiles * LC_T + 1);  // dense contracted list (H <= n)
  unsigned long long* rw = ws.alloc<unsigned long long>(tiles * LC_T + 1);
  LAUNCH(k_lc_link, dim3(static_cast<uint32_t>(tiles)), dim3(BLOCK), 0, st, toff, hidx, sp_succ, sp_w, rsucc, rw);
  HIP_CHECK(hipStreamSynchronize(st));
  const uint32_t H = hv[0], rhead = hv[1];
  if (std::getenv("CRDTM_LR_STATS")) std::fprintf(stderr, "crdtm list ranking: %llu entries -> %u chains\n",
                                                  static_cast<unsigned long long>(n), H);
  unsigned long long* rexcl = ws.alloc<unsigned long long>(static_cast<uint64_t>(H) + 1);
  if (H == 0 || rhead == NONE) {
    HIP_CHECK(hipMemsetAsync(rexcl, 0xFF, (static_cast<uint64_t>(H) + 1) * sizeof(unsigned long long), st));
  } else {
    r = list_rank_unpacked(rsucc, rw, H, rhead, rexcl, ws, st);
    if (r) return r;
  }
  LAUNCH(k_lc_expand<SINK>, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, toff, hidx, pre, rexcl, sink);
  return CRDTM_OK;
}

}  // namespace crdtm

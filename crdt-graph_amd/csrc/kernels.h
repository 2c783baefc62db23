// kernels.h — device helpers shared by the crdtm kernels (gfx950, wave64).
#pragma once

#include "common.h"

namespace crdtm {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 33;
  z *= 0xff51afd7ed558ccdULL;
  z ^= z >> 33;
  z *= 0xc4ceb9fe1a85ec53ULL;
  z ^= z >> 33;
  return z;
}

// Streaming stores, for what no later pass of the merge reads back (the op
// log, the node records): vector stores with the non-temporal hint, so the
// hundreds of MB they stream do not displace the slot records the next
// passes re-read from the MALL. (Built with -DCRDTM_NT=0: plain stores.)
#ifndef CRDTM_NT
#define CRDTM_NT 1
#endif
#ifndef CRDTM_NT_NODES
#define CRDTM_NT_NODES 1
#endif
template <class T>
__device__ __forceinline__ void st_node(T* p, T v) {  // (the node records' stores)
#if CRDTM_NT && CRDTM_NT_NODES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
template <class T>
__device__ __forceinline__ void st_stream(T* p, T v) {
#if CRDTM_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void st_stream16(void* p, uint4 v) {
#if CRDTM_NT
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
#else
  *reinterpret_cast<uint4*>(p) = v;
#endif
}
__device__ __forceinline__ void st_stream16(void* p, longlong2 v) {
  st_stream16(p, make_uint4(static_cast<uint32_t>(v.x), static_cast<uint32_t>(static_cast<unsigned long long>(v.x) >> 32),
                            static_cast<uint32_t>(v.y), static_cast<uint32_t>(static_cast<unsigned long long>(v.y) >> 32)));
}
__device__ __forceinline__ void st_stream4(void* p, uchar4 v) {
  st_stream(reinterpret_cast<uint32_t*>(p), static_cast<uint32_t>(v.x) | (static_cast<uint32_t>(v.y) << 8) |
                                                (static_cast<uint32_t>(v.z) << 16) | (static_cast<uint32_t>(v.w) << 24));
}

// replicaId ts = ts // 2^32 with Elm/JS (a / b) | 0 truncation (src/CRDTree/Timestamp.elm:16-18)
__host__ __device__ __forceinline__ int64_t replica_of(int64_t ts) { return ts / TWO32; }

// word-wise FNV-1a over 64-bit words (the canonical document hashes)
struct Fnv {
  unsigned long long h = 1469598103934665603ULL, n = 0;
  __device__ void put(long long w) {
    h ^= static_cast<unsigned long long>(w);
    h *= 1099511628211ULL;
    ++n;
  }
};

// ---- ts -> first Add index (open addressing, linear probing). Keys are stored
// XOR INT64_MIN so that an all-zero memset means "empty".
struct TsHash {
  unsigned long long* keys;  // ts ^ INT64_MIN, 0 = empty
  uint32_t* vals;            // min op index, 0xFFFFFFFF = none
  uint32_t mask;
};

__device__ __forceinline__ void tshash_insert(TsHash h, int64_t ts, uint32_t idx) {
  const unsigned long long k = static_cast<unsigned long long>(ts) ^ 0x8000000000000000ULL;
  uint32_t p = static_cast<uint32_t>(mix64(k)) & h.mask;
  for (;;) {
    unsigned long long prev = atomicCAS(&h.keys[p], 0ULL, k);
    if (prev == 0ULL || prev == k) {
      atomicMin(&h.vals[p], idx);
      return;
    }
    p = (p + 1) & h.mask;
  }
}

// the same from a first slot p whose key kk the caller has loaded (k: the
// stored form of the timestamp, ts ^ 2^63)
__device__ __forceinline__ uint32_t tshash_find_from(TsHash h, unsigned long long k, uint32_t p,
                                                     unsigned long long kk) {
  for (;;) {
    if (kk == k) return h.vals[p];
    if (kk == 0ULL) return NONE;
    p = (p + 1) & h.mask;
    kk = h.keys[p];
  }
}
__device__ __forceinline__ uint32_t tshash_find(TsHash h, int64_t ts) {
  const unsigned long long k = static_cast<unsigned long long>(ts) ^ 0x8000000000000000ULL;
  uint32_t p = static_cast<uint32_t>(mix64(k)) & h.mask;
  for (;;) {
    unsigned long long kk = h.keys[p];
    if (kk == k) return h.vals[p];
    if (kk == 0ULL) return NONE;
    p = (p + 1) & h.mask;
  }
}

// ---- ts -> first Add index, direct-addressed when counters are dense.
// A timestamp is replicaId * 2^32 + counter (src/CRDTree.elm:137, :348-350),
// and each replica's counters form a dense run, so when every Add ts is
// non-negative and the per-replica counter ranges add up to O(n) the index is
// a flat array: base[r] + (counter - cmin[r]). No hashing, no CAS, and ops of
// one replica land in one contiguous run (cache-friendly). Otherwise the
// open-addressing TsHash above serves.
constexpr uint32_t RID_BITS = 21;  // ts < 2^53
constexpr uint32_t RID_SLOTS = 1u << RID_BITS;

struct TsIndex {
  uint32_t dense;
  TsHash h;
  const uint2* rng;      // [RID_SLOTS] per replica {min counter, max counter}; min = 0xFFFFFFFF: no Add
  const uint32_t* base;  // [RID_SLOTS] exclusive scan of range sizes
  uint32_t* first;       // [total range] min op index, 0xFFFFFFFF = none
};

__device__ __forceinline__ uint32_t tsindex_slot(const TsIndex& x, int64_t ts) {
  if (ts <= 0) return NONE;
  const uint64_t r = static_cast<uint64_t>(ts) >> 32;
  if (r >= RID_SLOTS) return NONE;
  const uint32_t c = static_cast<uint32_t>(ts);
  const uint2 g = x.rng[r];
  if (c < g.x || c > g.y) return NONE;  // (an empty range {NONE, 0} holds no c; 2^32 - 1 is a counter)
  return x.base[r] + (c - g.x);
}

__device__ __forceinline__ uint32_t tsindex_find(const TsIndex& x, int64_t ts) {
  if (!x.dense) return tshash_find(x.h, ts);
  const uint32_t p = tsindex_slot(x, ts);
  return p == NONE ? NONE : x.first[p];
}

__device__ __forceinline__ void tsindex_insert(const TsIndex& x, int64_t ts, uint32_t idx) {
  if (!x.dense) { tshash_insert(x.h, ts, idx); return; }
  atomicMin(&x.first[tsindex_slot(x, ts)], idx);
}

// ---- (dict, key) -> slot hash used by the exact replay (single writer per entry).
struct SlotHash {
  uint32_t* dict;
  long long* key;
  uint32_t* slot;  // NONE = empty
  uint32_t mask;
};

__device__ __forceinline__ uint32_t slothash_pos(uint32_t d, int64_t k, uint32_t mask) {
  return static_cast<uint32_t>(mix64(static_cast<uint64_t>(k) ^ (static_cast<uint64_t>(d) * 0x9E3779B97F4A7C15ULL))) &
         mask;
}

__device__ __forceinline__ uint32_t slothash_find(const SlotHash& h, uint32_t d, int64_t k) {
  uint32_t p = slothash_pos(d, k, h.mask);
  for (;;) {
    uint32_t s = h.slot[p];
    if (s == NONE) return NONE;
    if (h.dict[p] == d && h.key[p] == k) return s;
    p = (p + 1) & h.mask;
  }
}

// Sequential insert (replay thread) — the key must be absent.
__device__ __forceinline__ void slothash_put_seq(const SlotHash& h, uint32_t d, int64_t k, uint32_t s) {
  uint32_t p = slothash_pos(d, k, h.mask);
  while (h.slot[p] != NONE) {
    if (h.dict[p] == d && h.key[p] == k) { h.slot[p] = s; return; }
    p = (p + 1) & h.mask;
  }
  h.dict[p] = d;
  h.key[p] = k;
  h.slot[p] = s;
}

// Parallel insert (build kernel) — distinct (d, k) per caller.
__device__ __forceinline__ void slothash_put_par(const SlotHash& h, uint32_t d, int64_t k, uint32_t s) {
  uint32_t p = slothash_pos(d, k, h.mask);
  for (;;) {
    if (atomicCAS(&h.slot[p], NONE, s) == NONE) {
      h.dict[p] = d;
      h.key[p] = k;
      return;
    }
    p = (p + 1) & h.mask;
  }
}

// Wave-aggregated counter increment: one atomic per wave; every lane of the
// wave must call it (pred selects the lanes that take a ticket).
__device__ __forceinline__ uint32_t wave_ticket(uint32_t* ctr, bool pred) {
  const unsigned long long m = __ballot(pred);
  const int lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (m) {
    const int leader = __ffsll(static_cast<long long>(m)) - 1;
    if (lane == leader) base = atomicAdd(ctr, static_cast<uint32_t>(__popcll(m)));
    base = __shfl(base, leader, 64);
  }
  return base + static_cast<uint32_t>(__popcll(m & ((1ULL << lane) - 1ULL)));
}

// Workgroup-aggregated tickets into NT counters: thread t takes the next
// index of counter `which` (NT or more: none). One device atomic per counter
// and workgroup call (a counter bumped by every wave still serialises ~12 ns
// per atomic on one word). Every thread of the workgroup must call it.
// GLOBAL = false: the counters live in LDS (s_ctr, this workgroup's running
// offsets into ranges it reserved before), no device atomic at all.
template <uint32_t NT, bool GLOBAL = true>
__device__ __forceinline__ uint32_t block_ticket(uint32_t* ctr, uint32_t which) {
  constexpr uint32_t NW = BLOCK / 64;
  __shared__ uint32_t s_cnt[NT][NW];
  __shared__ uint32_t s_base[NT];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned long long lt = (1ULL << lane) - 1ULL;
  uint32_t rank = 0;
#pragma unroll
  for (uint32_t k = 0; k < NT; ++k) {
    const unsigned long long m = __ballot(which == k);
    if (which == k) rank = static_cast<uint32_t>(__popcll(m & lt));
    if (lane == 0) s_cnt[k][wv] = static_cast<uint32_t>(__popcll(m));
  }
  __syncthreads();
  if (threadIdx.x < NT) {
    const uint32_t k = threadIdx.x;
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
      const uint32_t c = s_cnt[k][w];
      s_cnt[k][w] = tot;  // -> the waves' exclusive prefix
      tot += c;
    }
    if (GLOBAL) {
      s_base[k] = tot ? atomicAdd(&ctr[k], tot) : 0u;
    } else {
      s_base[k] = ctr[k];
      ctr[k] += tot;
    }
  }
  __syncthreads();
  const uint32_t r = which < NT ? s_base[which] + s_cnt[which][wv] + rank : NONE;
  __syncthreads();  // (the next call reuses the LDS)
  return r;
}

// wave64 inclusive scan of u32 (CDNA: 64 lanes, __shfl_up over width 64)
// The "barrier" of a one-wave workgroup: its memory accesses before are
// ordered before those after (a wave issues in order; the fence keeps the
// compiler from moving them and waits for the stores) without s_barrier —
// in the forest replay __syncthreads here cost 10% of the kernel.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ unsigned long long wave_incl_scan64(unsigned long long v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    unsigned long long t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// block-level OR/MAX reduction helpers (one atomic per block)
__device__ __forceinline__ uint32_t block_max(uint32_t v) {
  __shared__ uint32_t s[BLOCK / 64];
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = 0;
  for (int w = 0; w < BLOCK / 64; ++w) r = max(r, s[w]);
  __syncthreads();
  return r;
}
__device__ __forceinline__ uint32_t block_sum(uint32_t v) {
  __shared__ uint32_t s[BLOCK / 64];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = 0;
  for (int w = 0; w < BLOCK / 64; ++w) r += s[w];
  __syncthreads();
  return r;
}
__device__ __forceinline__ uint32_t block_min(uint32_t v) {
  __shared__ uint32_t s[BLOCK / 64];
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = NONE;
  for (int w = 0; w < BLOCK / 64; ++w) r = min(r, s[w]);
  __syncthreads();
  return r;
}

// the same for a workgroup of NT threads
template <uint32_t NT, class F>
__device__ __forceinline__ uint32_t block_reduce_t(uint32_t v, uint32_t id, F op) {
  __shared__ uint32_t s[NT / 64];
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = id;
  for (uint32_t w = 0; w < NT / 64; ++w) r = op(r, s[w]);
  __syncthreads();
  return r;
}

#define GRID_STRIDE(i, n) \
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += gridDim.x * blockDim.x)

}  // namespace crdtm

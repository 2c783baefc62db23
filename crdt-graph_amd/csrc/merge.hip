// merge.hip — the CRDTree batch merge on gfx950.
//
// Replaces the reference's sequential `apply (Batch ops)` (src/CRDTree.elm:
// 224-232, :265-350; src/Internal/Node.elm:51-163) for a whole batch.
//
// Two exact paths share one device tree state (engine.h TreeDev):
//  * closed form (fresh tree, guard holds): per-op status by level-synchronous
//    path resolution (K1), effective-parent pointer jumping + segmented sibling
//    sort (K2), tombstone scatter (K3), Euler tour + list ranking for the raw
//    `next` chains and the document order (K4), then a commit that writes the
//    tree state and appends the op log;
//  * exact replay (everything else): one lane replays the batch with the
//    reference's literal addAfterHelp/findInsertion/deleteHelp semantics,
//    including the findInsertion copy quirk, with an undo log for atomicity.
// DESIGN.md derives the closed form and its guard.

#include <cstring>

#include "engine.h"
#include "listrank.h"
#include "scan.h"

namespace crdtm {


struct Work {  // per-call device arrays of the closed form (sized by n ops)
  uint8_t* st;
  uint32_t* cur;
  uint32_t* leaf;
  uint32_t* addpar;
  uint32_t* dtime;
  uint8_t* dead;
  uint32_t* maxadd;
  uint4* nrec;    // per op, one line per lookup: {path begin, len | status << 16 | dead << 24, dict owner, chain death}
  uint32_t* tag;  // per op: PDR_REACHED, or the tombstoned node its path stopped at, or NONE (pdr.hip)
};

__device__ __forceinline__ uint32_t op_len(const OpsDev& o, uint32_t i) { return o.off[i + 1] - o.off[i]; }

// Four consecutive ops per lane, loaded with 16-byte vector loads (device
// inputs are 16-byte aligned: api.hip align_ops); the tail quad falls back
// to guarded scalar loads. Consecutive lanes take consecutive quads.
struct Quad {
  uint32_t cnt;  // valid ops (1..4)
  uint8_t kind[4];
  long long ts[4];
  uint32_t off[5];
};

__device__ __forceinline__ void load_quad(const OpsDev& o, uint32_t i0, Quad& q) {
  if (i0 + 4 <= o.n) {
    q.cnt = 4;
    const uchar4 k = *reinterpret_cast<const uchar4*>(o.kind + i0);
    q.kind[0] = k.x;
    q.kind[1] = k.y;
    q.kind[2] = k.z;
    q.kind[3] = k.w;
    const longlong2 a = *reinterpret_cast<const longlong2*>(o.ts + i0);
    const longlong2 b = *reinterpret_cast<const longlong2*>(o.ts + i0 + 2);
    q.ts[0] = a.x;
    q.ts[1] = a.y;
    q.ts[2] = b.x;
    q.ts[3] = b.y;
    const uint4 f = *reinterpret_cast<const uint4*>(o.off + i0);
    q.off[0] = f.x;
    q.off[1] = f.y;
    q.off[2] = f.z;
    q.off[3] = f.w;
    q.off[4] = o.off[i0 + 4];
  } else {
    q.cnt = o.n - i0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const bool v = k < q.cnt;
      q.kind[k] = v ? o.kind[i0 + k] : 0;
      q.ts[k] = v ? o.ts[i0 + k] : 0;
    }
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) q.off[k] = k <= q.cnt ? o.off[i0 + k] : 0;  // static indices: no scratch
  }
}

__device__ __forceinline__ void store_quad_u8(uint8_t* p, uint32_t i0, uint32_t cnt, const uint8_t v[4]) {
  if (cnt == 4) {
    *reinterpret_cast<uchar4*>(p + i0) = make_uchar4(v[0], v[1], v[2], v[3]);
  } else {
    for (uint32_t k = 0; k < cnt; ++k) p[i0 + k] = v[k];
  }
}

// Quads are strided over the grid: the blocks in flight cover one contiguous
// front of ops, so the slot-space lines that the ops of one replica touch
// (consecutive counters) are shared by concurrent blocks and stay cached.
#define QUAD_LOOP(i0, n)                                                                           \
  for (uint32_t i0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x); i0 < (n); i0 += 4 * gridDim.x * blockDim.x)

// XCD-chunked variant for kernels that scatter into slot space: the front is
// cut into 8 chunks, chunk j on the blocks with blockIdx % 8 == j % 8 (the
// hardware's round-robin XCD placement; speed only). A replica's consecutive
// ops within a chunk then write whole slot lines from ONE L2 instead of
// leaving partial lines in eight (measured: 7x write amplification).
#define QUAD_LOOP_XCD(i0, n)                                                                       \
  const uint32_t nq_ = ((n) + 3) / 4;                                                              \
  const bool x8_ = (gridDim.x & 7) == 0;                                                           \
  const uint32_t xc_ = x8_ ? blockIdx.x & 7 : 0, xy_ = x8_ ? blockIdx.x >> 3 : blockIdx.x;         \
  const uint32_t cq_ = (x8_ ? gridDim.x >> 3 : gridDim.x) * blockDim.x, xs_ = x8_ ? 8 : 1;         \
  for (uint32_t j_ = xc_, qd_ = xc_ * cq_ + xy_ * blockDim.x + threadIdx.x, i0 = 4 * qd_;         \
       j_ * cq_ < nq_; j_ += xs_, qd_ = j_ * cq_ + xy_ * blockDim.x + threadIdx.x, i0 = 4 * qd_)   \
    if (qd_ < nq_)

// A grid cap from the environment (A/B runs), else `def`.
static uint32_t env_grid(const char* name, uint32_t def) {
  const char* e = getenv(name);
  const int g = e ? atoi(e) : 0;
  return g >= 8 && g <= (1 << 20) ? static_cast<uint32_t>(g) : def;
}

inline uint32_t quad_grid(uint64_t n) {
  const uint64_t g = (((n + 3) / 4) + BLOCK - 1) / BLOCK;
  if (g >= 2048) return 2048;
  return g < 8 ? static_cast<uint32_t>(g ? g : 1) : static_cast<uint32_t>((g + 7) & ~7ULL);
}


// ---------------------------------------------------------------------------
// K1 — per-op status under sequential semantics (src/Internal/Node.elm:138-163,
// :56-90, :112-122; src/CRDTree.elm:298-325). Nodes are named by the index of
// the first Add of their timestamp; the root dict owner is ROOTN = n.
// ---------------------------------------------------------------------------

// Batch pre-pass: per-replica counter ranges of the Add timestamps (dense
// index layout), longest path, |x| < 2^53 range checks over ts, negative
// timestamps, Delete count and the largest replica id. The path elements'
// range check rides on the flat claim (k_fl_claim reads them anyway) and is a
// pass of its own (k_path_range) on the other paths.
// Replica ids below REP_DIRECT fold into a direct-mapped LDS table with
// no-return LDS atomics; larger ids go straight to the global table.
constexpr uint32_t REP_DIRECT = 4096;
// (PB = 1024 threads: 512 workgroups keep the range flush short, and the
// larger workgroups give every CU 32 waves to cover the memory latency)
constexpr uint32_t PRE_T = 1024;
template <uint32_t PB>
__global__ void __launch_bounds__(PB) __attribute__((amdgpu_waves_per_eu(PB == 1024 ? 8 : 4, 8))) k_pre(OpsDev o, uint2* rng, DevResult* dres) {
  __shared__ __attribute__((aligned(16))) uint32_t rlo[REP_DIRECT];
  __shared__ __attribute__((aligned(16))) uint32_t rhi[REP_DIRECT];
  for (uint32_t j = threadIdx.x; j < REP_DIRECT / 4; j += blockDim.x) {
    reinterpret_cast<uint4*>(rlo)[j] = make_uint4(NONE, NONE, NONE, NONE);
    reinterpret_cast<uint4*>(rhi)[j] = make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
  uint32_t mx = 0, bad = 0, neg = 0, ndel = 0, maxr = 0;
  auto fold = [&](const Quad& q) {
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (k >= q.cnt) break;
      const uint32_t L = q.off[k + 1] - q.off[k];
      mx = max(mx, L);
      if (q.kind[k] != CRDTM_ADD) {
        ++ndel;
        continue;
      }
      const long long ts = q.ts[k];
      if (ts >= TWO53 || ts <= -TWO53) {
        bad = 1;
      } else if (ts < 0) {
        neg = 1;
      } else if (L >= 1 && ts != 0) {
        const uint32_t r = static_cast<uint32_t>(static_cast<uint64_t>(ts) >> 32), c = static_cast<uint32_t>(ts);
        maxr = max(maxr, r);
        if (r < REP_DIRECT) {
          // the table only narrows towards the answer: a plain read that
          // already covers c makes the atomic unnecessary (same-address
          // reads broadcast, same-address atomics serialise)
          if (c < rlo[r]) atomicMin(&rlo[r], c);
          if (c > rhi[r]) atomicMax(&rhi[r], c);
        } else {
          atomicMin(&rng[r].x, c);
          atomicMax(&rng[r].y, c);
        }
      }
    }
  };
  // (512 workgroups keep the range flush short, so each thread keeps two
  // quads and four path pairs in flight to cover the memory latency)
  {
    const uint32_t qs = 4 * gridDim.x * blockDim.x;
    uint32_t i0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
    for (; i0 + qs < o.n; i0 += 2 * qs) {
      Quad qa, qb;
      load_quad(o, i0, qa);
      load_quad(o, i0 + qs, qb);
      fold(qa);
      fold(qb);
    }
    if (i0 < o.n) {
      Quad qa;
      load_quad(o, i0, qa);
      fold(qa);
    }
  }
  auto mxf = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
  maxr = block_reduce_t<PB>(maxr, 0u, mxf);  // (synchronises the block) only ids <= maxr were touched
  for (uint32_t j = threadIdx.x; j <= maxr && j < REP_DIRECT; j += blockDim.x) {
    if (rlo[j] <= rhi[j]) {  // (touched: a counter of 2^32 - 1 is a real range, not the NONE mark)
      atomicMin(&rng[j].x, rlo[j]);
      atomicMax(&rng[j].y, rhi[j]);
    }
  }
  mx = block_reduce_t<PB>(mx, 0u, mxf);
  bad = block_reduce_t<PB>(bad, 0u, mxf);
  neg = block_reduce_t<PB>(neg, 0u, mxf);
  ndel = block_reduce_t<PB>(ndel, 0u, [](uint32_t a, uint32_t b) { return a + b; });
  if (threadIdx.x == 0) {
    if (mx) atomicMax(&dres->max_len, mx);
    if (bad) atomicOr(&dres->bad_range, 1u);
    if (neg) atomicOr(&dres->has_negative, 1u);
    if (ndel) atomicAdd(&dres->n_del, ndel);
    if (maxr) atomicMax(&dres->max_replica, maxr);
  }
}

// |x| < 2^53 over every path element (16-byte loads over an even-aligned range)
__global__ void __launch_bounds__(BLOCK) k_path_range(OpsDev o, DevResult* dres) {
  const uint64_t np = o.n_path, npair = np / 2;
  auto out = [](long long v) { return v >= TWO53 || v <= -TWO53; };
  uint32_t bad = 0;
  const uint64_t ps = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t p = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
  for (; p + 3 * ps < npair; p += 4 * ps) {
    longlong2 v[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const longlong2*>(o.path + 2 * (p + u * ps));
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
      if (out(v[u].x) || out(v[u].y)) bad = 1;
  }
  for (; p < npair; p += ps) {
    const longlong2 v = *reinterpret_cast<const longlong2*>(o.path + 2 * p);
    if (out(v.x) || out(v.y)) bad = 1;
  }
  if ((np & 1) && blockIdx.x == 0 && threadIdx.x == 0 && out(o.path[np - 1])) bad = 1;
  bad = block_max(bad);
  if (threadIdx.x == 0 && bad) atomicOr(&dres->bad_range, 1u);
}

// The flat speculation's pre-pass (launched when every op may be an Add with
// a one-element path, n_path == n): the per-replica counter ranges of the
// timestamps (16-byte loads, ids below REP_SPEC in an LDS table), |ts| < 2^53,
// negative timestamps and the largest replica id, and the check that every
// op is an Add whose path is path[i] alone (kind, path_off[i] == i; else
// DevResult::spec_fail). The workgroup that finishes last lays the ranges end
// to end (base[], range_total, the slot words fl_nw), so the claim follows on
// the device without a host round trip.
constexpr uint32_t REP_SPEC = 256;
// BLIND: every op's min/max goes to the LDS table as a no-return atomic
// (nothing to wait for) instead of a read first and an atomic only when the
// read does not cover it (a typing replica's counters rise through the
// batch, so its maximum moves on nearly every op anyway)
template <uint32_t PB, bool BLIND>
__global__ void __launch_bounds__(PB) k_pre_ts(const long long* __restrict__ ts, const uint8_t* __restrict__ kind,
                                               const uint32_t* __restrict__ off, uint32_t n, uint2* rng,
                                               uint32_t* base, DevResult* dres) {
  __shared__ uint32_t rlo[REP_SPEC], rhi[REP_SPEC];
  __shared__ uint32_t s_last;
  __shared__ unsigned long long sw[PB / 64];
  for (uint32_t j = threadIdx.x; j < REP_SPEC; j += PB) {
    rlo[j] = NONE;
    rhi[j] = 0;
  }
  __syncthreads();
  uint32_t bad = 0, neg = 0, maxr = 0, vfail = 0;
  auto fold = [&](long long t) {
    if (t >= TWO53 || t <= -TWO53) {
      bad = 1;
    } else if (t < 0) {
      neg = 1;
    } else if (t != 0) {
      const uint32_t r = static_cast<uint32_t>(static_cast<uint64_t>(t) >> 32), c = static_cast<uint32_t>(t);
      maxr = max(maxr, r);
      if (r < REP_SPEC) {  // (the table only narrows: a covering read makes the atomic unnecessary)
        if (BLIND || c < rlo[r]) atomicMin(&rlo[r], c);
        if (BLIND || c > rhi[r]) atomicMax(&rhi[r], c);
      }
    }
  };
  {
    const longlong2* t2 = reinterpret_cast<const longlong2*>(ts);
    const uchar2* k2 = reinterpret_cast<const uchar2*>(kind);
    const uint2* o2 = reinterpret_cast<const uint2*>(off);
    auto verify = [&](uint32_t p, uchar2 k, uint2 f) {  // ops 2p, 2p + 1
      vfail |= (k.x | k.y) != CRDTM_ADD || f.x != 2 * p || f.y != 2 * p + 1;
    };
    const uint32_t np = n / 2, gs = gridDim.x * PB;
    uint32_t p = blockIdx.x * PB + threadIdx.x;
    for (; p + 3 * gs < np; p += 4 * gs) {  // four pairs in flight
      longlong2 v[4];
      uchar2 k[4];
      uint2 f[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        v[u] = t2[p + u * gs];
        k[u] = k2[p + u * gs];
        f[u] = o2[p + u * gs];
      }
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        fold(v[u].x);
        fold(v[u].y);
        verify(p + u * gs, k[u], f[u]);
      }
    }
    for (; p < np; p += gs) {
      const longlong2 v = t2[p];
      fold(v.x);
      fold(v.y);
      verify(p, k2[p], o2[p]);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (n & 1) {
        fold(ts[n - 1]);
        vfail |= kind[n - 1] != CRDTM_ADD || off[n - 1] != n - 1;
      }
      vfail |= off[n] != n;
    }
  }
  auto mxf = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
  maxr = block_reduce_t<PB>(maxr, 0u, mxf);  // (synchronises the block)
  for (uint32_t j = threadIdx.x; j <= maxr && j < REP_SPEC; j += PB)
    if (rlo[j] <= rhi[j]) {  // (touched: a counter of 2^32 - 1 is a real range, not the NONE mark)
      atomicMin(&rng[j].x, rlo[j]);
      atomicMax(&rng[j].y, rhi[j]);
    }
  bad = block_reduce_t<PB>(bad, 0u, mxf);
  neg = block_reduce_t<PB>(neg, 0u, mxf);
  vfail = block_reduce_t<PB>(vfail, 0u, mxf);
  if (threadIdx.x == 0) {
    if (vfail) atomicOr(&dres->spec_fail, 1u);
    if (bad) atomicOr(&dres->bad_range, 1u);
    if (neg) atomicOr(&dres->has_negative, 1u);
    if (maxr) atomicMax(&dres->max_replica, maxr);
    // (release: this workgroup's range atomics before its arrival)
    s_last = __hip_atomic_fetch_add(&dres->pre_done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
             gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // the last workgroup: base[r] = the sizes of the ranges before r (ids above
  // REP_SPEC - 1 make the speculation fail on the host; they are not laid out)
  const uint32_t nr =
      min(__hip_atomic_load(&dres->max_replica, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT), REP_SPEC - 1) + 1;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x / 64;
  unsigned long long sz = 0;  // (a range spans up to 2^32 counters: sizes and sums in 64 bits)
  if (threadIdx.x < nr) {
    const uint32_t lo = __hip_atomic_load(&rng[threadIdx.x].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t hi = __hip_atomic_load(&rng[threadIdx.x].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sz = lo <= hi ? static_cast<unsigned long long>(hi - lo) + 1ULL : 0ULL;  // (empty: {NONE, 0})
  }
  const unsigned long long inc = wave_incl_scan64(sz);
  if (lane == 63) sw[wave] = inc;
  __syncthreads();
  unsigned long long pre = inc - sz, tot = 0;
  for (uint32_t w = 0; w < PB / 64; ++w) {
    if (w < wave) pre += sw[w];
    tot += sw[w];
  }
  if (threadIdx.x < nr) base[threadIdx.x] = static_cast<uint32_t>(pre < NONE ? pre : NONE);
  if (threadIdx.x == 0) {
    const uint32_t q = static_cast<uint32_t>(tot < NONE - 64 ? tot : NONE - 64);
    dres->range_total = q;
    dres->fl_nw = (q + 63) / 64;
  }
}

// Per-op state of the level-synchronous (nested / hash-indexed) path.
__global__ void __launch_bounds__(BLOCK) k_work_init(OpsDev o, Work w) {
  GRID_STRIDE(i, o.n) {
    w.st[i] = op_len(o, i) == 0 ? ST_INVALID : ST_PENDING;
    w.cur[i] = o.n;
    w.addpar[i] = NONE;
    w.dtime[i] = NONE;
    w.tag[i] = NONE;
  }
}

// K1 node records (levels): written once per op here, then by its level
__global__ void __launch_bounds__(BLOCK) k_nrec_init(OpsDev o, Work w) {
  GRID_STRIDE(i, o.n) {
    const uint32_t b = o.off[i], L = o.off[i + 1] - b;
    w.nrec[i] = make_uint4(b, L | (static_cast<uint32_t>(ST_PENDING) << 16), NONE, NONE);
  }
}
__device__ __forceinline__ uint32_t nrec_len(const uint4& r) { return r.y & 0xFFFFu; }
__device__ __forceinline__ uint32_t nrec_st(const uint4& r) { return (r.y >> 16) & 0xFFu; }
__device__ __forceinline__ bool nrec_dead(const uint4& r) { return (r.y >> 24) & 1u; }

// Dense index layout: base[r] = exclusive scan of the range sizes over
// replicas 0..max_replica, one workgroup (max_replica is read on the device,
// so the host needs no copy of the ranges); the total goes to range_total.
__global__ void __launch_bounds__(BLOCK) k_range_base(const uint2* rng, uint32_t* base, DevResult* dres) {
  __shared__ unsigned long long sw[BLOCK / 64];
  const uint32_t nr = dres->max_replica + 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long carry = 0;
  for (uint32_t r0 = 0; r0 < nr; r0 += BLOCK) {
    const uint32_t r = r0 + threadIdx.x;
    unsigned long long sz = 0;  // (a range spans up to 2^32 counters: sizes and sums in 64 bits)
    if (r < nr) {
      const uint2 g = rng[r];
      sz = g.x <= g.y ? static_cast<unsigned long long>(g.y - g.x) + 1ULL : 0ULL;  // (empty: {NONE, 0})
    }
    const unsigned long long inc = wave_incl_scan64(sz);
    if (lane == 63) sw[wave] = inc;
    __syncthreads();
    unsigned long long pre = carry + (inc - sz), tot = 0;
    for (int w = 0; w < BLOCK / 64; ++w) {
      if (w < wave) pre += sw[w];
      tot += sw[w];
    }
    if (r < nr) base[r] = static_cast<uint32_t>(pre < NONE ? pre : NONE);
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) dres->range_total = static_cast<uint32_t>(carry < NONE ? carry : NONE);
}

// The replica range table lives in the context and is kept clean between
// calls: every merge resets the entries it touched (ids 0..max_replica).
__global__ void __launch_bounds__(BLOCK) k_range_reset(uint2* rng, uint32_t nr, const DevResult* dres) {
  if (nr == 0) nr = dres->max_replica + 1;
  GRID_STRIDE(r, nr) rng[r] = make_uint2(NONE, 0u);
}

void range_reset(crdtm_ctx* c, uint32_t nr) {
  LAUNCH(k_range_reset, dim3(nr ? std::min<uint32_t>(grid_for(nr), 1024) : 64), dim3(BLOCK), 0, c->stream, c->crange,
         nr, c->dres);
}

void launch_pre(crdtm_ctx* c, const OpsDev& o, hipStream_t s) {
  const uint32_t g = static_cast<uint32_t>(std::min<uint64_t>((o.n / 4 + PRE_T - 1) / PRE_T + 1, 512));
  LAUNCH(k_pre<PRE_T>, dim3(g), dim3(PRE_T), 0, s, o, c->crange, c->dres);
}

static __device__ __forceinline__ void dres_init_block(DevResult* d) {
  const uint32_t nw = sizeof(DevResult) / sizeof(uint32_t);
  uint32_t* w = reinterpret_cast<uint32_t*>(d);
  for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) w[j] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    d->err_index = NONE;
    d->first_del = NONE;
  }
}
__global__ void k_dres_init(DevResult* d) { dres_init_block(d); }

__global__ void __launch_bounds__(BLOCK) k_index_insert(OpsDev o, TsIndex x) {
  GRID_STRIDE(i, o.n) {
    if (o.kind[i] != CRDTM_ADD || op_len(o, i) == 0) continue;
    const long long ts = o.ts[i];
    if (ts != 0) tsindex_insert(x, ts, i);
  }
}

// Dense index without atomics: every Add stores its op index into its slot
// (one arbitrary writer wins among duplicates), then every Add that did not
// win takes an atomicMin, so the slot ends as the first Add of that
// timestamp. Batches without duplicate timestamps pay no atomic at all.
// The replica range table (base, min, max counter) is read from LDS when its
// nrep ids fit (as in k_fl_claim), else from the global table.
struct RangeLds {
  uint32_t* sbase;
  uint32_t* smin;
  uint32_t* smax;
  uint32_t nrep;
  __device__ __forceinline__ void load(const TsIndex& x) {
    for (uint32_t j = threadIdx.x; j < nrep; j += blockDim.x) {
      sbase[j] = x.base[j];
      const uint2 g = x.rng[j];
      smin[j] = g.x;
      smax[j] = g.y;
    }
    __syncthreads();
  }
  __device__ __forceinline__ uint32_t slot(const TsIndex& x, long long ts) const {
    if (!nrep) return tsindex_slot(x, ts);
    if (ts <= 0) return NONE;
    const uint64_t r = static_cast<uint64_t>(ts) >> 32;
    if (r >= nrep) return NONE;
    const uint32_t c = static_cast<uint32_t>(ts), lo = smin[r];
    if (c < lo || c > smax[r]) return NONE;  // (an empty range {NONE, 0} holds no c)
    return sbase[r] + (c - lo);
  }
};

__global__ void __launch_bounds__(BLOCK) k_index_store(OpsDev o, TsIndex x, uint32_t nrep) {
  extern __shared__ uint32_t srt[];  // [3 * nrep]
  RangeLds t{srt, srt + nrep, srt + 2 * nrep, nrep};
  t.load(x);
  QUAD_LOOP_XCD(i0, o.n) {
    Quad q;
    load_quad(o, i0, q);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (k >= q.cnt) break;
      if (q.kind[k] == CRDTM_ADD && q.off[k + 1] != q.off[k] && q.ts[k] > 0) x.first[t.slot(x, q.ts[k])] = i0 + k;
    }
  }
}

__global__ void __launch_bounds__(BLOCK) k_index_fix(OpsDev o, TsIndex x, uint32_t nrep) {
  extern __shared__ uint32_t srt[];  // [3 * nrep]
  RangeLds t{srt, srt + nrep, srt + 2 * nrep, nrep};
  t.load(x);
  QUAD_LOOP_XCD(i0, o.n) {
    Quad q;
    load_quad(o, i0, q);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (k >= q.cnt) break;
      if (q.kind[k] != CRDTM_ADD || q.off[k + 1] == q.off[k] || q.ts[k] <= 0) continue;
      uint32_t* f = &x.first[t.slot(x, q.ts[k])];
      if (*f != i0 + k) atomicMin(f, i0 + k);
    }
  }
}

// Fused K1 for the common single-level, Adds-only batch (a flat document):
// status, dict owner and the effective-parent seed in one pass.
__global__ void __launch_bounds__(BLOCK) k_flat_status(OpsDev o, Work w, TsIndex x, uint32_t* anc) {
  const uint32_t n = o.n;
  GRID_STRIDE(i, n) {
    if (w.st[i] != ST_PENDING) continue;  // L == 0: InvalidPath
    w.addpar[i] = n;                      // parent = the root
    const long long ts = o.ts[i];
    uint8_t s;
    if (ts == 0 || tsindex_find(x, ts) != i) {
      s = ST_ALREADY;  // key 0 is the sentinel / child ts parent exists
    } else {
      const long long k = o.path[o.off[i]];
      uint32_t a;
      if (k == 0) {
        a = SENT_T;
      } else {
        const uint32_t f = tsindex_find(x, k);
        a = (f != NONE && op_len(o, f) == 1) ? f : MISS_T;
      }
      s = (a == SENT_T || (a != MISS_T && a < i)) ? ST_APPLIED : ST_NOTFOUND;
      if (s == ST_APPLIED) {
        w.dead[i] = 0;
        anc[i] = a == SENT_T ? 2 * n : a;
      }
    }
    w.st[i] = s;
  }
}

// K1 by path length. Ops are bucketed by |path| and level j handles only the
// ops of length j, after every shorter op is final: their dict owner (L1),
// the leaf lookup, collisions and Delete times (L2), then statuses and each
// new node's chain death time (L3). Path resolution (src/Internal/Node.elm:
// 138-163) descends through keys; with timestamps unique per dict (the
// collision guard) the node of key k is tsindex_find(k), so the prefix
// [k1..k(j-1)] of op i names the node g = find(k(j-1)) exactly when g's own
// parent path equals [k1..k(j-2)]: then i's ancestors are g's, and i reaches
// g's children iff g was applied and no node of that chain was deleted before
// i (dtc = first Delete time over the chain, in the node record). Anything else takes the
// literal walk, one lookup per level.
__device__ __forceinline__ uint32_t lookup_child(const OpsDev& o, const Work& w, const TsIndex& h, uint32_t parent,
                                                 long long k, uint32_t lvl) {
  if (k == 0) return SENT_T;
  const uint32_t f = tsindex_find(h, k);
  if (f == NONE) return MISS_T;
  const uint4 r = w.nrec[f];
  if (nrec_len(r) != lvl || r.z != parent) return MISS_T;
  return f;
}

struct LevelLists {
  uint32_t* ops;          // op indices grouped by |path|
  uint32_t* fill;         // [MAXLV_BUCKET + 1] scatter cursors
};
constexpr uint32_t MAXLV_BUCKET = 64;  // longer paths: the per-level fallback

__global__ void __launch_bounds__(BLOCK) k_len_count(OpsDev o, uint32_t maxlen, uint32_t* cnt) {
  __shared__ uint32_t hist[MAXLV_BUCKET + 1];
  for (uint32_t j = threadIdx.x; j <= maxlen; j += blockDim.x) hist[j] = 0;
  __syncthreads();
  GRID_STRIDE(i, o.n) atomicAdd(&hist[op_len(o, i)], 1u);
  __syncthreads();
  for (uint32_t j = threadIdx.x; j <= maxlen; j += blockDim.x)
    if (hist[j]) atomicAdd(&cnt[j], hist[j]);
}

// one global atomic per (block, length): the block reserves its range, then
// ranks its ops in LDS (order inside a level does not matter)
struct LevelStart {
  uint32_t v[MAXLV_BUCKET + 1];
};

// A level-list entry: the op and its path offset (o.off[i]), so a level
// kernel loads the op's keys without a dependent offset load. The parent key
// path[L-2] is left to k_lv_dict: it shares lines with the prefix keys that
// kernel loads anyway (carried here it made k_len_scatter touch every line of
// the path array).
struct LvEnt {
  uint32_t i, b;
};
static_assert(sizeof(LvEnt) == 8, "one 8-byte load per entry");

__global__ void __launch_bounds__(BLOCK) k_len_scatter(OpsDev o, uint32_t maxlen, LevelStart start,
                                                       uint32_t* fill, LvEnt* lists) {
  __shared__ uint32_t hist[MAXLV_BUCKET + 1];
  __shared__ uint32_t base[MAXLV_BUCKET + 1];
  const uint32_t n = o.n;
  const uint32_t chunk = BLOCK * 8;
  for (uint32_t c0 = blockIdx.x * chunk; c0 < n; c0 += gridDim.x * chunk) {
    for (uint32_t j = threadIdx.x; j <= maxlen; j += blockDim.x) hist[j] = 0;
    __syncthreads();
    uint32_t L[8], r[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t i = c0 + u * BLOCK + threadIdx.x;
      b[u] = i < n ? o.off[i] : 0u;
      L[u] = i < n ? o.off[i + 1] - b[u] : NONE;
      r[u] = (L[u] != NONE) ? atomicAdd(&hist[L[u]], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j <= maxlen; j += blockDim.x)
      base[j] = hist[j] ? start.v[j] + atomicAdd(&fill[j], hist[j]) : 0u;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t i = c0 + u * BLOCK + threadIdx.x;
      if (L[u] != NONE) *reinterpret_cast<uint2*>(&lists[base[L[u]] + r[u]]) = make_uint2(i, b[u]);
    }
    __syncthreads();
  }
}

// L1: the dict of every op of length j (fast prefix check, else the walk).
// The prefix compare of paths up to LV_UNROLL keys is unrolled with
// level-uniform predicates, so the op's own keys load before the parent
// lookup resolves and the parent's keys load together.
constexpr uint32_t LV_UNROLL = 14;
constexpr uint32_t LV_PAIRS = (LV_UNROLL + 2) / 2;
// k[l] = path[base + l] for l + 2 < j, as 16-byte loads from the even index
// at or below base (half the load instructions and L2 line requests of
// 8-byte loads; the path array is 16-byte aligned, checked by the caller)
__device__ __forceinline__ void lv_keys(const long long* path, uint32_t base, uint32_t j, long long* k) {
  const uint32_t sh = base & 1u;
  const longlong2* p2 = reinterpret_cast<const longlong2*>(path + (base - sh));
  long long e[2 * LV_PAIRS];
#pragma unroll
  for (uint32_t m = 0; m < LV_PAIRS; ++m) {
    const longlong2 v = 2 * m < sh + j - 2 ? p2[m] : make_longlong2(0, 0);
    e[2 * m] = v.x;
    e[2 * m + 1] = v.y;
  }
#pragma unroll
  for (uint32_t l = 0; l < LV_UNROLL; ++l) k[l] = l + 2 < j ? (sh ? e[l + 1] : e[l]) : 0;
}

// |x| < 2^53 for the path elements of the level kernels: an op's keys
// [b, b + j - 1) here (its prefix and the parent's key, loaded anyway) and
// [b + j - 1] in k_lv_leaf, so every element of every op's path is checked
// once without a pass of its own over the path array (k_path_range)
__device__ __forceinline__ bool key_out(long long v) { return v >= TWO53 || v <= -TWO53; }
__device__ __forceinline__ void flag_bad_range(bool bad, DevResult* dres) {
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&dres->bad_range, 1u);
}

__global__ void __launch_bounds__(BLOCK) k_lv_dict(OpsDev o, Work w, TsIndex h, const LvEnt* list, uint32_t cnt,
                                                   uint32_t j, DevResult* dres) {
  const uint32_t n = o.n;
  const bool wide = (reinterpret_cast<uintptr_t>(o.path) & 15u) == 0 && j - 2 <= LV_UNROLL;
  bool bad = false;
  GRID_STRIDE(q, cnt) {
    const uint2 ev = *reinterpret_cast<const uint2*>(&list[q]);
    const uint32_t i = ev.x, b = ev.y;
    uint32_t cur = n;
    uint8_t s = ST_PENDING;
    if (j > 1) {
      const long long kp = o.path[b + j - 2];  // the parent's key
      long long own[LV_UNROLL];
      if (wide) {
        lv_keys(o.path, b, j, own);
      } else if (j - 2 <= LV_UNROLL) {
#pragma unroll
        for (uint32_t l = 0; l < LV_UNROLL; ++l) own[l] = l + 2 < j ? o.path[b + l] : 0;
      }
      bool ob = key_out(kp);
      if (j - 2 <= LV_UNROLL) {
#pragma unroll
        for (uint32_t l = 0; l < LV_UNROLL; ++l) ob |= l + 2 < j && key_out(own[l]);
      } else {
        for (uint32_t l = 0; l + 2 < j; ++l) ob |= key_out(o.path[b + l]);
      }
      bad |= ob;
      const uint32_t g = kp == 0 ? NONE : tsindex_find(h, kp);
      bool fast = g != NONE && g < i;
      uint32_t dg = NONE;
      if (fast) {
        const uint4 r = w.nrec[g];
        const uint32_t bg = r.x;
        dg = r.w;
        // independent loads (no early exit) so they issue together
        unsigned long long diff = 0;
        if (wide) {
          long long par[LV_UNROLL];
          lv_keys(o.path, bg, j, par);
#pragma unroll
          for (uint32_t l = 0; l < LV_UNROLL; ++l) diff |= static_cast<unsigned long long>(par[l] ^ own[l]);
        } else if (j - 2 <= LV_UNROLL) {
#pragma unroll
          for (uint32_t l = 0; l < LV_UNROLL; ++l)
            if (l + 2 < j) diff |= static_cast<unsigned long long>(o.path[bg + l] ^ own[l]);
        } else {
          for (uint32_t l = 0; l + 2 < j; ++l)
            diff |= static_cast<unsigned long long>(o.path[bg + l] ^ o.path[b + l]);
        }
        fast = nrec_len(r) == j - 1 && nrec_st(r) == ST_APPLIED && diff == 0;
      }
      if (fast && dg < i) {
        // the chain holds a node deleted before i: the descent stops at the
        // topmost such Tombstone (AlreadyApplied); which one is only needed
        // by the per-dict replay, which resolves TAG_LAZY from cur = g
        w.st[i] = ST_ALREADY;
        w.tag[i] = TAG_LAZY;
        w.cur[i] = g;
        continue;
      }
      if (fast) {
        cur = g;
      } else {  // the literal descent (k_lvl semantics, one level at a time)
        for (uint32_t l = 1; l < j; ++l) {
          const uint32_t tgt = lookup_child(o, w, h, cur, o.path[b + l - 1], l);
          if (tgt == MISS_T || (tgt != SENT_T && tgt >= i)) {  // child missing -> InvalidPath
            s = ST_INVALID;
            break;
          }
          if (tgt == SENT_T) {  // descending into the sentinel Tombstone
            s = ST_ALREADY;
            break;
          }
          if (w.dtime[tgt] < i) {  // descending into a Tombstone
            s = ST_ALREADY;
            w.tag[i] = tgt;
            break;
          }
          cur = tgt;
        }
      }
    }
    if (s != ST_PENDING) {
      w.st[i] = s;
      continue;
    }
    w.cur[i] = cur;
    if (o.kind[i] == CRDTM_ADD) {
      w.addpar[i] = cur;
      w.nrec[i].z = cur;
    }
  }
  flag_bad_range(bad, dres);
}

// L2: leaf lookup; collisions (the closed form names a node by its ts alone);
// the first Delete of a node that reaches it while its dict is live
// (deleteHelp, src/Internal/Node.elm:112-122).
__global__ void __launch_bounds__(BLOCK) k_lv_leaf(OpsDev o, Work w, TsIndex h, const LvEnt* list, uint32_t cnt,
                                                   uint32_t j, DevResult* dres) {
  bool bad = false;
  GRID_STRIDE(q, cnt) {
    const uint2 ev = *reinterpret_cast<const uint2*>(&list[q]);
    const uint32_t i = ev.x;
    const long long key = o.path[ev.y + j - 1];  // (range-checked for every op, pending or not)
    bad |= key_out(key);
    if (w.st[i] != ST_PENDING) continue;
    const uint32_t cur = w.cur[i];
    const uint32_t tgt = lookup_child(o, w, h, cur, key, j);
    w.leaf[i] = tgt;
    if (o.kind[i] == CRDTM_ADD) {
      const long long ts = o.ts[i];
      if (ts != 0) {
        const uint32_t f = tsindex_find(h, ts);
        if (f != i) {
          const uint4 r = w.nrec[f];
          if (nrec_len(r) != j || r.z != cur) atomicOr(&dres->guard, G_COLLISION);
          w.tag[i] = TAG_DUP;
        }
      } else {
        w.tag[i] = TAG_DUP;
      }
    } else if (tgt == SENT_T) {
      w.st[i] = ST_ALREADY;
    } else if (tgt == MISS_T || tgt > i) {
      w.st[i] = ST_NOTFOUND;
    } else {
      atomicMin(&w.dtime[tgt], i);
    }
  }
  flag_bad_range(bad, dres);
}

// L3: statuses of the ops that reached their dict; the chain death time of
// each new node (its own first Delete, or an ancestor's).
__global__ void __launch_bounds__(BLOCK) k_lv_fin(OpsDev o, Work w, TsIndex h, const LvEnt* list, uint32_t cnt,
                                                  uint32_t j) {
  const uint32_t n = o.n;
  GRID_STRIDE(q, cnt) {
    const uint32_t i = list[q].i;
    if (w.st[i] != ST_PENDING) continue;
    const uint32_t tg = w.tag[i];
    w.tag[i] = PDR_REACHED;
    if (o.kind[i] == CRDTM_DELETE) {
      w.st[i] = (w.dtime[w.leaf[i]] == i) ? ST_APPLIED : ST_ALREADY;
      continue;
    }
    uint8_t s;
    if (tg == TAG_DUP) s = ST_ALREADY;  // key 0 = the sentinel, or `child ts parent` exists (k_lv_leaf)
    else {
      const uint32_t a = w.leaf[i];
      s = (a == SENT_T || (a != MISS_T && a < i)) ? ST_APPLIED : ST_NOTFOUND;
    }
    w.st[i] = s;
    uint32_t dead = 0, dc = NONE;
    if (s == ST_APPLIED) {
      const uint32_t p = w.addpar[i];
      const uint32_t dt = w.dtime[i];
      if (p == n) {
        dead = dt != NONE;
        dc = dt;
      } else {
        const uint4 rp = w.nrec[p];
        dead = (dt != NONE || nrec_dead(rp)) ? 1u : 0u;
        dc = min(dt, rp.w);
      }
      w.dead[i] = static_cast<uint8_t>(dead);
    }
    w.nrec[i].y = j | (static_cast<uint32_t>(s) << 16) | (dead << 24);
    w.nrec[i].w = dc;
  }
}

// Batch accounting + the guard (DESIGN.md "Guard"): tombstones present in a
// dict while later Adds land in it can change findInsertion's walk. The
// common cases (no Deletes; Deletes after every Add) are decided from the
// batch-wide last applied Add and first applied Delete; only a batch that
// interleaves them pays the per-dict check (k_guard_dicts).
__global__ void __launch_bounds__(BLOCK) k_stats(OpsDev o, Work w, long long ts0, DevResult* dres) {
  uint32_t app = 0, alr = 0, err = NONE, own = 0, addapp = 0, last_add = 0, first_del = NONE;
  const long long id0 = replica_of(ts0);
  // four ops per lane: statuses and kinds as one 4-byte load each, the
  // timestamps as two 16-byte loads (independent of the statuses)
  QUAD_LOOP(i0, o.n) {
    Quad q;
    load_quad(o, i0, q);
    uint8_t sv[4];
    if (q.cnt == 4) {
      const uchar4 s4 = *reinterpret_cast<const uchar4*>(w.st + i0);
      sv[0] = s4.x;
      sv[1] = s4.y;
      sv[2] = s4.z;
      sv[3] = s4.w;
    } else {
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) sv[k] = k < q.cnt ? w.st[i0 + k] : ST_ALREADY;
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (k >= q.cnt) break;
      const uint32_t i = i0 + k;
      const uint8_t s = sv[k];
      if (s == ST_APPLIED) ++app;
      else if (s == ST_ALREADY) ++alr;
      else err = min(err, i);
      if (q.kind[k] == CRDTM_ADD) {
        if ((s == ST_APPLIED || s == ST_ALREADY) && replica_of(q.ts[k]) == id0) ++own;
        if (s == ST_APPLIED) {
          ++addapp;
          last_add = max(last_add, i + 1);
        }
      } else if (s == ST_APPLIED) {
        first_del = min(first_del, i);
      }
    }
  }
  app = block_sum(app);
  alr = block_sum(alr);
  own = block_sum(own);
  addapp = block_sum(addapp);
  err = block_min(err);
  last_add = block_max(last_add);
  first_del = block_min(first_del);
  if (threadIdx.x == 0) {
    atomicAdd(&dres->n_applied, app);
    atomicAdd(&dres->n_already, alr);
    atomicAdd(&dres->own_ok_adds, own);
    atomicAdd(&dres->n_adds_applied, addapp);
    if (err != NONE) atomicMin(&dres->err_index, err);
    if (last_add) atomicMax(&dres->last_add, last_add);
    if (first_del != NONE) atomicMin(&dres->first_del, first_del);
  }
}

// Per-dict guard, only when the batch interleaves Deletes before later Adds.
// (one atomic per wave and dict: the lanes of a wave hold consecutive ops,
// often of one dict — config 2's two big dicts took ~39k same-word atomics
// each, 363 us; a dict's lanes are peeled off by ballot, the highest lane
// holding the largest op index)
__global__ void __launch_bounds__(BLOCK) k_guard_maxadd(OpsDev o, Work w) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < o.n; i0 += gridDim.x * blockDim.x) {  // (wave-uniform trips)
    const uint32_t i = i0 + threadIdx.x;
    bool act = i < o.n && o.kind[i] == CRDTM_ADD && w.st[i] == ST_APPLIED;
    const uint32_t d = act ? w.addpar[i] : NONE;
    unsigned long long live = __ballot(act);
    while (live) {
      const uint32_t lead = static_cast<uint32_t>(__ffsll(static_cast<long long>(live))) - 1u;
      const uint32_t dk = __shfl(d, static_cast<int>(lead), 64);
      const unsigned long long same = __ballot(act && d == dk);
      const uint32_t top = 63u - static_cast<uint32_t>(__clzll(same));
      if (lane == top) atomicMax(&w.maxadd[dk], i + 1);
      if (act && d == dk) act = false;
      live &= ~same;
    }
  }
}

// (one atomic per wave that finds a violation: a same-word atomic per Delete
// serialised 1.8 ms on deep10m_il's 3.3M interleaved Deletes)
__global__ void __launch_bounds__(BLOCK) k_guard_del(OpsDev o, Work w, DevResult* dres) {
  for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < o.n; i0 += gridDim.x * blockDim.x) {
    const uint32_t i = i0 + threadIdx.x;
    bool v = false;
    if (i < o.n && o.kind[i] == CRDTM_DELETE && w.st[i] == ST_APPLIED) v = w.maxadd[w.addpar[w.leaf[i]]] > i + 1;
    if (__ballot(v) && (threadIdx.x & 63) == 0 &&
        !(__hip_atomic_load(&dres->guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & G_DEL_BEFORE_ADD))
      atomicOr(&dres->guard, G_DEL_BEFORE_ADD);  // (once set, the plain read skips the atomic)
  }
}

// ---------------------------------------------------------------------------
// K2 — placement. Closed form: with no tombstone in any skip walk,
// findInsertion (src/Internal/Node.elm:93-104) puts x after the subtree of its
// effective parent ep(x) = first node on x's anchor chain with a smaller ts
// (the dict's sentinel acts as -inf), among ep's children in descending ts.
// While jumping, the sentinel of dict P is the marker n + P (root dict: 2n).
// Document tree (uids 0..n+1): node x -> x, root sentinel -> n, super root
// -> n + 1. A node's children are first the roots of its own children dict
// (group 0: its sub-document) and then its ep-children in its parent's dict
// (group 1), each group in descending ts — the sentinel of a dict merged into
// its owner.
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t sent_uid(uint32_t owner, uint32_t n) { return owner == n ? 2 * n : n + owner; }

__global__ void __launch_bounds__(BLOCK) k_ep_init(OpsDev o, Work w, uint32_t* anc) {
  GRID_STRIDE(x, o.n) {
    if (o.kind[x] != CRDTM_ADD || w.st[x] != ST_APPLIED) continue;
    const uint32_t a = w.leaf[x];
    anc[x] = a == SENT_T ? sent_uid(w.addpar[x], o.n) : a;
  }
}

// Pointer jumping: follow other nodes' current candidates (relaxed agent-scope
// loads; a stale value is an older, still-valid candidate, so the walk is
// correct under any visibility and converges by doubling).
__global__ void __launch_bounds__(BLOCK) k_ep_jump(OpsDev o, Work w, uint32_t* anc, uint8_t* sent_present) {
  const uint32_t n = o.n;
  GRID_STRIDE(x, n) {
    if (o.kind[x] != CRDTM_ADD || w.st[x] != ST_APPLIED) continue;
    const long long tx = o.ts[x];
    uint32_t c = anc[x];
    while (c < n && o.ts[c] > tx) {
      c = __hip_atomic_load(&anc[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&anc[x], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (c >= n) sent_present[c - n] = 1;
  }
}

__device__ __forceinline__ bool doc_present(const OpsDev& o, const Work& w, const uint8_t* sp, uint32_t v) {
  const uint32_t n = o.n;
  if (v < n) return o.kind[v] == CRDTM_ADD && w.st[v] == ST_APPLIED;
  if (v == n) return sp[n] != 0;  // root sentinel: present when the root dict has nodes
  return v == n + 1;
}

// parent uid of a present v != super root
__device__ __forceinline__ uint32_t doc_up(const OpsDev& o, const uint32_t* anc, uint32_t v) {
  const uint32_t n = o.n;
  if (v == n) return n + 1;
  const uint32_t a = anc[v];
  if (a < n) return a;         // ep-child (group 1)
  return a == 2 * n ? n : a - n;  // a root of dict P: child of P (group 0) / of the root sentinel
}

__device__ __forceinline__ bool doc_group1(const OpsDev& o, const uint32_t* anc, uint32_t v) {
  return v < o.n && anc[v] < o.n;
}

// Workgroup exclusive sum of one value per thread (*total: the workgroup's sum).
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t v, uint32_t* total) {
  __shared__ uint32_t sw[BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v);
  if (lane == 63) sw[wave] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (int k = 0; k < BLOCK / 64; ++k) {
    if (k < wave) base += sw[k];
    tot += sw[k];
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// Grouping by the document parent without atomics: every uid gets the key
// = its parent uid (NONE: not in the document tree) for a stable radix sort,
// then the group sizes come from the sorted keys (the first position of each
// group, then its size at its last position) and one scan makes them the
// children CSR. (The counting sort it replaces paid one random device
// atomic per node twice, counting and placing: deep10m 0.67 ms.)
// Also the sibling sort key and k_links' cleared outputs.
__global__ void __launch_bounds__(BLOCK) k_doc_keys(OpsDev o, Work w, const uint32_t* anc, const uint8_t* sp,
                                                    uint32_t* key, uint32_t* val, long long* skey, uint32_t* fc,
                                                    uint32_t* ns, uint32_t* f1, uint32_t* nitems) {
  const uint32_t n = o.n, U = n + 1;  // uids 0 .. n (the super root n + 1 has no parent)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    fc[U] = ns[U] = f1[U] = NONE;
    *nitems = U;
  }
  GRID_STRIDE(v, U) {
    fc[v] = NONE;
    ns[v] = NONE;
    f1[v] = NONE;
    val[v] = v;
    if (!doc_present(o, w, sp, v)) {
      key[v] = NONE;
      continue;
    }
    key[v] = doc_up(o, anc, v);
    skey[v] = v < n ? (doc_group1(o, anc, v) ? (1LL << 60) : 0LL) + (TWO53 - o.ts[v]) : 0LL;
  }
}

__global__ void __launch_bounds__(BLOCK) k_doc_gstart(const uint32_t* sk, uint32_t m, uint32_t* gs) {
  GRID_STRIDE(k, m) {
    const uint32_t u = sk[k];
    if (u != NONE && (k == 0 || sk[k - 1] != u)) gs[u] = k;
  }
}

__global__ void __launch_bounds__(BLOCK) k_doc_gcount(const uint32_t* sk, uint32_t m, const uint32_t* gs,
                                                      uint32_t* cnt) {
  GRID_STRIDE(k, m) {
    const uint32_t u = sk[k];
    if (u != NONE && (k + 1 == m || sk[k + 1] != u)) cnt[u] = k + 1 - gs[u];
  }
}

// fc = first child, ns = next sibling, f1 = first ep-child (group 1)
// pu[p] = the parent uid of carr[p] (the grouping sort's keys: sorting
// within a group keeps them); the neighbours' come from the adjacent lanes.
__global__ void __launch_bounds__(BLOCK) k_links(OpsDev o, const uint32_t* anc, const uint32_t* pu,
                                                 const uint32_t* total, const uint32_t* carr, uint32_t* fc,
                                                 uint32_t* ns, uint32_t* f1) {
  const uint32_t tot = *total;
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t p0 = blockIdx.x * blockDim.x; p0 < tot; p0 += gridDim.x * blockDim.x) {
    const uint32_t p = p0 + threadIdx.x;
    const bool valid = p < tot;
    const uint32_t v = valid ? carr[p] : NONE, u = valid ? pu[p] : NONE;
    const bool g1 = valid && doc_group1(o, anc, v);
    uint32_t up = __shfl_up(u, 1, 64), un = __shfl_down(u, 1, 64), vn = __shfl_down(v, 1, 64);
    bool g1p = __shfl_up(g1 ? 1u : 0u, 1, 64) != 0;
    if (!valid) continue;
    if (lane == 0 && p > 0) {
      up = pu[p - 1];
      g1p = doc_group1(o, anc, carr[p - 1]);
    }
    if (lane == 63 && p + 1 < tot) {
      un = pu[p + 1];
      vn = carr[p + 1];
    }
    const bool first = p == 0 || up != u;
    if (first) fc[u] = v;
    if (g1 && (first || !g1p)) f1[u] = v;
    ns[v] = (p + 1 < tot && un == u) ? vn : NONE;
  }
}

// Euler tour: entry 2v = enter v, 2v+1 = leave v. The weight of enter v is
// (1 << 32) | visible(v) (wbits 0b1x): the high word counts tour nodes
// (pre-order rank), the low word counts visible nodes (document rank).
__global__ void __launch_bounds__(BLOCK) k_euler(OpsDev o, Work w, const uint32_t* anc, const uint8_t* sp,
                                                 const uint32_t* fc, const uint32_t* ns, uint2* ent) {
  const uint32_t n = o.n, U = n + 2;
  GRID_STRIDE(v, U) {
    if (!doc_present(o, w, sp, v)) {
      ent[2 * v] = make_uint2(ABSENT, 0u);
      ent[2 * v + 1] = make_uint2(ABSENT, 0u);
      continue;
    }
    uint32_t after;
    if (v == n + 1) after = NONE;
    else if (ns[v] != NONE) after = 2 * ns[v];
    else after = 2 * doc_up(o, anc, v) + 1;
    uint32_t vis = 0;
    if (v < n) {
      const uint32_t p = w.addpar[v];
      vis = (w.dtime[v] == NONE && (p == n || !w.dead[p])) ? 1u : 0u;
    }
    const uint32_t f = fc[v];
    if (f == NONE && v != n + 1) {
      // a leaf: enter goes straight on and its leave entry is off the tour
      // (its rank = enter's + 1, k_next): ~45% fewer tour steps at deep10m
      ent[2 * v] = make_uint2(after, 2u | vis);
      ent[2 * v + 1] = make_uint2(ABSENT, 0u);
    } else {
      ent[2 * v] = make_uint2(f != NONE ? 2 * f : 2 * v + 1, 2u | vis);
      ent[2 * v + 1] = make_uint2(after, 0u);
    }
  }
}

// order[rank] = {node, its dict owner} (NONE for the sentinels): k_next
// takes the dict of the node after a subtree with the node itself, one
// gather instead of two
__global__ void __launch_bounds__(BLOCK) k_order(OpsDev o, Work w, const uint8_t* sp,
                                                 const unsigned long long* excl, uint2* order) {
  const uint32_t n = o.n, U = n + 2;
  GRID_STRIDE(v, U) {
    if (!doc_present(o, w, sp, v)) continue;
    order[static_cast<uint32_t>(excl[2 * v] >> 32)] = make_uint2(v, v < n ? w.addpar[v] : NONE);
  }
}

// next(x) within its dict (DESIGN.md "Raw next chains"): the first ep-child
// of x, else the pre-order successor of x's whole subtree when that node
// lives in the same dict.
__global__ void __launch_bounds__(BLOCK) k_next(OpsDev o, Work w, const unsigned long long* excl,
                                                const uint2* order, const uint32_t* f1, uint32_t* nextn) {
  const uint32_t n = o.n;
  // tour nodes = enter-weights before leave(super root)
  const uint32_t total = static_cast<uint32_t>(excl[2 * (n + 1) + 1] >> 32);
  GRID_STRIDE(x, n) {
    if (o.kind[x] != CRDTM_ADD || w.st[x] != ST_APPLIED) continue;
    uint32_t y = f1[x];  // (the first ep-child: in x's own dict)
    if (y == NONE) {
      // the tour node after x's subtree: leave x's rank, or for a leaf (its
      // leave entry off the tour, ~0) enter's + 1 (one 16-byte load)
      const ulonglong2 ex = *reinterpret_cast<const ulonglong2*>(excl + 2 * static_cast<uint64_t>(x));
      const uint32_t j = ex.y != ~0ULL ? static_cast<uint32_t>(ex.y >> 32) : static_cast<uint32_t>(ex.x >> 32) + 1u;
      if (j < total) {
        const uint2 e = order[j];
        y = e.y == w.addpar[x] ? e.x : NONE;
      }
    }
    nextn[x] = y;
  }
}

// ---------------------------------------------------------------------------
// K3 + commit — tombstones, kept/live flags, op log, tree state.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(BLOCK) k_commit_flags(OpsDev o, Work w, uint32_t* appl, uint32_t* plen,
                                                        uint32_t* kept, uint32_t* live) {
  const uint32_t n = o.n;
  GRID_STRIDE(i, n) {
    const bool a = w.st[i] == ST_APPLIED;
    if (appl) appl[i] = a;  // (null when every op applied: the log is the batch)
    if (plen) plen[i] = a ? op_len(o, i) : 0;
    uint32_t k = 0, l = 0;
    if (a && o.kind[i] == CRDTM_ADD) {
      const uint32_t p = w.addpar[i];
      k = (p == n || !w.dead[p]) ? 1 : 0;
      l = (k && w.dtime[i] == NONE) ? 1 : 0;
    }
    if (kept) kept[i] = k;
    if (live) live[i] = l;
  }
}

struct CommitArgs {
  uint32_t base_slot;     // first new slot
  uint32_t n_kept;        // K
  uint32_t base_dict;     // first new dict
  uint32_t log_base;
};

__global__ void __launch_bounds__(BLOCK) k_commit_nodes(OpsDev o, Work w, TreeDev T, CommitArgs a,
                                                        const uint32_t* kslot, const uint32_t* lslot,
                                                        const uint32_t* logidx, const uint32_t* nextn,
                                                        const uint32_t* fc, const unsigned long long* excl,
                                                        uint32_t* doc) {
  const uint32_t n = o.n;
  GRID_STRIDE(x, n) {
    if (o.kind[x] != CRDTM_ADD || w.st[x] != ST_APPLIED) continue;
    const uint32_t p = w.addpar[x];
    if (p != n && w.dead[p]) continue;  // dict discarded (owner or an ancestor tombstoned)
    const uint32_t slot = a.base_slot + kslot[x];
    const bool tomb = w.dtime[x] != NONE;
    T.s_key[slot] = o.ts[x];
    T.s_dict[slot] = p == n ? 0u : a.base_dict + lslot[p];
    T.s_next[slot] = nextn[x] != NONE ? a.base_slot + kslot[nextn[x]] : NONE;
    T.s_src[slot] = a.log_base + (logidx ? logidx[x] : x);
    T.s_flags[slot] = tomb ? F_TOMB : 0;
    if (!tomb) {
      const uint32_t dd = a.base_dict + lslot[x];
      const uint32_t ss = a.base_slot + a.n_kept + lslot[x];
      T.s_child[slot] = dd;
      T.s_key[ss] = 0;
      T.s_dict[ss] = dd;
      const uint32_t f = fc[x];  // first root of x's own dict (group 0), if any
      T.s_next[ss] = (f != NONE && w.addpar[f] == x) ? a.base_slot + kslot[f] : NONE;
      T.s_src[ss] = NONE;
      T.s_child[ss] = NONE;
      T.s_flags[ss] = F_TOMB | F_SENT;
      T.d_sent[dd] = ss;
      T.d_owner[dd] = slot;
      doc[static_cast<uint32_t>(excl[2 * x])] = slot;  // document rank (low word) -> slot
    } else {
      T.s_child[slot] = NONE;
    }
  }
}

__global__ void k_commit_root(OpsDev o, TreeDev T, const uint32_t* kslot, const uint32_t* fc, uint32_t base_slot) {
  const uint32_t f = fc[o.n];  // root sentinel's first child
  T.s_next[0] = f != NONE ? base_slot + kslot[f] : NONE;
}

// Append applied ops to the log (operations, src/CRDTree.elm:311).
// One block per chunk of BLOCK ops: the op records first, then the chunk's
// path elements (contiguous in the input) one per thread, each finding its op
// by a binary search over the chunk's offsets in LDS (coalesced reads; writes
// contiguous across applied ops).
__global__ void __launch_bounds__(BLOCK) k_log(OpsDev o, const uint8_t* st, TreeDev T, uint32_t log_base,
                                               uint32_t lpath_base, const uint32_t* logidx, const uint32_t* lpoff) {
  __shared__ uint32_t soff[BLOCK + 1];
  __shared__ uint32_t sdst[BLOCK];
  const uint32_t n = o.n;
  const uint32_t chunks = (n + BLOCK - 1) / BLOCK;
  for (uint32_t c = blockIdx.x; c < chunks; c += gridDim.x) {
    const uint32_t i0 = c * BLOCK, cnt = min(static_cast<uint32_t>(BLOCK), n - i0);
    const uint32_t t = threadIdx.x;
    if (t < cnt) {
      const uint32_t i = i0 + t;
      soff[t] = o.off[i];
      uint32_t dst = NONE;
      if (st[i] == ST_APPLIED) {
        // logidx / lpoff null: every op applied, log index = op index and
        // path offsets = the batch's (off[0] == 0)
        const uint32_t li = log_base + (logidx ? logidx[i] : i);
        const bool add = o.kind[i] == CRDTM_ADD;
        T.l_kind[li] = o.kind[i];
        T.l_ts[li] = add ? o.ts[i] : 0;
        T.l_val[li] = add ? o.val[i] : 0;
        dst = lpath_base + (lpoff ? lpoff[i] : soff[t]);
        T.l_off[li] = dst;
      }
      sdst[t] = dst;
    }
    if (t == 0) soff[cnt] = o.off[i0 + cnt];
    __syncthreads();
    const uint32_t p0 = soff[0], p1 = soff[cnt];
    for (uint32_t p = p0 + t; p < p1; p += BLOCK) {
      uint32_t lo = 0, hi = cnt;  // last op j with soff[j] <= p
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (soff[mid] <= p) lo = mid;
        else hi = mid;
      }
      const uint32_t d = sdst[lo];
      if (d != NONE) T.l_path[d + (p - soff[lo])] = o.path[p];
    }
    __syncthreads();
  }
}

__global__ void k_log_totals(DevResult* d, uint32_t n, uint32_t npath) {
  d->log_n = n;
  d->log_npath = npath;
}

__global__ void k_log_tail(TreeDev T, uint32_t log_base, const uint32_t* n_app, uint32_t lpath_base,
                           const uint32_t* n_path) {
  T.l_off[log_base + *n_app] = lpath_base + *n_path;
}

// replicas[replicaId t] := t, last writer wins (src/CRDTree.elm:313). For a
// Delete t is the deleted node's key (Operation.timestamp, src/Internal/Operation.elm:100-101).
__device__ __forceinline__ long long op_t(const OpsDev& o, uint32_t i) {
  return o.kind[i] == CRDTM_ADD ? o.ts[i] : o.path[o.off[i + 1] - 1];
}

// Each block folds rep_per * BLOCK consecutive ops into a direct-mapped LDS
// table (replica id < REP_DIRECT -> 1 + its last applied op; other ids go
// straight to the global table), loading four ops per thread at a time so the
// dependent loads of op_t overlap. Same-address LDS atomics serialise, and a
// batch has few replicas, so each wave first reduces per replica: the lanes
// of one replica hold consecutive op indices, the highest of them publishes.
// The block then publishes one atomicMax per replica it saw; the first
// publisher of a replica (the table entry was 0) appends it to `rlist`, so the
// output pass visits the touched replicas only.
// ops per thread: 16 on large batches (fewer table flushes), 4 on small ones (more workgroups in flight)
inline uint32_t rep_per(uint32_t n) { return n >= (1u << 22) ? 16u : 4u; }
constexpr uint32_t REP_ROUNDS = 1;
// replica rl (offset id) saw op v - 1: the LDS table for small ids, else the
// global table (its first publisher appends it to the touched list)
__device__ __forceinline__ void rep_publish(uint32_t* rv, uint32_t* rtab, uint32_t* rlist, uint32_t* rcount,
                                            uint32_t rl, uint32_t v, uint32_t& mr) {
  constexpr uint32_t OFF = 1u << (REPLICA_BITS - 1);
  const uint32_t d = rl - OFF;  // (ids below 0 wrap high: global table)
  if (d < REP_DIRECT) {
    atomicMax(&rv[d], v);
    mr = max(mr, d);
  } else if (atomicMax(&rtab[rl], v) == 0) {
    rlist[atomicAdd(rcount, 1u)] = rl;
  }
}
__global__ void __launch_bounds__(BLOCK) k_rep_max(OpsDev o, const uint8_t* st, uint32_t* rtab, uint32_t* rlist,
                                                   uint32_t* rcount, uint32_t per) {
  __shared__ uint32_t rv[REP_DIRECT];
  for (uint32_t j = threadIdx.x; j < REP_DIRECT; j += blockDim.x) rv[j] = 0;
  __syncthreads();
  const uint32_t n = o.n;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t b0 = blockIdx.x * (BLOCK * per) + threadIdx.x;
  constexpr uint32_t OFF = 1u << (REPLICA_BITS - 1);
  uint32_t mr = 0;
  for (uint32_t k0 = 0; k0 < per; k0 += 4) {
    uint32_t ii[4];
    bool ok[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      ii[u] = b0 + (k0 + u) * BLOCK;
      ok[u] = ii[u] < n && st[ii[u]] == ST_APPLIED;
    }
    long long t[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) t[u] = ok[u] ? op_t(o, ii[u]) : 0;
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t r = static_cast<uint32_t>(replica_of(t[u]) + OFF);
      bool pend = ok[u];
      // up to REP_ROUNDS replicas per wave reduce first (one atomic each); a
      // wave holding more (many replicas interleaved) sends the rest to the
      // table lane by lane -- different words, so those atomics run in parallel
      // (1 round measured best: incremental batch 0.398 -> 0.391 ms, 4 rounds
      // and more cost a ballot loop per extra replica)
      uint32_t round = 0;
      for (unsigned long long m = __ballot(pend); m && round < REP_ROUNDS; m = __ballot(pend), ++round) {
        const uint32_t rl = __builtin_amdgcn_readlane(r, static_cast<uint32_t>(__builtin_ctzll(m)));
        const unsigned long long mm = __ballot(pend && r == rl);
        if (lane == 63u - static_cast<uint32_t>(__builtin_clzll(mm))) rep_publish(rv, rtab, rlist, rcount, rl, ii[u] + 1, mr);
        if (r == rl) pend = false;
      }
      if (pend) rep_publish(rv, rtab, rlist, rcount, r, ii[u] + 1, mr);
    }
  }
  mr = block_max(mr);  // (synchronises the block) only ids <= mr were touched
  for (uint32_t j = threadIdx.x; j <= mr; j += blockDim.x)
    if (rv[j] && atomicMax(&rtab[j + OFF], rv[j]) == 0) rlist[atomicAdd(rcount, 1u)] = j + OFF;
}

inline uint32_t rep_grid(uint32_t n) { return grid_for(n, BLOCK * rep_per(n)); }

// One thread per touched replica: the winner is op rtab[r] - 1; the entry is
// cleared (the table stays clean between calls).
__global__ void __launch_bounds__(BLOCK) k_rep_out(OpsDev o, uint32_t* rtab, const uint32_t* rlist,
                                                   const uint32_t* rcount, long long* out, uint32_t* n_out,
                                                   long long* inl) {
  const uint32_t nr = *rcount;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nr; k += gridDim.x * blockDim.x) {
    const uint32_t r = rlist[k];
    const uint32_t i = rtab[r] - 1;
    rtab[r] = 0;
    const long long t = op_t(o, i);
    out[2 * k] = replica_of(t);
    out[2 * k + 1] = t;
    if (k < REP_INLINE) {
      inl[2 * k] = replica_of(t);
      inl[2 * k + 1] = t;
    }
    if (k == 0) *n_out = nr;
  }
}

// st == nullptr: every op applied (the flat speculation writes no statuses)
__global__ void __launch_bounds__(BLOCK) k_status_out(const uint8_t* st, uint32_t n, uint32_t err, uint8_t* out) {
  GRID_STRIDE(i, n) {
    uint8_t s = st ? st[i] : static_cast<uint8_t>(ST_APPLIED);
    if (i > err) s = CRDTM_ST_UNREACHED;
    else if (s == ST_INVALID || s == ST_NOTFOUND) s = CRDTM_ST_ERROR;
    out[i] = s;
  }
}

// ---------------------------------------------------------------------------
// Exact replay (one lane per tree): the reference's literal sequential
// semantics over the slot state, including the findInsertion copy quirk
// (src/Internal/Node.elm:87-89 with leftTs != key(left)) as a persistent deep
// copy of the copied node's children. In-place edits of committed slots are
// undo-logged so that an error leaves the tree unchanged.
// ---------------------------------------------------------------------------
struct ReplayArgs {
  TreeDev T;
  SlotHash H;
  uint32_t* dhead;   // per dict: first member slot
  uint32_t* mnext;   // per slot: next member of the same dict
  uint32_t* undo;    // triples (slot, field, old)
  uint32_t undo_cap;
  uint32_t* queue;   // deep-copy BFS queue of (src dict, dst dict)
  uint32_t queue_cap;
  uint32_t committed_slots;
  uint32_t n_slots, n_dicts;
  uint32_t cap_slots, cap_dicts;
  uint32_t hash_limit;
  uint32_t log_base;
  long long ts0;
  uint32_t root_dict;   // 0 for a tree state; a document's own root dict in a forest
  uint32_t src_is_op;   // forest: s_src = global op index (no log is kept)
};

enum : uint32_t { UF_NEXT = 0, UF_SRC = 1, UF_CHILD = 2, UF_FLAGS = 3 };

struct Replayer {
  ReplayArgs a;
  uint32_t slots, dicts, inserted, undo_n;
  bool overflow;

  __device__ void log_undo(uint32_t s, uint32_t field, uint32_t old) {
    if (s >= a.committed_slots) return;
    if (undo_n + 1 > a.undo_cap) { overflow = true; return; }
    a.undo[3 * undo_n] = s;
    a.undo[3 * undo_n + 1] = field;
    a.undo[3 * undo_n + 2] = old;
    ++undo_n;
  }
  __device__ void set_next(uint32_t s, uint32_t v) { log_undo(s, UF_NEXT, a.T.s_next[s]); a.T.s_next[s] = v; }
  __device__ void set_src(uint32_t s, uint32_t v) { log_undo(s, UF_SRC, a.T.s_src[s]); a.T.s_src[s] = v; }
  __device__ void set_child(uint32_t s, uint32_t v) { log_undo(s, UF_CHILD, a.T.s_child[s]); a.T.s_child[s] = v; }
  __device__ void set_flags(uint32_t s, uint32_t v) { log_undo(s, UF_FLAGS, a.T.s_flags[s]); a.T.s_flags[s] = static_cast<uint8_t>(v); }

  __device__ void rollback() {
    while (undo_n > 0) {
      --undo_n;
      const uint32_t s = a.undo[3 * undo_n], f = a.undo[3 * undo_n + 1], v = a.undo[3 * undo_n + 2];
      if (f == UF_NEXT) a.T.s_next[s] = v;
      else if (f == UF_SRC) a.T.s_src[s] = v;
      else if (f == UF_CHILD) a.T.s_child[s] = v;
      else a.T.s_flags[s] = static_cast<uint8_t>(v);
    }
  }

  __device__ uint32_t new_slot(uint32_t d, long long key, uint32_t next, uint32_t src, uint32_t child, uint8_t flags) {
    if (slots >= a.cap_slots || inserted + 1 > a.hash_limit) { overflow = true; return NONE; }
    const uint32_t s = slots++;
    a.T.s_key[s] = key;
    a.T.s_dict[s] = d;
    a.T.s_next[s] = next;
    a.T.s_src[s] = src;
    a.T.s_child[s] = child;
    a.T.s_flags[s] = flags;
    slothash_put_seq(a.H, d, key, s);
    ++inserted;
    a.mnext[s] = a.dhead[d];
    a.dhead[d] = s;
    return s;
  }

  __device__ uint32_t new_dict(uint32_t owner) {
    if (dicts >= a.cap_dicts) { overflow = true; return NONE; }
    const uint32_t d = dicts++;
    a.dhead[d] = NONE;
    a.T.d_owner[d] = owner;
    a.T.d_sent[d] = NONE;
    return d;
  }

  // The children dict of live node s, created on first use: a dict holding
  // only its sentinel (emptyChildren, src/Internal/Node.elm:46-48).
  __device__ uint32_t materialise(uint32_t s) {
    const uint32_t dd = new_dict(s);
    if (dd == NONE) return NONE;
    const uint32_t ss = new_slot(dd, 0, NONE, NONE, NONE, F_TOMB | F_SENT);
    if (ss == NONE) return NONE;
    a.T.d_sent[dd] = ss;
    set_child(s, dd);
    return dd;
  }

  // Persistent copy of dict `src` (and every dict below it) into `dst`.
  __device__ void deep_copy(uint32_t src, uint32_t dst) {
    uint32_t qh = 0, qt = 0;
    a.queue[0] = src;
    a.queue[1] = dst;
    qt = 1;
    while (qh < qt && !overflow) {
      const uint32_t sd = a.queue[2 * qh], dd = a.queue[2 * qh + 1];
      ++qh;
      for (uint32_t m = a.dhead[sd]; m != NONE && !overflow; m = a.mnext[m]) {
        const uint8_t fl = a.T.s_flags[m];
        const uint32_t nm = new_slot(dd, a.T.s_key[m], NONE, a.T.s_src[m], NONE, fl);
        if (nm == NONE) break;
        if (fl & F_SENT) a.T.d_sent[dd] = nm;
        const uint32_t c = a.T.s_child[m];
        if (c != NONE) {
          const uint32_t nc = new_dict(nm);
          if (nc == NONE) break;
          a.T.s_child[nm] = nc;
          if (qt + 1 > a.queue_cap) { overflow = true; break; }
          a.queue[2 * qt] = c;
          a.queue[2 * qt + 1] = nc;
          ++qt;
        }
      }
      // re-link `next` keys inside the copy
      for (uint32_t m = a.dhead[sd]; m != NONE && !overflow; m = a.mnext[m]) {
        const uint32_t nx = a.T.s_next[m];
        if (nx == NONE) continue;
        const uint32_t nm = slothash_find(a.H, dd, a.T.s_key[m]);
        a.T.s_next[nm] = slothash_find(a.H, dd, a.T.s_key[nx]);
      }
    }
  }

  // One op; returns ST_* (src/CRDTree.elm:275-295 with src/Internal/Node.elm).
  __device__ uint8_t op(const OpsDev& o, uint32_t i, uint32_t applied) {
    const uint32_t b = o.off[i], L = o.off[i + 1] - b;
    if (L == 0) return ST_INVALID;
    uint32_t d = a.root_dict;
    for (uint32_t l = 0; l + 1 < L; ++l) {  // update: descend
      const uint32_t s = slothash_find(a.H, d, o.path[b + l]);
      if (s == NONE) return ST_INVALID;
      if (a.T.s_flags[s] & F_TOMB) return ST_ALREADY;
      d = a.T.s_child[s];
      if (d == NONE) {  // an implicit empty children dict: materialise it
        d = materialise(s);
        if (d == NONE) return ST_PENDING;
      }
    }
    const long long k = o.path[b + L - 1];
    if (o.kind[i] == CRDTM_DELETE) {  // deleteHelp
      const uint32_t s = slothash_find(a.H, d, k);
      if (s == NONE) return ST_NOTFOUND;
      if (a.T.s_flags[s] & F_TOMB) return ST_ALREADY;
      set_flags(s, a.T.s_flags[s] | F_TOMB);
      set_child(s, NONE);  // Tombstone drops the children
      return ST_APPLIED;
    }
    const long long ts = o.ts[i];  // addAfterHelp
    if (slothash_find(a.H, d, ts) != NONE) return ST_ALREADY;
    const uint32_t found = slothash_find(a.H, d, k);
    if (found == NONE) return ST_NOTFOUND;
    long long nkey = k;  // findInsertion
    uint32_t node = found;
    for (;;) {
      const uint32_t rn = a.T.s_next[node];
      if (rn == NONE) break;
      uint32_t live = rn;
      while (live != NONE && (a.T.s_flags[live] & F_TOMB)) live = a.T.s_next[live];
      if (live == NONE) break;
      const long long rk = a.T.s_key[rn];
      if (ts > rk) break;
      nkey = rk;
      node = live;
    }
    // the new Node's children {0: Tombstone} (src/Internal/Node.elm:85) stay
    // implicit until something descends into it
    const uint32_t x = new_slot(d, ts, a.T.s_next[node], a.src_is_op ? i : a.log_base + applied, NONE, 0);
    if (x == NONE) return ST_PENDING;
    const uint32_t ls = slothash_find(a.H, d, nkey);
    // x is reachable from the dict's sentinel iff its predecessor is (an Add
    // anchored at an orphan hangs off the chain)
    if (a.T.s_flags[ls] & F_ORPHAN) a.T.s_flags[x] |= F_ORPHAN;
    if (ls == node) {
      set_next(node, x);
    } else {
      // copy quirk: slot nkey := copy of node with next = ts; the entries
      // between it and node drop off the chain (orphans) when it was on it.
      if (!(a.T.s_flags[ls] & F_ORPHAN)) {
        for (uint32_t q = a.T.s_next[ls]; q != NONE; q = a.T.s_next[q]) {
          set_flags(q, a.T.s_flags[q] | F_ORPHAN);
          if (q == node) break;
        }
      }
      set_src(ls, a.T.s_src[node]);
      set_flags(ls, (a.T.s_flags[node] & ~F_ORPHAN) | (a.T.s_flags[ls] & F_ORPHAN));
      set_next(ls, x);
      const uint32_t c = a.T.s_child[node];
      uint32_t nc = NONE;
      if (c != NONE) {
        nc = new_dict(ls);
        if (nc == NONE) return ST_PENDING;
        deep_copy(c, nc);
        if (overflow) return ST_PENDING;
      }
      set_child(ls, nc);
    }
    return overflow ? ST_PENDING : ST_APPLIED;
  }
};

__global__ void k_replay(OpsDev o, ReplayArgs args, uint8_t* st, DevResult* dres) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Replayer r;
  r.a = args;
  r.slots = args.n_slots;
  r.dicts = args.n_dicts;
  r.inserted = args.n_slots;
  r.undo_n = 0;
  r.overflow = false;
  long long ts = args.ts0;
  uint32_t applied = 0, already = 0, err = NONE, code = 0;
  for (uint32_t i = 0; i < o.n; ++i) {
    const uint8_t s = r.op(o, i, applied);
    if (r.overflow) break;
    st[i] = s;
    if (s == ST_INVALID || s == ST_NOTFOUND) {
      err = i;
      code = s == ST_INVALID ? CRDTM_INVALID_PATH : CRDTM_OPERATION_FAILED;
      break;
    }
    if (s == ST_APPLIED) ++applied;
    else ++already;
    // incrementTimestamp (src/CRDTree.elm:337-343): Ok Adds of the own replica
    if (o.kind[i] == CRDTM_ADD && replica_of(o.ts[i]) == replica_of(ts)) ++ts;
  }
  if (r.overflow || err != NONE) r.rollback();
  dres->replay_overflow = r.overflow ? 1u : 0u;
  dres->err_index = err;
  dres->replay_err_code = code;
  dres->n_applied = applied;
  dres->n_already = already;
  dres->replay_slots = r.slots;
  dres->replay_dicts = r.dicts;
  dres->replay_timestamp = ts;
}

// Build the (dict, key) -> slot hash and the dict member lists of the state.
__global__ void __launch_bounds__(BLOCK) k_replay_index(TreeDev T, uint32_t n_slots, SlotHash H, uint32_t* dhead,
                                                        uint32_t* mnext) {
  GRID_STRIDE(s, n_slots) {
    const uint32_t d = T.s_dict[s];
    slothash_put_par(H, d, T.s_key[s], s);
    mnext[s] = atomicExch(&dhead[d], s);
  }
}

// ---------------------------------------------------------------------------
// Generic linearisation of a tree state (document order of any state, e.g.
// after a replay): entries enter(s) = s, exit(d) = S + d. A dict is alive when
// every owner up its chain is an on-chain live node.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(BLOCK) k_dict_alive_init(TreeDev T, uint32_t n_dicts, uint8_t* ok, uint32_t* up) {
  GRID_STRIDE(d, n_dicts) {
    if (d == 0) { ok[d] = 1; up[d] = 0; continue; }
    const uint32_t o = T.d_owner[d];
    const bool good = o != NONE && T.s_child[o] == d && !(T.s_flags[o] & (F_TOMB | F_ORPHAN));
    ok[d] = good ? 1 : 0;
    up[d] = good ? T.s_dict[o] : 0;
  }
}

__global__ void __launch_bounds__(BLOCK) k_dict_alive_jump(uint32_t n_dicts, uint8_t* ok, uint32_t* up,
                                                           uint8_t* ok2, uint32_t* up2) {
  GRID_STRIDE(d, n_dicts) {
    const uint32_t u = up[d];
    ok2[d] = ok[d] & ok[u];
    up2[d] = up[u];
  }
}

__global__ void __launch_bounds__(BLOCK) k_lin_entries(TreeDev T, uint32_t S, uint32_t D, const uint8_t* alive,
                                                       uint2* ent) {
  GRID_STRIDE(e, S + D) {
    if (e < S) {
      const uint32_t s = e;
      const uint8_t f = T.s_flags[s];
      if (!alive[T.s_dict[s]] || (f & F_ORPHAN)) { ent[e] = make_uint2(ABSENT, 0u); continue; }
      const uint32_t c = T.s_child[s];
      uint32_t nx;
      if (!(f & F_TOMB) && c != NONE) nx = T.d_sent[c];
      else nx = T.s_next[s] != NONE ? T.s_next[s] : S + T.s_dict[s];
      ent[e] = make_uint2(nx, (f & F_TOMB) ? 0u : 1u);
    } else {
      const uint32_t d = e - S;
      if (!alive[d]) { ent[e] = make_uint2(ABSENT, 0u); continue; }
      if (d == 0) { ent[e] = make_uint2(NONE, 0u); continue; }
      const uint32_t o = T.d_owner[d];
      ent[e] = make_uint2(T.s_next[o] != NONE ? T.s_next[o] : S + T.s_dict[o], 0u);
    }
  }
}

__global__ void __launch_bounds__(BLOCK) k_lin_doc(TreeDev T, uint32_t S, const unsigned long long* excl,
                                                   uint32_t* doc, uint64_t cap) {
  GRID_STRIDE(s, S) {
    const unsigned long long e = excl[s];
    if (e == ~0ULL) continue;
    const uint8_t f = T.s_flags[s];
    if (f & (F_TOMB | F_ORPHAN)) continue;
    if (e < cap) doc[static_cast<uint32_t>(e)] = s;
  }
}

// ---------------------------------------------------------------------------
// Forest: many independent documents, each replayed
// exactly by one lane (documents are the parallel axis; cfg-5 streams
// interleave Deletes with concurrent inserts, where the closed form's guard
// rarely holds). Each lane owns a region of the slot/dict/hash arenas sized
// from its op count, and ends by hashing its visible document with the same
// canonical words as the oracle (FNV-1a over depth, value, path).
// ---------------------------------------------------------------------------
struct ForestArgs {
  TreeDev T;               // shared slot/dict arrays (per-document regions)
  const uint32_t* doc_off; // [n_docs + 1] ops of document d = [doc_off[d], doc_off[d+1])
  uint32_t n_docs;
  long long ts0;
  uint32_t* dhead;
  uint32_t* mnext;
  uint32_t* hdict;
  long long* hkey;
  uint32_t* hslot;
  uint32_t* queue;
  int32_t* code;
  uint32_t* err;
  uint32_t* applied;
  unsigned long long* vhash;
  unsigned long long* vwords;
  long long* tstamp;
  uint32_t* overflow;
};

__host__ __device__ __forceinline__ uint64_t forest_slot_cap(uint32_t nops) { return 2ULL * nops + 64; }
__host__ __device__ __forceinline__ uint64_t forest_dict_cap(uint32_t nops) { return nops + 32; }
__host__ __device__ __forceinline__ uint32_t forest_hash_cap(uint32_t nops) {
  uint32_t h = 64;
  while (h < 2 * forest_slot_cap(nops)) h <<= 1;
  return h;
}

__global__ void __launch_bounds__(64) k_forest(OpsDev o, ForestArgs f, const uint64_t* sbase, const uint64_t* dbase,
                                               const uint64_t* hbase, const uint8_t* fb) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= f.n_docs || !fb[d]) return;  // served by k_forest_prep / k_forest_wave
  {
    uint32_t* hs = f.hslot + hbase[d];  // this document's hash region starts empty
    for (uint32_t p = 0, H = forest_hash_cap(f.doc_off[d + 1] - f.doc_off[d]); p < H; ++p) hs[p] = NONE;
  }
  const uint32_t ob = f.doc_off[d], oe = f.doc_off[d + 1], nops = oe - ob;
  const uint32_t s0 = static_cast<uint32_t>(sbase[d]), d0 = static_cast<uint32_t>(dbase[d]);
  const uint32_t H = forest_hash_cap(nops);
  // fresh document: root dict d0 with its sentinel slot s0
  Replayer r;
  r.a.T = f.T;
  r.a.H.dict = f.hdict + hbase[d];
  r.a.H.key = f.hkey + hbase[d];
  r.a.H.slot = f.hslot + hbase[d];
  r.a.H.mask = H - 1;
  r.a.dhead = f.dhead;
  r.a.mnext = f.mnext;
  r.a.undo = nullptr;
  r.a.undo_cap = 0;
  r.a.queue = f.queue + 2 * dbase[d];
  r.a.queue_cap = static_cast<uint32_t>(forest_dict_cap(nops));
  r.a.committed_slots = s0;  // nothing to undo: every slot of the document is new
  r.a.n_slots = s0;
  r.a.n_dicts = d0;
  r.a.cap_slots = s0 + static_cast<uint32_t>(forest_slot_cap(nops));
  r.a.cap_dicts = d0 + static_cast<uint32_t>(forest_dict_cap(nops));
  r.a.hash_limit = H / 2;
  r.a.log_base = 0;
  r.a.ts0 = f.ts0;
  r.a.root_dict = d0;
  r.a.src_is_op = 1;
  r.slots = s0;
  r.dicts = d0;
  r.inserted = 0;
  r.undo_n = 0;
  r.overflow = false;
  f.dhead[d0] = NONE;
  f.T.d_owner[d0] = NONE;
  r.dicts = d0 + 1;
  const uint32_t root = r.new_slot(d0, 0, NONE, NONE, NONE, F_TOMB | F_SENT);
  f.T.d_sent[d0] = root;
  long long ts = f.ts0;
  uint32_t applied = 0, err = NONE;
  int32_t code = CRDTM_OK;
  for (uint32_t i = ob; i < oe; ++i) {
    const uint8_t s = r.op(o, i, applied);
    if (r.overflow) break;
    if (s == ST_INVALID || s == ST_NOTFOUND) {
      err = i - ob;
      code = s == ST_INVALID ? CRDTM_INVALID_PATH : CRDTM_OPERATION_FAILED;
      break;
    }
    if (s == ST_APPLIED) ++applied;
    if (o.kind[i] == CRDTM_ADD && replica_of(o.ts[i]) == replica_of(ts)) ++ts;
  }
  f.overflow[d] = r.overflow ? 1u : 0u;
  f.code[d] = code;
  f.err[d] = err;
  f.applied[d] = applied;
  f.tstamp[d] = ts;
  // visible document, pre-order (the oracle's dumpVisible words)
  Fnv h;
  if (code == CRDTM_OK && !r.overflow) {
    constexpr int MAXD = 64;
    uint32_t stack[MAXD];
    int depth = 0;
    stack[0] = root;
    while (depth >= 0) {
      uint32_t nx = f.T.s_next[stack[depth]];
      while (nx != NONE && (f.T.s_flags[nx] & F_TOMB)) nx = f.T.s_next[nx];
      if (nx == NONE) { --depth; continue; }
      stack[depth] = nx;
      const uint32_t src = f.T.s_src[nx];
      const uint32_t pb = o.off[src], pe = o.off[src + 1];
      h.put(depth);
      h.put(static_cast<long long>(o.val[src]));
      h.put(static_cast<long long>(pe - pb));
      for (uint32_t j = pb; j + 1 < pe; ++j) h.put(o.path[j]);
      h.put(o.ts[src]);
      const uint32_t c = f.T.s_child[nx];
      if (c != NONE && depth + 1 < MAXD) stack[++depth] = f.T.d_sent[c];
      else if (c != NONE) f.overflow[d] = 2u;
    }
  }
  f.vhash[d] = h.h;
  f.vwords[d] = h.n;
}

// ---------------------------------------------------------------------------
// Flat closed form in timestamp-slot space: a fresh tree, a single-level
// Adds-only batch, and a dense timestamp index. Node q = the dense slot of
// its timestamp (base[replica] + counter - min counter[replica]), so slot order IS
// timestamp order (src/Internal/Node.elm:100 compares the Int key), and a
// replica's typing run x_c -> x_{c+1} -> ... occupies consecutive slots: the
// effective-parent chains, the child counting, the Euler tour and the
// list-ranking walks step through memory sequentially instead of hopping
// ~R ops apart. The root dict's sentinel (key 0, -inf in the order) is node
// Q. anc[q] = ABSENT marks a slot without an applied Add.
// ---------------------------------------------------------------------------

// K1 (flat). Slot records rec[q] = {x: the anchor code of slot q's Add (its
// anchor slot, Q = the dict's sentinel, or `anone` = anchor key not in the
// batch) tagged with the merge's epoch, y: that Add's op index} (y is valid
// only where x is present; one 8-byte record, so the claim scatters one store
// per op and a reader of both halves touches one line). rec is the context's
// own buffer (engine.h crdtm_ctx::fl_rec): every flat merge takes the next
// epoch (1..62), so a slot whose word carries another epoch holds no Add and
// nothing clears the buffer between merges (a clearing pass wrote 80 MB per
// 10M-slot merge); the buffer is zeroed when the epochs wrap. Narrow mode
// packs the epoch into the top 6 bits of x and needs Q < 2^26 - 2; wide mode
// (larger Q) keeps full 32-bit anchor codes and clears x to FR_EMPTY before
// each merge (k_fl_init).
constexpr uint32_t FR_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t FR_ABITS = 26;
constexpr uint32_t FR_EPOCHS = 62;  // (epoch 63 with a missing anchor would read as FR_EMPTY)
struct FlatRec {
  uint2* rec;
  uint32_t ep;     // epoch << FR_ABITS (narrow), 0 (wide)
  uint32_t amask;  // anchor code field
  uint32_t anone;  // code of a missing anchor
  // the flat speculation launches the merge before the host knows the slot
  // range: the kernels then read it here (range_total; the host passed an
  // upper bound for grids and buffers) and the replica count (max_replica)
  const uint32_t* qd = nullptr;
  const uint32_t* nrd = nullptr;
  // (the bound stays the limit: a batch whose range exceeds it reads as cut
  // off, and the host discards the speculation)
  __device__ __forceinline__ uint32_t q(uint32_t Q) const { return qd ? min(*qd, Q) : Q; }
  __device__ __forceinline__ uint32_t nrep(uint32_t nr) const { return nrd ? min(nr, *nrd + 1u) : nr; }
  __device__ __forceinline__ bool present(uint32_t w) const { return w != FR_EMPTY && (w & ~amask) == ep; }
  __device__ __forceinline__ uint32_t code(uint32_t qa) const { return (qa == NONE ? anone : qa) | ep; }
  // slot, Q (the sentinel) or NONE
  __device__ __forceinline__ uint32_t anchor(uint32_t w) const {
    const uint32_t a = w & amask;
    return a == anone ? NONE : a;
  }
};

// K1 (flat), one pass over the ops: every Add writes its slot record with
// one plain 8-byte store (an arbitrary duplicate wins), and the pass folds
// what the batch accounting needs when every op applies — the last Add
// index per replica (replicas table), the own-replica Add count
// (incrementTimestamp), the Adds with a slot, and the ops that would not
// apply on their own (empty path: InvalidPath, its smallest index to
// err_index; ts 0: the sentinel's key, AlreadyApplied). The order's slot
// pass (k_run_expand with `chk`) then checks every slot's Add against its
// anchor and counts the slots: as many slots as keyed Adds means no duplicate
// timestamps. Only a batch where some op does not apply runs the per-op
// k_fl_status.
// track_rep = 0: k_run_expand folds the replicas table from the records
// instead (slot order: a wave's slots stay inside one replica's range, no
// per-op LDS atomics).
// log_to_tree: the flat speculation (fresh tree, every op applies) also
// appends the batch to the log here (it IS the log: same CSR layout, path
// elements [0, n_path)), so the ops stream from HBM once for both.
// SIMPLE: every op is an Add with a one-element path (k_pre: no Delete, the
// longest path 1 and as many path elements as ops), so op i's anchor is
// path[i]: the pass reads the timestamps, anchors (and values for the log) as
// 16-byte vectors and writes the log's kinds and offsets without reading them.
// VERIFY (the speculation launched without the pre-pass's kinds and path
// lengths): the pass also checks that every op is an Add whose path is
// path[i] alone (kind, and path_off[i] == i), else DevResult::spec_fail.
// SPEC (the flat speculation's instance): log_to_tree, no per-op replica
// tracking, the range table in LDS — the other cases' branches compiled out.
template <bool SIMPLE, bool VERIFY, bool SPEC = false>
__global__ void __launch_bounds__(BLOCK) k_fl_claim(OpsDev o, TsIndex x, uint32_t Q, FlatRec fr,
                                                    long long ts0, uint32_t* rtab, DevResult* dres,
                                                    uint32_t track_rep, uint32_t nrep, TreeDev T,
                                                    uint32_t log_to_tree) {
  Q = fr.q(Q);
  nrep = fr.nrep(nrep);
  if (SPEC) {
    log_to_tree = 1;
    track_rep = 0;
  }
  // dynamic LDS: the replica range table (nrep ids: {base, min, max counter}
  // in one 16-byte entry, one LDS read per lookup) when it fits, else
  // lookups go to the global table; rv when track_rep
  extern __shared__ __attribute__((aligned(16))) uint32_t scl[];
  uint4* stab = reinterpret_cast<uint4*>(scl);
  uint32_t* rv = scl + 4 * nrep;
  for (uint32_t j = threadIdx.x; j < nrep; j += blockDim.x) {
    const uint2 g = x.rng[j];
    stab[j] = make_uint4(x.base[j], g.x, g.y, 0u);
  }
  if (track_rep)
    for (uint32_t j = threadIdx.x; j < REP_DIRECT; j += blockDim.x) rv[j] = 0;
  __syncthreads();
  auto slot = [&](long long ts) -> uint32_t {
    if (!SPEC && !nrep) return tsindex_slot(x, ts);
    if (ts <= 0) return NONE;
    const uint64_t r = static_cast<uint64_t>(ts) >> 32;
    if (r >= nrep) return NONE;
    const uint4 e = stab[r];
    const uint32_t c = static_cast<uint32_t>(ts), lo = e.y;
    if (c < lo || c > e.z) return NONE;  // (an empty range {NONE, 0} holds no c)
    return e.x + (c - lo);
  };
  const long long id0 = replica_of(ts0);
  uint32_t keys = 0, own = 0, slow = 0, err = NONE, mr = 0, bad = 0, vfail = 0;
  // the slot records are staged in LDS and stored grouped by replica (a
  // replica's ops of one iteration hold consecutive counters: whole lines of
  // its slot run), instead of one scattered 8-byte store per op beside the
  // log's streaming stores (tools/claim_bench.hip: 146 -> 101 us for the
  // same bytes)
  __shared__ uint32_t s_cnt[64], s_off[64];
  __shared__ uint2 s_rec[4 * BLOCK];
  __shared__ uint32_t s_q[4 * BLOCK];
  const uint32_t nq_ = (o.n + 3) / 4;  // (QUAD_LOOP_XCD, with every thread in every iteration)
  const bool x8_ = (gridDim.x & 7) == 0;
  const uint32_t xc_ = x8_ ? blockIdx.x & 7 : 0, xy_ = x8_ ? blockIdx.x >> 3 : blockIdx.x;
  const uint32_t cq_ = (x8_ ? gridDim.x >> 3 : gridDim.x) * blockDim.x, xs_ = x8_ ? 8 : 1;
  for (uint32_t j_ = xc_; j_ * cq_ < nq_; j_ += xs_) {
    const uint32_t qd_ = j_ * cq_ + xy_ * blockDim.x + threadIdx.x, i0 = 4 * qd_;
    uint32_t sq[4] = {NONE, NONE, NONE, NONE}, sb[4] = {0u, 0u, 0u, 0u};
    uint2 sv[4];
    if (qd_ < nq_) {
    Quad qd;
    long long pk[4];  // the path element of each op (flat: |path| <= 1)
    if (VERIFY) {
      if (i0 + 4 <= o.n) {
        const uchar4 k4 = *reinterpret_cast<const uchar4*>(o.kind + i0);
        const uint4 f4 = *reinterpret_cast<const uint4*>(o.off + i0);
        vfail |= (k4.x | k4.y | k4.z | k4.w) != CRDTM_ADD ||
                 (f4.x != i0) | (f4.y != i0 + 1) | (f4.z != i0 + 2) | (f4.w != i0 + 3);
      } else {
        for (uint32_t i = i0; i < o.n; ++i) vfail |= o.kind[i] != CRDTM_ADD || o.off[i] != i;
      }
      if (i0 + 4 >= o.n) vfail |= o.off[o.n] != o.n;
    }
    if (SIMPLE) {
      if (i0 + 4 <= o.n) {
        qd.cnt = 4;
        const longlong2 a = *reinterpret_cast<const longlong2*>(o.ts + i0);
        const longlong2 b = *reinterpret_cast<const longlong2*>(o.ts + i0 + 2);
        const longlong2 c = *reinterpret_cast<const longlong2*>(o.path + i0);
        const longlong2 d = *reinterpret_cast<const longlong2*>(o.path + i0 + 2);
        qd.ts[0] = a.x; qd.ts[1] = a.y; qd.ts[2] = b.x; qd.ts[3] = b.y;
        pk[0] = c.x; pk[1] = c.y; pk[2] = d.x; pk[3] = d.y;
      } else {
        qd.cnt = o.n - i0;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
          qd.ts[k] = k < qd.cnt ? o.ts[i0 + k] : 0;
          pk[k] = k < qd.cnt ? o.path[i0 + k] : 0;
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < 5; ++k) qd.off[k] = i0 + k;
    } else {
      load_quad(o, i0, qd);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) pk[k] = (k < qd.cnt && qd.off[k + 1] != qd.off[k]) ? o.path[qd.off[k]] : 0;
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) bad |= (pk[k] >= TWO53 || pk[k] <= -TWO53) ? 1u : 0u;  // (|x| < 2^53)
    if (log_to_tree) {
      if (qd.cnt == 4) {  // (streaming stores: nothing in the merge reads the log back)
        if (SIMPLE) {
          st_stream4(T.l_kind + i0, make_uchar4(CRDTM_ADD, CRDTM_ADD, CRDTM_ADD, CRDTM_ADD));
          st_stream16(T.l_path + i0, make_longlong2(pk[0], pk[1]));
          st_stream16(T.l_path + i0 + 2, make_longlong2(pk[2], pk[3]));
        } else {
          st_stream4(T.l_kind + i0, make_uchar4(qd.kind[0], qd.kind[1], qd.kind[2], qd.kind[3]));
        }
        st_stream16(T.l_ts + i0, make_longlong2(qd.ts[0], qd.ts[1]));
        st_stream16(T.l_ts + i0 + 2, make_longlong2(qd.ts[2], qd.ts[3]));
        st_stream16(T.l_off + i0, make_uint4(qd.off[0], qd.off[1], qd.off[2], qd.off[3]));
        st_stream16(T.l_val + i0, *reinterpret_cast<const uint4*>(o.val + i0));
      } else {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {  // (static indices: no scratch)
          if (k < qd.cnt) {
            T.l_kind[i0 + k] = SIMPLE ? static_cast<uint8_t>(CRDTM_ADD) : qd.kind[k];
            T.l_ts[i0 + k] = qd.ts[k];
            T.l_off[i0 + k] = qd.off[k];
            T.l_val[i0 + k] = o.val[i0 + k];
            if (SIMPLE) T.l_path[i0 + k] = pk[k];
          }
        }
      }
      if (i0 + qd.cnt == o.n) T.l_off[o.n] = SIMPLE ? o.n : o.off[o.n];
      if (!SIMPLE) {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
          if (k < qd.cnt && qd.off[k + 1] != qd.off[k]) T.l_path[qd.off[k]] = pk[k];
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (k >= qd.cnt) continue;
      const uint32_t i = i0 + k;
      if (!SIMPLE && qd.off[k + 1] == qd.off[k]) {  // update [] = InvalidPath (src/Internal/Node.elm:147-148)
        ++slow;
        err = min(err, i);
        continue;
      }
      const long long ts = qd.ts[k];
      if (replica_of(ts) == id0) ++own;
      const uint32_t q = slot(ts);
      if (q >= Q) {  // ts 0: the sentinel's key (AlreadyApplied); (or past a speculation's bound)
        ++slow;
        continue;
      }
      ++keys;
      const long long kk = pk[k];
      uint32_t qa = kk == 0 ? Q : slot(kk);
      if (qa > Q) qa = NONE;
      sq[k] = q;  // (stored below: fr.rec[q] = {anchor code, op index})
      sv[k] = make_uint2(fr.code(qa), i);
      sb[k] = static_cast<uint32_t>(static_cast<uint64_t>(ts) >> 32) & 63u;
      if (track_rep) {
        const uint32_t rr = static_cast<uint32_t>(static_cast<uint64_t>(ts) >> 32);
        if (rr < REP_DIRECT) {
          atomicMax(&rv[rr], i + 1);
          mr = max(mr, rr);
        } else {
          atomicMax(&rtab[rr + (1u << (REPLICA_BITS - 1))], i + 1);
        }
      }
    }
    }
    // the staged stores: counting sort of the iteration's records by bucket
    for (uint32_t b = threadIdx.x; b < 64; b += blockDim.x) s_cnt[b] = 0;
    __syncthreads();
    uint32_t pos[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) pos[k] = sq[k] != NONE ? atomicAdd(&s_cnt[sb[k]], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < 64) {
      const uint32_t c = s_cnt[threadIdx.x];
      s_off[threadIdx.x] = wave_incl_scan(c) - c;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
      if (sq[k] != NONE) {
        const uint32_t e = s_off[sb[k]] + pos[k];
        s_rec[e] = sv[k];
        s_q[e] = sq[k];
      }
    __syncthreads();
    const uint32_t tot = s_off[63] + s_cnt[63];
    for (uint32_t e = threadIdx.x; e < tot; e += blockDim.x) fr.rec[s_q[e]] = s_rec[e];
    __syncthreads();
  }
  mr = block_max(mr);  // (synchronises the block) only ids <= mr were touched
  if (track_rep)
    for (uint32_t j = threadIdx.x; j <= mr; j += blockDim.x)
      if (rv[j]) atomicMax(&rtab[j + (1u << (REPLICA_BITS - 1))], rv[j]);
  keys = block_sum(keys);
  own = block_sum(own);
  slow = block_sum(slow);
  err = block_min(err);
  bad = block_max(bad);
  if (VERIFY) vfail = block_max(vfail);
  if (threadIdx.x == 0) {  // 16 shards a line apart: ~12 ns per atomic on one word
    if (VERIFY && vfail) atomicOr(&dres->spec_fail, 1u);
    if (bad) atomicOr(&dres->bad_range, 1u);
    uint32_t* sh = dres->fl_part + 32 * (blockIdx.x & 15);
    if (keys) atomicAdd(&sh[1], keys);
    if (own) atomicAdd(&sh[2], own);
    if (slow) atomicAdd(&sh[3], slow);
    if (err != NONE) atomicMin(&dres->err_index, err);
  }
}

// Status of every op (update / addAfterHelp, src/Internal/Node.elm:56-90,
// :138-163) when some op does not apply (k_fl_claim's records are final by
// then), fused with the batch accounting and the replicas fold: every
// applied Add's replica keeps its last op index in a direct-mapped LDS table
// (ids < REP_DIRECT), flushed once per workgroup into the replica table.
__global__ void __launch_bounds__(BLOCK) k_fl_status(OpsDev o, uint8_t* st, TsIndex x, uint32_t Q, FlatRec fr,
                                                     long long ts0, uint32_t* rtab, DevResult* dres) {
  __shared__ uint32_t rv[REP_DIRECT];
  for (uint32_t j = threadIdx.x; j < REP_DIRECT; j += blockDim.x) rv[j] = 0;
  __syncthreads();
  const long long id0 = replica_of(ts0);
  uint32_t app = 0, alr = 0, own = 0, err = NONE, dup = 0;
  QUAD_LOOP_XCD(i0, o.n) {
    Quad qd;
    load_quad(o, i0, qd);
    uint8_t s4[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (k >= qd.cnt) continue;
      const uint32_t i = i0 + k;
      uint8_t s;
      const long long ts = qd.ts[k];
      if (qd.off[k + 1] == qd.off[k]) {
        s = ST_INVALID;  // update [] = InvalidPath (src/Internal/Node.elm:147-148)
      } else {
        const uint32_t q = tsindex_slot(x, ts);
        if (q == NONE) {
          s = ST_ALREADY;  // ts 0 is the sentinel's key (:63-65)
        } else {
          const uint32_t fi = fr.rec[q].y;
          if (fi != i) {
            s = ST_ALREADY;  // `child ts parent` exists (:63-65)
            if (i < fi) {    // lost the store race to a later duplicate: take the slot (decided again)
              atomicMin(&fr.rec[q].y, i);
              dup = 1;
            }
          } else {
            const long long kk = o.path[qd.off[k]];
            const uint32_t qa = kk == 0 ? Q : tsindex_slot(x, kk);
            fr.rec[q].x = fr.code(qa);  // (the op index may have reached the slot after a duplicate's anchor)
            bool ok = qa == Q;          // anchored at the sentinel
            if (!ok && qa != NONE) {    // anchor Added before (:68-70)
              const uint2 ra = fr.rec[qa];
              ok = fr.present(ra.x) && ra.y < i;
            }
            s = ok ? ST_APPLIED : ST_NOTFOUND;
          }
        }
      }
      s4[k] = s;
      if (s == ST_APPLIED) {
        ++app;
        const uint32_t rr = static_cast<uint32_t>(static_cast<uint64_t>(ts) >> 32);
        if (rr < REP_DIRECT) atomicMax(&rv[rr], i + 1);
        else atomicMax(&rtab[rr + (1u << (REPLICA_BITS - 1))], i + 1);
      } else if (s == ST_ALREADY) {
        ++alr;
      } else {
        err = min(err, i);
      }
      // incrementTimestamp (src/CRDTree.elm:337-343): Ok Adds of the own replica
      if ((s == ST_APPLIED || s == ST_ALREADY) && replica_of(ts) == id0) ++own;
    }
    store_quad_u8(st, i0, qd.cnt, s4);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < REP_DIRECT; j += blockDim.x)
    if (rv[j]) atomicMax(&rtab[j + (1u << (REPLICA_BITS - 1))], rv[j]);
  app = block_sum(app);
  alr = block_sum(alr);
  own = block_sum(own);
  err = block_min(err);
  dup = block_max(dup);
  if (threadIdx.x == 0) {
    if (app) {
      atomicAdd(&dres->n_applied, app);
      atomicAdd(&dres->n_adds_applied, app);
    }
    if (alr) atomicAdd(&dres->n_already, alr);
    if (own) atomicAdd(&dres->own_ok_adds, own);
    if (err != NONE) atomicMin(&dres->err_index, err);
    if (dup) atomicOr(&dres->dup_fix, 1u);
  }
}

// Before a second commit: forget the speculative one's order and collection words.
__global__ void k_fl_commit_reset(DevResult* d) {
  d->run_fail = 0;
  d->n_replica_out = 0;
}

// A fresh tree's root sentinel points nowhere (crdtm_tree_reset, and after an
// unconfirmed speculative commit).
// (d: the result block's init rides on the tree reset, crdtm_ctx::dres_ready)
__global__ void k_reset_root(uint32_t* s_next, DevResult* d) {
  if (threadIdx.x == 0) s_next[0] = NONE;
  if (d) dres_init_block(d);
}

// Before the second status pass: forget the first pass's accounting.
__global__ void k_fl_stat_reset(DevResult* d) {
  d->n_applied = 0;
  d->n_adds_applied = 0;
  d->n_already = 0;
  d->own_ok_adds = 0;
  d->err_index = NONE;
  d->dup_fix = 0;
}

// replicas[r] := ts of replica r's last applied Add (flat: Adds only, ids in
// [0, max_replica]); clears the table entries it reads, and (rng_clear, the
// merge's last launch before its result read) the replica range entries.
__device__ __forceinline__ void fl_rep_collect(OpsDev o, uint32_t nr, uint32_t* rtab, long long* out,
                                               uint32_t* n_out, long long* inl, uint2* rng_clear) {
  GRID_STRIDE(r, nr) {
    if (rng_clear) rng_clear[r] = make_uint2(NONE, 0u);
    uint32_t* e = &rtab[r + (1u << (REPLICA_BITS - 1))];
    const uint32_t v = *e;
    if (!v) continue;
    *e = 0;
    if (!out) continue;  // clear only (a merge that did not commit)
    const uint32_t k = atomicAdd(n_out, 1u);
    out[2 * k] = r;
    out[2 * k + 1] = o.ts[v - 1];
    if (k < REP_INLINE) {  // (the host reads these with the result block)
      inl[2 * k] = r;
      inl[2 * k + 1] = o.ts[v - 1];
    }
  }
}
__global__ void __launch_bounds__(BLOCK) k_fl_rep_collect(OpsDev o, uint32_t nr, uint32_t* rtab, long long* out,
                                                          uint32_t* n_out, long long* inl, uint2* rng_clear) {
  fl_rep_collect(o, nr, rtab, out, n_out, inl, rng_clear);
}
// (the collection's arguments, when it rides on k_fl_next)
struct RepCollect {
  OpsDev o;
  uint32_t nr;
  uint32_t* rtab;
  long long* out;
  uint32_t* n_out;
  long long* inl;
  uint2* rng_clear;
};

// Runs. A run is a maximal slot interval [h, e) whose every slot but h is
// anchored at the slot before it (a replica's typing run: consecutive
// counters are consecutive slots); an absent slot is a run of its own with
// no node (a "hole" run). The run of a slot is not stored per slot: every
// word of 64 slots keeps the bit mask of its run heads (hm) and the number
// of heads before it (hb, an exclusive scan of the masks' popcounts), so
// run(q) = hb[q / 64] + popcount(hm[q / 64] up to q) - 1 — 12 bytes per 64
// slots, small enough to stay in L2 while the walks below look runs up (a
// 4-byte run id per slot was a 40 MB array written by a look-back scan and
// read back by every walk step and by the slot pass).
struct RunMask {
  const unsigned long long* hm;
  const uint32_t* hb;
};
__device__ __forceinline__ uint32_t run_of(const RunMask& rm, uint32_t q) {
  const uint32_t w = q >> 6;
  const unsigned long long below = (2ULL << (q & 63)) - 1ULL;  // (q & 63 == 63: every bit)
  return rm.hb[w] + static_cast<uint32_t>(__popcll(rm.hm[w] & below)) - 1u;
}

// The key of slot q from the replica range tables: the replica r with
// base[r] <= q (the largest such r: an empty range shares its base with the
// next replica) and counter min[r] + q - base[r] (slot order = timestamp
// order, src/CRDTree.elm:137).
__device__ __forceinline__ long long fl_key(uint32_t q, const uint32_t* sb, const uint32_t* sc, uint32_t nrep,
                                            uint32_t& rep) {
  uint32_t lo = 0, hi = nrep;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sb[mid] <= q) lo = mid;
    else hi = mid;
  }
  rep = lo;
  return (static_cast<long long>(lo) << 32) | static_cast<long long>(sc[lo] + (q - sb[lo]));
}

// One pass over the slot records in slot order, one wave per word of 64
// slots (lane = slot):
//  * the run heads by ballot (a missing anchor only occurs in a batch that
//    fails, which the flat speculation discards): hm, and the count per word;
//  * the node record of every present slot (tree slot 1 + its compacted
//    index; key recomputed from the slot, tables in LDS when the replica ids
//    fit, else the op's ts; implicit empty children dict): coalesced stores
//    of a streaming pass, instead of the per-slot stores of the rank pass;
//  * with `chk` (the flat speculation) the claim's check: every present
//    slot's Add must come after its anchor's (addAfterHelp,
//    src/Internal/Node.elm:68-70; inside a run the anchor is the slot before,
//    whose record the neighbouring lane holds), the present slots are counted
//    (as many as keyed Adds: no duplicate timestamps), and the replicas table
//    is folded (a wave's slots usually lie in one replica's range: one LDS
//    atomic per wave and replica).
// The trip count is wave-uniform, so every lane takes part in the ballots.
constexpr uint32_t RM_UNROLL = 4;       // k_run_heads: words per wave and iteration
constexpr uint32_t RM_BUCKETS = 2048;   // k_run_mask: slot buckets of the replica lookup
constexpr uint32_t RM_MASK_UNROLL = 2;  // k_run_mask (48 VGPRs, full occupancy; 4 words: 68, 120 -> 110 us at flat10m)
// DEVQ: the speculation without the host round trip (FlatRec::qd): the slot
// range and replica count come from the device (the tree's slot capacity
// covers the host's bound, so a speculation the host will discard stays in
// bounds).
template <uint32_t U, bool DEVQ>
__global__ void __launch_bounds__(BLOCK) k_run_mask(FlatRec fr, uint32_t Q, unsigned long long* hm, uint32_t* hc,
                                                   TreeDev T, const uint32_t* qc, const uint32_t* logidx, OpsDev o,
                                                   TsIndex x, uint32_t nrep, DevResult* chk, uint32_t* rtab) {
  extern __shared__ uint32_t smk[];  // dynamic: 3 * nrep words when the tables fit (HOST_RANGES)
  // (DEVQ, the speculation: the tables fit, no compaction, every op applies
  // — the branches for the other cases are compiled out)
  const bool lds = DEVQ || nrep <= HOST_RANGES;
  if (DEVQ) {
    qc = nullptr;
    logidx = nullptr;
  }
  if (DEVQ) {
    Q = fr.q(Q);
    nrep = fr.nrep(nrep);
  }
  uint32_t* sb = smk;
  uint32_t* sc = smk + nrep;
  uint32_t* srv = smk + 2 * nrep;  // (chk) largest op index + 1 per replica
  // the replica of a word's first slot: the slot's bucket of 2^sh slots
  // names the last replica starting at or before the bucket (LDS), a few
  // steps on from there (one dependent LDS read per word instead of a
  // binary search's seven)
  __shared__ uint16_t sbk[RM_BUCKETS];
  uint32_t sh = 0;
  while ((static_cast<uint64_t>(Q) >> sh) >= RM_BUCKETS) ++sh;
  if (lds) {
    for (uint32_t j = threadIdx.x; j < nrep; j += blockDim.x) {
      sb[j] = x.base[j];
      sc[j] = x.rng[j].x;
      srv[j] = 0;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < RM_BUCKETS; b += blockDim.x) {
      const uint32_t q0 = b << sh;
      uint32_t lo = 0, hi = nrep;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sb[mid] <= q0) lo = mid;
        else hi = mid;
      }
      sbk[b] = static_cast<uint16_t>(lo);
    }
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = (Q + 63) >> 6;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwave = (gridDim.x * blockDim.x) >> 6;
  uint32_t present = 0, err = NONE;
  // Loads are unconditional (clamped indices) and the next iteration's are
  // issued before this one's stores: a load behind an exec-masked branch,
  // or behind the stores, made the compiler wait for everything in flight
  // (gfx9 counts loads and stores in issue order) twice per iteration.
  const uint32_t qmax = Q ? Q - 1 : 0u;
  uint2 nq[U], np;
  auto load = [&](uint32_t w0) {
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) nq[u] = fr.rec[min(((w0 + u) << 6) + lane, qmax)];
    np = fr.rec[w0 ? (w0 << 6) - 1 : 0u];  // (the slot before the first word: one address for the wave)
  };
  if (wave * U < nw) load(wave * U);
  for (uint32_t w0 = wave * U; w0 < nw; w0 += nwave * U) {
    uint2 rq[U], rp[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) rq[u] = nq[u];
    const uint2 rprev = w0 ? np : make_uint2(FR_EMPTY, 0u);
    if (w0 + nwave * U < nw) load(w0 + nwave * U);
    // the slot before each lane's: the neighbouring lane's, the previous
    // word's last for lane 0
    uint2 ra[U];
    unsigned long long m[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t q = ((w0 + u) << 6) + lane;
      const uint32_t px = __shfl_up(rq[u].x, 1, 64), py = __shfl_up(rq[u].y, 1, 64);
      const uint2 last = u ? make_uint2(__shfl(rq[u - 1].x, 63, 64), __shfl(rq[u - 1].y, 63, 64)) : rprev;
      rp[u] = lane ? make_uint2(px, py) : last;
      const bool pres = q < Q && fr.present(rq[u].x);
      const uint32_t qa = fr.anchor(rq[u].x);
      const bool cont = pres && q > 0 && fr.present(rp[u].x) && qa == q - 1;
      m[u] = __ballot(q < Q && !cont);
      // the anchors' records of run heads anchored elsewhere (the check)
      ra[u] = make_uint2(FR_EMPTY, 0u);
      if (chk && pres && qa != Q && qa != NONE && qa + 1 != q) ra[u] = fr.rec[qa];
    }
    {  // the words' head masks and counts: one store per iteration, lane u for word u
      unsigned long long mv = 0;
#pragma unroll
      for (uint32_t u = 0; u < U; ++u)
        if (lane == u) mv = m[u];
      if (lane < U && w0 + lane < nw) {
        hm[w0 + lane] = mv;
        hc[w0 + lane] = static_cast<uint32_t>(__popcll(mv));
      }
    }
    uint32_t rep[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t q = ((w0 + u) << 6) + lane;
      const bool pres = q < Q && fr.present(rq[u].x);
      rep[u] = NONE;
      const uint32_t fi = rq[u].y;
      // the replica of the word's first slot, looked up once for the wave
      // (uniform LDS reads); a lane past that replica's range (a word that
      // straddles two ranges) searches for itself
      uint32_t wr = 0, wlo = NONE, whi = 0;
      if (lds) {
        const uint32_t q0 = (w0 + u) << 6;
        uint32_t lo = sbk[min(q0 >> sh, RM_BUCKETS - 1)];
        while (lo + 1 < nrep && sb[lo + 1] <= q0) ++lo;
        wr = lo;
        wlo = sb[lo];
        whi = lo + 1 < nrep ? sb[lo + 1] : NONE;
      }
      if (pres) {  // (streaming stores: the merge does not read them back)
        const uint32_t slot = 1 + (qc ? qc[q] : q);
        long long key;
        if (!lds) {
          key = o.ts[fi];
        } else if (q >= wlo && q < whi) {
          rep[u] = wr;
          key = (static_cast<long long>(wr) << 32) | static_cast<long long>(sc[wr] + (q - wlo));
        } else {
          key = fl_key(q, sb, sc, nrep, rep[u]);
        }
        st_node(T.s_key + slot, key);
        st_node(T.s_dict + slot, 0u);
        st_node(T.s_src + slot, logidx ? logidx[fi] : fi);
        st_node(T.s_flags + slot, static_cast<uint8_t>(0));
        st_node(T.s_child + slot, NONE);
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {  // (after the stores: the wait covers the anchor loads only)
      const uint32_t q = ((w0 + u) << 6) + lane;
      const bool pres = q < Q && fr.present(rq[u].x);
      const uint32_t qa = fr.anchor(rq[u].x);
      const uint32_t fi = rq[u].y;
      if (chk && pres) {
        ++present;
        if (qa != Q) {
          bool ok = false;  // an Add at the anchor, before this one
          if (qa + 1 == q) ok = fr.present(rp[u].x) && rp[u].y < fi;
          else if (qa != NONE) ok = fr.present(ra[u].x) && ra[u].y < fi;
          if (!ok) err = min(err, fi);
        }
      }
      if (chk && lds) {  // (wave-uniform) replicas[r] := its last Add
        const unsigned long long mr = __ballot(rep[u] != NONE);
        if (mr) {
          const uint32_t r0 = __shfl(rep[u], __ffsll(static_cast<long long>(mr)) - 1, 64);
          if (__ballot(rep[u] != NONE && rep[u] != r0) == 0) {
            uint32_t v = rep[u] != NONE ? fi + 1 : 0u;
#pragma unroll
            for (int o2 = 32; o2 > 0; o2 >>= 1) v = max(v, __shfl_xor(v, o2, 64));
            if (lane == 0) atomicMax(&srv[r0], v);
          } else if (rep[u] != NONE) {
            atomicMax(&srv[rep[u]], fi + 1);
          }
        }
      }
    }
  }
  if (!chk) return;  // (grid-uniform)
  present = block_sum(present);  // (synchronises the block: srv complete)
  err = block_min(err);
  if (lds)
    for (uint32_t j = threadIdx.x; j < nrep; j += blockDim.x)
      if (srv[j]) atomicMax(&rtab[j + (1u << (REPLICA_BITS - 1))], srv[j]);
  if (threadIdx.x == 0) {
    if (present) atomicAdd(&chk->fl_part[32 * (blockIdx.x & 15)], present);
    if (err != NONE) atomicMin(&chk->err_index, err);
  }
}

// Per run: its head slot and the head's anchor (ABSENT: a hole run; a
// missing anchor reads as the sentinel so that the speculative walks stay in
// bounds), hh[r] = {head, anchor}; k_run_ep replaces the anchor by the
// head's effective parent.
// (hasch: every run's has-a-child flag cleared, for k_run_ep to set)
__global__ void __launch_bounds__(BLOCK) k_run_heads(FlatRec fr, uint32_t Q, RunMask rm, uint2* hh,
                                                     uint8_t* hasch) {
  Q = fr.q(Q);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = (Q + 63) >> 6;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwave = (gridDim.x * blockDim.x) >> 6;
  const unsigned long long lt = (1ULL << lane) - 1ULL;
  for (uint32_t w0 = wave * RM_UNROLL; w0 < nw; w0 += nwave * RM_UNROLL) {
    unsigned long long m[RM_UNROLL];
    uint32_t x[RM_UNROLL], b[RM_UNROLL];
#pragma unroll
    for (uint32_t u = 0; u < RM_UNROLL; ++u) {  // every load in flight first
      const uint32_t w = w0 + u;
      m[u] = w < nw ? rm.hm[w] : 0ULL;
      b[u] = w < nw ? rm.hb[w] : 0u;
      x[u] = ((m[u] >> lane) & 1ULL) ? fr.rec[(w << 6) + lane].x : FR_EMPTY;
    }
#pragma unroll
    for (uint32_t u = 0; u < RM_UNROLL; ++u) {
      if (!((m[u] >> lane) & 1ULL)) continue;
      uint32_t a = ABSENT;
      if (fr.present(x[u])) {
        a = fr.anchor(x[u]);
        if (a == NONE) a = Q;
      }
      const uint32_t r = b[u] + static_cast<uint32_t>(__popcll(m[u] & lt));
      hh[r] = make_uint2(((w0 + u) << 6) + lane, a);
      if (hasch) hasch[r] = 0;
    }
  }
}

// Counting-sort scatter; single-child parents (the common case in a typing
// stream) take a plain store. The root sentinel's children are placed by
// k_fl_root_* instead (already in order, no sort).
__global__ void __launch_bounds__(BLOCK) k_fl_scatter(uint32_t Q, const uint32_t* anc, const uint32_t* start,
                                                      uint32_t* fill, uint32_t* carr) {
  GRID_STRIDE(q, Q) {
    const uint32_t p = anc[q];
    if (p == ABSENT || p == Q) continue;
    const uint32_t b = start[p];
    carr[start[p + 1] - b == 1 ? b : b + atomicAdd(&fill[p], 1u)] = q;
  }
}

// The root sentinel's children in descending slot order by an ordered
// compaction: every workgroup owns a contiguous slot chunk, counts its root
// children, and (after a scan of the counts) writes them in slot order from
// the back of the segment.
__global__ void __launch_bounds__(BLOCK) k_fl_root_count(uint32_t Q, const uint32_t* anc, uint32_t* bcnt) {
  const uint32_t chunk = (Q + gridDim.x - 1) / gridDim.x;
  const uint32_t b0 = blockIdx.x * chunk, b1 = min(Q, b0 + chunk);
  uint32_t c = 0;
  for (uint32_t q = b0 + threadIdx.x; q < b1; q += blockDim.x) c += anc[q] == Q ? 1u : 0u;
  c = block_sum(c);
  if (threadIdx.x == 0) bcnt[blockIdx.x] = c;
}

__global__ void __launch_bounds__(BLOCK) k_fl_root_place(uint32_t Q, const uint32_t* anc, const uint32_t* boff,
                                                         const uint32_t* start, uint32_t* carr) {
  const uint32_t chunk = (Q + gridDim.x - 1) / gridDim.x;
  const uint32_t b0 = blockIdx.x * chunk, b1 = min(Q, b0 + chunk);
  const uint32_t seg = start[Q], R = start[Q + 1] - seg;
  uint32_t run = boff[blockIdx.x];
  for (uint32_t t0 = b0; t0 < b1; t0 += blockDim.x) {
    const uint32_t q = t0 + threadIdx.x;
    const uint32_t f = (q < b1 && anc[q] == Q) ? 1u : 0u;
    uint32_t tot;
    const uint32_t j = run + block_excl_sum(f, &tot);
    if (f) carr[seg + (R - 1 - j)] = q;
    run += tot;
  }
}

__global__ void __launch_bounds__(BLOCK) k_fl_links(const uint32_t* anc, const uint32_t* start, const uint32_t* total,
                                                    const uint32_t* carr, uint32_t* ns) {
  const uint32_t tot = *total;
  GRID_STRIDE(pos, tot) {
    const uint32_t v = carr[pos];
    ns[v] = (pos + 1 < start[anc[v] + 1]) ? carr[pos + 1] : NONE;
  }
}

// K4: Euler tour entries computed on the fly for the list ranking:
// enter(u) = 2u, leave(u) = 2u + 1; the enter of a node weighs 1, so a
// node's rank is its document position. The ranks go straight into
// order[rank] = node (no tour or rank arrays in HBM).
struct FlatEulerSrc {
  uint32_t Q;
  const uint32_t* anc;    // ep per node, ABSENT = no node
  const uint32_t* start;  // children segment of u: carr[start[u] .. start[u+1])
  const uint32_t* carr;
  const uint32_t* ns;     // next sibling
  __device__ __forceinline__ uint2 operator()(uint64_t e) const {
    const uint32_t u = static_cast<uint32_t>(e >> 1);
    const uint32_t p = u < Q ? anc[u] : Q;
    if (p == ABSENT) return make_uint2(ABSENT, 0u);
    if (!(e & 1)) {
      const uint32_t b = start[u], en = start[u + 1];
      return make_uint2(b < en ? 2 * carr[b] : 2 * u + 1, u < Q ? 1u : 0u);
    }
    if (u == Q) return make_uint2(NONE, 0u);
    const uint32_t s = ns[u];
    return make_uint2(s != NONE ? 2 * s : 2 * p + 1, 0u);
  }
};

// doc[rank] = the tree slot of the node (1 + its compacted slot index).
struct FlatDocSink {
  uint32_t Q;
  uint32_t* doc;
  const uint32_t* qc;  // exclusive scan of node presence, nullptr when slots have no holes
  static constexpr bool kOffList = false;
  __device__ __forceinline__ void operator()(uint64_t e, unsigned long long r) const {
    if (e & 1) return;
    const uint32_t u = static_cast<uint32_t>(e >> 1);
    if (u < Q) doc[static_cast<uint32_t>(r)] = 1 + (qc ? qc[u] : u);
  }
};

// Commit. Node q -> tree slot 1 + qc(q) (slot order = timestamp order), its
// children dict implicit (engine.h TreeDev). Within the root dict the raw
// `next` chain is the document order (no tombstones): k_fl_next links
// doc[r] -> doc[r + 1] and the root sentinel (slot 0) -> doc[0].
// (The flat speculation may run this over more ranks than slots when its
// guess fails: entries past the document are then stale, and `cap` keeps
// the stores inside the slot arrays; the result is discarded.)
// (rc.nr > 0: the replicas collection of the merge's end, k_fl_rep_collect,
// rides on this launch)
__global__ void __launch_bounds__(BLOCK) k_fl_next(uint32_t K, const uint32_t* doc, TreeDev T, uint64_t cap,
                                                   RepCollect rc) {
  if (rc.nr) fl_rep_collect(rc.o, rc.nr, rc.rtab, rc.out, rc.n_out, rc.inl, rc.rng_clear);
  GRID_STRIDE(r, K) {
    const uint32_t d = doc[r];
    if (d < cap) T.s_next[d] = r + 1 < K ? doc[r + 1] : NONE;
    if (r == 0) T.s_next[0] = doc[0];
  }
}

__global__ void __launch_bounds__(BLOCK) k_fl_present(uint32_t Q, FlatRec fr, uint32_t* f) {
  GRID_STRIDE(q, Q) f[q] = fr.present(fr.rec[q].x) ? 1u : 0u;
}

// Log append into a fresh tree when every op applied: the log is the batch
// itself (same CSR layout, path elements [0, n_path)). SIMPLE (k_fl_claim):
// op i is an Add whose one path element is path[i], so the kinds and offsets
// are written without reading them; four ops per lane, 16-byte accesses.
template <bool SIMPLE>
__global__ void __launch_bounds__(BLOCK) k_fl_log_copy(OpsDev o, TreeDev T) {
  if (SIMPLE) {
    QUAD_LOOP(i0, o.n) {
      if (i0 + 4 <= o.n) {
        *reinterpret_cast<uchar4*>(T.l_kind + i0) = make_uchar4(CRDTM_ADD, CRDTM_ADD, CRDTM_ADD, CRDTM_ADD);
        *reinterpret_cast<longlong2*>(T.l_ts + i0) = *reinterpret_cast<const longlong2*>(o.ts + i0);
        *reinterpret_cast<longlong2*>(T.l_ts + i0 + 2) = *reinterpret_cast<const longlong2*>(o.ts + i0 + 2);
        *reinterpret_cast<uint4*>(T.l_off + i0) = make_uint4(i0, i0 + 1, i0 + 2, i0 + 3);
        *reinterpret_cast<uint4*>(T.l_val + i0) = *reinterpret_cast<const uint4*>(o.val + i0);
        *reinterpret_cast<longlong2*>(T.l_path + i0) = *reinterpret_cast<const longlong2*>(o.path + i0);
        *reinterpret_cast<longlong2*>(T.l_path + i0 + 2) = *reinterpret_cast<const longlong2*>(o.path + i0 + 2);
      } else {
        for (uint32_t i = i0; i < o.n; ++i) {
          T.l_kind[i] = CRDTM_ADD;
          T.l_ts[i] = o.ts[i];
          T.l_off[i] = i;
          T.l_val[i] = o.val[i];
          T.l_path[i] = o.path[i];
        }
      }
      if (i0 + 4 >= o.n) T.l_off[o.n] = o.n;
    }
    return;
  }
  GRID_STRIDE(i, o.n + 1) {
    T.l_off[i] = o.off[i];
    if (i == o.n) continue;
    T.l_kind[i] = o.kind[i];
    T.l_ts[i] = o.ts[i];
    T.l_val[i] = o.val[i];
  }
  const uint64_t np = o.n_path;
  for (uint64_t p = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; p < np;
       p += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    T.l_path[p] = o.path[p];
}

// ---------------------------------------------------------------------------
// K4 (flat): the document order by run decomposition. A run is a maximal
// interval of present slots [h, h + len) each anchored at the slot before it
// (RunIdGen), so ep(q) = q - 1 inside (the first node below q on its anchor
// chain). A node's children all have larger slots (an effective parent has
// the smaller timestamp), so q + 1 is the smallest, i.e. the LAST child of q
// in the descending order (src/Internal/Node.elm:93-104 via the closed form,
// DESIGN.md): the pre-order visits q, then q's other ("side") children's
// subtrees, then q + 1. Every side child heads a run ("child run" of q's run,
// attached at q), so a slot's document rank is pos(head) + the run's slots
// before it + the subtrees of the run's child runs attached below it; the
// subtree of run r has T(r) = len(r) + the subtrees of its child runs; and a
// child run r of slot j starts at pos(j) + 1 + (the subtrees of j's other
// child runs with a larger slot). Runs form a shallow tree (flat10m: 1.0M
// runs, depth <= 11): T comes bottom-up, pos(head) top-down as a sum along
// the run's ancestor chain. Everything between the run scan and the final
// expansion works on the 1M runs, not the 10M slots. A run tree deeper than
// RUN_MAXD takes the generic Euler-tour list ranking instead (run_fail).
// ---------------------------------------------------------------------------
constexpr uint32_t RUN_MAXD = 64;
constexpr uint32_t EX_ITERS = 128;  // k_run_expand keeps its run-mask words in LDS up to this many iterations

// One 16-byte record per run, so that a walk over runs (the bottom-up climb,
// the top-down chain) takes every field it needs from one line:
// rr[r] = {parent run (NONE: a child of the root sentinel, or a hole run),
//          length (after k_run_tree_up: w, the head's rank minus its parent
//          run head's rank), sorted positions [z, w) of its child runs
//          ({NONE, 0}: none)}.
struct RunArr {
  const uint32_t* nR;        // device: number of runs
  uint2* hh;                 // {head slot, anchor of the head (ABSENT: a hole run), then its effective parent}
  uint4* rr;                 // {par, len -> w, er.x, er.y}
  const uint32_t* qd;        // (the flat speculation: the slot range on the device, FlatRec::qd)
  unsigned long long* ca;    // children arrived << 32 | their subtree sizes
  uint32_t* tk;              // subtree sizes in sorted order (k_run_tree_up writes T(r) at kinv[r])
  const uint32_t* kinv;      // run -> its position in the sorted order
  uint32_t* posh;            // document rank of the head
  uint8_t* hasch = nullptr;  // run -> 1 when some run is its child (k_run_sizes: leaves)
};

#define RUN_LOOP(r) for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x, nr_ = *a.nR; r < nr_; r += gridDim.x * blockDim.x)

// K2a at run granularity. Inside a run ep(q) = q - 1; only a head needs its
// effective parent (the first node on its anchor chain below it), and only a
// head anchored at a larger slot walks: the chain runs down through whole
// runs (a run's slots are all larger than x when its head is), so each step
// jumps from the run holding d to its head's anchor (flat10m: 0.49M walks,
// mean 3.7 steps, at most 23). hh[].y is overwritten with ep as walks
// finish; a concurrent reader then sees ep(h) instead of anchor(h), which
// skips only nodes > h > x, so every walk stays exact. A walk only descends
// to smaller heads, so the runs are taken from the last one down (the grid
// starts with the largest slots): most steps then meet an effective parent
// already resolved. Each step is one look-up of the run masks (L2) and one
// 8-byte {head, anchor} load. Then the run's parent run (the run holding ep),
// its length, and the sibling sort's input (key = attach slot, the root
// sentinel = Q, hole runs Q + 1) listed in descending run order, so the
// stable sort leaves siblings at one slot in descending slot order.
// COHERENT: the {head, anchor} words are read and the effective parents
// written at agent scope (past the XCDs' L2s, so a walk sees what walks on
// other XCDs resolved); else through the L2 (a walk may then read an anchor
// another XCD already replaced by its effective parent: also exact, see
// above, only possibly longer).
template <bool COHERENT>
__device__ __forceinline__ uint2 hh_load(const uint2* p) {
  const unsigned long long v =
      COHERENT ? __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT)
               : *reinterpret_cast<const unsigned long long*>(p);
  return make_uint2(static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32));
}
template <bool COHERENT>
__device__ __forceinline__ void hh_store_ep(uint2* p, uint32_t d) {
  if (COHERENT) __hip_atomic_store(&p->y, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else p->y = d;
}
template <bool COHERENT>
__global__ void __launch_bounds__(BLOCK) k_run_ep(RunArr a, uint32_t Q, RunMask rm, FlatRec fr, uint32_t* skey,
                                                  uint32_t* sval) {
  Q = fr.q(Q);
  const uint32_t R = *a.nR;
  RUN_LOOP(k) {
    const uint32_t r = R - 1 - k;
    const uint2 me = a.hh[r];
    const uint32_t x = me.x;
    uint32_t d = me.y;
    const uint32_t hn = r + 1 < R ? a.hh[r + 1].x : Q;
    if (d == ABSENT) {  // a hole run
      a.rr[r] = make_uint4(NONE, 0u, NONE, 0u);  // (child range [z, w): none)
      a.ca[r] = 0;
      skey[R - 1 - r] = Q + 1;
      sval[R - 1 - r] = r;
      continue;
    }
    if (d < Q && d > x) {
      // (a valid batch's anchors form a forest of present slots; a failing
      // batch run by the flat speculation may anchor at a slot without a node
      // or hold a cycle: those walks end at the sentinel, which keeps every
      // walk finite and in bounds, and the speculation is discarded)
      for (uint32_t steps = 0; d < Q && d > x; ++steps) {
        const uint2 hj = hh_load<COHERENT>(a.hh + run_of(rm, d));
        if (hj.x <= x || steps > R) {
          d = Q;
          break;
        }
        d = hj.y;
      }
      if (d >= Q) d = Q;
      hh_store_ep<COHERENT>(&a.hh[r], d);
    } else if (d == x) {  // (self-anchored: a failing batch)
      d = Q;
      hh_store_ep<COHERENT>(&a.hh[r], d);
    }
    // (an anchor at a slot without a node — a failing batch, whose speculation
    // the slot pass's check discards — is left as it is: its run is a hole
    // run with a smaller index, so the run tree stays a forest and every
    // later index stays in range; a batch that reaches the commit after its
    // statuses has every anchor present)
    // (len: a hole after the run is a run of its own)
    const uint32_t P = d == Q ? NONE : run_of(rm, d);
    a.rr[r] = make_uint4(P, hn - x, NONE, 0u);
    if (a.hasch && P != NONE) a.hasch[P] = 1;  // (the same value from every child: plain stores)
    a.ca[r] = 0;
    skey[R - 1 - r] = d;
    sval[R - 1 - r] = r;
  }
}

// The generic order's input (a run tree deeper than RUN_MAXD): ep per slot
// (q - 1 inside a run, the walked effective parent at a head, ABSENT = no
// node), into anc.
__global__ void __launch_bounds__(BLOCK) k_run_ep_slots(RunArr a, uint32_t Q, RunMask rm, FlatRec fr,
                                                        uint32_t* anc) {
  GRID_STRIDE(q, Q) {
    if (!fr.present(fr.rec[q].x)) {
      anc[q] = ABSENT;
      continue;
    }
    const uint2 h = a.hh[run_of(rm, q)];
    anc[q] = h.x == q ? h.y : q - 1;
  }
}

// Bottom-up subtree sizes in one launch: every leaf run climbs its chain of
// ancestors; a child announces its size with ONE 64-bit device-scope atomic
// {arrivals += 1, sizes += T} (memory-side, coherent across the XCDs), and
// the child that arrives last holds the sum of all its siblings' sizes in
// the returned value, so it finalises the parent and climbs on. Any depth.
// Leaves are taken in sibling order, where a parent's children sit side by
// side: a wave sums its leaves per parent first (one atomic per wave and
// parent; a parent with thousands of children would otherwise serialise
// thousands of atomics on one word, ~12 ns each).
// (ex: the record of x, loaded by the step that reached x; the parent's
// record loads beside the atomic, so a level costs one round trip)
__device__ __forceinline__ void run_climb(RunArr& a, uint32_t x, uint4 ex, uint32_t t) {
  for (;;) {
    a.tk[a.kinv[x]] = t;
    const uint32_t p = ex.x;
    if (p == NONE) return;
    const unsigned long long old = atomicAdd(&a.ca[p], (1ULL << 32) | t);
    const uint4 e = a.rr[p];
    if (static_cast<uint32_t>(old >> 32) + 1u != e.w - e.z) return;
    t = e.y + static_cast<uint32_t>(old) + t;
    x = p;
    ex = e;
  }
}

__global__ void __launch_bounds__(BLOCK) k_run_tree_up(RunArr a, const uint32_t* sarr) {
  const uint32_t R = *a.nR;
  const int lane = threadIdx.x & 63;
  for (uint32_t k0 = blockIdx.x * blockDim.x; k0 < R; k0 += gridDim.x * blockDim.x) {
    const uint32_t k = k0 + threadIdx.x;
    uint32_t key = NONE - 1 - static_cast<uint32_t>(lane);  // (distinct per idle lane)
    unsigned long long v = 0;                                // leaves << 32 | their sizes
    if (k < R) {
      const uint4 e = a.rr[sarr[k]];
      key = e.x;
      if (e.w <= e.z) {  // (no child runs: [NONE, 0))
        const uint32_t t = e.y;
        a.tk[k] = t;  // (kinv[r] == k)
        v = (1ULL << 32) | t;
      }
    }
    // segmented inclusive sum over lanes with the same parent (contiguous)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long ov = __shfl_up(v, o, 64);
      const uint32_t ok = __shfl_up(key, o, 64);
      if (lane >= o && ok == key) v += ov;
    }
    const uint32_t nk = __shfl_down(key, 1, 64);
    if ((lane == 63 || nk != key) && key < NONE - 64 && (v >> 32)) {
      const unsigned long long old = atomicAdd(&a.ca[key], v);
      const uint4 e = a.rr[key];
      if (static_cast<uint32_t>(old >> 32) + static_cast<uint32_t>(v >> 32) == e.w - e.z)
        run_climb(a, key, e, e.y + static_cast<uint32_t>(old) + static_cast<uint32_t>(v));
    }
  }
}

// Round 6: the subtree sizes and the child-run ranges in one launch, and the
// offsets w by a segmented scan (k_run_gstart and k_run_w gone). Per sorted
// position k (a child run c attached at slot p of parent run P, or a root
// sentinel child):
//  * the ends of each parent's child range [z, w) come from the neighbours'
//    parents (lanes of one wave hold consecutive positions), written into
//    rr[P].z / .w for the expansion;
//  * offk[k] = SEGF when k starts a parent's range | (p - head(P) + 1), the
//    part of w(c) before the sibling subtrees (0 for root children);
//  * completion without child counts: P's counter (ca, high half) receives
//    +1 per child that arrives (leaves in this pass, inner runs when their
//    own subtree completes), +z from the lane at z and -w from the lane at
//    w - 1; it is back at 0 exactly when every child has arrived (a partial
//    sum is 0 only when what is missing adds nothing). A wave that holds a
//    parent's whole range of leaves completes it without an atomic (most
//    parents: 263k parents of ~1M runs at flat10m, 3.4 children each). The
//    run that completes a parent climbs on with T(P) = len(P) + the sizes.
// Leaves come from hasch (k_run_ep). Any depth.
constexpr uint32_t SEGF = 0x80000000u;
constexpr uint32_t PAR_ROOT = NONE - 1, PAR_HOLE = NONE - 2;

__device__ __forceinline__ void run_climb2(RunArr& a, uint32_t x, uint4 ex, uint32_t t) {
  for (;;) {
    a.tk[a.kinv[x]] = t;
    const uint32_t p = ex.x;
    if (p == NONE) return;
    const unsigned long long add = (1ULL << 32) | t;
    const unsigned long long old = atomicAdd(&a.ca[p], add);
    const uint4 e = a.rr[p];
    const unsigned long long nv = old + add;
    if ((nv >> 32) != 0) return;
    t = e.y + static_cast<uint32_t>(nv);
    x = p;
    ex = e;
  }
}

__global__ void __launch_bounds__(BLOCK) k_run_sizes(RunArr a, uint32_t Q, const uint32_t* sarr, const uint32_t* pk,
                                                     RunMask rm, uint32_t* offk) {
  if (a.qd) Q = min(*a.qd, Q);  // (FlatRec::q: the bound stays the limit)
  const uint32_t R = *a.nR;
  const uint32_t lane = threadIdx.x & 63;
  auto par = [&](uint32_t x) -> uint32_t {
    return x < Q ? run_of(rm, x) : (x == Q ? PAR_ROOT : (x == Q + 1 ? PAR_HOLE : NONE));
  };
  for (uint32_t k0 = blockIdx.x * blockDim.x; k0 < R; k0 += gridDim.x * blockDim.x) {
    const uint32_t k = k0 + threadIdx.x;
    const bool valid = k < R;
    const uint32_t r = valid ? sarr[k] : 0u;
    const uint32_t p = valid ? pk[k] : Q + 2;
    const uint32_t pq = (lane == 0 && valid && k > 0) ? pk[k - 1] : Q + 2;  // (the neighbours outside the wave)
    const uint32_t pn = (lane == 63 && k + 1 < R) ? pk[k + 1] : Q + 2;
    const uint4 e = valid ? a.rr[r] : make_uint4(NONE, 0u, NONE, 0u);
    const bool leaf = valid && !a.hasch[r];
    const uint32_t P = par(p);
    uint32_t Pp = __shfl_up(P, 1, 64), Pn = __shfl_down(P, 1, 64);
    if (lane == 0) Pp = par(pq);
    if (lane == 63) Pn = par(pn);
    const bool start = valid && Pp != P, end = valid && Pn != P;
    const bool real = valid && P < PAR_HOLE;  // (a parent run, not the root sentinel or a hole)
    uint32_t off = 0;
    if (real) {
      const unsigned long long m = rm.hm[p >> 6] & ((2ULL << (p & 63)) - 1ULL);  // (the word run_of read)
      const uint32_t hp = m ? (p & ~63u) + 63u - static_cast<uint32_t>(__clzll(m)) : a.hh[P].x;
      off = p - hp + 1u;
      if (start) a.rr[P].z = k;
      if (end) a.rr[P].w = k + 1;
    }
    if (valid) offk[k] = (start ? SEGF : 0u) | off;
    if (leaf) a.tk[k] = e.y;  // (kinv[r] == k)
    uint32_t hi = 0, lo = 0;
    if (real) {
      hi = (leaf ? 1u : 0u) + (start ? k : 0u) - (end ? k + 1u : 0u);
      lo = leaf ? e.y : 0u;
    }
    unsigned long long v = (static_cast<unsigned long long>(hi) << 32) | lo;
    const uint32_t key = real ? P : NONE - 4 - lane;  // (distinct per lane without a parent run)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // segmented inclusive sum over the lanes of one parent (contiguous)
      const unsigned long long ov = __shfl_up(v, o, 64);
      const uint32_t ok = __shfl_up(key, o, 64);
      if (lane >= static_cast<uint32_t>(o) && ok == key) v += ov;
    }
    const uint32_t kp = __shfl_up(key, 1, 64), kn = __shfl_down(key, 1, 64);
    const unsigned long long gs = __ballot(lane == 0 || kp != key);  // the groups' first lanes
    const uint32_t f = 63u - static_cast<uint32_t>(__clzll(gs & ((2ULL << lane) - 1ULL)));
    const bool fstart = __shfl(start ? 1u : 0u, static_cast<int>(f), 64) != 0;
    if (real && (lane == 63 || kn != key)) {  // the group's last lane
      if (fstart && end && (v >> 32) == 0) {  // the whole range, every child a leaf
        const uint4 ep = a.rr[P];
        run_climb2(a, P, ep, ep.y + static_cast<uint32_t>(v));
      } else if (v != 0) {
        const unsigned long long old = atomicAdd(&a.ca[P], v);
        const uint4 ep = a.rr[P];
        const unsigned long long nv = old + v;
        if ((nv >> 32) == 0) run_climb2(a, P, ep, ep.y + static_cast<uint32_t>(nv));
      }
    }
  }
}

// The offsets w by a segmented inclusive scan of the sizes in sorted order
// (a parent's child range is one segment; the root sentinel's children one
// more): its epilogue writes w(c) = the sizes of c's siblings sorted before
// it + offk, and the expansion reads the inclusive values (xs & ~SEGF).
struct SegSumOp {
  static __device__ __forceinline__ uint32_t id() { return 0u; }
  static __device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b) {
    return (b & SEGF) ? b : ((a & SEGF) | ((a & ~SEGF) + b));
  }
};
struct RunSizeGen {
  static constexpr bool kStriped = true;
  static constexpr bool kEpilogue = false;
  const uint32_t* tk;
  const uint32_t* offk;
  __device__ __forceinline__ bool aligned(uint64_t b) const {
    return ((reinterpret_cast<uintptr_t>(tk + b) | reinterpret_cast<uintptr_t>(offk + b)) & 15) == 0;
  }
  __device__ __forceinline__ uint4 load4(uint64_t b) const {
    const uint4 t = *reinterpret_cast<const uint4*>(tk + b), f = *reinterpret_cast<const uint4*>(offk + b);
    return make_uint4(t.x | (f.x & SEGF), t.y | (f.y & SEGF), t.z | (f.z & SEGF), t.w | (f.w & SEGF));
  }
  __device__ __forceinline__ void load(uint64_t b, uint64_t n, uint32_t* v) const {
#pragma unroll
    for (int j = 0; j < DS_ITEMS; ++j) v[j] = b + j < n ? (tk[b + j] | (offk[b + j] & SEGF)) : 0u;
  }
};

// w(c) = the sizes of c's siblings sorted before it (the segmented scan one
// position back, 0 at a range's start) + offk (a grid-wide pass: the scan's
// few large tiles would serialise these random stores)
__global__ void __launch_bounds__(BLOCK) k_run_w2(RunArr a, uint32_t Q, const uint32_t* sarr, const uint32_t* pk,
                                                  const uint32_t* xs, const uint32_t* offk) {
  if (a.qd) Q = min(*a.qd, Q);
  RUN_LOOP(k) {
    const uint32_t f = offk[k], r = sarr[k], p = pk[k];
    if (p > Q) continue;  // (hole runs)
    const uint32_t ex = (f & SEGF) ? 0u : (xs[k - 1] & ~SEGF);
    a.rr[r].y = ex + (f & ~SEGF);
  }
}

// The subtree sizes in sorted order (tk, written by k_run_tree_up at each
// run's sorted position), summed inclusively by the xs scan:
// S(k) = the sizes of the first k entries = k ? xs[k - 1] : 0.
__device__ __forceinline__ uint32_t run_S(const uint32_t* xs, uint32_t k) { return k ? xs[k - 1] : 0u; }

// Per parent run P the sorted positions er = [x, y) of its child runs
// (contiguous: P owns a contiguous slot range and the list is by slot); the
// first position of the root sentinel's children to *groot. Neighbours'
// parents come from the adjacent lanes (a wave holds consecutive positions).
// (a parent run comes from the run masks of its attach slot, L2-resident,
// instead of a gather of the child's record)
__global__ void __launch_bounds__(BLOCK) k_run_gstart(RunArr a, uint32_t Q, const uint32_t* pk, RunMask rm,
                                                      uint32_t* groot) {
  if (a.qd) Q = min(*a.qd, Q);  // (FlatRec::q: the bound stays the limit)
  const uint32_t R = *a.nR;
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t k0 = blockIdx.x * blockDim.x; k0 < R; k0 += gridDim.x * blockDim.x) {
    const uint32_t k = k0 + threadIdx.x;
    const uint32_t p = k < R ? pk[k] : Q + 1;
    const uint32_t P = p < Q ? run_of(rm, p) : NONE;
    uint32_t Pp = __shfl_up(P, 1, 64), Pn = __shfl_down(P, 1, 64);
    if (k >= R) continue;
    if (p == Q && (k == 0 || pk[k - 1] != Q)) *groot = k;
    if (p >= Q) continue;
    if (lane == 0) Pp = k ? (pk[k - 1] < Q ? run_of(rm, pk[k - 1]) : NONE) : NONE;
    if (lane == 63 || k + 1 == R) Pn = k + 1 < R && pk[k + 1] < Q ? run_of(rm, pk[k + 1]) : NONE;
    if (Pp != P) a.rr[P].z = k;
    if (Pn != P) a.rr[P].w = k + 1;
  }
}

// w(r): the head's rank minus its parent run head's rank (root children:
// the rank itself). Inside the parent run P, slot p is preceded by p - head(P)
// slots of P and by the subtrees of P's child runs attached before p; run r
// itself comes after p and after its siblings at p with a larger slot (the
// ones sorted before it): together, the child runs of P sorted before r.
__global__ void __launch_bounds__(BLOCK) k_run_w(RunArr a, uint32_t Q, const uint32_t* sarr, const uint32_t* pk,
                                                 const uint32_t* xs, const uint32_t* groot, RunMask rm) {
  if (a.qd) Q = min(*a.qd, Q);  // (FlatRec::q: the bound stays the limit)
  RUN_LOOP(k) {
    const uint32_t r = sarr[k], p = pk[k];
    if (p > Q) continue;  // (hole runs)
    // (w replaces the length in the record: k_run_tree_up has used it)
    if (p == Q) {
      a.rr[r].y = run_S(xs, k) - run_S(xs, *groot);
    } else {
      const uint32_t P = run_of(rm, p);  // (= the record's parent: the run holding the attach slot)
      a.rr[r].y = run_S(xs, k) - run_S(xs, a.rr[P].z) + (p - a.hh[P].x) + 1u;
    }
  }
}

// head ranks: the sum of w along the ancestor chain; a chain longer than
// RUN_MAXD flags the generic path instead (quadratic walks on deep trees)
__global__ void __launch_bounds__(BLOCK) k_run_pos(RunArr a, DevResult* dres) {
  RUN_LOOP(r) {
    const uint4 e = a.rr[r];
    uint32_t s = e.y, d = 0;
    for (uint32_t x = e.x; x != NONE;) {
      if (++d > RUN_MAXD) {
        atomicOr(&dres->run_fail, 1u);
        break;
      }
      const uint4 f = a.rr[x];  // (one record: the ancestor's w and its parent)
      s += f.y;
      x = f.x;
    }
    a.posh[r] = s;
  }
}

// Per slot, the document order: doc[rank] = tree slot, where rank = the
// head's rank + the slots of the run before q + the subtrees of the run's
// child runs attached at slots below q (child runs at q itself follow q; the
// run's child runs are contiguous in the sorted list with ascending attach
// slots: a binary search finds the first one at or above q, most runs have
// none). The run of q comes from the run masks of its word, which the
// workgroup stages in LDS for all its iterations (gfx9 waits on its vector
// memory counter in order, so a global prefetch of them would be waited for
// before this slot's dependent loads).
__global__ void __launch_bounds__(BLOCK) k_run_expand(RunArr a, uint32_t Q, uint32_t K, RunMask rm,
                                                      const uint32_t* pk, const uint32_t* xs, const uint32_t* qc,
                                                      uint32_t* doc, FlatRec fr, uint32_t lds_iters, uint32_t seg) {
  extern __shared__ uint32_t smw[];  // [lds_iters * waves] {mask lo, mask hi, base}
  Q = fr.q(Q);  // (the host sized the LDS staging for its bound: at least these iterations)
  const uint32_t iters = (Q + gridDim.x * blockDim.x - 1) / (gridDim.x * blockDim.x);
  const bool mlds = iters <= lds_iters;
  const uint32_t wpb = blockDim.x >> 6;
  if (mlds) {
    const uint32_t nw = (Q + 63) >> 6;
    for (uint32_t j = threadIdx.x; j < iters * wpb; j += blockDim.x) {
      const uint32_t w = (blockIdx.x + (j / wpb) * gridDim.x) * wpb + j % wpb;
      const unsigned long long m = w < nw ? rm.hm[w] : 0ULL;
      smw[3 * j] = static_cast<uint32_t>(m);
      smw[3 * j + 1] = static_cast<uint32_t>(m >> 32);
      smw[3 * j + 2] = w < nw ? rm.hb[w] : 0u;
    }
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, stride = gridDim.x * blockDim.x;
  const unsigned long long below = (2ULL << lane) - 1ULL;
  auto run_at = [&](uint32_t it, uint32_t q) -> uint32_t {
    unsigned long long mq;
    uint32_t bq;
    if (mlds) {
      const uint32_t* e = smw + 3 * (it * wpb + (threadIdx.x >> 6));
      mq = (static_cast<unsigned long long>(e[1]) << 32) | e[0];
      bq = e[2];
    } else {
      mq = rm.hm[q >> 6];
      bq = rm.hb[q >> 6];
    }
    return bq + static_cast<uint32_t>(__popcll(mq & below)) - 1u;
  };
  // the run records of the lane's next slot load before this slot's search
  // (software pipelined: their round trip overlaps this one's)
  uint32_t q0 = blockIdx.x * blockDim.x;
  uint2 hn = make_uint2(0u, ABSENT);
  uint32_t pn = 0;
  uint4 en = make_uint4(0u, 0u, 0u, 0u);
  auto fetch = [&](uint32_t it, uint32_t q) {
    if (q < Q) {
      const uint32_t r = run_at(it, q);
      hn = a.hh[r];
      pn = a.posh[r];
      en = a.rr[r];
    }
  };
  fetch(0, q0 + threadIdx.x);
  for (uint32_t it = 0; q0 < Q; q0 += stride, ++it) {
    const uint32_t q = q0 + threadIdx.x;
    // (a slot without a node is a hole run of its own, its anchor ABSENT:
    // presence comes with the run's record, not from a pass over the slot
    // records)
    const uint2 h = hn;
    const uint32_t ph = pn;
    const uint4 er = en;
    hn = make_uint2(0u, ABSENT);
    if (q0 + stride < Q) fetch(it + 1, q + stride);
    if (q >= Q || h.y == ABSENT) continue;
    uint32_t p = ph + (q - h.x);
    const uint32_t e0 = er.z, e1 = er.w;
    if (e1 > e0) {
      uint32_t lo = e0, hi = e1;  // first k with pk[k] >= q
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pk[mid] < q) lo = mid + 1;
        else hi = mid;
      }
      if (lo > e0) p += seg ? (xs[lo - 1] & ~SEGF) : xs[lo - 1] - run_S(xs, e0);
    }
    if (p < K) doc[p] = 1 + (qc ? qc[q] : q);  // (a rank past K: a speculation that fails)
  }
}

// child counts of every node (the generic K2b/K4 fallback)
__global__ void __launch_bounds__(BLOCK) k_fl_count(uint32_t Q, const uint32_t* ep, uint32_t* cnt) {
  uint32_t hot = 0;
  GRID_STRIDE(x, Q) {
    const uint32_t d = ep[x];
    if (d == ABSENT) continue;
    if (d == Q) ++hot;
    else atomicAdd(&cnt[d], 1u);
  }
  hot = block_sum(hot);
  if (threadIdx.x == 0 && hot) atomicAdd(&cnt[Q], hot);
}

// ---------------------------------------------------------------------------
// Host orchestration
// ---------------------------------------------------------------------------
thread_local crdtm_ctx* g_prof = nullptr;

void mark_begin(crdtm_ctx* c, hipStream_t st) {
  if (!c->profile) return;
  if (c->pending) hipEventDestroy(c->pending);
  c->pending = nullptr;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return;
  hipEventRecord(e, st);
  c->pending = e;
}

void mark(crdtm_ctx* c, const char* name, hipStream_t st) {
  if (!c->profile || !c->pending) return;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return;
  hipEventRecord(e, st);
  c->marks.push_back({name, c->pending, e});
  c->pending = nullptr;
}

template <class T>
static int grow_array(T*& p, uint64_t old_n, uint64_t new_n) {
  T* q = nullptr;
  HIP_CHECK(hipMalloc(&q, new_n * sizeof(T) + 256));
  if (p) {
    if (old_n) HIP_CHECK(hipMemcpy(q, p, old_n * sizeof(T), hipMemcpyDeviceToDevice));
    HIP_CHECK(hipFree(p));
  }
  p = q;
  return CRDTM_OK;
}

DevStore::~DevStore() {
  void* ps[] = {d.s_key, d.s_next, d.s_src, d.s_child, d.s_dict, d.s_flags, d.d_sent,
                d.d_owner, d.l_kind, d.l_ts, d.l_val, d.l_off, d.l_path, d.doc};
  for (void* p : ps)
    if (p) hipFree(p);
}

static int grow_tree_arrays(crdtm_tree* t, const TreeCaps& need);

// Grows the state's arrays (keeping their contents); never called on a
// store other versions share (api.hip unshares before every write).
int grow_tree(crdtm_tree* t, const TreeCaps& need) {
  if (!t->store) t->store = std::make_shared<DevStore>();
  const int r = grow_tree_arrays(t, need);
  t->store->d = t->d;  // the store owns whatever grow_array left in place
  return r;
}

static int grow_tree_arrays(crdtm_tree* t, const TreeCaps& need) {
  HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
  TreeCaps& c = t->cap;
  auto bump = [](uint64_t have, uint64_t want) { return want <= have ? have : (want + want / 4 + 1024); };
  if (need.slots > c.slots) {
    uint64_t n = bump(c.slots, need.slots);
    int r = 0;
    if ((r = grow_array(t->d.s_key, t->n_slots, n)) || (r = grow_array(t->d.s_next, t->n_slots, n)) ||
        (r = grow_array(t->d.s_src, t->n_slots, n)) || (r = grow_array(t->d.s_child, t->n_slots, n)) ||
        (r = grow_array(t->d.s_dict, t->n_slots, n)) || (r = grow_array(t->d.s_flags, t->n_slots, n)))
      return r;
    c.slots = n;
  }
  if (need.dicts > c.dicts) {
    uint64_t n = bump(c.dicts, need.dicts);
    int r = 0;
    if ((r = grow_array(t->d.d_sent, t->n_dicts, n)) || (r = grow_array(t->d.d_owner, t->n_dicts, n))) return r;
    c.dicts = n;
  }
  if (need.log > c.log) {
    uint64_t n = bump(c.log, need.log);
    int r = 0;
    if ((r = grow_array(t->d.l_kind, t->log_n, n)) || (r = grow_array(t->d.l_ts, t->log_n, n)) ||
        (r = grow_array(t->d.l_val, t->log_n, n)) || (r = grow_array(t->d.l_off, t->log_n + 1, n + 1)))
      return r;
    c.log = n;
  }
  if (need.lpath > c.lpath) {
    uint64_t n = bump(c.lpath, need.lpath);
    int r = grow_array(t->d.l_path, t->log_npath, n);
    if (r) return r;
    c.lpath = n;
  }
  if (need.doc > c.doc) {
    uint64_t n = bump(c.doc, need.doc);
    int r = grow_array(t->d.doc, t->doc_valid ? t->doc_n : 0, n);  // (the incremental merge reads it)
    if (r) return r;
    c.doc = n;
  }
  return CRDTM_OK;
}

// Copy on write: before a version that shares its arrays with another is
// written, it takes a private copy of the live portions (one device copy of
// the state, the same order of bytes as one merge writes).
int unshare_tree(crdtm_tree* t, bool keep_contents) {
  if (!t->store || t->store.use_count() == 1) return CRDTM_OK;
  HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
  const TreeDev old = t->d;
  const TreeCaps cap = t->cap;
  t->d = TreeDev{};
  t->cap = TreeCaps{};
  t->store.reset();
  int r = grow_tree(t, cap);  // fresh private arrays of the same capacity
  if (r) return r;
  if (!keep_contents) return CRDTM_OK;
  auto cp = [&](void* dst, const void* src, uint64_t bytes) -> int {
    if (bytes) HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, t->ctx->stream));
    return CRDTM_OK;
  };
  const uint64_t S = t->n_slots, D = t->n_dicts, Ln = t->log_n;
  if ((r = cp(t->d.s_key, old.s_key, S * 8)) || (r = cp(t->d.s_next, old.s_next, S * 4)) ||
      (r = cp(t->d.s_src, old.s_src, S * 4)) || (r = cp(t->d.s_child, old.s_child, S * 4)) ||
      (r = cp(t->d.s_dict, old.s_dict, S * 4)) || (r = cp(t->d.s_flags, old.s_flags, S)) ||
      (r = cp(t->d.d_sent, old.d_sent, D * 4)) || (r = cp(t->d.d_owner, old.d_owner, D * 4)) ||
      (r = cp(t->d.l_kind, old.l_kind, Ln)) || (r = cp(t->d.l_ts, old.l_ts, Ln * 8)) ||
      (r = cp(t->d.l_val, old.l_val, Ln * 4)) || (r = cp(t->d.l_off, old.l_off, (Ln + 1) * 4)) ||
      (r = cp(t->d.l_path, old.l_path, t->log_npath * 8)) ||
      (r = cp(t->d.doc, old.doc, (t->doc_valid ? t->doc_n : 0) * 4)))
    return r;
  HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
  return CRDTM_OK;
}

static uint32_t pow2_at_least(uint64_t x) {
  uint64_t p = 1024;
  while (p < x) p <<= 1;
  return static_cast<uint32_t>(p);
}

// Reads the device result block. A scan whose look-back gave up has written
// partial prefixes: report it as an engine error before anything is used.
// The host waits for the result block by polling an event recorded after the
// copy: a blocking stream synchronisation sleeps and wakes ~15 us after the
// copy ends, idling the device between the merge's phases and calls.
int sync_read(crdtm_ctx* c) {
  c->dres_ready = false;
  HIP_CHECK(hipMemcpyAsync(c->hres, c->dres, sizeof(DevResult), hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(hipEventRecord(c->ev_sync, c->stream));
  for (;;) {
    const hipError_t e = hipEventQuery(c->ev_sync);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) HIP_CHECK(e);
    spin_pause();
  }
  if (c->hres->scan_err) {
    std::fprintf(stderr, "crdtm: a device scan's look-back did not resolve\n");
    return CRDTM_E_HIP;
  }
  return CRDTM_OK;
}

// Replicas table entries collected by the commit (inline in the result
// block when they fit, else one copy).
int take_replicas(crdtm_tree* t, const long long* rep_dev) {
  const DevResult& h = *t->ctx->hres;
  const uint32_t nrep = h.n_replica_out;
  if (!nrep) return CRDTM_OK;
  const long long* hv = h.rep_inline;
  std::vector<long long> big;
  if (nrep > REP_INLINE) {
    big.resize(2 * static_cast<size_t>(nrep));
    HIP_CHECK(hipMemcpy(big.data(), rep_dev, big.size() * sizeof(long long), hipMemcpyDeviceToHost));
    hv = big.data();
  }
  for (uint32_t k = 0; k < nrep; ++k) t->replicas[hv[2 * k]] = hv[2 * k + 1];
  return CRDTM_OK;
}

__global__ void __launch_bounds__(BLOCK) k_post_flags(OpsDev o, const uint8_t* st, uint32_t* appl, uint32_t* plen) {
  GRID_STRIDE(i, o.n) {
    const bool a = st[i] == ST_APPLIED;
    appl[i] = a;
    plen[i] = a ? o.off[i + 1] - o.off[i] : 0;
  }
}

// replicas[replicaId t] := t, last writer wins, over the applied ops: fold
// into c->rtab, collect the touched replicas into `rep` (+ the inline copy).
static_assert(offsetof(DevResult, n_rep_list) == offsetof(DevResult, n_replica_out) + sizeof(uint32_t),
              "one memset clears both counters");
int replica_fold(crdtm_ctx* c, const OpsDev& o, const uint8_t* st, long long* rep, Arena& ws, hipStream_t s,
                 bool zeroed) {
  uint32_t* rlist = ws.alloc<uint32_t>(std::min<uint64_t>(o.n, REPLICA_SLOTS) + 1);
  return replica_fold_into(c, o, st, rep, rlist, s, zeroed);
}

// (rlist: min(n, REPLICA_SLOTS) + 1 words, taken by the caller)
int replica_fold_into(crdtm_ctx* c, const OpsDev& o, const uint8_t* st, long long* rep, uint32_t* rlist,
                      hipStream_t s, bool zeroed) {
  DevResult* dr = c->dres;
  const uint32_t n = o.n;
  if (!zeroed) HIP_CHECK(hipMemsetAsync(&dr->n_replica_out, 0, 2 * sizeof(uint32_t), s));  // n_replica_out, n_rep_list
  LAUNCH(k_rep_max, dim3(rep_grid(n)), dim3(BLOCK), 0, s, o, st, c->rtab, rlist, &dr->n_rep_list, rep_per(n));
  LAUNCH(k_rep_out, dim3(64), dim3(BLOCK), 0, s, o, c->rtab, rlist, &dr->n_rep_list, rep, &dr->n_replica_out,
         dr->rep_inline);
  return CRDTM_OK;
}

// Append the applied ops to the log and fold replicas; shared by both paths.
int post_pass(crdtm_tree* t, const OpsDev& o, const uint8_t* st, Arena& ws) {
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  const uint32_t n = o.n;
  uint32_t* appl = ws.alloc<uint32_t>(n + 1);
  uint32_t* plen = ws.alloc<uint32_t>(n + 1);
  long long* rep = ws.alloc<long long>(2 * static_cast<uint64_t>(n) + 2);
  LAUNCH(k_post_flags, dim3(grid_for(n)), dim3(BLOCK), 0, s, o, st, appl, plen);
  DevResult* dr = c->dres;
  int r;
  if ((r = scan_excl_u32(appl, appl, n, &dr->log_n, ws, s))) return r;
  if ((r = scan_excl_u32(plen, plen, n, &dr->log_npath, ws, s))) return r;
  LAUNCH(k_log, dim3(grid_for(n)), dim3(BLOCK), 0, s, o, st, t->d, static_cast<uint32_t>(t->log_n),
                     static_cast<uint32_t>(t->log_npath), appl, plen);
  LAUNCH(k_log_tail, dim3(1), dim3(1), 0, s, t->d, static_cast<uint32_t>(t->log_n), &dr->log_n,
                     static_cast<uint32_t>(t->log_npath), &dr->log_npath);
  if ((r = replica_fold(c, o, st, rep, ws, s))) return r;
  if ((r = sync_read(c))) return r;
  if ((r = take_replicas(t, rep))) return r;
  t->last_begin = t->log_n;
  t->log_n += c->hres->log_n;
  t->log_npath += c->hres->log_npath;
  t->last_end = t->log_n;
  return CRDTM_OK;
}

static int run_replay(crdtm_tree* t, const OpsDev& o, uint8_t* st, crdtm_result* res, uint32_t guard) {
  if (t->remerge) return R_INCR;  // replay the batch alone on the untouched state instead
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  uint64_t nadd = o.n;  // upper bound on new nodes
  uint64_t extra = 64;
  const size_t arena_mark = c->ws.used;
  for (int attempt = 0; attempt < 8; ++attempt) {
    TreeCaps need = t->cap;
    need.slots = std::max<uint64_t>(need.slots, t->n_slots + 2 * nadd + extra);
    need.dicts = std::max<uint64_t>(need.dicts, t->n_dicts + nadd + extra);
    need.log = std::max<uint64_t>(need.log, t->log_n + o.n + 1);
    need.lpath = std::max<uint64_t>(need.lpath, t->log_npath + o.n_path + 1);
    int r = grow_tree(t, need);
    if (r) return r;
    Arena& ws = c->ws;
    ws.used = arena_mark;
    const uint64_t slot_cap = t->cap.slots;
    const uint32_t H = pow2_at_least(2 * slot_cap);
    SlotHash hh;
    hh.dict = ws.alloc<uint32_t>(H);
    hh.key = ws.alloc<long long>(H);
    hh.slot = ws.alloc<uint32_t>(H);
    hh.mask = H - 1;
    uint32_t* dhead = ws.alloc<uint32_t>(t->cap.dicts);
    uint32_t* mnext = ws.alloc<uint32_t>(slot_cap);
    const uint32_t undo_cap = static_cast<uint32_t>(4 * static_cast<uint64_t>(o.n) + 4 * extra + 1024);
    uint32_t* undo = ws.alloc<uint32_t>(3 * static_cast<uint64_t>(undo_cap));
    const uint32_t qcap = static_cast<uint32_t>(t->cap.dicts);
    uint32_t* queue = ws.alloc<uint32_t>(2 * static_cast<uint64_t>(qcap) + 2);
    HIP_CHECK(hipMemsetAsync(hh.slot, 0xFF, H * sizeof(uint32_t), s));
    HIP_CHECK(hipMemsetAsync(dhead, 0xFF, t->cap.dicts * sizeof(uint32_t), s));
    LAUNCH(k_replay_index, dim3(grid_for(t->n_slots)), dim3(BLOCK), 0, s, t->d,
                       static_cast<uint32_t>(t->n_slots), hh, dhead, mnext);
    ReplayArgs a;
    a.T = t->d;
    a.H = hh;
    a.dhead = dhead;
    a.mnext = mnext;
    a.undo = undo;
    a.undo_cap = undo_cap;
    a.queue = queue;
    a.queue_cap = qcap;
    a.committed_slots = static_cast<uint32_t>(t->n_slots);
    a.n_slots = static_cast<uint32_t>(t->n_slots);
    a.n_dicts = static_cast<uint32_t>(t->n_dicts);
    a.cap_slots = static_cast<uint32_t>(slot_cap);
    a.cap_dicts = static_cast<uint32_t>(t->cap.dicts);
    a.hash_limit = H / 2;
    a.log_base = static_cast<uint32_t>(t->log_n);
    a.ts0 = t->timestamp;
    a.root_dict = 0;
    a.src_is_op = 0;
    HIP_CHECK(hipMemsetAsync(c->dres, 0, sizeof(DevResult), s));
    LAUNCH(k_replay, dim3(1), dim3(64), 0, s, o, a, st, c->dres);
    if ((r = sync_read(c))) return r;
    const DevResult& h = *c->hres;
    if (h.replay_overflow) {
      extra = extra * 4 + t->n_slots;  // deep copies need more room
      continue;
    }
    res->path_taken = CRDTM_PATH_REPLAY;
    res->guard = guard;
    if (h.err_index != NONE) {
      res->code = static_cast<int32_t>(h.replay_err_code);
      res->err_index = h.err_index;
      return CRDTM_OK;
    }
    res->n_applied = h.n_applied;
    res->n_already = h.n_already;
    res->serial_ops = o.n;  // the whole batch in order on one lane
    res->serial_dicts = 1;
    res->serial_max = o.n;
    const long long new_ts = h.replay_timestamp;
    const uint32_t new_slots = h.replay_slots, new_dicts = h.replay_dicts;
    if ((r = post_pass(t, o, st, ws))) return r;
    t->n_slots = new_slots;
    t->n_dicts = new_dicts;
    t->timestamp = new_ts;
    t->doc_valid = false;
    res->code = CRDTM_OK;
    return CRDTM_OK;
  }
  return CRDTM_E_NOMEM;
}

__global__ void __launch_bounds__(BLOCK) k_fl_init(uint32_t Q, uint2* rec) {
  GRID_STRIDE(q, Q) rec[q].x = FR_EMPTY;
}

// The slot records of one flat merge: a new epoch of the context's anchor
// buffer (grown and zeroed when needed, zeroed when the epochs wrap; wide
// mode clears it instead), the op indices from the arena.
static int flat_rec(crdtm_ctx* c, uint32_t Q, FlatRec& fr) {
  hipStream_t s = c->stream;
  if (c->fl_cap < static_cast<uint64_t>(Q) + 1) {
    HIP_CHECK(hipStreamSynchronize(s));
    if (c->fl_rec) HIP_CHECK(hipFree(c->fl_rec));
    c->fl_rec = nullptr;
    const uint64_t cap = std::max<uint64_t>(static_cast<uint64_t>(Q) + 1 + Q / 4, 1 << 16);
    HIP_CHECK(hipMalloc(&c->fl_rec, cap * sizeof(uint2)));
    c->fl_cap = cap;
    c->fl_epoch = FR_EPOCHS;  // (forces the zeroing below)
  }
  fr.rec = c->fl_rec;
  const bool narrow = static_cast<uint64_t>(Q) + 2 < (1ULL << FR_ABITS) - 1;
  if (narrow) {
    if (++c->fl_epoch > FR_EPOCHS) {
      HIP_CHECK(hipMemsetAsync(c->fl_rec, 0, c->fl_cap * sizeof(uint2), s));  // (epoch 0 is never current)
      c->fl_epoch = 1;
    }
    fr.ep = c->fl_epoch << FR_ABITS;
    fr.amask = (1u << FR_ABITS) - 1u;
    fr.anone = fr.amask;
  } else {
    fr.ep = 0;
    fr.amask = ~0u;
    fr.anone = FR_EMPTY - 1u;
    c->fl_epoch = FR_EPOCHS;  // (the next narrow merge zeroes the buffer first)
    LAUNCH(k_fl_init, dim3(grid_for(Q, BLOCK, 4096)), dim3(BLOCK), 0, s, Q, fr.rec);
  }
  return CRDTM_OK;
}

// Flat closed form: launches K2/K4 (the order), the commit and the replica
// collection for K nodes; nothing synchronises. The flat order's run tree
// may be too deep (DevResult::run_fail, read with the final result): then
// flat_order_fallback recomputes `doc` and the chain.
struct FlatBufs {
  FlatRec fr;
  uint32_t* anc;
  uint32_t* cnt;
  uint32_t* fill;
  uint32_t* qc;
  RunMask rm;       // slot -> its run
  uint2* hh;        // run -> {head slot, effective parent of its head}
  long long* rep;
};

static void fl_log_copy(crdtm_ctx* c, const OpsDev& o, const TreeDev& T, bool simple) {
  if (simple)
    LAUNCH(k_fl_log_copy<true>, dim3(quad_grid(o.n)), dim3(BLOCK), 0, c->stream, o, T);
  else
    LAUNCH(k_fl_log_copy<false>, dim3(grid_for(o.n + 1)), dim3(BLOCK), 0, c->stream, o, T);
}

static int flat_order_commit(crdtm_tree* t, const OpsDev& o, const TsIndex& ix, uint32_t Q, uint32_t maxr,
                             const uint8_t* st, uint32_t K, bool all_applied, bool log_done, bool simple,
                             bool check, FlatBufs& fb) {
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  DevResult* dr = c->dres;
  const uint32_t n = o.n;
  const uint32_t g = grid_for(n);
  const FlatRec& fr = fb.fr;
  int r;
  fb.qc = nullptr;
  if (K > 0) {
    // ---- runs: head masks per word of 64 slots, their scan, {head, anchor} per run ----
    const uint32_t gq = grid_for(Q);
    const uint32_t NW = (Q + 63) / 64;
    RunArr ra;
    ra.nR = &dr->run_count;
    ra.qd = fr.qd;
    // (a run per present slot at most, plus a hole run per absent slot)
    ra.hh = fb.hh = ws.alloc<uint2>(Q + 1);
    unsigned long long* hm = ws.alloc<unsigned long long>(NW + 1);
    uint32_t* hc = ws.alloc<uint32_t>(NW + 1);
    uint32_t* hb = ws.alloc<uint32_t>(NW + 1);
    fb.rm = RunMask{hm, hb};
    uint32_t* logidx = nullptr;
    if (!all_applied) {  // compacted log (its scans share the ctx scan pool: main stream)
      logidx = ws.alloc<uint32_t>(n + 1);
      uint32_t* plen = ws.alloc<uint32_t>(n + 1);
      LAUNCH(k_post_flags, dim3(g), dim3(BLOCK), 0, s, o, st, logidx, plen);
      if ((r = scan_excl_u32(logidx, logidx, n, &dr->log_n, ws, s))) return r;
      if ((r = scan_excl_u32(plen, plen, n, &dr->log_npath, ws, s))) return r;
      LAUNCH(k_log, dim3(g), dim3(BLOCK), 0, s, o, st, t->d, 0u, 0u, logidx, plen);
      LAUNCH(k_log_tail, dim3(1), dim3(1), 0, s, t->d, 0u, &dr->log_n, 0u, &dr->log_npath);
    }
    uint32_t* qc = nullptr;
    if (!fr.qd && Q != K) {  // slots with no node: compact (the speculation confirms there are none)
      qc = fb.qc = ws.alloc<uint32_t>(Q);
      LAUNCH(k_fl_present, dim3(gq), dim3(BLOCK), 0, s, Q, fr, qc);
      if ((r = scan_excl_u32(qc, qc, Q, nullptr, ws, s))) return r;
    }
    // (A/B: CRDTM_MASK_U = words per wave and iteration, 1 / 2 / 4;
    // CRDTM_MASK_GRID = the workgroup cap)
    static const uint32_t mask_u = [] {
      const char* e = getenv("CRDTM_MASK_U");
      const uint32_t u = e ? static_cast<uint32_t>(atoi(e)) : RM_MASK_UNROLL;
      return (u == 1 || u == 4) ? u : RM_MASK_UNROLL;
    }();
    // (1,024 workgroups: 0.689 -> 0.659 ms per flat10m step against 2,048;
    // 512: 0.70)
    static const uint32_t mask_grid = env_grid("CRDTM_MASK_GRID", 1024);
    const uint32_t gw = std::max<uint32_t>(1, std::min<uint32_t>(mask_grid, (NW + mask_u * (BLOCK / 64) - 1) /
                                                                                 (mask_u * (BLOCK / 64))));
    const size_t mshm = maxr + 1 <= HOST_RANGES ? 3 * (maxr + 1) * sizeof(uint32_t) : 0;
    const bool dq = fr.qd != nullptr;  // (the kernel's DEVQ instance assumes the speculation's shape)
    auto mask_launch = [&](auto kern, const char* name) {
      prof_begin(s);
      hipLaunchKernelGGL(kern, dim3(gw), dim3(BLOCK), mshm, s, fr, Q, hm, hc, t->d, qc, logidx, o, ix, maxr + 1,
                         check ? dr : nullptr, c->rtab);
      prof_mark(name, s);
    };
    static const bool diag_mask2 = [] {  // (diagnostic: the pass twice, the second on a warm memory system)
      const char* e = getenv("CRDTM_DIAG_MASK2");
      return e && e[0] == '1';
    }();
    if (diag_mask2) mask_launch(dq ? k_run_mask<RM_MASK_UNROLL, true> : k_run_mask<RM_MASK_UNROLL, false>, "k_run_mask");
    if (mask_u == 1) mask_launch(dq ? k_run_mask<1, true> : k_run_mask<1, false>, "k_run_mask");
    else if (mask_u == 4) mask_launch(dq ? k_run_mask<4, true> : k_run_mask<4, false>, "k_run_mask");
    else mask_launch(dq ? k_run_mask<RM_MASK_UNROLL, true> : k_run_mask<RM_MASK_UNROLL, false>, "k_run_mask");
    if ((r = dscan<SumOp, false>(ArrGen{hc}, hb, NW, &dr->run_count, ws, s, nullptr, fr.qd ? &dr->fl_nw : nullptr,
                                 "k_dscan_runs")))
      return r;
    // (env CRDTM_RUN_V2=0: round 5's k_run_gstart, k_run_tree_up, scan, k_run_w)
    static const bool run_v2 = [] {
      const char* e = getenv("CRDTM_RUN_V2");
      return !(e && e[0] == '0');
    }();
    ra.hasch = run_v2 ? ws.alloc<uint8_t>(Q + 1) : nullptr;
    static const uint32_t heads_grid = env_grid("CRDTM_HEADS_GRID", 4096);
    LAUNCH(k_run_heads, dim3(grid_for(64ULL * NW, BLOCK, heads_grid)), dim3(BLOCK), 0, s, fr, Q, fb.rm, ra.hh,
           ra.hasch);
    // ---- K2a (heads' effective parents), parent runs, sibling order (stable radix sort by attach slot) ----
    ra.rr = ws.alloc<uint4>(Q + 1);
    ra.ca = ws.alloc<unsigned long long>(Q + 1);
    uint32_t* kinv = ws.alloc<uint32_t>(Q + 1);
    ra.kinv = kinv;
    ra.posh = ws.alloc<uint32_t>(Q + 1);
    uint32_t* sk[2] = {ws.alloc<uint32_t>(Q + 1), ws.alloc<uint32_t>(Q + 1)};
    uint32_t* sv[2] = {ws.alloc<uint32_t>(Q + 1), ws.alloc<uint32_t>(Q + 1)};
    uint32_t* xs = ws.alloc<uint32_t>(Q + 1);
    uint32_t* groot = fb.cnt;  // one word: the root sentinel's first child in the sorted list
    static const uint32_t run_grid = env_grid("CRDTM_RUN_GRID", 2048);
    const uint32_t gr = grid_for(Q, BLOCK, run_grid);
    // (env CRDTM_EP_COHERENT=1: the walks read and write at agent scope)
    static const bool ep_coh = [] {
      const char* e = getenv("CRDTM_EP_COHERENT");
      return e && e[0] == '1';
    }();
    if (ep_coh) LAUNCH(k_run_ep<true>, dim3(gr), dim3(BLOCK), 0, s, ra, Q, fb.rm, fr, sk[0], sv[0]);
    else LAUNCH(k_run_ep<false>, dim3(gr), dim3(BLOCK), 0, s, ra, Q, fb.rm, fr, sk[0], sv[0]);
    uint32_t *pk = nullptr, *sarr = nullptr;  // attach slot, run: siblings grouped by slot, slots ascending
    // (measured and reverted in round 5: a bucket sort — bucket histograms,
    // one scatter, an LDS bitonic sort per bucket — was 3.4 ms against 0.09:
    // attach slots concentrate on the document's early slots, so 53 buckets
    // of 16k slots held 4k-28k runs and sorted in global memory)
    {
      uint32_t sbits = 8;
      while (sbits < 32 && ((static_cast<uint64_t>(Q) + 1) >> sbits) != 0) sbits += 8;
      if ((r = radix_sort_pairs(sk[0], sv[0], sk[1], sv[1], ra.nR, Q, sbits, ws, s, &pk, &sarr, kinv))) return r;
      ra.tk = pk == sk[0] ? sk[1] : sk[0];  // (free after the sort)
      if (!run_v2) LAUNCH(k_run_gstart, dim3(gr), dim3(BLOCK), 0, s, ra, Q, pk, fb.rm, groot);
    }
    // ---- subtree sizes (one launch, in sorted order), head ranks, the document order ----
    if (run_v2) {
      uint32_t* offk = ws.alloc<uint32_t>(Q + 1);
      LAUNCH(k_run_sizes, dim3(gr), dim3(BLOCK), 0, s, ra, Q, sarr, pk, fb.rm, offk);
      if ((r = dscan<SegSumOp, true>(RunSizeGen{ra.tk, offk}, xs, Q, nullptr, ws, s, nullptr, ra.nR, "k_dscan_seg")))
        return r;
      LAUNCH(k_run_w2, dim3(gr), dim3(BLOCK), 0, s, ra, Q, sarr, pk, xs, offk);
    } else {
      LAUNCH(k_run_tree_up, dim3(gr), dim3(BLOCK), 0, s, ra, sarr);
      if ((r = dscan<SumOp, true>(ArrGen{ra.tk}, xs, Q, nullptr, ws, s, nullptr, ra.nR, "k_dscan_xs"))) return r;
      LAUNCH(k_run_w, dim3(gr), dim3(BLOCK), 0, s, ra, Q, sarr, pk, xs, groot, fb.rm);
    }
    LAUNCH(k_run_pos, dim3(gr), dim3(BLOCK), 0, s, ra, dr);
    // ---- the document order, the chain ----
    static const uint32_t ex_grid = env_grid("CRDTM_EX_GRID", 2048);
    const uint32_t gx = grid_for(Q, BLOCK, ex_grid);
    const uint32_t ex_iters = (Q + gx * BLOCK - 1) / (gx * BLOCK);
    LAUNCH(k_run_expand, dim3(gx), dim3(BLOCK),
           ex_iters <= EX_ITERS ? 3 * ex_iters * (BLOCK / 64) * sizeof(uint32_t) : 0, s, ra, Q, K, fb.rm, pk, xs, qc,
           t->d.doc, fr, ex_iters <= EX_ITERS ? ex_iters : 0u, run_v2 ? 1u : 0u);
    // (measured and reverted in round 5: the raw `next` written in slot order
    // by the expansion — the run's next slot, the first child run at the
    // slot, or the successor of the run's sub-document found by a walk up in
    // k_run_pos — cost 36 + 32 us more there than this pass's 33 us)
    static const uint32_t next_grid = env_grid("CRDTM_NEXT_GRID", 1u << 20);
    fb.rep = ws.alloc<long long>(2 * static_cast<uint64_t>(maxr) + 2);
    // (the replicas collection rides on this launch: it is the merge's last
    // when the log was written by the claim)
    RepCollect rc{o, 0u, c->rtab, fb.rep, &dr->n_replica_out, dr->rep_inline, check ? c->crange : nullptr};
    const bool rep_here = !(all_applied && !log_done);
    if (rep_here) rc.nr = maxr + 1;
    LAUNCH(k_fl_next, dim3(grid_for(K, BLOCK, next_grid)), dim3(BLOCK), 0, s, K, t->d.doc, t->d, t->cap.slots, rc);
    if (rep_here) return CRDTM_OK;
    if (all_applied && !log_done) fl_log_copy(c, o, t->d, simple);
  } else if (all_applied && !log_done) {
    fl_log_copy(c, o, t->d, simple);
  }
  if (!fb.rep) fb.rep = ws.alloc<long long>(2 * static_cast<uint64_t>(maxr) + 2);
  // (the speculation's commit is the merge's last: the range table is reset here too)
  LAUNCH(k_fl_rep_collect, dim3(grid_for(maxr + 1)), dim3(BLOCK), 0, s, o, maxr + 1, c->rtab, fb.rep,
         &dr->n_replica_out, dr->rep_inline, check ? c->crange : nullptr);
  return CRDTM_OK;
}

// The generic order for a run tree deeper than RUN_MAXD: children of every
// node, Euler tour + list ranking, then the chain.
static int flat_order_fallback(crdtm_tree* t, uint32_t Q, uint32_t K, FlatBufs& fb) {
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  DevResult* dr = c->dres;
  const uint32_t U = Q + 1;
  const uint32_t gq = grid_for(Q);
  uint32_t* anc = fb.anc;
  uint32_t* cnt = fb.cnt;
  uint32_t* fill = fb.fill;
  uint32_t* qc = fb.qc;
  int r;
  {  // ep per slot (the run path keeps it per run)
    RunArr ra{};
    ra.hh = fb.hh;
    LAUNCH(k_run_ep_slots, dim3(gq), dim3(BLOCK), 0, s, ra, Q, fb.rm, fb.fr, anc);
  }
  // ---- a run tree deeper than RUN_MAXD: children of every node, Euler tour + list ranking ----
  uint32_t* carr = ws.alloc<uint32_t>(U);
  uint32_t* ns = ws.alloc<uint32_t>(U);
  HIP_CHECK(hipMemsetAsync(cnt, 0, (U + 1) * sizeof(uint32_t), s));
  HIP_CHECK(hipMemsetAsync(fill, 0, (U + 1) * sizeof(uint32_t), s));
  LAUNCH(k_fl_count, dim3(grid_for(Q, BLOCK, 2048)), dim3(BLOCK), 0, s, Q, anc, cnt);
  uint32_t* n_child = &dr->n_sentinels;  // scratch word for the scan total
  if ((r = scan_excl_u32(cnt, cnt, U + 1, n_child, ws, s))) return r;
  LAUNCH(k_fl_scatter, dim3(gq), dim3(BLOCK), 0, s, Q, anc, cnt, fill, carr);
  {
    const uint32_t gb = grid_for(Q, BLOCK, 2048);
    uint32_t* bc = ws.alloc<uint32_t>(gb + 1);
    LAUNCH(k_fl_root_count, dim3(gb), dim3(BLOCK), 0, s, Q, anc, bc);
    if ((r = scan_excl_u32(bc, bc, gb, nullptr, ws, s))) return r;
    LAUNCH(k_fl_root_place, dim3(gb), dim3(BLOCK), 0, s, Q, anc, bc, cnt, carr);
  }
  if ((r = segmented_sort_desc_id(cnt, U, carr, U, ws, s, dr, Q))) return r;
  LAUNCH(k_fl_links, dim3(gq), dim3(BLOCK), 0, s, anc, cnt, n_child, carr, ns);
  if ((r = list_rank_fused(FlatEulerSrc{Q, anc, cnt, carr, ns}, 2ULL * U, 2 * Q, FlatDocSink{Q, t->d.doc, qc},
                           ws, s)))
    return r;
  LAUNCH(k_fl_next, dim3(grid_for(K)), dim3(BLOCK), 0, s, K, t->d.doc, t->d, t->cap.slots, RepCollect{});
  return CRDTM_OK;
}

// Flat closed form (see the k_fl_* kernels): the index `ix` is dense and
// already built; Q = its slot range. The common case — every op is the only
// Add of its timestamp and applies — is speculated: its order and commit are
// queued right behind the claim, and the claim's own counters, read with the
// final result, confirm it (one host round trip for the whole merge). A
// batch where some op does not apply is then decided op by op and committed
// again (the tree is fresh: its root sentinel is restored in between).
// devq (the speculation launched without a host round trip, apply_flat_spec):
// Q and maxr are upper bounds, the kernels read the true values on the device;
// the result read then checks the batch's shape (SIMPLE, dense, replica ids
// below REP_SPEC) and returns with *done = false when it is not one this path
// serves (the caller runs the general path from the top).
static int apply_flat(crdtm_tree* t, const OpsDev& o, const TsIndex& ix, uint32_t Q, uint32_t maxr, uint8_t* st,
                      uint8_t* st_out, crdtm_result* res, bool simple, RangeReset& rr, bool devq = false,
                      bool* done = nullptr) {
  if (done) *done = true;
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  DevResult* dr = c->dres;
  const uint32_t n = o.n;
  const uint32_t g = grid_for(n);
  const uint32_t U = Q + 1;  // nodes + the root sentinel
  FlatBufs fb{};
  fb.anc = ws.alloc<uint32_t>(U);
  fb.cnt = ws.alloc<uint32_t>(U + 1);
  fb.fill = ws.alloc<uint32_t>(U + 1);
  int r;
  auto grow_for = [&](uint32_t K, uint32_t applied) -> int {
    TreeCaps need = t->cap;
    need.slots = std::max<uint64_t>(need.slots, 1ULL + K + 1);
    need.dicts = std::max<uint64_t>(need.dicts, 2);
    need.log = std::max<uint64_t>(need.log, t->log_n + applied + 1);
    need.lpath = std::max<uint64_t>(need.lpath, t->log_npath + o.n_path + 1);
    need.doc = std::max<uint64_t>(need.doc, 1ULL + K);
    if (need.slots > t->cap.slots || need.dicts > t->cap.dicts || need.log > t->cap.log ||
        need.lpath > t->cap.lpath || need.doc > t->cap.doc)
      return grow_tree(t, need);
    return CRDTM_OK;
  };
  // speculation (below): every op applies, so the claim also writes the log
  // (devq: slots up to the bound Q, which the device's range may reach)
  const bool spec = (devq || Q >= n) && !t->remerge;
  if (spec && (r = grow_for(devq ? Q : n, n))) return r;
  if ((r = flat_rec(c, Q, fb.fr))) return r;
  if (devq) {
    fb.fr.qd = &dr->range_total;
    fb.fr.nrd = &dr->max_replica;
  }
  // replicas table: folded by the check over slot order when the range table fits in LDS
  // (16 bytes per replica in the claim's LDS table: up to 3,840 replicas there)
  const uint32_t nrep = maxr + 1 <= HOST_RANGES && maxr + 1 <= 3840 ? maxr + 1 : 0u;
  const uint32_t shm = (4 * nrep + (nrep ? 0 : REP_DIRECT)) * sizeof(uint32_t);
  // (devq: k_pre_ts has checked the kinds and offsets; k_fl_claim<true, true> checks them itself)
  static const uint32_t claim_grid = env_grid("CRDTM_CLAIM_GRID", 1024) & ~7u;  // (XCD chunks: a multiple of 8; 1,024 after the LDS staging: 0.610 -> 0.604 ms at flat10m)
  if (simple && spec && devq && nrep)
    LAUNCH((k_fl_claim<true, false, true>), dim3(std::min(quad_grid(n), std::max(8u, claim_grid))), dim3(BLOCK), shm,
           s, o, ix, Q, fb.fr, t->timestamp, c->rtab, dr, 0u, nrep, t->d, 1u);
  else if (simple)
    LAUNCH((k_fl_claim<true, false>), dim3(std::min(quad_grid(n), std::max(8u, claim_grid))), dim3(BLOCK), shm, s, o,
           ix, Q, fb.fr, t->timestamp,
           c->rtab, dr, nrep ? 0u : 1u, nrep, t->d, spec ? 1u : 0u);
  else
    LAUNCH((k_fl_claim<false, false>), dim3(quad_grid(n)), dim3(BLOCK), shm, s, o, ix, Q, fb.fr, t->timestamp,
           c->rtab, dr, nrep ? 0u : 1u, nrep, t->d, spec ? 1u : 0u);
  auto finish = [&](uint32_t K, uint32_t applied, uint32_t already, uint64_t npath, long long new_ts) -> int {
    int rr = take_replicas(t, fb.rep);
    if (rr) return rr;
    res->path_taken = CRDTM_PATH_CLOSED_FORM;
    res->n_applied = applied;
    res->n_already = already;
    t->flat_clean = true;  // one dict of live nodes (no Deletes on this path), doc covers them
    t->n_slots = 1ULL + K;
    t->n_dicts = 1;
    t->last_begin = t->log_n;
    t->log_n += applied;
    t->log_npath += npath;
    t->last_end = t->log_n;
    t->timestamp = new_ts;
    t->doc_n = K;
    t->doc_valid = true;
    return CRDTM_OK;
  };
  // ---- speculation: every op applies (writes the state before the check,
  // so never inside an incremental re-merge) ----
  if (spec) {
    if ((r = flat_order_commit(t, o, ix, Q, maxr, st, n, true, true, simple, true, fb))) return r;
    if (st_out) LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, nullptr, n, NONE, st_out);
    rr.armed = false;  // (k_fl_rep_collect reset the range table: no launch after the result read)
    if ((r = sync_read(c))) return r;
    const DevResult& h = *c->hres;
    uint32_t present = 0, keys = 0, own = 0, slow = 0;  // (k_run_expand / k_fl_claim shards)
    for (int k = 0; k < 16; ++k) {
      present += h.fl_part[32 * k];
      keys += h.fl_part[32 * k + 1];
      own += h.fl_part[32 * k + 2];
      slow += h.fl_part[32 * k + 3];
    }
    if (devq) {
      // the shape the launches assumed: every op an Add with a one-element
      // path, non-negative timestamps, a dense range within the bound, replica
      // ids below REP_SPEC; else nothing of this merge is kept
      if (h.spec_fail || h.has_negative || h.max_replica >= REP_SPEC || h.range_total > Q ||
          h.range_total > 4ULL * n + 65536) {
        LAUNCH(k_reset_root, dim3(1), dim3(1), 0, s, t->d.s_next, nullptr);
        *done = false;
        return CRDTM_OK;
      }
      // (the shape first: k_pre_ts range-checks every op's ts, a Delete's
      // too, which the reference ignores — a batch with a Delete is not one
      // this path serves, and the general path checks only what it reads)
      if (h.bad_range) return CRDTM_E_RANGE;  // (every op an Add: its ts or path element is out of range)
      Q = h.range_total;  // (known from here: the later launches take the host's values)
      maxr = h.max_replica;
      fb.fr.qd = nullptr;
      fb.fr.nrd = nullptr;
      if (t->max_depth < 1) t->max_depth = 1;
    }
    if (h.bad_range) return CRDTM_E_RANGE;  // (k_fl_claim's path check; the caller restores the fresh tree)
    const long long new_ts = t->timestamp + own - t->own_bias;
    // (devq: the merge assumed no slot without a node, Q == n)
    const bool every = h.err_index == NONE && slow == 0 && present == keys && keys == n && (!devq || Q == n);
    if (every && replica_of(new_ts) == replica_of(t->timestamp)) {
      if (h.run_fail && (r = flat_order_fallback(t, Q, n, fb))) return r;
      res->guard = 0;
      return finish(n, n, 0, o.n_path, new_ts);
    }
    // not confirmed: the fresh tree's only reachable change is its root sentinel's `next`
    LAUNCH(k_reset_root, dim3(1), dim3(1), 0, s, t->d.s_next, nullptr);
    // the replica ranges again (reset above; k_pre's other results are idempotent, no Delete here)
    launch_pre(c, o, s);
    LAUNCH(k_range_base, dim3(1), dim3(BLOCK), 0, s, c->crange, const_cast<uint32_t*>(ix.base), dr);
    rr.armed = true;
  }
  // ---- per-op statuses: duplicates, ts 0, errors ----
  LAUNCH(k_fl_rep_collect, dim3(grid_for(maxr + 1)), dim3(BLOCK), 0, s, o, maxr + 1, c->rtab, nullptr, nullptr,
         nullptr, nullptr);
  LAUNCH(k_fl_stat_reset, dim3(1), dim3(1), 0, s, dr);
  LAUNCH(k_fl_status, dim3(quad_grid(n)), dim3(BLOCK), 0, s, o, st, ix, Q, fb.fr, t->timestamp, c->rtab, dr);
  if ((r = sync_read(c))) return r;
  if (c->hres->dup_fix) {  // a smaller duplicate took its slot: the records are final now, decide again
    LAUNCH(k_fl_rep_collect, dim3(grid_for(maxr + 1)), dim3(BLOCK), 0, s, o, maxr + 1, c->rtab, nullptr, nullptr,
           nullptr, nullptr);
    LAUNCH(k_fl_stat_reset, dim3(1), dim3(1), 0, s, dr);
    LAUNCH(k_fl_status, dim3(quad_grid(n)), dim3(BLOCK), 0, s, o, st, ix, Q, fb.fr, t->timestamp, c->rtab, dr);
    if ((r = sync_read(c))) return r;
  }
  const DevResult h1 = *c->hres;
  if (h1.bad_range) return CRDTM_E_RANGE;
  uint32_t guard = 0;
  const long long new_ts = t->timestamp + h1.own_ok_adds - t->own_bias;
  if (replica_of(new_ts) != replica_of(t->timestamp)) guard |= G_REPLICA_DRIFT;
  res->guard = guard;
  if (guard || h1.err_index != NONE)  // no commit: leave the replica table clean
    LAUNCH(k_fl_rep_collect, dim3(grid_for(maxr + 1)), dim3(BLOCK), 0, s, o, maxr + 1, c->rtab, nullptr, nullptr,
           nullptr, nullptr);
  if (guard) {
    r = run_replay(t, o, st, res, guard);
    if (r == CRDTM_OK && st_out)
      LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, st, n,
             res->err_index >= 0 ? static_cast<uint32_t>(res->err_index) : NONE, st_out);
    return r;
  }
  res->path_taken = CRDTM_PATH_CLOSED_FORM;
  if (h1.err_index != NONE) {
    uint8_t est = 0;
    HIP_CHECK(hipMemcpy(&est, st + h1.err_index, 1, hipMemcpyDeviceToHost));
    res->code = est == ST_INVALID ? CRDTM_INVALID_PATH : CRDTM_OPERATION_FAILED;
    res->err_index = h1.err_index;
    if (st_out) LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, st, n, h1.err_index, st_out);
    return CRDTM_OK;
  }
  const uint32_t K = h1.n_adds_applied;
  const bool all_applied = h1.n_applied == n;
  if ((r = grow_for(K, h1.n_applied))) return r;
  LAUNCH(k_fl_commit_reset, dim3(1), dim3(1), 0, s, dr);
  if ((r = flat_order_commit(t, o, ix, Q, maxr, st, K, all_applied, spec, simple, false, fb))) return r;
  if (st_out) LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, st, n, NONE, st_out);
  if ((r = sync_read(c))) return r;
  if (c->hres->run_fail && (r = flat_order_fallback(t, Q, K, fb))) return r;
  return finish(K, h1.n_applied, h1.n_already, all_applied ? o.n_path : c->hres->log_npath, new_ts);
}

static int apply_core(crdtm_tree* t, const OpsDev& o, uint8_t* st_out, crdtm_result* res) {
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;  // reset by the caller (inputs may live in it)
  const uint32_t n = o.n;
  res->err_index = -1;
  res->code = CRDTM_OK;
  if (n == 0) {
    res->path_taken = CRDTM_PATH_CLOSED_FORM;
    t->last_begin = t->last_end = t->log_n;
    return CRDTM_OK;
  }
  Work w;
  w.st = ws.alloc<uint8_t>(n);
  uint32_t* rbase = ws.alloc<uint32_t>(RID_SLOTS + 1);
  DevResult* dr = c->dres;
  const bool dres_ready = c->dres_ready;  // (the tree reset's launch initialised it)
  c->dres_ready = false;
  // (env CRDTM_FORCE_REPLAY=1: every batch takes the one-lane sequential
  // replay, so the cost of that fallback is measurable on any workload)
  const char* fe = getenv("CRDTM_FORCE_REPLAY");
  const bool force_replay = fe && fe[0] == '1';
  // The flat speculation (config 3's shape): a fresh tree and as many path
  // elements as ops, so every op may be an Add whose path is its anchor
  // alone. The pre-pass reads the timestamps only, the claim checks the
  // kinds and path offsets, and the whole merge is queued at once with the
  // slot range read on the device (no host round trip between the pre-pass
  // and the claim). The result read confirms the shape; a batch of another
  // shape leaves nothing behind and takes the general path below.
  // (env CRDTM_FLAT_SPEC=0: off)
  static const bool spec_on = [] {
    const char* e = getenv("CRDTM_FLAT_SPEC");
    return !(e && e[0] == '0');
  }();
  if (spec_on && !force_replay && t->n_slots == 1 && t->log_n == 0 && !t->remerge && o.n_path == n) {
    // slot range bound: the radix sort's key width for n (at least 64k
    // slots: small batches with counter gaps), within the dense limit
    uint32_t b = 8;
    while (b < 32 && ((static_cast<uint64_t>(n) + 2) >> b) != 0) b += 8;
    const uint64_t qcap = std::min<uint64_t>(std::max<uint64_t>((1ULL << b) - 2, 65536), 4ULL * n + 65536);
    if (qcap + 2 < (1ULL << FR_ABITS) - 1) {
      if (!dres_ready) LAUNCH(k_dres_init, dim3(1), dim3(64), 0, s, dr);
      // (env CRDTM_PRE_GRID: workgroups; CRDTM_PRE_BLIND=1: no-return atomics only)
      static const uint32_t pre_grid = env_grid("CRDTM_PRE_GRID", 256);  // (256 x 1024 threads: 55 -> 48 us at flat10m)
      static const bool pre_blind = [] {
        const char* e = getenv("CRDTM_PRE_BLIND");
        return e && e[0] == '1';
      }();
      const uint32_t gp = static_cast<uint32_t>(std::min<uint64_t>((n / 2 + PRE_T - 1) / PRE_T + 1, pre_grid));
      if (pre_blind)
        LAUNCH((k_pre_ts<PRE_T, true>), dim3(gp), dim3(PRE_T), 0, s, o.ts, o.kind, o.off, n, c->crange, rbase, dr);
      else
        LAUNCH((k_pre_ts<PRE_T, false>), dim3(gp), dim3(PRE_T), 0, s, o.ts, o.kind, o.off, n, c->crange, rbase, dr);
      RangeReset spec_clean{c};  // (nr 0: up to the device's max_replica)
      TsIndex ix;
      ix.rng = c->crange;
      ix.base = rbase;
      ix.dense = 1;
      ix.h = TsHash{nullptr, nullptr, 0};
      ix.first = nullptr;
      bool done = false;
      int rs = apply_flat(t, o, ix, static_cast<uint32_t>(qcap), REP_SPEC - 1, w.st, st_out, res, true, spec_clean,
                          true, &done);
      if (rs || done) return rs;
    }
  }
  LAUNCH(k_dres_init, dim3(1), dim3(64), 0, s, dr);
  // (512 workgroups: each flushes its replica ranges and counters with
  // device-scope atomics that serialise per word, ~12 ns each)
  // (measured: 512 beats 1024 and 2048 workgroups on flat10m and deep10m)
  launch_pre(c, o, s);
  LAUNCH(k_range_base, dim3(1), dim3(BLOCK), 0, s, c->crange, rbase, dr);
  RangeReset keep_clean{c};  // resets the context's replica ranges on every exit
  int r;
  if ((r = sync_read(c))) return r;
  // (explicit from here: the replay paths reset the DevResult)
  keep_clean.nr = c->hres->max_replica + 1;
  if (c->hres->bad_range) return CRDTM_E_RANGE;
  const uint32_t maxlen = c->hres->max_len;
  if (t->max_depth < maxlen) t->max_depth = maxlen;
  const uint32_t g = grid_for(n);
  if (force_replay || t->n_slots != 1 || t->log_n != 0) {
    // incremental merge into existing state: exact replay
    if (o.n_path) {
      LAUNCH(k_path_range, dim3(std::min<uint32_t>(grid_for(o.n_path / 2 + 1), 1024)), dim3(BLOCK), 0, s, o, dr);
      if ((r = sync_read(c))) return r;
      if (c->hres->bad_range) return CRDTM_E_RANGE;
    }
    r = run_replay(t, o, w.st, res, force_replay ? G_FORCED : G_NOT_FRESH);
    if (r == CRDTM_OK && st_out)
      LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, w.st, n,
             res->err_index >= 0 ? static_cast<uint32_t>(res->err_index) : NONE, st_out);
    return r;
  }
  const uint32_t maxr = c->hres->max_replica;
  const uint64_t range_total = c->hres->range_total;
  // ts index: dense per-replica runs when possible, else an open-addressing hash
  TsIndex ix;
  ix.rng = c->crange;
  ix.base = rbase;
  ix.dense = (!c->hres->has_negative && range_total <= 4ULL * n + 65536) ? 1u : 0u;
  const bool flat = maxlen == 1 && c->hres->n_del == 0;
  // path elements' range check: the flat claim and the level kernels check
  // the elements they load (every element of every op's path); otherwise one
  // streaming pass on the side stream, joined before the next result read,
  // which checks it before anything is written
  const bool levels = !flat && maxlen <= MAXLV_BUCKET;
  const bool side_range = !(ix.dense && flat) && !levels && o.n_path;
  if (side_range) {
    HIP_CHECK(hipEventRecord(c->ev_fork, s));
    HIP_CHECK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
    LAUNCH(k_path_range, dim3(std::min<uint32_t>(grid_for(o.n_path / 2 + 1), 1024)), dim3(BLOCK), 0, c->side, o,
           dr);
    HIP_CHECK(hipEventRecord(c->ev_join, c->side));
  }
  auto range_ok = [&]() -> int {  // (after a sync_read that followed the join)
    return c->hres->bad_range ? CRDTM_E_RANGE : CRDTM_OK;
  };
  if (ix.dense) {
    ix.h = TsHash{nullptr, nullptr, 0};
    ix.first = nullptr;
    // (simple: every op an Add whose path is its anchor alone, op i's at path[i])
    if (flat)
      return apply_flat(t, o, ix, static_cast<uint32_t>(range_total), maxr, w.st, st_out, res, o.n_path == n,
                        keep_clean);
    ix.first = ws.alloc<uint32_t>(range_total + 1);
    HIP_CHECK(hipMemsetAsync(ix.first, 0xFF, (range_total + 1) * sizeof(uint32_t), s));
    const uint32_t nrep = maxr + 1 <= HOST_RANGES ? maxr + 1 : 0u;
    LAUNCH(k_index_store, dim3(quad_grid(n)), dim3(BLOCK), 3 * nrep * sizeof(uint32_t), s, o, ix, nrep);
    LAUNCH(k_index_fix, dim3(quad_grid(n)), dim3(BLOCK), 3 * nrep * sizeof(uint32_t), s, o, ix, nrep);
  } else {
    const uint32_t H = pow2_at_least(2 * static_cast<uint64_t>(n));
    ix.first = nullptr;
    ix.h.keys = ws.alloc<unsigned long long>(H);
    ix.h.vals = ws.alloc<uint32_t>(H);
    ix.h.mask = H - 1;
    HIP_CHECK(hipMemsetAsync(ix.h.keys, 0, H * sizeof(unsigned long long), s));
    HIP_CHECK(hipMemsetAsync(ix.h.vals, 0xFF, H * sizeof(uint32_t), s));
    LAUNCH(k_index_insert, dim3(g), dim3(BLOCK), 0, s, o, ix);
  }
  w.cur = ws.alloc<uint32_t>(n);
  w.leaf = ws.alloc<uint32_t>(n);
  w.addpar = ws.alloc<uint32_t>(n);
  w.dtime = ws.alloc<uint32_t>(n);
  w.dead = ws.alloc<uint8_t>(n);
  w.maxadd = ws.alloc<uint32_t>(n + 1);
  w.tag = ws.alloc<uint32_t>(n);
  uint32_t* anc = ws.alloc<uint32_t>(n);
  LAUNCH(k_work_init, dim3(g), dim3(BLOCK), 0, s, o, w);
  if (flat) {
    LAUNCH(k_flat_status, dim3(g), dim3(BLOCK), 0, s, o, w, ix, anc);
  } else {
    HIP_CHECK(hipMemsetAsync(w.maxadd, 0, (n + 1) * sizeof(uint32_t), s));
    if (maxlen > MAXLV_BUCKET) {  // paths this deep are not bucketed: exact replay
      HIP_CHECK(hipStreamWaitEvent(s, c->ev_join, 0));
      if ((r = sync_read(c)) || (r = range_ok())) return r;
      r = run_replay(t, o, w.st, res, G_DEEP_PATH);
      if (r == CRDTM_OK && st_out)
        LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, w.st, n,
               res->err_index >= 0 ? static_cast<uint32_t>(res->err_index) : NONE, st_out);
      return r;
    }
    // bucket the ops by |path| (one small copy back for the level sizes)
    uint32_t* lcnt = ws.alloc<uint32_t>(2 * (MAXLV_BUCKET + 1));
    uint32_t* lfill = lcnt + (MAXLV_BUCKET + 1);
    LvEnt* lists = ws.alloc<LvEnt>(n);
    w.nrec = ws.alloc<uint4>(n);
    LAUNCH(k_nrec_init, dim3(g), dim3(BLOCK), 0, s, o, w);
    HIP_CHECK(hipMemsetAsync(lcnt, 0, 2 * (MAXLV_BUCKET + 1) * sizeof(uint32_t), s));
    LAUNCH(k_len_count, dim3(grid_for(n, BLOCK, 1024)), dim3(BLOCK), 0, s, o, maxlen, lcnt);
    uint32_t hc[MAXLV_BUCKET + 1];
    HIP_CHECK(hipMemcpyAsync(hc, lcnt, (maxlen + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (int rw = stream_wait(s)) return rw;
    LevelStart hs{};
    uint32_t acc = 0;
    for (uint32_t j = 0; j <= maxlen; ++j) {
      hs.v[j] = acc;
      acc += hc[j];
    }
    LAUNCH(k_len_scatter, dim3(grid_for(n, BLOCK * 8, 2048)), dim3(BLOCK), 0, s, o, maxlen, hs, lfill, lists);
    for (uint32_t lvl = 1; lvl <= maxlen; ++lvl) {
      const uint32_t c = hc[lvl];
      if (!c) continue;
      const LvEnt* lst = lists + hs.v[lvl];
      static const uint32_t lv_grid = env_grid("CRDTM_LV_GRID", 1u << 20);  // (A/B)
      static const uint32_t lv_lds = env_grid("CRDTM_LV_LDS", 40000);
      const uint32_t gl = grid_for(c, BLOCK, lv_grid);
      // (k_lv_dict reserves 40 KB of LDS it does not use: at most 3 workgroups
      // per CU, so the lines of the prefix keys its lanes load stay in L2
      // between the load instructions; measured 1.27 -> 1.17 ms on deep10m)
      LAUNCH(k_lv_dict, dim3(gl), dim3(BLOCK), lv_lds, s, o, w, ix, lst, c, lvl, dr);
      LAUNCH(k_lv_leaf, dim3(gl), dim3(BLOCK), 0, s, o, w, ix, lst, c, lvl, dr);
      LAUNCH(k_lv_fin, dim3(gl), dim3(BLOCK), 0, s, o, w, ix, lst, c, lvl);
    }
  }
  HIP_CHECK(hipMemsetAsync(&dr->first_del, 0xFF, sizeof(uint32_t), s));
  LAUNCH(k_stats, dim3(quad_grid(n)), dim3(BLOCK), 0, s, o, w, t->timestamp, dr);
  if (side_range) HIP_CHECK(hipStreamWaitEvent(s, c->ev_join, 0));
  if ((r = sync_read(c)) || (r = range_ok())) return r;
  if (c->hres->first_del != NONE && c->hres->last_add > c->hres->first_del + 1) {
    LAUNCH(k_guard_maxadd, dim3(g), dim3(BLOCK), 0, s, o, w);
    LAUNCH(k_guard_del, dim3(g), dim3(BLOCK), 0, s, o, w, dr);
    if ((r = sync_read(c))) return r;
  }
  DevResult h1 = *c->hres;
  uint32_t guard = h1.guard;
  const long long id0 = replica_of(t->timestamp);
  const long long new_ts = t->timestamp + h1.own_ok_adds - t->own_bias;
  if (replica_of(new_ts) != id0) guard |= G_REPLICA_DRIFT;
  res->guard = guard;
  if (guard == G_DEL_BEFORE_ADD) {
    // one lane per children dict (pdr.hip); conflicts fall through to the replay
    PdrIn pin;
    pin.ix = ix;
    pin.tag = w.tag;
    pin.cur = w.cur;
    pin.leaf = w.leaf;
    pin.addpar = w.addpar;
    pin.dtime = w.dtime;
    pin.maxlen = maxlen;
    bool handled = false;
    if ((r = pdr_apply(t, o, pin, w.st, res, &handled))) return r;
    if (handled) {
      res->guard = guard;
      if (st_out)
        LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, w.st, n,
               res->err_index >= 0 ? static_cast<uint32_t>(res->err_index) : NONE, st_out);
      return CRDTM_OK;
    }
  }
  if (guard) {
    // exact sequential replay decides statuses (and errors) itself
    r = run_replay(t, o, w.st, res, guard);
    if (r == CRDTM_OK && st_out)
      LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, w.st, n,
                         res->err_index >= 0 ? static_cast<uint32_t>(res->err_index) : NONE, st_out);
    return r;
  }
  res->path_taken = CRDTM_PATH_CLOSED_FORM;
  if (h1.err_index != NONE) {
    // error class of the first failing op
    uint8_t est = 0;
    HIP_CHECK(hipMemcpy(&est, w.st + h1.err_index, 1, hipMemcpyDeviceToHost));
    res->code = est == ST_INVALID ? CRDTM_INVALID_PATH : CRDTM_OPERATION_FAILED;
    res->err_index = h1.err_index;
    if (st_out) LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, w.st, n, h1.err_index, st_out);
    return CRDTM_OK;
  }
  res->n_applied = h1.n_applied;
  res->n_already = h1.n_already;

  // ---- the op log depends on the statuses only, so it is written on the
  // side stream while K2/K4 run here ----
  // every op applied: the log is the batch (identity log index, the batch's
  // path offsets), so the two log scans are skipped
  const bool every = h1.n_applied == n;
  uint32_t* appl = nullptr;
  uint32_t* plen = nullptr;
  if (every) {
    LAUNCH(k_log_totals, dim3(1), dim3(1), 0, s, dr, n, static_cast<uint32_t>(o.n_path));
  } else {
    appl = ws.alloc<uint32_t>(n + 1);
    plen = ws.alloc<uint32_t>(n + 1);
    LAUNCH(k_post_flags, dim3(g), dim3(BLOCK), 0, s, o, w.st, appl, plen);
    if ((r = scan_excl_u32(appl, appl, n, &dr->log_n, ws, s))) return r;
    if ((r = scan_excl_u32(plen, plen, n, &dr->log_npath, ws, s))) return r;
  }
  TreeCaps need = t->cap;
  need.slots = std::max<uint64_t>(need.slots, 1 + 2ULL * h1.n_adds_applied + 1);
  need.dicts = std::max<uint64_t>(need.dicts, 1 + h1.n_adds_applied + 1);
  need.log = std::max<uint64_t>(need.log, t->log_n + h1.n_applied + 1);
  need.lpath = std::max<uint64_t>(need.lpath, t->log_npath + o.n_path + 1);
  need.doc = std::max<uint64_t>(need.doc, h1.n_adds_applied + 1);
  // capacity changes synchronise; they only happen on the first calls
  if (need.slots > t->cap.slots || need.dicts > t->cap.dicts || need.log > t->cap.log ||
      need.lpath > t->cap.lpath || need.doc > t->cap.doc) {
    if ((r = grow_tree(t, need))) return r;
  }
  long long* rep = ws.alloc<long long>(2 * static_cast<uint64_t>(n) + 2);

  // ---- K2: effective parents, document tree, sibling sort ----
  const uint32_t U = n + 2;
  uint8_t* sp = ws.alloc<uint8_t>(n + 1);
  uint32_t* cnt = ws.alloc<uint32_t>(U + 1);
  uint32_t* fill = ws.alloc<uint32_t>(U + 1);
  long long* skey = ws.alloc<long long>(U);
  uint32_t* carr = ws.alloc<uint32_t>(U);
  uint32_t* fc = ws.alloc<uint32_t>(U);
  uint32_t* ns = ws.alloc<uint32_t>(U);
  uint32_t* f1 = ws.alloc<uint32_t>(U);
  HIP_CHECK(hipMemsetAsync(sp, 0, n + 1, s));
  HIP_CHECK(hipMemsetAsync(cnt, 0, (U + 1) * sizeof(uint32_t), s));
  if (!flat) LAUNCH(k_ep_init, dim3(g), dim3(BLOCK), 0, s, o, w, anc);
  HIP_CHECK(hipEventRecord(c->ev_fork, s));
  HIP_CHECK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
  // (forked after k_ep_init, so the log copy overlaps the latency-bound
  // pointer jumping instead of the streaming passes; full grids: a small
  // background grid starves k_log's chunk loop)
  LAUNCH(k_log, dim3(g), dim3(BLOCK), 0, c->side, o, w.st, t->d, static_cast<uint32_t>(t->log_n),
         static_cast<uint32_t>(t->log_npath), appl, plen);
  LAUNCH(k_log_tail, dim3(1), dim3(1), 0, c->side, t->d, static_cast<uint32_t>(t->log_n), &dr->log_n,
         static_cast<uint32_t>(t->log_npath), &dr->log_npath);
  HIP_CHECK(hipEventRecord(c->ev_join, c->side));
  struct Join {  // every exit waits for the side stream (the arena is reused by the next call)
    crdtm_ctx* c;
    ~Join() { hipStreamWaitEvent(c->stream, c->ev_join, 0); }
  } join{c};
  LAUNCH(k_ep_jump, dim3(g), dim3(BLOCK), 0, s, o, w, anc, sp);
  const uint32_t gU = grid_for(U);
  uint32_t* sk = nullptr;  // the parent uid of every carr position
  {  // children of every document node, grouped by a radix sort on the parent uid (CSR in cnt, items in carr)
    const uint32_t m = n + 1;  // uids that may have a parent
    uint32_t* ka = ws.alloc<uint32_t>(m);
    uint32_t* kb = ws.alloc<uint32_t>(m);
    uint32_t* vb = ws.alloc<uint32_t>(m);
    uint32_t* nitems = ws.alloc<uint32_t>(1);
    const uint32_t gm = grid_for(m, BLOCK, 2048);
    LAUNCH(k_doc_keys, dim3(gm), dim3(BLOCK), 0, s, o, w, anc, sp, ka, carr, skey, fc, ns, f1, nitems);
    uint32_t kbits = 8;  // NONE (no parent) must sort after every uid <= n + 1
    while (kbits < 32 && ((static_cast<uint64_t>(n) + 2) >> kbits) != 0) kbits += 8;
    uint32_t* sv = nullptr;
    if ((r = radix_sort_pairs(ka, carr, kb, vb, nitems, m, kbits, ws, s, &sk, &sv))) return r;
    carr = sv;  // (the children in parent order: the CSR's items)
    LAUNCH(k_doc_gstart, dim3(gm), dim3(BLOCK), 0, s, sk, m, fill);
    LAUNCH(k_doc_gcount, dim3(gm), dim3(BLOCK), 0, s, sk, m, fill, cnt);
  }
  uint32_t* n_child_total = &dr->n_sentinels;  // scratch word for the scan total
  if ((r = scan_excl_u32(cnt, cnt, U + 1, n_child_total, ws, s))) return r;
  if ((r = segmented_sort(cnt, U, carr, U, skey, ws, s, dr))) return r;
  LAUNCH(k_links, dim3(grid_for(U, BLOCK, 4096)), dim3(BLOCK), 0, s, o, anc, sk, n_child_total, carr, fc, ns, f1);

  // ---- K4: Euler tour + list ranking ----
  const uint64_t E = 2ULL * U;
  uint2* ent = ws.alloc<uint2>(E);
  unsigned long long* excl = ws.alloc<unsigned long long>(E);
  LAUNCH(k_euler, dim3(gU), dim3(BLOCK), 0, s, o, w, anc, sp, fc, ns, ent);
  if ((r = list_rank_packed(ent, E, 2 * (n + 1), excl, ws, s))) return r;
  uint2* order = ws.alloc<uint2>(U);
  uint32_t* nextn = ws.alloc<uint32_t>(n);
  LAUNCH(k_order, dim3(gU), dim3(BLOCK), 0, s, o, w, sp, excl, order);
  LAUNCH(k_next, dim3(g), dim3(BLOCK), 0, s, o, w, excl, order, f1, nextn);

  // ---- K3 + commit ----
  uint32_t* kept = ws.alloc<uint32_t>(n + 1);
  uint32_t* live = ws.alloc<uint32_t>(n + 1);
  LAUNCH(k_commit_flags, dim3(g), dim3(BLOCK), 0, s, o, w, nullptr, nullptr, kept, live);
  if ((r = scan_excl_u32(kept, kept, n, &dr->n_nodes_kept, ws, s))) return r;
  if ((r = scan_excl_u32(live, live, n, &dr->n_live_kept, ws, s))) return r;
  if ((r = sync_read(c))) return r;
  const uint32_t K = c->hres->n_nodes_kept;
  CommitArgs ca;
  ca.base_slot = 1;
  ca.n_kept = K;
  ca.base_dict = 1;
  ca.log_base = static_cast<uint32_t>(t->log_n);
  LAUNCH(k_commit_nodes, dim3(g), dim3(BLOCK), 0, s, o, w, t->d, ca, kept, live, appl, nextn, fc, excl,
                     t->d.doc);
  LAUNCH(k_commit_root, dim3(1), dim3(1), 0, s, o, t->d, kept, fc, 1u);
  // (the replica fold stays here: beside the order kernels its hot table
  // lines slowed both streams)
  if ((r = replica_fold(c, o, w.st, rep, ws, s))) return r;
  if (st_out) LAUNCH(k_status_out, dim3(g), dim3(BLOCK), 0, s, w.st, n, NONE, st_out);
  HIP_CHECK(hipStreamWaitEvent(s, c->ev_join, 0));
  if ((r = sync_read(c))) return r;
  const DevResult& h2 = *c->hres;
  if ((r = take_replicas(t, rep))) return r;
  t->n_slots = 1 + static_cast<uint64_t>(h2.n_nodes_kept) + h2.n_live_kept;
  t->n_dicts = 1 + static_cast<uint64_t>(h2.n_live_kept);
  t->last_begin = t->log_n;
  t->log_n += h2.log_n;
  t->log_npath += h2.log_npath;
  t->last_end = t->log_n;
  t->timestamp = new_ts;
  t->doc_n = h2.n_live_kept;  // visible nodes = kept live nodes
  t->doc_valid = true;
  return CRDTM_OK;
}

// ---------------------------------------------------------------------------
// Incremental merges: apply into a tree that already holds state
// (src/CRDTree.elm:265-269 on any tree; the steady state of a replica that
// applies remote batches). The state is a pure function of its log: every
// logged op was Applied, in log order, and every op that was not logged
// (AlreadyApplied) changed nothing. So `apply batch state` equals
// `apply (log ++ batch) init` with the log's ops all Applied again, and that
// runs on the parallel fresh-tree paths (closed form, per-dict replay)
// instead of the one-lane replay over a rebuilt slot index. The outputs
// that are not a function of the log are carried over: the timestamp (the
// log's own-replica Adds are not counted again; AlreadyApplied ones never
// reached the log), lastOperation (the log suffix) and the statuses (the
// batch part). Nothing writes the state before the batch's last check (no
// flat speculation), so an error or a path that needs the sequential replay
// (R_INCR) leaves the state untouched and the batch is replayed alone.
// Cost: O(log + batch) parallel work per call, against O(batch) serial
// dependent steps plus an O(state) index rebuild for the replay.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(BLOCK) k_cat_ops(OpsDev lg, OpsDev b, uint32_t L, uint32_t LP, uint8_t* kind,
                                                   long long* ts, uint32_t* off, uint32_t* val) {
  GRID_STRIDE(i, L + b.n + 1) {
    if (i < L) {
      kind[i] = lg.kind[i];
      ts[i] = lg.ts[i];
      val[i] = lg.val[i];
      off[i] = lg.off[i];
    } else {
      const uint32_t j = i - L;
      if (j < b.n) {
        kind[i] = b.kind[j];
        ts[i] = b.ts[j];
        val[i] = b.val[j];
      }
      off[i] = LP + b.off[j];
    }
  }
}

// own-replica Adds of the log (incrementTimestamp, src/CRDTree.elm:337-343)
__global__ void __launch_bounds__(BLOCK) k_own_log(const uint8_t* kind, const long long* ts, uint32_t L, long long rid,
                                                   unsigned long long* out) {
  uint32_t c = 0;
  GRID_STRIDE(i, L) c += (kind[i] == CRDTM_ADD && replica_of(ts[i]) == rid) ? 1u : 0u;
  c = block_sum(c);
  if (threadIdx.x == 0 && c) atomicAdd(out, static_cast<unsigned long long>(c));
}

static bool remerge_wanted(const crdtm_tree* t, uint32_t n) {
  if (t->log_n + static_cast<uint64_t>(n) >= 0x7FFFFFF0ULL || t->max_depth > MAXLV_BUCKET) return false;
  const char* e = getenv("CRDTM_INCREMENTAL");
  if (e && !strcmp(e, "replay")) return false;
  if (e && !strcmp(e, "remerge")) return true;
  // parallel work over log + batch (~0.1-1 ns per op) against ~5 us of
  // dependent device accesses per replayed op
  return t->log_n <= 4096ULL * n;
}

static int apply_batch_paths(crdtm_tree* t, const OpsDev& o, uint8_t* st_out, crdtm_result* res) {
  const bool fresh = t->n_slots == 1 && t->log_n == 0;
  if (!fresh && o.n && ilr_wanted(t, o.n)) {  // per children dict on the state itself (ilr.hip)
    bool handled = false;
    const int r = ilr_apply(t, o, st_out, res, &handled);
    if (r != CRDTM_OK || handled) return r;
  }
  t->ilr_valid = false;  // (every other path rewrites or extends the state without its index)
  if (fresh || o.n == 0 || !remerge_wanted(t, o.n)) return apply_core(t, o, st_out, res);
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  const size_t mark0 = ws.used;
  const uint32_t L = static_cast<uint32_t>(t->log_n);
  const uint64_t LP = t->log_npath;
  OpsDev lg;
  lg.n = L;
  lg.kind = t->d.l_kind;
  lg.ts = t->d.l_ts;
  lg.off = t->d.l_off;
  lg.val = t->d.l_val;
  OpsDev m;
  m.n = L + o.n;
  m.n_path = LP + o.n_path;
  auto* kind = ws.alloc<uint8_t>(m.n + 1);
  auto* ts = ws.alloc<long long>(m.n + 1);
  auto* off = ws.alloc<uint32_t>(m.n + 1);
  auto* path = ws.alloc<long long>(m.n_path + 1);
  auto* val = ws.alloc<uint32_t>(m.n + 1);
  auto* own = ws.alloc<unsigned long long>(1);
  uint8_t* st2 = st_out ? ws.alloc<uint8_t>(m.n + 1) : nullptr;
  LAUNCH(k_cat_ops, dim3(grid_for(m.n + 1)), dim3(BLOCK), 0, s, lg, o, L, static_cast<uint32_t>(LP), kind, ts, off,
         val);
  if (LP) HIP_CHECK(hipMemcpyAsync(path, t->d.l_path, LP * 8, hipMemcpyDeviceToDevice, s));
  if (o.n_path) HIP_CHECK(hipMemcpyAsync(path + LP, o.path, o.n_path * 8, hipMemcpyDeviceToDevice, s));
  HIP_CHECK(hipMemsetAsync(own, 0, sizeof(*own), s));
  LAUNCH(k_own_log, dim3(grid_for(L, BLOCK, 1024)), dim3(BLOCK), 0, s, kind, ts, L, replica_of(t->timestamp), own);
  unsigned long long own_h = 0;
  HIP_CHECK(hipMemcpyAsync(&own_h, own, sizeof(own_h), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  m.kind = kind;
  m.ts = ts;
  m.off = off;
  m.path = path;
  m.val = val;
  // the host-side state the fresh paths overwrite; restored unless the batch commits
  struct Saved {
    uint64_t n_slots, n_dicts, log_n, log_npath, doc_n, last_begin, last_end;
    bool doc_valid;
    uint32_t max_depth;
    int64_t timestamp;
  } sv{t->n_slots, t->n_dicts, t->log_n, t->log_npath, t->doc_n, t->last_begin, t->last_end,
       t->doc_valid, t->max_depth, t->timestamp};
  auto restore = [&]() {
    t->n_slots = sv.n_slots;
    t->n_dicts = sv.n_dicts;
    t->log_n = sv.log_n;
    t->log_npath = sv.log_npath;
    t->doc_n = sv.doc_n;
    t->last_begin = sv.last_begin;
    t->last_end = sv.last_end;
    t->doc_valid = sv.doc_valid;
    t->max_depth = sv.max_depth;
    t->timestamp = sv.timestamp;
    t->remerge = false;
    t->own_bias = 0;
  };
  t->n_slots = 1;
  t->n_dicts = 1;
  t->log_n = 0;
  t->log_npath = 0;
  t->remerge = true;
  t->own_bias = static_cast<int64_t>(own_h);
  int r;
  try {
    r = apply_core(t, m, st2, res);
  } catch (...) {
    restore();
    throw;
  }
  t->remerge = false;
  t->own_bias = 0;
  if (r == R_INCR || (r == CRDTM_OK && res->code != CRDTM_OK && res->err_index < static_cast<int64_t>(L))) {
    // a sequential path (or, defensively, a log op that did not re-apply):
    // the state is untouched; replay the batch alone on it
    restore();
    ws.used = mark0;
    std::memset(res, 0, sizeof(*res));
    res->err_index = -1;
    return apply_core(t, o, st_out, res);
  }
  if (r != CRDTM_OK) return r;
  res->flags |= CRDTM_FLAG_REMERGE;
  if (res->code != CRDTM_OK) {
    restore();
    res->err_index -= L;
  } else {
    res->n_applied -= L;
    t->last_begin = sv.log_n;
    t->last_end = t->log_n;
    if (t->log_n != sv.log_n + res->n_applied) {
      std::fprintf(stderr, "crdtm: incremental re-merge log mismatch\n");
      return CRDTM_E_HIP;
    }
    if (t->max_depth < sv.max_depth) t->max_depth = sv.max_depth;
  }
  if (st_out) HIP_CHECK(hipMemcpyAsync(st_out, st2 + L, o.n, hipMemcpyDeviceToDevice, s));
  return CRDTM_OK;
}

// Every apply: an adds-only batch into a clean flat document takes the
// incremental closed form (incr.hip); the rest the paths above. The flat-clean
// mark and the key index describe the state, so they follow it: any other
// commit clears them (the flat closed form sets flat_clean again), a failing
// batch leaves both as they were.
int apply_batch(crdtm_tree* t, const OpsDev& o, uint8_t* st_out, crdtm_result* res) {
  const bool fresh = t->n_slots == 1 && t->log_n == 0;
  const bool was_clean = t->flat_clean, was_kidx = t->kidx_valid;
  if (!fresh && o.n) {
    bool handled = false;
    int r = finc_apply(t, o, st_out, res, &handled);
    if (r != CRDTM_OK || handled) {
      t->ilr_valid = false;
      if (r != CRDTM_OK) {
        t->flat_clean = was_clean;
        t->kidx_valid = false;
      }
      return r;
    }
  }
  t->flat_clean = false;
  t->kidx_valid = false;
  const bool was_gapped = t->doc_gapped;  // (after finc_apply: it may have written `doc` back)
  t->doc_gapped = false;  // (the general paths write `doc`, or leave it to linearize)
  const int r = apply_batch_paths(t, o, st_out, res);
  if (r != CRDTM_OK || res->code != CRDTM_OK) {  // the state is unchanged
    t->flat_clean = was_clean;
    t->kidx_valid = was_kidx && r == CRDTM_OK;
    t->doc_gapped = was_gapped && t->kidx_valid;
    if (was_gapped && !t->doc_gapped) t->doc_valid = false;  // (an engine error: linearize from the state)
  }
  return r;
}

// The chain order of every dict of the state, for the level replay's
// findInsertion walks (ilr.hip): every dict's chain (sentinel, then `next`
// by `next`; orphans are on none) laid end to end in dict order — a chain's
// last entry is followed by the next dict's sentinel — and list-ranked.
// R[slot] = its position (NONE: an orphan), G[position] = the slot there.
// Every dict's chain occupies consecutive positions, whether or not its
// owner is visible (ops reach a dict by key, not through the document).
__global__ void __launch_bounds__(BLOCK) k_snap_links(TreeDev T, uint32_t S, uint32_t D, uint2* ent) {
  GRID_STRIDE(s, S) {
    if (T.s_flags[s] & F_ORPHAN) {
      ent[s] = make_uint2(ABSENT, 0u);
      continue;
    }
    uint32_t nx = T.s_next[s];
    if (nx == NONE) {  // the chain's end: the next dict's sentinel
      for (uint32_t d = T.s_dict[s] + 1; d < D; ++d)
        if ((nx = T.d_sent[d]) != NONE) break;
    }
    ent[s] = make_uint2(nx, 1u);
  }
}
__global__ void __launch_bounds__(BLOCK) k_snap_scatter(uint32_t S, const unsigned long long* excl, uint32_t* R,
                                                        uint32_t* G) {
  GRID_STRIDE(s, S) {
    const unsigned long long r = excl[s];
    const bool on = r != ~0ULL && r < S;
    R[s] = on ? static_cast<uint32_t>(r) : NONE;
    if (on) G[r] = s;
  }
}
int chain_snapshot(crdtm_tree* t, uint32_t* R, uint32_t* G, Arena& ws, hipStream_t s) {
  const uint32_t S = static_cast<uint32_t>(t->n_slots), D = static_cast<uint32_t>(t->n_dicts);
  uint2* ent = ws.alloc<uint2>(S);
  unsigned long long* excl = ws.alloc<unsigned long long>(S);
  LAUNCH(k_snap_links, dim3(grid_for(S)), dim3(BLOCK), 0, s, t->d, S, D, ent);
  int r = list_rank(ent, S, 0u /* the root dict's sentinel */, excl, ws, s);
  if (r) return r;
  HIP_CHECK(hipMemsetAsync(G, 0xFF, static_cast<uint64_t>(S) * sizeof(uint32_t), s));
  LAUNCH(k_snap_scatter, dim3(grid_for(S)), dim3(BLOCK), 0, s, S, excl, R, G);
  return CRDTM_OK;
}

int linearize(crdtm_tree* t) {
  crdtm_ctx* c = t->ctx;
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  ws.reset();
  if (t->doc_gapped) {  // current in the incremental merge's gapped order: compact it
    int r = fi_materialize(t);
    if (r) return r;
  }
  if (t->doc_valid) return CRDTM_OK;
  const uint32_t S = static_cast<uint32_t>(t->n_slots), D = static_cast<uint32_t>(t->n_dicts);
  uint8_t* ok = ws.alloc<uint8_t>(D);
  uint8_t* ok2 = ws.alloc<uint8_t>(D);
  uint32_t* up = ws.alloc<uint32_t>(D);
  uint32_t* up2 = ws.alloc<uint32_t>(D);
  LAUNCH(k_dict_alive_init, dim3(grid_for(D)), dim3(BLOCK), 0, s, t->d, D, ok, up);
  // pointer doubling up the owner chain (depth bounded by the longest path)
  uint32_t rounds = 1;
  while ((1u << rounds) < t->max_depth + 2) ++rounds;
  rounds += 1;
  for (uint32_t k = 0; k < rounds; ++k) {
    LAUNCH(k_dict_alive_jump, dim3(grid_for(D)), dim3(BLOCK), 0, s, D, ok, up, ok2, up2);
    std::swap(ok, ok2);
    std::swap(up, up2);
  }
  const uint64_t E = static_cast<uint64_t>(S) + D;
  uint2* ent = ws.alloc<uint2>(E);
  unsigned long long* excl = ws.alloc<unsigned long long>(E);
  LAUNCH(k_lin_entries, dim3(grid_for(E)), dim3(BLOCK), 0, s, t->d, S, D, ok, ent);
  int r = list_rank(ent, E, 0u /* root sentinel slot */, excl, ws, s);
  if (r) return r;
  TreeCaps need = t->cap;
  need.doc = std::max<uint64_t>(need.doc, S + 1);
  if (need.doc > t->cap.doc && ((r = unshare_tree(t, true)) || (r = grow_tree(t, need)))) return r;
  LAUNCH(k_lin_doc, dim3(grid_for(S)), dim3(BLOCK), 0, s, t->d, S, excl, t->d.doc, t->cap.doc);
  // number of visible entries = weight sum up to the end: excl at exit(0)
  unsigned long long tot = 0;
  HIP_CHECK(hipMemcpyAsync(&tot, excl + S, sizeof(tot), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  t->doc_n = (tot == ~0ULL || tot > S) ? 0 : tot;
  t->doc_valid = true;
  return CRDTM_OK;
}

}  // namespace crdtm

namespace crdtm {

// the context's pinned staging buffer, at least `bytes` (grown, contents lost)
static char* host_pinned(crdtm_ctx* c, size_t bytes) {
  if (bytes > c->pin_cap) {
    if (c->pin) hipHostFree(c->pin);
    c->pin = nullptr;
    c->pin_cap = 0;
    const size_t cap = std::max<size_t>(bytes, 1u << 20);
    if (hipHostMalloc(reinterpret_cast<void**>(&c->pin), cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    c->pin_cap = cap;
  }
  return c->pin;
}

int forest_apply(crdtm_ctx* c, int64_t replica_id, const OpsDev& o, const uint32_t* doc_off_host, uint64_t n_docs,
                 int32_t* code, int64_t* err, uint32_t* applied, uint64_t* vhash, uint64_t* vwords,
                 int64_t* tstamp) {
  hipStream_t s = c->stream;
  Arena& ws = c->ws;
  // the per-document tables go up and the results come back through the
  // pinned staging buffer, one copy each way: [doc_off u32 | pad | slot,
  // dict, hash bases u64] up; [code, err, applied, overflow u32 | vhash,
  // vwords, tstamp u64] down
  const uint64_t N1 = n_docs + 1;
  const size_t in_off = (N1 * 4 + 7) & ~size_t{7};
  const size_t in_b = in_off + 3 * N1 * 8;
  const size_t out_off = (4 * n_docs * 4 + 7) & ~size_t{7};
  const size_t out_b = out_off + 3 * n_docs * 8;
  char* pin = host_pinned(c, std::max(in_b, out_b));
  if (!pin) return CRDTM_E_NOMEM;
  memcpy(pin, doc_off_host, N1 * 4);
  uint64_t* sb = reinterpret_cast<uint64_t*>(pin + in_off);
  uint64_t* db = sb + N1;
  uint64_t* hb = db + N1;
  sb[0] = db[0] = hb[0] = 0;
  for (uint64_t d = 0; d < n_docs; ++d) {
    const uint32_t nops = doc_off_host[d + 1] - doc_off_host[d];
    sb[d + 1] = sb[d] + forest_slot_cap(nops);
    db[d + 1] = db[d] + forest_dict_cap(nops);
    hb[d + 1] = hb[d] + forest_hash_cap(nops);
  }
  const uint64_t S = sb[n_docs], D = db[n_docs], Hn = hb[n_docs];
  if (S >= 0xFFFFFFF0ULL || D >= 0xFFFFFFF0ULL) return CRDTM_E_ARG;
  ForestArgs f;
  f.T.s_key = ws.alloc<long long>(S);
  f.T.s_next = ws.alloc<uint32_t>(S);
  f.T.s_src = ws.alloc<uint32_t>(S);
  f.T.s_child = ws.alloc<uint32_t>(S);
  f.T.s_dict = ws.alloc<uint32_t>(S);
  f.T.s_flags = ws.alloc<uint8_t>(S);
  f.T.d_sent = ws.alloc<uint32_t>(D);
  f.T.d_owner = ws.alloc<uint32_t>(D);
  f.dhead = ws.alloc<uint32_t>(D);
  f.mnext = ws.alloc<uint32_t>(S);
  f.hdict = ws.alloc<uint32_t>(Hn);
  f.hkey = ws.alloc<long long>(Hn);
  f.hslot = ws.alloc<uint32_t>(Hn);
  f.queue = ws.alloc<uint32_t>(2 * D);
  char* din = ws.alloc<char>(in_b);
  uint32_t* doff = reinterpret_cast<uint32_t*>(din);
  uint64_t* dsb = reinterpret_cast<uint64_t*>(din + in_off);
  uint64_t* ddb = dsb + N1;
  uint64_t* dhb = ddb + N1;
  char* dout = ws.alloc<char>(out_b);
  f.code = reinterpret_cast<int32_t*>(dout);
  f.err = reinterpret_cast<uint32_t*>(dout) + n_docs;
  f.applied = reinterpret_cast<uint32_t*>(dout) + 2 * n_docs;
  f.overflow = reinterpret_cast<uint32_t*>(dout) + 3 * n_docs;
  f.vhash = reinterpret_cast<unsigned long long*>(dout + out_off);
  f.vwords = f.vhash + n_docs;
  f.tstamp = reinterpret_cast<long long*>(f.vwords + n_docs);
  f.doc_off = doff;
  f.n_docs = static_cast<uint32_t>(n_docs);
  f.ts0 = replica_id * TWO32;
  HIP_CHECK(hipMemcpyAsync(din, pin, in_b, hipMemcpyHostToDevice, s));
  uint8_t* fb = ws.alloc<uint8_t>(n_docs);
  HIP_CHECK(hipMemsetAsync(fb, 0, n_docs, s));
  uint32_t* opw = ws.alloc<uint32_t>(o.n + 1);
  uint16_t* sent = ws.alloc<uint16_t>(n_docs);
  longlong2* vt = ws.alloc<longlong2>(n_docs * FL_SLOTS);
  // the flat documents (forest.hip), then the rest (k_forest)
  if (int rf = forest_flat_launch(o, doff, f.n_docs, f.ts0, opw, sent, fb, vt, f.code, f.err, f.applied, f.vhash,
                                  f.vwords, f.tstamp, f.overflow, s))
    return rf;
  LAUNCH(k_forest, dim3(static_cast<uint32_t>((n_docs + 63) / 64)), dim3(64), 0, s, o, f, dsb, ddb, dhb, fb);
  HIP_CHECK(hipMemcpyAsync(pin, dout, out_b, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  const uint32_t* hc = reinterpret_cast<const uint32_t*>(pin);
  const unsigned long long* h8 = reinterpret_cast<const unsigned long long*>(pin + out_off);
  memcpy(code, hc, n_docs * 4);
  if (applied) memcpy(applied, hc + 2 * n_docs, n_docs * 4);
  if (vhash) memcpy(vhash, h8, n_docs * 8);
  if (vwords) memcpy(vwords, h8 + n_docs, n_docs * 8);
  if (tstamp) memcpy(tstamp, h8 + 2 * n_docs, n_docs * 8);
  int rc = CRDTM_OK;
  for (uint64_t d = 0; d < n_docs; ++d) {
    const uint32_t e = hc[n_docs + d];
    if (err) err[d] = e == NONE ? -1 : static_cast<int64_t>(e);
    if (hc[3 * n_docs + d]) {  // a document outgrew its arena (deep copies): reported, never silently wrong
      code[d] = CRDTM_E_NOMEM;
      rc = CRDTM_E_NOMEM;
    }
  }
  return rc;
}

uint64_t forest_ws_bytes(const uint32_t* doc_off_host, uint64_t n_docs, uint64_t n_ops, uint64_t n_path) {
  uint64_t S = 0, D = 0, H = 0;
  for (uint64_t d = 0; d < n_docs; ++d) {
    const uint32_t nops = doc_off_host[d + 1] - doc_off_host[d];
    S += forest_slot_cap(nops);
    D += forest_dict_cap(nops);
    H += forest_hash_cap(nops);
  }
  return S * 29 + D * 20 + H * 16 + n_docs * (96 + 16 * FL_SLOTS) + n_ops * 32 + n_path * 8 + (64ULL << 20);
}

}  // namespace crdtm

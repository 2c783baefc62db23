// scan.h — single-pass device-wide scans (decoupled look-back) for crdtm.
#pragma once

#include "engine.h"

namespace crdtm {

// ---------------------------------------------------------------------------
// Single-pass scan with decoupled look-back (u32, sum or max). A workgroup
// takes the next tile by ticket (so every predecessor tile has started),
// publishes its aggregate, and wave 0 looks back over up to 64 predecessors
// at a time until it meets an inclusive prefix. Status words pack
// {flag (1 = aggregate, 2 = prefix) : 2, epoch : 30, value : 32} and move
// through agent-scope atomics (coherent across the XCDs' L2s); a word from an
// earlier call carries an older epoch and reads as "not yet published", so
// the status pool is never cleared. The workgroup that draws the last ticket
// resets the ticket counter. Every element is read once and written once.
// Spins are bounded; an exhausted spin sets *err (by default the context's
// DevResult::scan_err, which sync_read turns into CRDTM_E_HIP before any
// result is used). `out` may alias the input (in-place scans): no restrict.
// ---------------------------------------------------------------------------
constexpr int DS_ITEMS = 32;
constexpr int DS_TILE = BLOCK * DS_ITEMS;

__device__ __forceinline__ unsigned long long ds_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ds_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint32_t DS_EPOCH_MASK = (1u << 30) - 1;

// The look-back of tile `tile` with aggregate `agg`, by one whole wave: it
// publishes the aggregate, folds the predecessors' words (64 at a time, from
// the farthest lane down to the nearest, in front of the nearer windows'
// prefix) until it meets an inclusive prefix, publishes its own, and returns
// the exclusive prefix (in every lane).
template <class OP>
__device__ __forceinline__ uint32_t ds_lookback(unsigned long long* status, uint32_t tile, uint32_t agg,
                                                uint32_t epoch, uint32_t* err) {
  const int lane = threadIdx.x & 63;
  const unsigned long long ep = static_cast<unsigned long long>(epoch) << 32;
  uint32_t prefix = OP::id();
  if (tile == 0) {
    if (lane == 0) ds_store(&status[0], (2ULL << 62) | ep | agg);
    return prefix;
  }
  if (lane == 0) ds_store(&status[tile], (1ULL << 62) | ep | agg);
  long long j = static_cast<long long>(tile) - 1;
  uint32_t spins = 0;
  for (;;) {
    const long long idx = j - lane;
    const unsigned long long s = idx >= 0 ? ds_load(&status[idx]) : ((2ULL << 62) | ep | OP::id());
    const uint32_t flag = ((s >> 32) & DS_EPOCH_MASK) == epoch ? static_cast<uint32_t>(s >> 62) : 0u;
    const uint32_t val = static_cast<uint32_t>(s);
    const unsigned long long pm = __ballot(flag == 2), im = __ballot(flag == 0);
    uint32_t upto = 64;  // lanes that contribute
    if (pm) upto = __ffsll(static_cast<long long>(pm));  // lowest prefix lane p -> lanes 0..p
    const unsigned long long need = upto == 64 ? ~0ULL : ((1ULL << upto) - 1);
    if (im & need) {
      if (++spins > (1u << 24)) {  // bounded: never hang the device
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    // lane j holds tile (tile - 1 - j): fold from the farthest lane down
    // to lane 0 (the nearest), then in front of the nearer windows' prefix
    uint32_t c = static_cast<uint32_t>(lane) < upto ? val : OP::id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_down(c, o, 64);
      if (lane + o < 64) c = OP::op(t, c);
    }
    c = __shfl(c, 0, 64);
    prefix = OP::op(c, prefix);
    if (pm) break;
    j -= 64;
  }
  if (lane == 0) ds_store(&status[tile], (2ULL << 62) | ep | OP::op(prefix, agg));
  return prefix;
}

template <class OP, bool INCL, class GEN>
__global__ void __launch_bounds__(BLOCK) k_dscan(GEN gen, uint32_t* out, uint64_t n,
                                                 unsigned long long* __restrict__ status, uint32_t* __restrict__ ticket,
                                                 uint32_t ntiles, uint32_t epoch, uint32_t* __restrict__ total,
                                                 uint32_t* __restrict__ err, const uint32_t* n_dev) {
  __shared__ uint32_t s_tile, s_prefix;
  __shared__ uint32_t sw[BLOCK / 64];
  // full tiles move through LDS so that HBM sees lane-contiguous 16-byte
  // accesses (a lane's DS_ITEMS consecutive items would otherwise make every
  // vector load/store instruction touch one 16-byte piece of 64 lines)
  __shared__ __attribute__((aligned(16))) uint32_t sx[DS_TILE];
  // a device-side item count (<= n): the workgroups past its tiles leave
  // before drawing a ticket (the host launches for n: a launch sized for 10M
  // slots over 1M runs had 1,100 idle workgroups serialising ~12 ns each on
  // the ticket word)
  if (n_dev && *n_dev < n) {
    n = *n_dev;
    ntiles = n ? static_cast<uint32_t>((n - 1) / DS_TILE) + 1u : 1u;
    if (blockIdx.x >= ntiles) return;
  }
  if (threadIdx.x == 0) {
    s_tile = atomicAdd(ticket, 1u);
    if (s_tile == ntiles - 1) atomicExch(ticket, 0u);  // every ticket is drawn: ready for the next scan
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t b = static_cast<uint64_t>(tile) * DS_TILE + static_cast<uint64_t>(threadIdx.x) * DS_ITEMS;
  uint32_t v[DS_ITEMS];
  const uint64_t tb = static_cast<uint64_t>(tile) * DS_TILE;
  const bool full = tb + DS_TILE <= n;
  if (GEN::kStriped && full && gen.aligned(tb)) {
#pragma unroll
    for (int j = 0; j < DS_ITEMS / 4; ++j) {
      const uint32_t x = (j * BLOCK + threadIdx.x) * 4;
      *reinterpret_cast<uint4*>(sx + x) = gen.load4(tb + x);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < DS_ITEMS; j += 4) {
      const uint4 y = *reinterpret_cast<const uint4*>(sx + threadIdx.x * DS_ITEMS + j);
      v[j] = y.x;
      v[j + 1] = y.y;
      v[j + 2] = y.z;
      v[j + 3] = y.w;
    }
  } else {
    gen.load(b, n, v);
  }
  uint32_t acc = OP::id();
#pragma unroll
  for (int j = 0; j < DS_ITEMS; ++j) acc = OP::op(acc, v[j]);
  // workgroup exclusive scan of the per-thread totals (every combination in
  // item order, earlier operand first: OP need not commute — the segmented
  // sum of the flat order's run sizes does not)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = acc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc = OP::op(t, inc);
  }
  if (lane == 63) sw[wave] = inc;
  __syncthreads();
  uint32_t texcl = __shfl_up(inc, 1, 64);
  if (lane == 0) texcl = OP::id();
  uint32_t agg = OP::id(), wpre = OP::id();
  for (int w = 0; w < BLOCK / 64; ++w) {
    if (w < wave) wpre = OP::op(wpre, sw[w]);
    agg = OP::op(agg, sw[w]);
  }
  texcl = OP::op(wpre, texcl);
  if (wave == 0) {
    const uint32_t prefix = ds_lookback<OP>(status, tile, agg, epoch, err);
    if (lane == 0) {
      s_prefix = prefix;
      if (total && tile == ntiles - 1) *total = OP::op(prefix, agg);
    }
  }
  __syncthreads();
  uint32_t run = OP::op(s_prefix, texcl);
  const uint32_t start = run;
#pragma unroll
  for (int j = 0; j < DS_ITEMS; ++j) {
    const uint32_t x = v[j];
    if (INCL) {
      run = OP::op(run, x);
      v[j] = run;
    } else {
      v[j] = run;
      run = OP::op(run, x);
    }
  }
  // a generator may consume the scanned values of its own items (items b ..
  // b + DS_ITEMS, `start` = the prefix before them) before they are stored
  if constexpr (GEN::kEpilogue) gen.epilogue(b, n, v, start);
  if (full && (reinterpret_cast<uintptr_t>(out + tb) & 15) == 0) {
    // (every lane finished reading sx: the look-back's __syncthreads lie between)
#pragma unroll
    for (int j = 0; j < DS_ITEMS; j += 4)
      *reinterpret_cast<uint4*>(sx + threadIdx.x * DS_ITEMS + j) = make_uint4(v[j], v[j + 1], v[j + 2], v[j + 3]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < DS_ITEMS / 4; ++j) {
      const uint32_t x = (j * BLOCK + threadIdx.x) * 4;
      *reinterpret_cast<uint4*>(out + tb + x) = *reinterpret_cast<const uint4*>(sx + x);
    }
  } else if (b + DS_ITEMS <= n) {
#pragma unroll
    for (int j = 0; j < DS_ITEMS; j += 4)
      *reinterpret_cast<uint4*>(out + b + j) = make_uint4(v[j], v[j + 1], v[j + 2], v[j + 3]);
  } else {
    for (int j = 0; j < DS_ITEMS; ++j)
      if (b + j < n) out[b + j] = v[j];
  }
}

struct SumOp {
  static __device__ __forceinline__ uint32_t id() { return 0u; }
  static __device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b) { return a + b; }
};

struct ArrGen {
  static constexpr bool kStriped = true;  // k_dscan may load full tiles lane-contiguously
  static constexpr bool kEpilogue = false;
  const uint32_t* in;
  __device__ __forceinline__ bool aligned(uint64_t b) const { return (reinterpret_cast<uintptr_t>(in + b) & 15) == 0; }
  __device__ __forceinline__ uint4 load4(uint64_t b) const { return *reinterpret_cast<const uint4*>(in + b); }
  __device__ __forceinline__ void load(uint64_t b, uint64_t n, uint32_t* v) const {
    if (b + DS_ITEMS <= n && (reinterpret_cast<uintptr_t>(in + b) & 15) == 0) {
#pragma unroll
      for (int j = 0; j < DS_ITEMS; j += 4) {
        const uint4 x = *reinterpret_cast<const uint4*>(in + b + j);
        v[j] = x.x;
        v[j + 1] = x.y;
        v[j + 2] = x.z;
        v[j + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < DS_ITEMS; ++j) v[j] = b + j < n ? in[b + j] : 0u;
    }
  }
};

// n_dev (optional): the item count on the device, at most n (the grid covers n).
template <class OP, bool INCL, class GEN>
int dscan(GEN gen, uint32_t* out, uint64_t n, uint32_t* total, Arena& ws, hipStream_t st, uint32_t* err,
          const uint32_t* n_dev = nullptr, const char* label = "k_dscan") {
  if (n == 0) {
    if (total) HIP_CHECK(hipMemsetAsync(total, 0, sizeof(uint32_t), st));
    return CRDTM_OK;
  }
  const uint64_t tiles = (n + DS_TILE - 1) / DS_TILE;
  ws.scan_epoch = (ws.scan_epoch % DS_EPOCH_MASK) + 1;  // 1..2^30-1; zeroed memory never matches
  unsigned long long* status = ws.scan_status;
  uint32_t* ticket = ws.scan_ticket;
  if (!status || tiles > ws.scan_cap) {  // beyond the pool: a zeroed status array of its own
    status = ws.alloc<unsigned long long>(tiles + 1);
    ticket = reinterpret_cast<uint32_t*>(status + tiles);
    HIP_CHECK(hipMemsetAsync(status, 0, (tiles + 1) * sizeof(unsigned long long), st));
  }
  if (!err) err = ws.scan_err;
  auto* kfn = &k_dscan<OP, INCL, GEN>;
  prof_begin(st);
  hipLaunchKernelGGL(kfn, dim3(static_cast<uint32_t>(tiles)), dim3(BLOCK), 0, st, gen, out, n, status, ticket,
                     static_cast<uint32_t>(tiles), ws.scan_epoch, total, err, n_dev);
  prof_mark(label, st);
  return CRDTM_OK;
}

struct MaxOp {
  static __device__ __forceinline__ uint32_t id() { return 0u; }
  static __device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b) { return a > b ? a : b; }
};

}  // namespace crdtm

// claim_bench.hip — what bounds the flat claim (merge.hip k_fl_claim)?
// Standalone variants over a synthetic config-3-shaped batch (10M Adds, 64
// replicas interleaved, counters rising per replica): the op log copy alone,
// the slot-record scatter alone, both (the claim's shape), and both with the
// records staged through LDS by replica before the stores.
//
//   hipcc -O3 --offload-arch=gfx950 tools/claim_bench.hip -o build/claim_bench && build/claim_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__);            \
      return 1;                                                              \
    }                                                                        \
  } while (0)

constexpr uint32_t B = 256;
constexpr uint32_t NR = 64;

struct Args {
  const long long* ts;
  const long long* path;
  const uint32_t* val;
  uint32_t n;
  const uint32_t* base;  // per replica
  const uint32_t* cmin;
  uint8_t* l_kind;
  long long* l_ts;
  uint32_t* l_off;
  uint32_t* l_val;
  long long* l_path;
  uint2* rec;
};

__device__ __forceinline__ void nt16(void* p, uint4 v) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
}
__device__ __forceinline__ void nt16(void* p, longlong2 v) {
  nt16(p, make_uint4((uint32_t)v.x, (uint32_t)((unsigned long long)v.x >> 32), (uint32_t)v.y,
                     (uint32_t)((unsigned long long)v.y >> 32)));
}

// MODE bit 0: write the log; bit 1: scatter the records; bit 2: stage them in LDS
template <int MODE>
__global__ void __launch_bounds__(B) k_claim(Args a) {
  __shared__ uint32_t sb[NR], sc[NR];
  __shared__ uint32_t cnt[NR], off[NR];
  __shared__ uint2 st[B * 4];
  __shared__ uint32_t sq[B * 4];
  for (uint32_t j = threadIdx.x; j < NR; j += B) {
    sb[j] = a.base[j];
    sc[j] = a.cmin[j];
  }
  __syncthreads();
  const uint32_t nq = (a.n + 3) / 4;
  const uint32_t xc = blockIdx.x & 7, xy = blockIdx.x >> 3, cq = (gridDim.x >> 3) * B;
  for (uint32_t j = xc;; j += 8) {  // XCD chunks, as QUAD_LOOP_XCD
    const uint32_t qd = j * cq + xy * B + threadIdx.x;
    if (j * cq >= nq) break;
    const bool act = qd < nq;
    const uint32_t i0 = 4 * qd;
    longlong2 t0{}, t1{}, p0{}, p1{};
    uint4 v{};
    if (act) {
      t0 = *reinterpret_cast<const longlong2*>(a.ts + i0);
      t1 = *reinterpret_cast<const longlong2*>(a.ts + i0 + 2);
      p0 = *reinterpret_cast<const longlong2*>(a.path + i0);
      p1 = *reinterpret_cast<const longlong2*>(a.path + i0 + 2);
      v = *reinterpret_cast<const uint4*>(a.val + i0);
    }
    if ((MODE & 1) && act) {
      *reinterpret_cast<uint32_t*>(a.l_kind + i0) = 0u;
      nt16(a.l_ts + i0, t0);
      nt16(a.l_ts + i0 + 2, t1);
      nt16(a.l_off + i0, make_uint4(i0, i0 + 1, i0 + 2, i0 + 3));
      nt16(a.l_val + i0, v);
      nt16(a.l_path + i0, p0);
      nt16(a.l_path + i0 + 2, p1);
    }
    if (MODE & 2) {
      const long long tt[4] = {t0.x, t0.y, t1.x, t1.y}, pp[4] = {p0.x, p0.y, p1.x, p1.y};
      uint32_t q[4];
      uint2 rv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t r = (uint32_t)((unsigned long long)tt[k] >> 32) % NR;
        q[k] = sb[r] + ((uint32_t)tt[k] - sc[r]);
        const uint32_t ra = (uint32_t)((unsigned long long)pp[k] >> 32) % NR;
        const uint32_t qa = pp[k] ? sb[ra] + ((uint32_t)pp[k] - sc[ra]) : 0xFFFFFFFFu;
        rv[k] = make_uint2(qa, i0 + k);
      }
      if (!(MODE & 4)) {
        if (act)
#pragma unroll
          for (int k = 0; k < 4; ++k) a.rec[q[k]] = rv[k];
      } else {
        // counting sort of the block's 1024 records by replica in LDS, then
        // lane-contiguous stores (consecutive lanes: the same replica's slots)
        for (uint32_t r = threadIdx.x; r < NR; r += B) cnt[r] = 0;
        __syncthreads();
        uint32_t pos[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          pos[k] = act ? atomicAdd(&cnt[(uint32_t)((unsigned long long)tt[k] >> 32) % NR], 1u) : 0u;
        __syncthreads();
        if (threadIdx.x < 64) {
          uint32_t c = threadIdx.x < NR ? cnt[threadIdx.x] : 0u, inc = c;
          for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(inc, o, 64);
            if ((int)threadIdx.x >= o) inc += t;
          }
          if (threadIdx.x < NR) off[threadIdx.x] = inc - c;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (act) {
            const uint32_t s = off[(uint32_t)((unsigned long long)tt[k] >> 32) % NR] + pos[k];
            st[s] = rv[k];
            sq[s] = q[k];
          }
        __syncthreads();
        const uint32_t tot = off[NR - 1] + cnt[NR - 1];
        for (uint32_t s = threadIdx.x; s < tot; s += B) a.rec[sq[s]] = st[s];
        __syncthreads();
      }
    }
  }
}

int main() {
  const uint32_t n = 10000000;
  std::vector<long long> ts(n), path(n);
  std::vector<uint32_t> val(n), cnt(NR, 0), base(NR), cmin(NR, 1);
  uint32_t x = 0xC0FFEE03u;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
  std::vector<long long> last(NR, 0);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = rnd() % NR;
    const uint32_t c = ++cnt[r];
    ts[i] = ((long long)r << 32) | c;
    if (last[r] && rnd() % 10) path[i] = last[r];
    else path[i] = i ? ts[rnd() % i] : 0;
    last[r] = ts[i];
    val[i] = i;
  }
  uint32_t acc = 0;
  for (uint32_t r = 0; r < NR; ++r) {
    base[r] = acc;
    acc += cnt[r];
  }
  Args a{};
  a.n = n;
  long long *dts, *dpath, *lts, *lpath;
  uint32_t *dval, *db, *dc, *loff, *lval;
  uint8_t* lkind;
  uint2* rec;
  CK(hipMalloc(&dts, n * 8ULL));
  CK(hipMalloc(&dpath, n * 8ULL));
  CK(hipMalloc(&dval, n * 4ULL));
  CK(hipMalloc(&db, NR * 4));
  CK(hipMalloc(&dc, NR * 4));
  CK(hipMalloc(&lts, n * 8ULL));
  CK(hipMalloc(&lpath, n * 8ULL));
  CK(hipMalloc(&loff, n * 4ULL + 16));
  CK(hipMalloc(&lval, n * 4ULL));
  CK(hipMalloc(&lkind, n + 64ULL));
  CK(hipMalloc(&rec, n * 8ULL));
  CK(hipMemcpy(dts, ts.data(), n * 8ULL, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpath, path.data(), n * 8ULL, hipMemcpyHostToDevice));
  CK(hipMemcpy(dval, val.data(), n * 4ULL, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, base.data(), NR * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, cmin.data(), NR * 4, hipMemcpyHostToDevice));
  a.ts = dts; a.path = dpath; a.val = dval; a.base = db; a.cmin = dc;
  a.l_kind = lkind; a.l_ts = lts; a.l_off = loff; a.l_val = lval; a.l_path = lpath; a.rec = rec;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](auto kern, const char* name, double mb) {
    for (uint32_t grid : {1024u, 2048u, 4096u}) {
      for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(B), 0, 0, a);
      hipEventRecord(e0);
      const int reps = 10;
      for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(B), 0, 0, a);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / reps;
      printf("%-28s grid %5u %8.1f us  %6.2f TB/s (%.0f MB)\n", name, grid, us, mb / us, mb);
    }
  };
  run(k_claim<1>, "log only", 200 + 250);
  run(k_claim<2>, "records only (scatter)", 160 + 80);
  run(k_claim<3>, "log + records (claim)", 200 + 250 + 80);
  run(k_claim<7>, "log + records staged", 200 + 250 + 80);
  run(k_claim<6>, "records staged only", 160 + 80);
  return 0;
}

// mask_bench.hip — what bounds the flat slot-order pass (merge.hip
// k_run_mask)? Standalone variants over 10M slots: read the 8-byte slot
// records, write the five node-record columns (key 8 B, source, dict,
// children 4 B, flags 1 B), with streaming or plain stores, with or without
// the per-word head masks and the byte column, one or more words per wave.
//
//   hipcc -O3 --offload-arch=gfx950 tools/mask_bench.hip -o abtest/mask_bench && abtest/mask_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint32_t B = 256;

struct Args {
  const uint2* rec;
  uint32_t Q;
  long long* s_key;
  uint32_t* s_src;
  uint32_t* s_dict;
  uint8_t* s_flags;
  uint32_t* s_child;
  unsigned long long* hm;
  uint32_t* hc;
};

template <class T>
__device__ __forceinline__ void st(T* p, T v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// F bit 0: streaming stores; bit 1: no flags column; bit 2: head masks;
// bit 3: the masks written by one vector store per iteration
template <uint32_t U, int F>
__global__ void __launch_bounds__(B) k_mask(Args a) {
  const bool nt = F & 1;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = (a.Q + 63) >> 6;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwave = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t w0 = wave * U; w0 < nw; w0 += nwave * U) {
    uint2 rq[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t q = ((w0 + u) << 6) + lane;
      rq[u] = q < a.Q ? a.rec[q] : make_uint2(0u, 0u);
    }
    unsigned long long mm[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t q = ((w0 + u) << 6) + lane;
      const uint32_t px = __shfl_up(rq[u].x, 1, 64);
      mm[u] = __ballot(q < a.Q && rq[u].x != px + 1);
      if (q >= a.Q) continue;
      const uint32_t slot = 1 + q;
      st(a.s_key + slot, (long long)rq[u].x << 8, nt);
      st(a.s_dict + slot, 0u, nt);
      st(a.s_src + slot, rq[u].y, nt);
      if (!(F & 2)) st(a.s_flags + slot, (uint8_t)0, nt);
      st(a.s_child + slot, 0xFFFFFFFFu, nt);
    }
    if (F & 4) {
      if (F & 8) {
        unsigned long long m = 0;
#pragma unroll
        for (uint32_t u = 0; u < U; ++u)
          if (lane == u) m = mm[u];
        if (lane < U && w0 + lane < nw) {
          a.hm[w0 + lane] = m;
          a.hc[w0 + lane] = (uint32_t)__popcll(m);
        }
      } else if (lane == 0) {
#pragma unroll
        for (uint32_t u = 0; u < U; ++u)
          if (w0 + u < nw) {
            a.hm[w0 + u] = mm[u];
            a.hc[w0 + u] = (uint32_t)__popcll(mm[u]);
          }
      }
    }
  }
}

int main() {
  const uint32_t Q = 10000000;
  Args a{};
  a.Q = Q;
  uint2* rec;
  hipMalloc(&rec, Q * 8ULL);
  hipMemset(rec, 1, Q * 8ULL);
  a.rec = rec;
  hipMalloc(&a.s_key, (Q + 2) * 8ULL);
  hipMalloc(&a.s_src, (Q + 2) * 4ULL);
  hipMalloc(&a.s_dict, (Q + 2) * 4ULL);
  hipMalloc(&a.s_flags, (Q + 2) * 1ULL);
  hipMalloc(&a.s_child, (Q + 2) * 4ULL);
  hipMalloc(&a.hm, (Q / 64 + 2) * 8ULL);
  hipMalloc(&a.hc, (Q / 64 + 2) * 4ULL);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name) {
    for (uint32_t grid : {1024u, 2048u}) {
      for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(B), 0, 0, a);
      hipEventRecord(e0);
      const int reps = 10;
      for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(B), 0, 0, a);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / reps;
      printf("%-40s grid %5u %8.1f us  %6.2f TB/s of 290 MB\n", name, grid, us, 290.0 / us);
    }
  };
  run(k_mask<2, 1 | 4>, "U2 nt masks (run_mask's shape)");
  run(k_mask<2, 0 | 4>, "U2 plain masks");
  run(k_mask<2, 1>, "U2 nt no masks");
  run(k_mask<2, 1 | 2 | 4>, "U2 nt masks, no flags column");
  run(k_mask<2, 1 | 4 | 8>, "U2 nt masks by one vector store");
  run(k_mask<4, 1 | 4 | 8>, "U4 nt masks by one vector store");
  run(k_mask<1, 1 | 4>, "U1 nt masks");
  return 0;
}

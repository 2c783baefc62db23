// pre_bench.hip — what bounds the flat pre-pass (merge.hip k_pre_ts)? Its
// main loop over a config-3-shaped batch (10M Adds, 64 replicas, counters
// rising per replica) with the per-replica min/max fold in LDS on or off,
// the kind/offset check on or off, and a contiguous chunk per workgroup
// whose last iteration is folded first (a rising counter then rarely moves
// the table: fewer LDS atomics).
//
//   hipcc -O3 --offload-arch=gfx950 tools/pre_bench.hip -o abtest/pre_bench && abtest/pre_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

constexpr uint32_t PB = 1024;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr long long TWO53 = 1LL << 53;

// F bit 0: fold; bit 1: verify; bit 2: chunked, last iteration first
template <int F>
__global__ void __launch_bounds__(PB) k_pre(const long long* __restrict__ ts, const uint8_t* __restrict__ kind,
                                            const uint32_t* __restrict__ off, uint32_t n, uint2* rng,
                                            uint32_t* sink) {
  __shared__ uint32_t rlo[256], rhi[256];
  for (uint32_t j = threadIdx.x; j < 256; j += PB) {
    rlo[j] = NONE;
    rhi[j] = 0;
  }
  __syncthreads();
  uint32_t bad = 0, neg = 0, maxr = 0, vfail = 0;
  auto fold = [&](long long t) {
    if (t >= TWO53 || t <= -TWO53) bad = 1;
    else if (t < 0) neg = 1;
    else if (t != 0) {
      const uint32_t r = (uint32_t)((unsigned long long)t >> 32), c = (uint32_t)t;
      maxr = max(maxr, r);
      if ((F & 1) && r < 256) {
        if (c < rlo[r]) atomicMin(&rlo[r], c);
        if (c > rhi[r]) atomicMax(&rhi[r], c);
      }
    }
  };
  const longlong2* t2 = reinterpret_cast<const longlong2*>(ts);
  const uchar2* k2 = reinterpret_cast<const uchar2*>(kind);
  const uint2* o2 = reinterpret_cast<const uint2*>(off);
  auto verify = [&](uint32_t p, uchar2 k, uint2 f) { vfail |= (k.x | k.y) != 0 || f.x != 2 * p || f.y != 2 * p + 1; };
  const uint32_t np = n / 2;
  auto body4 = [&](uint32_t p, uint32_t stride) {  // four pairs, every load first
    longlong2 v[4];
    uchar2 k[4];
    uint2 f[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t pp = min(p + u * stride, np - 1);
      v[u] = t2[pp];
      if (F & 2) {
        k[u] = k2[pp];
        f[u] = o2[pp];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      if (p + u * stride >= np) continue;
      fold(v[u].x);
      fold(v[u].y);
      if (F & 2) verify(p + u * stride, k[u], f[u]);
    }
  };
  if (!(F & 4)) {
    const uint32_t gs = gridDim.x * PB;
    for (uint32_t p = blockIdx.x * PB + threadIdx.x; p < np; p += 4 * gs) body4(p, gs);
  } else {
    // the workgroup's contiguous chunk of pairs, in iterations of 4 x PB
    const uint32_t chunk = ((np + gridDim.x - 1) / gridDim.x + 4 * PB - 1) / (4 * PB) * (4 * PB);
    const uint32_t p0 = blockIdx.x * chunk, p1 = min(np, p0 + chunk);
    if (p0 < p1) {
      const uint32_t last = p0 + ((p1 - p0 - 1) / (4 * PB)) * (4 * PB);
      body4(last + threadIdx.x, PB);  // the largest counters first: the maxima settle at once
      for (uint32_t p = p0; p < last; p += 4 * PB) body4(p + threadIdx.x, PB);
    }
  }
  __syncthreads();
  if (threadIdx.x < 256 && rlo[threadIdx.x] != NONE) {
    atomicMin(&rng[threadIdx.x].x, rlo[threadIdx.x]);
    atomicMax(&rng[threadIdx.x].y, rhi[threadIdx.x]);
  }
  if ((bad | neg | vfail) && maxr == 12345) atomicAdd(sink, 1u);
}

int main() {
  const uint32_t n = 10000000;
  std::vector<long long> ts(n);
  std::vector<uint32_t> off(n + 1), cnt(64, 0);
  uint32_t x = 0xC0FFEE03u;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = 1 + rnd() % 64;
    ts[i] = ((long long)r << 32) | ++cnt[r - 1];
    off[i] = i;
  }
  off[n] = n;
  long long* dts;
  uint8_t* dk;
  uint32_t *doff, *sink;
  uint2* rng;
  hipMalloc(&dts, n * 8ULL);
  hipMalloc(&dk, n);
  hipMalloc(&doff, (n + 1) * 4ULL);
  hipMalloc(&rng, 256 * 8);
  hipMalloc(&sink, 4);
  hipMemcpy(dts, ts.data(), n * 8ULL, hipMemcpyHostToDevice);
  hipMemset(dk, 0, n);
  hipMemcpy(doff, off.data(), (n + 1) * 4ULL, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name, double mb) {
    for (uint32_t grid : {128u, 256u, 512u}) {
      for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(PB), 0, 0, dts, dk, doff, n, rng, sink);
      hipEventRecord(e0);
      const int reps = 10;
      for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(PB), 0, 0, dts, dk, doff, n, rng, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / reps;
      printf("%-34s grid %4u %7.1f us  %5.2f TB/s (%.0f MB)\n", name, grid, us, mb / us, mb);
    }
  };
  run(k_pre<3>, "fold + verify (k_pre_ts)", 130);
  run(k_pre<2>, "verify, no fold", 130);
  run(k_pre<1>, "fold, no verify", 80);
  run(k_pre<0>, "loads only", 80);
  run(k_pre<7>, "fold + verify, chunked, last first", 130);
  run(k_pre<5>, "fold, chunked, last first", 80);
  return 0;
}

// pmc_calibrate.hip — known-byte-count kernels for calibrating rocprofv3's
// FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns the crdtm
// kernels use (MI355X_MICROARCH.md, HBM: "calibrate on a known byte count in
// your own access pattern before trusting an absolute").
//
//   hipcc -O3 --offload-arch=gfx950 tools/pmc_calibrate.hip -o build/pmc_calibrate
//   rocprofv3 --pmc FETCH_SIZE -d <dir> -o run --output-format csv -- build/pmc_calibrate
//
// Every kernel touches a 1 GiB region once (4x the Infinity Cache), so the
// memory-side counters see every byte; the expected bytes are printed.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint64_t BYTES = 1ULL << 30;

template <class T>
__global__ void rd(const T* __restrict__ p, uint64_t n, unsigned* sink) {
  T acc{};
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (*reinterpret_cast<const unsigned*>(&acc) == 0x12345678u) atomicAdd(sink, 1u);
}

__global__ void rd16(const uint4* __restrict__ p, uint64_t n, unsigned* sink) {
  uint4 acc{};
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) atomicAdd(sink, 1u);
}

template <class T>
__global__ void wr(T* __restrict__ p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = static_cast<T>(i);
}

__global__ void wr16(uint4* __restrict__ p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

// one 4-byte (or 8-byte) gather per 128-byte line, lines in a random order:
// the gather pattern of pointer-chasing kernels (every line fetched once)
// (lines is a power of two: multiplying by an odd constant permutes [0, lines))
__device__ __forceinline__ uint64_t perm(uint64_t i, uint64_t m) { return (i * 0x9E3779B1ULL) & (m - 1); }
__global__ void gather4(const unsigned* __restrict__ p, uint64_t lines, unsigned* sink) {
  unsigned acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= p[perm(i, lines) * 32];
  if (acc == 0x12345678u) atomicAdd(sink, 1u);
}
__global__ void scatter4(unsigned* __restrict__ p, uint64_t lines) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x)
    p[perm(i, lines) * 32] = (unsigned)i;
}

int main() {
  void* buf = nullptr;
  unsigned* sink = nullptr;
  if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, BYTES);
  (void)hipDeviceSynchronize();
  const dim3 g(4096), b(256);
  const uint64_t lines = BYTES / 128;
  hipLaunchKernelGGL(rd<uint8_t>, g, b, 0, 0, (const uint8_t*)buf, BYTES, sink);
  hipLaunchKernelGGL(rd<unsigned>, g, b, 0, 0, (const unsigned*)buf, BYTES / 4, sink);
  hipLaunchKernelGGL(rd<unsigned long long>, g, b, 0, 0, (const unsigned long long*)buf, BYTES / 8, sink);
  hipLaunchKernelGGL(rd16, g, b, 0, 0, (const uint4*)buf, BYTES / 16, sink);
  hipLaunchKernelGGL(wr<uint8_t>, g, b, 0, 0, (uint8_t*)buf, BYTES);
  hipLaunchKernelGGL(wr<unsigned>, g, b, 0, 0, (unsigned*)buf, BYTES / 4);
  hipLaunchKernelGGL(wr<unsigned long long>, g, b, 0, 0, (unsigned long long*)buf, BYTES / 8);
  hipLaunchKernelGGL(wr16, g, b, 0, 0, (uint4*)buf, BYTES / 16);
  hipLaunchKernelGGL(gather4, g, b, 0, 0, (const unsigned*)buf, lines, sink);
  hipLaunchKernelGGL(scatter4, g, b, 0, 0, (unsigned*)buf, lines);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("streams: %llu bytes each (rd<u8>, rd<u32>, rd<u64>, rd16, wr<u8>, wr<u32>, wr<u64>, wr16)\n",
              (unsigned long long)BYTES);
  std::printf("gather4/scatter4: %llu lines touched (one 4-byte access per 128-byte line)\n",
              (unsigned long long)lines);
  (void)hipFree(buf);
  (void)hipFree(sink);
  return 0;
}

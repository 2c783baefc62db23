// Host cost of one kernel launch on this runtime, by launch API: the
// hipLaunchKernelGGL path, hipModuleLaunchKernel on a function handle taken
// once (hipGetFuncBySymbol), and hipExtLaunchKernel. A null kernel with a
// 64-byte argument block, 2000 launches per method, stream synchronised
// around each run.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

struct Args64 {
  unsigned long long w[8];
};
struct Args512 {
  unsigned long long w[64];
};
__global__ void k_null(Args64 a, int* out) {
  if (a.w[0] == 12345 && threadIdx.x == 0) *out = 1;
}
__global__ void k_null512(Args512 a, int* out) {
  if (a.w[0] == 12345 && threadIdx.x == 0) *out = 1;
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int* out;
  hipMalloc(&out, 4);
  Args64 a{};
  const int N = 2000;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 100; ++i) launch();
    hipStreamSynchronize(s);
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < N; ++i) launch();
    auto t1 = std::chrono::high_resolution_clock::now();
    hipStreamSynchronize(s);
    auto t2 = std::chrono::high_resolution_clock::now();
    printf("%-22s host %.2f us/launch, to completion %.2f us/launch\n", name,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
  };
  run("hipLaunchKernelGGL", [&] { hipLaunchKernelGGL(k_null, dim3(64), dim3(256), 0, s, a, out); });
  hipFunction_t f = nullptr;
  if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&k_null)) != hipSuccess) printf("no hipGetFuncBySymbol\n");
  void* params[] = {&a, &out};
  if (f) run("hipModuleLaunchKernel", [&] { hipModuleLaunchKernel(f, 64, 1, 1, 256, 1, 1, 0, s, params, nullptr); });
  run("hipLaunchKernel", [&] {
    hipLaunchKernel(reinterpret_cast<const void*>(&k_null), dim3(64), dim3(256), params, 0, s);
  });
  run("hipExtLaunchKernel", [&] {
    hipExtLaunchKernel(reinterpret_cast<const void*>(&k_null), dim3(64), dim3(256), params, 0, s, nullptr, nullptr, 0);
  });
  Args512 b{};
  run("GGL 512-byte args", [&] { hipLaunchKernelGGL(k_null512, dim3(64), dim3(256), 0, s, b, out); });
  hipStream_t sp;
  hipStreamCreateWithPriority(&sp, hipStreamDefault, 0);
  std::swap(s, sp);
  run("GGL default-flag stream", [&] { hipLaunchKernelGGL(k_null, dim3(64), dim3(256), 0, s, a, out); });
  run("GGL 512 default stream", [&] { hipLaunchKernelGGL(k_null512, dim3(64), dim3(256), 0, s, b, out); });
  run("GGL 4096 blocks", [&] { hipLaunchKernelGGL(k_null, dim3(4096), dim3(256), 0, s, a, out); });
  run("GGL 16k shm", [&] { hipLaunchKernelGGL(k_null, dim3(64), dim3(256), 16384, s, a, out); });
  return 0;
}

// ldsbench.hip — LDS random-lookup throughput vs independent chains per lane
// (diagnostic tool, not part of the engine): a 128 KiB table of u16 "next
// row" entries walked like k_scan_fast's automaton (e = T[e + col]), with C
// independent chains per lane, 16 waves per CU.  Reports G lookups/s.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ldsbench tools/ldsbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(1);                                                \
    }                                                         \
  } while (0)

constexpr int kRows = 1000, kRowU16 = 65;

template <int C>
__global__ __launch_bounds__(1024) void k_chain(uint32_t* out, int iters, uint32_t seed) {
  __shared__ uint16_t T[kRows * kRowU16];
  for (int i = threadIdx.x; i < kRows * kRowU16; i += 1024) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    T[i] = (uint16_t)((h % kRows) * kRowU16);
  }
  __syncthreads();
  uint32_t e[C], m = 0, x = threadIdx.x * 0x9E3779B9u + blockIdx.x;
#pragma unroll
  for (int c = 0; c < C; ++c) e[c] = ((threadIdx.x * 7 + c * 131) % kRows) * kRowU16;
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const uint32_t col = (x >> (c * 6 + 2)) & 63;
      e[c] = T[e[c] + col];
      m = m > e[c] ? m : e[c];
    }
  }
  out[blockIdx.x * 1024 + threadIdx.x] = m;
}

int main() {
  uint32_t* o;
  CK(hipMalloc(&o, 1 << 22));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, int chains, auto launch) {
    launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 4; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    const double lookups = (double)cus * 1024 * 4096 * chains;
    printf("%-10s %8.3f ms  %8.1f G lookups/s\n", name, best, lookups / (best * 1e-3) / 1e9);
  };
  run("chains1", 1, [&] { hipLaunchKernelGGL(k_chain<1>, dim3(cus), dim3(1024), 0, 0, o, 4096, 1u); });
  run("chains2", 2, [&] { hipLaunchKernelGGL(k_chain<2>, dim3(cus), dim3(1024), 0, 0, o, 4096, 1u); });
  run("chains4", 4, [&] { hipLaunchKernelGGL(k_chain<4>, dim3(cus), dim3(1024), 0, 0, o, 4096, 1u); });
  return 0;
}

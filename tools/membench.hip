// membench.hip — access-pattern microbenchmarks for the k_scan_fast design
// (diagnostic tool, not part of the engine).  Reads N bytes with different
// per-lane layouts and reports GB/s:
//   coalesced : each wave instruction reads 1 KiB contiguous (lane i: +16 i)
//   span4k    : each lane streams its own 4 KiB span, 16 B per load (the scan's layout)
//   span4k_x  : span4k with span index swizzled across lanes/waves
//   slot128   : each lane owns 128 contiguous bytes of an 8 KiB wave region
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/membench tools/membench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__device__ inline uint32_t mix(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

__global__ __launch_bounds__(1024) void k_coalesced(const uint8_t* d, uint64_t n, uint32_t* out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = t * 16; i + 16 <= n; i += nt * 16) acc ^= mix(*(const uint4*)(d + i));
  if (acc == 0x12345678) out[0] = acc;
}

template <int SWZ>
__global__ __launch_bounds__(1024) void k_span(const uint8_t* d, uint64_t n, uint32_t* out) {
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t spans = n / 4096;
  uint64_t gl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (SWZ) gl = (gl * 2654435761ull) % lanes;  // scatter lanes over spans
  uint32_t acc = 0;
  for (uint64_t s = gl; s < spans; s += lanes) {
    const uint8_t* p = d + s * 4096;
    uint4 cur[8], nxt[8];
    for (int k = 0; k < 8; ++k) nxt[k] = *(const uint4*)(p + 16 * k);
    for (int step = 0; step < 32; ++step) {
      for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
      if (step + 1 < 32)
        for (int k = 0; k < 8; ++k) nxt[k] = *(const uint4*)(p + 128 * (step + 1) + 16 * k);
      for (int k = 0; k < 8; ++k) acc ^= mix(cur[k]);
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}

// each lane streams its own 4 KiB span in STEP-byte steps (prefetch one step ahead)
template <int STEP, int NT>
__global__ __launch_bounds__(NT) void k_span_step(const uint8_t* d, uint64_t n, uint32_t* out) {
  constexpr int V = STEP / 16;
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t spans = n / 4096;
  const uint64_t gl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (uint64_t s = gl; s < spans; s += lanes) {
    const uint8_t* p = d + s * 4096;
    uint4 cur[V], nxt[V];
    for (int k = 0; k < V; ++k) nxt[k] = *(const uint4*)(p + 16 * k);
    for (int step = 0; step < 4096 / STEP; ++step) {
      for (int k = 0; k < V; ++k) cur[k] = nxt[k];
      if (step + 1 < 4096 / STEP)
        for (int k = 0; k < V; ++k) nxt[k] = *(const uint4*)(p + STEP * (step + 1) + 16 * k);
      for (int k = 0; k < V; ++k) acc ^= mix(cur[k]);
      for (int q = 0; q < STEP / 2; ++q) acc = acc * 1664525u + 1013904223u;  // ~compute per byte
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}

__global__ __launch_bounds__(1024) void k_slot(const uint8_t* d, uint64_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t regions = n / 8192;
  uint32_t acc = 0;
  for (uint64_t r = wave; r < regions; r += nw) {
    const uint8_t* p = d + r * 8192 + lane * 128;
    uint4 v[8];
    for (int k = 0; k < 8; ++k) v[k] = *(const uint4*)(p + 16 * k);
    for (int k = 0; k < 8; ++k) acc ^= mix(v[k]);
  }
  if (acc == 0x12345678) out[0] = acc;
}

int lds_main();

int main(int argc, char** argv) {
  if (argc > 2) return lds_main();
  const uint64_t n = (argc > 1 ? strtoull(argv[1], 0, 10) : 8ull) << 30;
  uint8_t* d;
  uint32_t* o;
  CK(hipMalloc(&d, n));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(d, 1, n));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    printf("%-12s %8.3f ms  %8.1f GB/s\n", name, best, n / (best * 1e-3) / 1e9);
  };
  run("coalesced", [&] { hipLaunchKernelGGL(k_coalesced, dim3(cus * 4), dim3(1024), 0, 0, d, n, o); });
  run("span4k", [&] { hipLaunchKernelGGL(k_span<0>, dim3(cus), dim3(1024), 0, 0, d, n, o); });
  run("span4k_2x", [&] { hipLaunchKernelGGL(k_span<0>, dim3(cus * 2), dim3(1024), 0, 0, d, n, o); });
  run("span4k_x", [&] { hipLaunchKernelGGL(k_span<1>, dim3(cus), dim3(1024), 0, 0, d, n, o); });
  run("step128x16w", [&] { hipLaunchKernelGGL((k_span_step<128, 1024>), dim3(cus), dim3(1024), 0, 0, d, n, o); });
  run("step64x16w", [&] { hipLaunchKernelGGL((k_span_step<64, 1024>), dim3(cus), dim3(1024), 0, 0, d, n, o); });
  run("step64x24w", [&] { hipLaunchKernelGGL((k_span_step<64, 768>), dim3(cus * 2), dim3(768), 0, 0, d, n, o); });
  run("step32x24w", [&] { hipLaunchKernelGGL((k_span_step<32, 768>), dim3(cus * 2), dim3(768), 0, 0, d, n, o); });
  run("slot128", [&] { hipLaunchKernelGGL(k_slot, dim3(cus), dim3(1024), 0, 0, d, n, o); });
  run("slot128_4x", [&] { hipLaunchKernelGGL(k_slot, dim3(cus * 4), dim3(1024), 0, 0, d, n, o); });
  return 0;
}

// ---- LDS lookup chains: ds_read_u16 vs ds_read_b32 on a 64 KiB table ----
template <int W>
__global__ __launch_bounds__(1024) void k_lds_chain(const uint32_t* seed, uint32_t* out, int iters) {
  __shared__ uint32_t tab[16384];
  for (int i = threadIdx.x; i < 16384; i += 1024) tab[i] = (i * 2654435761u) & 0x3FFFu;
  __syncthreads();
  uint32_t e = (threadIdx.x * 7919u + blockIdx.x) & 0x3FFFu;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    if (W == 16) {
      e = ((const uint16_t*)tab)[(e ^ it) & 0x7FFF];
    } else {
      e = tab[(e ^ it) & 0x3FFF] & 0x3FFF;
    }
    acc += e;
  }
  if (acc == 0x12345678) out[0] = acc;
}

int lds_main() {
  uint32_t* o;
  CK(hipMalloc(&o, 64));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 4096;
  for (int w : {16, 32}) {
    float best = 1e9;
    for (int r = 0; r < 4; ++r) {
      CK(hipEventRecord(a));
      if (w == 16) hipLaunchKernelGGL(k_lds_chain<16>, dim3(cus), dim3(1024), 0, 0, (const uint32_t*)nullptr, o, iters);
      else hipLaunchKernelGGL(k_lds_chain<32>, dim3(cus), dim3(1024), 0, 0, (const uint32_t*)nullptr, o, iters);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    const double lookups = (double)cus * 1024 * iters;
    printf("lds chain u%-2d %8.3f ms  %8.1f G lookups/s\n", w, best, lookups / (best * 1e-3) / 1e9);
  }
  return 0;
}

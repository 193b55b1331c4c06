// micro_region.hip — diagnostic (not product): the cost of k_pk_probe's region layout. One
// 1024-thread workgroup per slice p (1024 slices) walks its G = 256 regions of L pairs (config B:
// L ~ 384) in chunks of K = 7 pairs per lane (one chunk per region, the next region's chunk in flight)
// and writes one 8-B output per pair densely. Layouts: "g-major" region (g, p) at (g * P + p) * cap
// (what k_pk_part writes: each partitioning workgroup's regions contiguous), "p-major" at
// (p * G + g) * cap (each slice's regions contiguous), and the contiguous persistent walk as the
// reference. Prints ms and copy-equivalent GB/s.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int K = 7;
constexpr uint32_t P = 1024, G = 256, L = 384, CAP = 512;

template <bool GMAJOR>
__global__ __launch_bounds__(1024) void k_regions(const uint2* __restrict__ reg, uint2* __restrict__ out) {
  extern __shared__ uint32_t unused_lds[];
  if (threadIdx.x == 0 && reg == nullptr) unused_lds[0] = 0;
  const uint32_t p = blockIdx.x, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  auto src = [&](uint32_t g) { return reg + (GMAJOR ? (uint64_t(g) * P + p) : (uint64_t(p) * G + g)) * CAP; };
  uint2 cur[K], nxt[K];
  auto load = [&](uint2 (&v)[K], uint32_t g) {
    const uint2* s = src(g);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t i = min(uint32_t(j * 64) + lane, L - 1);
      const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(s + i));
      v[j] = make_uint2(uint32_t(x), uint32_t(x >> 32));
    }
  };
  uint32_t g = wid;
  load(cur, g);
  const uint64_t obase = uint64_t(p) * G * L;
  for (; g < G; g += 16) {
    load(nxt, g + 16 < G ? g + 16 : g);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t i = uint32_t(j * 64) + lane;
      uint2* d = out + obase + uint64_t(g) * L + (i < L ? i : 0);
      if (i < L) __builtin_nontemporal_store((uint64_t(cur[j].x ^ 0x5A5A5A5Au) << 32) | cur[j].y, reinterpret_cast<uint64_t*>(d));
    }
#pragma unroll
    for (int j = 0; j < K; ++j) cur[j] = nxt[j];
  }
}

template <bool GMAJOR>
void run(const char* name, const uint2* reg, uint2* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_regions<GMAJOR>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const size_t lds = 150 * 1024;  // k_pk_probe's occupancy: one workgroup per CU
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_regions<GMAJOR>, dim3(P), dim3(1024), lds, 0, reg, out);
  CK(hipGetLastError());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_regions<GMAJOR>, dim3(P), dim3(1024), lds, 0, reg, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double bytes = 16.0 * P * G * L;
  printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBs\": %.0f}\n", name, ms, bytes / ms / 1e6);
}

int main() {
  uint2 *reg, *out;
  const uint64_t nreg = uint64_t(P) * G * CAP, nout = uint64_t(P) * G * L;
  CK(hipMalloc(&reg, nreg * 8));
  CK(hipMalloc(&out, nout * 8));
  CK(hipMemset(reg, 0x33, nreg * 8));
  run<true>("g-major (k_pk_part layout)", reg, out);
  run<false>("p-major", reg, out);
  run<true>("g-major (k_pk_part layout)", reg, out);
  run<false>("p-major", reg, out);
  return 0;
}

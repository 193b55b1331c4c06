// micro_occ.hip — diagnostic (not product): does k_pk_probe's shape gain from two workgroups per CU?
// A persistent walk over 1e8 8-B pairs (next chunk of K pairs per lane in flight, as k_pk_probe
// walks its regions), L dependent random LDS lookups per pair into a per-workgroup LDS table, one
// 8-B output per pair. Variants: one 1024-thread workgroup per CU with a 150 KB table against two
// per CU with 75 KB tables (and 4 x 512 threads with 37 KB), for L = 0 (pure copy), 2, 3.
// Prints the kernel time and the copy-equivalent GB/s (1.6 GB moved).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int BLOCK, int K, int L>
__global__ __launch_bounds__(BLOCK) void k_walk(const uint2* __restrict__ in, uint2* __restrict__ out, uint64_t n,
                                                uint32_t words) {
  extern __shared__ uint32_t tab[];
  for (uint32_t i = threadIdx.x; i < words; i += BLOCK) tab[i] = i * 0x9E3779B1u;
  __syncthreads();
  constexpr uint64_t kChunk = uint64_t(BLOCK) * K;
  const uint64_t nch = n / kChunk;
  uint2 cur[K], nxt[K];
  uint64_t c = blockIdx.x;
  auto load = [&](uint2 (&v)[K], uint64_t ch) {
    const uint64_t b = (ch < nch ? ch : nch - 1) * kChunk;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(in + b + j * BLOCK + threadIdx.x));
      v[j] = make_uint2(uint32_t(x), uint32_t(x >> 32));
    }
  };
  load(cur, c);
  for (; c < nch; c += gridDim.x) {
    load(nxt, c + gridDim.x);
    uint32_t r[K];
#pragma unroll
    for (int j = 0; j < K; ++j) r[j] = cur[j].x;
#pragma unroll
    for (int l = 0; l < L; ++l) {
#pragma unroll
      for (int j = 0; j < K; ++j) r[j] = tab[__umulhi(r[j] ^ (l * 0x85EBCA6Bu), words)] ^ cur[j].x;
    }
    const uint64_t b = c * kChunk;
#pragma unroll
    for (int j = 0; j < K; ++j)
      __builtin_nontemporal_store((uint64_t(r[j]) << 32) | cur[j].y,
                                  reinterpret_cast<uint64_t*>(out + b + j * BLOCK + threadIdx.x));
#pragma unroll
    for (int j = 0; j < K; ++j) cur[j] = nxt[j];
  }
}

template <int BLOCK, int K, int L>
void run(const char* name, const uint2* in, uint2* out, uint64_t n, int cus, int per_cu, uint32_t words) {
  auto kern = k_walk<BLOCK, K, L>;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const size_t lds = size_t(words) * 4;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(cus * per_cu), dim3(BLOCK), lds, 0, in, out, n, words);
  CK(hipGetLastError());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(cus * per_cu), dim3(BLOCK), lds, 0, in, out, n, words);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("{\"variant\": \"%s\", \"block\": %d, \"per_cu\": %d, \"lds_kb\": %.1f, \"K\": %d, \"L\": %d, \"ms\": %.4f, \"GBs\": %.0f}\n",
         name, BLOCK, per_cu, lds / 1024.0, K, L, ms, 16.0 * n / ms / 1e6);
}

int main() {
  const uint64_t n = 100000000ull / (1024 * 8 * 4) * (1024 * 8 * 4);
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint2 *in, *out;
  CK(hipMalloc(&in, n * 8));
  CK(hipMalloc(&out, n * 8));
  CK(hipMemset(in, 0x5A, n * 8));
  for (int L : {0, 2, 3}) {
    if (L == 0) {
      run<1024, 8, 0>("1x1024", in, out, n, cus, 1, 38000);
      run<1024, 8, 0>("2x1024", in, out, n, cus, 2, 19000);
      run<512, 8, 0>("4x512", in, out, n, cus, 4, 9500);
    } else if (L == 2) {
      run<1024, 8, 2>("1x1024", in, out, n, cus, 1, 38000);
      run<1024, 8, 2>("2x1024", in, out, n, cus, 2, 19000);
      run<512, 8, 2>("4x512", in, out, n, cus, 4, 9500);
    } else {
      run<1024, 8, 3>("1x1024", in, out, n, cus, 1, 38000);
      run<1024, 8, 3>("2x1024", in, out, n, cus, 2, 19000);
      run<512, 8, 3>("4x512", in, out, n, cus, 4, 9500);
    }
  }
  return 0;
}

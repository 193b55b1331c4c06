// micro_slices.hip — diagnostic (not product): what k_pk_probe's shape would gain from smaller LDS
// slices. One workgroup per slice, non-persistent like k_pk_probe: stage the slice image (`words` u32
// from HBM into LDS, all loads of a batch issued before the first LDS write), then walk the slice's
// contiguous run of 8-B pairs in chunks of K per lane (the next chunk in flight), L dependent random
// LDS lookups per pair, one 8-B output per pair. Same 1e8 pairs and the same total image bytes in
// every variant: 1024 slices of ~150 KB (one 1024-thread workgroup per CU) against 2048 of ~75 KB
// (two per CU) and 4096 of ~37 KB with 512 threads (four per CU).
// Prints ms and the copy-equivalent GB/s (pairs in + outputs out).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int BLOCK, int K, int L>
__device__ __forceinline__ void slice_walk(const uint2* __restrict__ in, const uint32_t* __restrict__ img,
                                           uint2* __restrict__ out, uint32_t per_slice, uint32_t words,
                                           uint32_t* tab, uint64_t s, bool stage, int ilv = 0, uint32_t nsl = 0) {
  // ilv bit 0: outputs chunk-interleaved over the slices (chunk c of slice s at chunk c * nsl + s),
  // bit 1: inputs likewise; otherwise each slice's pairs / outputs are one contiguous run
  constexpr uint64_t kChunk = uint64_t(BLOCK) * K;
  const uint32_t nch = (per_slice + kChunk - 1) / kChunk;
  const uint2* src = (ilv & 2) ? in : in + s * per_slice;
  uint2* dst = (ilv & 1) ? out : out + s * per_slice;
  const auto cin = [&](uint32_t c) { return (ilv & 2) ? (uint64_t(c) * nsl + s) * kChunk : uint64_t(c) * kChunk; };
  const auto cout = [&](uint32_t c) { return (ilv & 1) ? (uint64_t(c) * nsl + s) * kChunk : uint64_t(c) * kChunk; };
  uint2 cur[K], nxt[K];
  auto load = [&](uint2 (&v)[K], uint32_t ch) __attribute__((always_inline)) {
    const uint32_t cc = ch < nch ? ch : nch - 1;
    const uint64_t b = cin(cc);
    const uint32_t lim = per_slice - 1 - cc * uint32_t(kChunk);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint64_t i = b + min(uint32_t(j * BLOCK) + threadIdx.x, lim);
      const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(src + i));
      v[j] = make_uint2(uint32_t(x), uint32_t(x >> 32));
    }
  };
  load(cur, 0);  // the first chunk in flight while the slice is staged (as k_pk_probe does)
  const uint32_t* im = img + s * words;
  constexpr int kStage = 12;
  for (uint32_t k0 = threadIdx.x; stage && k0 < words; k0 += BLOCK * kStage) {
    uint32_t a[kStage];
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const uint32_t k = k0 + u * BLOCK;
      a[u] = k < words ? im[k] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const uint32_t k = k0 + u * BLOCK;
      if (k < words) tab[k] = a[u] * 0x9E3779B1u;
    }
  }
  __syncthreads();
  for (uint32_t c = 0; c < nch; ++c) {
    load(nxt, c + 1);
    uint32_t r[K];
#pragma unroll
    for (int j = 0; j < K; ++j) r[j] = cur[j].x;
#pragma unroll
    for (int l = 0; l < L; ++l) {
#pragma unroll
      for (int j = 0; j < K; ++j) r[j] = tab[__umulhi(r[j] ^ (l * 0x85EBCA6Bu), words)] ^ cur[j].x;
    }
    const uint64_t b = cout(c);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t i = c * uint32_t(kChunk) + uint32_t(j * BLOCK) + threadIdx.x;
      if (i < per_slice)
        __builtin_nontemporal_store((uint64_t(r[j]) << 32) | cur[j].y,
                                    reinterpret_cast<uint64_t*>(dst + b + uint32_t(j * BLOCK) + threadIdx.x));
    }
#pragma unroll
    for (int j = 0; j < K; ++j) cur[j] = nxt[j];
  }
}

// MODE 0: one workgroup per slice; 1: the same without staging (LDS left as is); 2: persistent,
// workgroup g takes slices g, g + grid, ... (stage, barrier, walk, barrier); 3 / 4 / 5: MODE 0 with
// outputs / inputs / both chunk-interleaved over the slices
template <int BLOCK, int K, int L, int MODE>
__global__ __launch_bounds__(BLOCK) void k_slice(const uint2* __restrict__ in, const uint32_t* __restrict__ img,
                                                 uint2* __restrict__ out, uint32_t per_slice, uint32_t words,
                                                 uint32_t nslices) {
  extern __shared__ uint32_t tab[];
  if (MODE == 2) {
    for (uint32_t s = blockIdx.x; s < nslices; s += gridDim.x) {
      slice_walk<BLOCK, K, L>(in, img, out, per_slice, words, tab, s, true);
      __syncthreads();
    }
  } else {
    slice_walk<BLOCK, K, L>(in, img, out, per_slice, words, tab, blockIdx.x, MODE != 1, MODE >= 3 ? MODE - 2 : 0,
                            nslices);
  }
}

template <int BLOCK, int K, int L, int MODE = 0>
void run(const char* name, const uint2* in, const uint32_t* img, uint2* out, uint64_t n, uint32_t slices,
         uint32_t words, uint32_t grid = 0) {
  auto kern = k_slice<BLOCK, K, L, MODE>;
  if (!grid) grid = slices;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const size_t lds = size_t(words) * 4;
  const uint32_t per = uint32_t(n / slices);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), lds, 0, in, img, out, per, words, slices);
  CK(hipGetLastError());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), lds, 0, in, img, out, per, words, slices);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("{\"variant\": \"%s\", \"mode\": %d, \"slices\": %u, \"block\": %d, \"lds_kb\": %.1f, \"K\": %d, \"L\": %d, \"ms\": %.4f, \"GBs\": %.0f}\n",
         name, MODE, slices, BLOCK, lds / 1024.0, K, L, ms, 16.0 * double(per) * slices / ms / 1e6);
}

template <int L>
void sweep(const uint2* in, const uint32_t* img, uint2* out, uint64_t n) {
  run<1024, 7, L>("1x1024", in, img, out, n, 1024, 37000);
  run<1024, 7, L, 1>("1x1024 nostage", in, img, out, n, 1024, 37000);
  run<1024, 7, L, 2>("1x1024 persistent", in, img, out, n, 1024, 37000, 256);
  run<1024, 7, L, 3>("1x1024 out-ilv", in, img, out, n, 1024, 37000);
  run<1024, 7, L, 4>("1x1024 in-ilv", in, img, out, n, 1024, 37000);
  run<1024, 7, L, 5>("1x1024 both-ilv", in, img, out, n, 1024, 37000);
  run<1024, 7, L>("2x1024", in, img, out, n, 2048, 18500);
  run<512, 7, L>("2x512", in, img, out, n, 2048, 18500);
  run<512, 7, L>("4x512", in, img, out, n, 4096, 9250);
  run<256, 7, L>("4x256", in, img, out, n, 4096, 9250);
}

int main() {
  const uint64_t n = 100000000ull;
  uint2 *in, *out;
  uint32_t* img;
  const uint64_t room = 110000000ull;  // interleaved layouts address whole chunks: 14 x 1024 x 7168 pairs
  CK(hipMalloc(&in, room * 8));
  CK(hipMalloc(&out, room * 8));
  CK(hipMalloc(&img, 1024ull * 37000 * 4));
  CK(hipMemset(in, 0x5A, room * 8));
  CK(hipMemset(img, 0x33, 1024ull * 37000 * 4));
  sweep<0>(in, img, out, n);
  sweep<2>(in, img, out, n);
  CK(hipFree(in));
  CK(hipFree(out));
  CK(hipFree(img));
  return 0;
}

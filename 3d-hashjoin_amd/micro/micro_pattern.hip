// micro_pattern.hip — diagnostic (not product): HBM throughput of the two access patterns a
// radix partition can put on the memory system, at the config B probe size (1e8 pairs, 800 MB).
//   seq       read pairs sequentially, write pairs sequentially (the copy floor)
//   rd128     read 128-B pieces in a scattered order, write pairs sequentially
//   rd64      same with 64-B pieces
//   wr128     read pairs sequentially, write 128-B pieces in a scattered order
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t scramble(uint32_t x, uint32_t n) {  // a permutation of [0, n) for n = 2^k
  x *= 0x9E3779B1u;
  x ^= x >> 15;
  x *= 0x85EBCA6Bu;
  return x & (n - 1);
}

// PIECE pairs per piece; piece q of the output comes from piece scramble(q) of the input (READ) or
// the other way round. One wave moves 64 / PIECE... pieces per step; 8 steps in flight.
template <int PIECE, int MODE>  // 0 sequential, 1 scattered reads, 2 scattered writes
__global__ __launch_bounds__(256) void k_piece(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                              uint32_t npieces) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
  const uint64_t nwaves = uint64_t(gridDim.x) * 4;
  constexpr uint32_t kPer = 64 / PIECE;  // pieces per wave step
  constexpr int kU = 8;
  for (uint64_t q0 = wave * kPer * kU; q0 < npieces; q0 += nwaves * kPer * kU) {
    uint64_t v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t q = uint32_t(q0 + u * kPer + lane / PIECE);
      const uint32_t src = MODE == 1 ? scramble(q, npieces) : q;
      v[u] = q < npieces ? __builtin_nontemporal_load(in + uint64_t(src) * PIECE + lane % PIECE) : 0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t q = uint32_t(q0 + u * kPer + lane / PIECE);
      const uint32_t dst = MODE == 2 ? scramble(q, npieces) : q;
      if (q < npieces) out[uint64_t(dst) * PIECE + lane % PIECE] = v[u];
    }
  }
}

int main() {
  const uint64_t n = 1ull << 27;  // 134M pairs (1 GiB), power of two for the permutation
  uint64_t *a, *b;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, n * 8));
  CK(hipMemset(a, 1, n * 8));
  CK(hipMemset(b, 0, n * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto kern, uint32_t npieces) {
    hipLaunchKernelGGL(kern, dim3(4096), dim3(256), 0, 0, a, b, npieces);
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kern, dim3(4096), dim3(256), 0, 0, a, b, npieces);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-28s %8.3f ms  %7.0f GB/s (read + write)\n", name, ms, 2.0 * n * 8 / (ms * 1e-3) / 1e9);
  };
  run("sequential", k_piece<16, 0>, uint32_t(n / 16));
  run("rd 128-B pieces scattered", k_piece<16, 1>, uint32_t(n / 16));
  run("rd 64-B pieces scattered", k_piece<8, 1>, uint32_t(n / 8));
  run("rd 256-B pieces scattered", k_piece<32, 1>, uint32_t(n / 32));
  run("wr 128-B pieces scattered", k_piece<16, 2>, uint32_t(n / 16));
  run("wr 64-B pieces scattered", k_piece<8, 2>, uint32_t(n / 8));
  run("wr 256-B pieces scattered", k_piece<32, 2>, uint32_t(n / 32));
  printf("ok\n");
  return 0;
}

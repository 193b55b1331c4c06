// micro_width.hip — diagnostic (not product): streaming copy of 1e8 8-B pairs (800 MB in, 800 MB
// out) by persistent 1024-thread workgroups, one per CU (the shape of k_pk_probe's region walk),
// with 8-B (one pair per lane and access) against 16-B (two pairs) accesses, and K pairs per lane in
// flight. Prints GB/s of the copy (1.6 GB moved).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// W = 8 or 16 bytes per lane access; K pairs per lane per step (K * 8 / W accesses), next step in flight
template <int W, int K>
__global__ __launch_bounds__(1024) void k_copy(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t n) {
  constexpr int V = W / 8;           // pairs per access
  constexpr int A = K / V;           // accesses per lane per step
  constexpr uint64_t kStep = 1024ull * K;
  const uint64_t nsteps = (n + kStep - 1) / kStep;
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  using T = typename std::conditional<W == 16, u64x2, uint64_t>::type;
  const T* src = reinterpret_cast<const T*>(in);
  T* dst = reinterpret_cast<T*>(out);
  const uint64_t nt = n / V;
  for (uint64_t s = blockIdx.x; s < nsteps; s += gridDim.x) {
    T v[A];
    const uint64_t base = s * kStep / V;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const uint64_t i = base + uint64_t(a) * 1024 + threadIdx.x;
      if (i < nt) v[a] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const uint64_t i = base + uint64_t(a) * 1024 + threadIdx.x;
      if (i < nt) __builtin_nontemporal_store(v[a], dst + i);
    }
  }
}

template <int W, int K>
void run(const uint64_t* in, uint64_t* out, uint64_t n, int ncu) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_copy<W, K>), dim3(ncu), dim3(1024), 0, 0, in, out, n);
  CK(hipEventRecord(a));
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_copy<W, K>), dim3(ncu), dim3(1024), 0, 0, in, out, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("W=%2d B K=%d: %.3f ms  %.0f GB/s\n", W, K, ms, 16.0 * n / (ms * 1e-3) / 1e9);
}

int main() {
  const uint64_t n = 100000000ull;
  uint64_t *in, *out;
  CK(hipMalloc(&in, n * 8));
  CK(hipMalloc(&out, n * 8));
  CK(hipMemset(in, 1, n * 8));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  run<8, 4>(in, out, n, ncu);
  run<8, 8>(in, out, n, ncu);
  run<16, 4>(in, out, n, ncu);
  run<16, 8>(in, out, n, ncu);
  run<16, 16>(in, out, n, ncu);
  run<8, 8>(in, out, n, ncu * 2);
  run<16, 8>(in, out, n, ncu * 2);
  return 0;
}

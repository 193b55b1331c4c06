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
template <int W, int K, int SW = W>
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
      if constexpr (SW == W) {
        if (i < nt) __builtin_nontemporal_store(v[a], dst + i);
      } else if constexpr (SW == 8) {  // 16-B loads, two 8-B stores
        if (i < nt) {
          __builtin_nontemporal_store(v[a].x, out + 2 * i);
          __builtin_nontemporal_store(v[a].y, out + 2 * i + 1);
        }
      } else {  // SW == 17: 16-B stores misaligned by 8 B (output shifted by one pair)
        typedef T Ta8 __attribute__((aligned(8)));
        if (i < nt - 1) *reinterpret_cast<Ta8*>(out + 2 * i + 1) = v[a];
      }
    }
  }
}

// Reading 12-B tuples {k, a, b} for their key word a (config B's S relation, 1.2 GB): MODE 0 one 4-B
// load per tuple (stride 12), 1 one 8-B load per tuple (the aligned 8 B holding the key), 2 three
// 16-B loads per 4 tuples. 8 tuples per thread and step, one 1024-thread workgroup per CU.
template <int MODE>
__global__ __launch_bounds__(1024) void k_keys(const uint32_t* __restrict__ t, uint64_t n, uint32_t* __restrict__ sink) {
  constexpr uint64_t kStep = 8192;
  uint32_t acc = 0;
  for (uint64_t s = blockIdx.x; s * kStep < n; s += gridDim.x) {
    const uint64_t base = s * kStep;
    if constexpr (MODE == 0) {
      uint32_t k[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint64_t i = base + j * 1024 + threadIdx.x;
        k[j] = i < n ? t[3 * i + 1] : 0u;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += k[j] * 0x9E3779B1u;
    } else if constexpr (MODE == 1) {
      uint2 k[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint64_t i = base + j * 1024 + threadIdx.x;
        k[j] = i < n ? *reinterpret_cast<const uint2*>(t + ((3 * i + 1) & ~1ull)) : make_uint2(0, 0);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += (((base + j * 1024 + threadIdx.x) & 1) ? k[j].x : k[j].y) * 0x9E3779B1u;
    } else {
      uint4 w[6];
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const uint64_t i = base + g * 4096 + 4 * threadIdx.x;  // 4 tuples = 3 x 16 B
        const uint4* p = reinterpret_cast<const uint4*>(t + 3 * i);
#pragma unroll
        for (int c = 0; c < 3; ++c) w[3 * g + c] = i + 4 <= n ? p[c] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < 2; ++g) acc += (w[3 * g].y + w[3 * g + 1].x + w[3 * g + 1].w + w[3 * g + 2].z) * 0x9E3779B1u;
    }
  }
  sink[blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <int MODE>
void run_keys(const uint32_t* t, uint64_t n, uint32_t* sink, int ncu) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_keys<MODE>), dim3(ncu), dim3(1024), 0, 0, t, n, sink);
  CK(hipEventRecord(a));
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_keys<MODE>), dim3(ncu), dim3(1024), 0, 0, t, n, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("keys MODE=%d: %.3f ms  %.0f GB/s (12-B tuples)\n", MODE, ms, 12.0 * n / (ms * 1e-3) / 1e9);
}

template <int W, int K, int SW = W>
void run(const uint64_t* in, uint64_t* out, uint64_t n, int ncu) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_copy<W, K, SW>), dim3(ncu), dim3(1024), 0, 0, in, out, n);
  CK(hipEventRecord(a));
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_copy<W, K, SW>), dim3(ncu), dim3(1024), 0, 0, in, out, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("W=%2d B SW=%2d K=%d grid=%d: %.3f ms  %.0f GB/s\n", W, SW, K, ncu, ms, 16.0 * n / (ms * 1e-3) / 1e9);
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
  run<16, 4, 8>(in, out, n, ncu);
  run<16, 8, 8>(in, out, n, ncu);
  run<16, 4, 17>(in, out, n, ncu);
  run<16, 8, 17>(in, out, n, ncu);
  run<8, 8>(in, out, n, ncu * 2);
  run<16, 8>(in, out, n, ncu * 2);
  uint32_t* tup;
  CK(hipMalloc(&tup, n * 12));
  CK(hipMemset(tup, 3, n * 12));
  run_keys<0>(tup, n, reinterpret_cast<uint32_t*>(out), ncu);
  run_keys<1>(tup, n, reinterpret_cast<uint32_t*>(out), ncu);
  run_keys<2>(tup, n, reinterpret_cast<uint32_t*>(out), ncu);
  return 0;
}

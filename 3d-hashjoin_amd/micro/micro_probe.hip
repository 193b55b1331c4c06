// micro_probe.hip — diagnostic microbenchmark for the probe kernel's components (not product).
// Variants over |S| = 1e8 AoS {k,a,b} tuples, interleaved in one process (rule 24):
//   stream_plain : strided 4-B key loads, hash, per-thread sum
//   stream_nt    : same with non-temporal loads
//   stream_x4    : 16-B coalesced loads of the tuple stream, key extracted through LDS
//   lookup_small : stream_plain + dir/entry lookups in an L2-resident table
//   lookup_big   : stream_plain + dir/entry lookups in an IC-resident 120 MB table
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../csrc/hj3d_device.hpp"

using namespace hj3d;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int B = 256;

template <bool NT>
__global__ __launch_bounds__(B) void k_stream(const uint32_t* __restrict__ t, uint64_t n, unsigned long long* out) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * B + threadIdx.x; i < n; i += uint64_t(gridDim.x) * B) {
    const uint32_t k = NT ? __builtin_nontemporal_load(t + 3 * i + 1) : t[3 * i + 1];
    acc += murmur32(k);
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

template <int ITEMS>
__global__ __launch_bounds__(B) void k_stream_items(const uint32_t* __restrict__ t, uint64_t n, unsigned long long* out) {
  uint32_t acc = 0;
  const uint64_t stride = uint64_t(gridDim.x) * B * ITEMS;
  for (uint64_t base = uint64_t(blockIdx.x) * B * ITEMS; base < n; base += stride) {
    uint32_t k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + uint64_t(j) * B + threadIdx.x;
      k[j] = i < n ? __builtin_nontemporal_load(t + 3 * i + 1) : 0u;
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) acc += murmur32(k[j]);
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

// 16-B loads: a block stages 256 tuples (3 KB) = 192 uint4 through LDS.
__global__ __launch_bounds__(B) void k_stream_x4(const uint32_t* __restrict__ t, uint64_t n, unsigned long long* out) {
  __shared__ uint32_t lds[B * 3];
  uint32_t acc = 0;
  for (uint64_t base = uint64_t(blockIdx.x) * B; base < n; base += uint64_t(gridDim.x) * B) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* src = reinterpret_cast<const u32x4*>(t + 3 * base);
    if (threadIdx.x < 192 && base + B <= n) {
      const u32x4 v = __builtin_nontemporal_load(src + threadIdx.x);
      reinterpret_cast<u32x4*>(lds)[threadIdx.x] = v;
    }
    __syncthreads();
    const uint64_t i = base + threadIdx.x;
    if (i < n) acc += murmur32(lds[3 * threadIdx.x + 1]);
    __syncthreads();
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

template <int ITEMS>
__global__ __launch_bounds__(B) void k_lookup(const uint32_t* __restrict__ t, uint64_t n, FastMod fm,
                                              const uint32_t* __restrict__ off, const uint2* __restrict__ ent,
                                              unsigned long long* out) {
  uint32_t acc = 0;
  const uint64_t stride = uint64_t(gridDim.x) * B * ITEMS;
  for (uint64_t base = uint64_t(blockIdx.x) * B * ITEMS; base < n; base += stride) {
    uint32_t h[ITEMS], s[ITEMS], e[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + uint64_t(j) * B + threadIdx.x;
      h[j] = murmur32(i < n ? __builtin_nontemporal_load(t + 3 * i + 1) : 0u);
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t b = fm.mod(h[j]);
      s[j] = off[b];
      e[j] = off[b + 1];
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      if (e[j] > s[j]) acc += ent[s[j]].y;
    }
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const uint64_t n = 100000000ull;
  uint32_t* t;
  unsigned long long* out;
  CK(hipMalloc(&t, n * 12));
  CK(hipMalloc(&out, 8));
  std::vector<uint32_t> h(3 * n);
  for (uint64_t i = 0; i < n; ++i) { h[3 * i] = uint32_t(i); h[3 * i + 1] = uint32_t(mix64(i) % 10000000); h[3 * i + 2] = 0; }
  CK(hipMemcpy(t, h.data(), n * 12, hipMemcpyHostToDevice));
  auto mk = [&](uint32_t nb, uint32_t** off, uint2** ent) {
    std::vector<uint32_t> o(nb + 1);
    for (uint32_t b = 0; b <= nb; ++b) o[b] = b;  // one entry per bucket
    std::vector<uint2> e(nb);
    for (uint32_t b = 0; b < nb; ++b) e[b] = make_uint2(b, b);
    CK(hipMalloc(off, (nb + 1) * 4));
    CK(hipMalloc(ent, nb * 8));
    CK(hipMemcpy(*off, o.data(), (nb + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(*ent, e.data(), nb * 8, hipMemcpyHostToDevice));
  };
  uint32_t *offS, *offB;
  uint2 *entS, *entB;
  mk(262144, &offS, &entS);
  mk(10000000, &offB, &entB);
  const FastMod fmS = FastMod::make(262144), fmB = FastMod::make(10000000);
  for (int round = 0; round < 3; ++round) {
    for (unsigned g : {2048u, 8192u, 65536u}) {
      printf("grid %6u  stream_plain %.3f  stream_nt %.3f  x4 %.3f  items4 %.3f  items8 %.3f  lookup_small4 %.3f  lookup_small8 %.3f  lookup_big4 %.3f  lookup_big8 %.3f\n", g,
             timeit([&] { hipLaunchKernelGGL(k_stream<false>, dim3(g), dim3(B), 0, 0, t, n, out); }, 5),
             timeit([&] { hipLaunchKernelGGL(k_stream<true>, dim3(g), dim3(B), 0, 0, t, n, out); }, 5),
             timeit([&] { hipLaunchKernelGGL(k_stream_x4, dim3(g), dim3(B), 0, 0, t, n, out); }, 5),
             timeit([&] { hipLaunchKernelGGL(k_stream_items<4>, dim3(g), dim3(B), 0, 0, t, n, out); }, 5),
             timeit([&] { hipLaunchKernelGGL(k_stream_items<8>, dim3(g), dim3(B), 0, 0, t, n, out); }, 5),
             timeit([&] { hipLaunchKernelGGL(k_lookup<4>, dim3(g), dim3(B), 0, 0, t, n, fmS, offS, entS, out); }, 5),
             timeit([&] { hipLaunchKernelGGL(k_lookup<8>, dim3(g), dim3(B), 0, 0, t, n, fmS, offS, entS, out); }, 5),
             timeit([&] { hipLaunchKernelGGL(k_lookup<4>, dim3(g), dim3(B), 0, 0, t, n, fmB, offB, entB, out); }, 5),
             timeit([&] { hipLaunchKernelGGL(k_lookup<8>, dim3(g), dim3(B), 0, 0, t, n, fmB, offB, entB, out); }, 5));
    }
  }
  return 0;
}

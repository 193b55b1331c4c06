// micro_lds_atomic.hip — LDS atomic-with-return throughput on gfx950 (diagnostic, not product).
// Each workgroup (1024 threads) performs R rounds of one LDS op per thread on random counters:
//   mode 0: atomicAdd-return on 1018 shared u32 counters
//   mode 1: atomicAdd-return on per-wave private counters (16 x 1018)
//   mode 2: atomicAdd without using the result (no return)
//   mode 3: plain ds_read + ds_write on per-wave private counters (lost updates, timing only)
//   mode 4: ds_read only
//   mode 5: atomicCAS (compare-and-swap with return) on 1018 shared counters
//   mode 6: atomicMin without return on 1018 shared counters
//   mode 7: atomicAdd + atomicMin without return on one random slot (k_nagg pass A's hit path)
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void k(unsigned* out, int rounds) {
  __shared__ unsigned cnt[16 * 1024];
  for (int i = threadIdx.x; i < 16 * 1024; i += 1024) cnt[i] = 0;
  __syncthreads();
  unsigned x = threadIdx.x * 2654435761u + blockIdx.x * 40503u, acc = 0;
  const unsigned wbase = (threadIdx.x >> 6) * 1024;
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      x = x * 1664525u + 1013904223u;
      const unsigned p = (x >> 8) % 1018u;
      if (MODE == 0) acc += atomicAdd(&cnt[p], 1u);
      if (MODE == 1) acc += atomicAdd(&cnt[wbase + p], 1u);
      if (MODE == 2) atomicAdd(&cnt[p], 1u);
      if (MODE == 3) { const unsigned v = cnt[wbase + p]; cnt[wbase + p] = v + 1; acc += v; }
      if (MODE == 4) acc += cnt[wbase + p];
      if (MODE == 5) acc += atomicCAS(&cnt[p], x, x + 1u);
      if (MODE == 6) atomicMin(&cnt[p], x);
      if (MODE == 7) { atomicAdd(&cnt[p], 1u); atomicMin(&cnt[1024 + p], x); }
    }
  }
  __syncthreads();
  if (acc == 0x12345u) out[0] = cnt[threadIdx.x];
  if (threadIdx.x == 0) out[blockIdx.x + 1] = cnt[7];
}

int main() {
  unsigned* out;
  CK(hipMalloc(&out, 1 << 20));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int G = 256, R = 100;
  auto run = [&](const char* nm, auto kern) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(1024), 0, 0, out, R);
    hipDeviceSynchronize();
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(G), dim3(1024), 0, 0, out, R);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double ops = double(G) * 1024 * 16 * R;
    // cycles per wave-instruction per CU at 2.4 GHz
    printf("%-36s %8.3f ms  %6.1f cyc per wave-op per CU\n", nm, ms, ms * 1e-3 * 2.4e9 / (ops / 64 / G));
  };
  run("atomic rtn, shared 1018", k<0>);
  run("atomic rtn, per-wave private", k<1>);
  run("atomic no-return, shared", k<2>);
  run("plain read+write, private", k<3>);
  run("plain read only", k<4>);
  run("atomicCAS rtn, shared", k<5>);
  run("atomicMin no-return, shared", k<6>);
  run("atomicAdd + atomicMin no-return", k<7>);
  return 0;
}

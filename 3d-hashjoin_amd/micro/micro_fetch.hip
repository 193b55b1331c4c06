// micro_fetch.hip — diagnostic (not product): calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access widths the hj3d kernels use, on KNOWN byte counts (MI355X_MICROARCH.md,
// HBM section: FETCH_SIZE reads half the bytes of a 16-B-per-lane streaming read; other widths are
// uncalibrated). Every pattern touches a 3 GiB buffer (beyond the 256 MiB Infinity Cache) once, so
// its algorithmic bytes are the HBM bytes; run each kernel under `rocprofv3 --pmc FETCH_SIZE` /
// `--pmc WRITE_SIZE` and divide the counter by the printed `bytes` to get the per-pattern factor.
//   r16   16-B loads per lane, streaming                   (known: x 2, the guide's calibration)
//   r8    8-B loads per lane, streaming                    (k_pk_probe's pairs, k_nagg's pairs)
//   r4    4-B loads per lane, streaming                    (k_expand_light's sub rows, key columns)
//   r4s12 4-B loads at a 12-B stride                       (key word of a {k, a, b} tuple)
//   r4x2  two 4-B loads per 8-B pair, back to back         (explicit-row k_pk_part)
//   g64   4-B gather, one per distinct 64-B sector         (bytes = sectors x 64)
//   g128  4-B gather, one per distinct 128-B line          (bytes = lines x 128 if whole lines move)
//   w8    8-B streaming stores                             (pairs, output)
//   w4    4-B streaming stores                             (sub rows)
//   w4r   4-B scattered stores filling every word of each 128-B line once, lines in random order
//         within 1 MiB windows (k_nagg's sub-row scatter after its lines complete)
// Usage: micro_fetch <pattern>|all  (prints one JSON line per pattern: name, bytes, ms).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint64_t kBytes = 3ull << 30;  // 3 GiB

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ a, uint64_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    const T v = a[i];
    uint32_t w[sizeof(T) / 4];
    memcpy(w, &v, sizeof(T));
#pragma unroll
    for (int k = 0; k < int(sizeof(T) / 4); ++k) acc ^= w[k];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// 4-B loads at a word stride (n items)
__global__ __launch_bounds__(256) void k_read_stride(const uint32_t* __restrict__ a, uint64_t n, uint32_t stride,
                                                     uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) acc ^= a[i * stride];
  if (acc == 0x12345678u) sink[0] = acc;
}

// two 4-B loads per 8-B pair (key word, row word), back to back
__global__ __launch_bounds__(256) void k_read_x2(const uint32_t* __restrict__ a, uint64_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    acc ^= a[2 * i];
    acc += a[2 * i + 1];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// 4-B gather: item i reads the first word of unit perm(i) (units of `unit` bytes; perm = a
// multiplicative bijection mod n, n prime-free of the multiplier: every unit exactly once)
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ a, uint64_t n, uint32_t unit_words,
                                                uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    const uint64_t u = (i * 2654435761ull) % n;  // n a power of two: odd multiplier -> bijection
    acc ^= a[u * unit_words];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename T>
__global__ __launch_bounds__(256) void k_write(T* __restrict__ a, uint64_t n) {
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    T v;
    memset(&v, int(i & 0x7F), sizeof(T));
    a[i] = v;
  }
}

// 4-B scattered stores: word i goes to a position inside its 1 MiB window given by a bijection of
// the window's words (every word once; consecutive lanes far apart)
__global__ __launch_bounds__(256) void k_write_scatter(uint32_t* __restrict__ a, uint64_t n) {
  constexpr uint64_t kWin = (1u << 20) / 4;  // words per window
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    const uint64_t w = i / kWin, k = i % kWin;
    a[w * kWin + (k * 40503ull) % kWin] = uint32_t(i);
  }
}

int main(int argc, char** argv) {
  const char* which = argc > 1 ? argv[1] : "all";
  uint8_t* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, kBytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * 16;
  auto run = [&](const char* name, uint64_t bytes, auto&& launch) {
    if (strcmp(which, "all") != 0 && strcmp(which, name) != 0) return;
    launch();  // warm (page tables)
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"pattern\": \"%s\", \"bytes\": %llu, \"ms\": %.4f, \"GBs\": %.1f}\n", name, (unsigned long long)bytes, ms,
           bytes / (ms * 1e6));
  };
  const uint64_t n4 = kBytes / 4;
  run("r16", kBytes, [&] { hipLaunchKernelGGL((k_read<uint4>), dim3(grid), dim3(256), 0, 0, (const uint4*)buf, kBytes / 16, sink); });
  run("r8", kBytes, [&] { hipLaunchKernelGGL((k_read<uint2>), dim3(grid), dim3(256), 0, 0, (const uint2*)buf, kBytes / 8, sink); });
  run("r4", kBytes, [&] { hipLaunchKernelGGL((k_read<uint32_t>), dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, n4, sink); });
  run("r4s12", kBytes, [&] { hipLaunchKernelGGL(k_read_stride, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, n4 / 3, 3u, sink); });
  run("r4x2", kBytes, [&] { hipLaunchKernelGGL(k_read_x2, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, kBytes / 8, sink); });
  // 2 GiB of units (a power of two: the gather's bijection), one 4-B read per unit
  const uint64_t span = 2ull << 30;
  run("g64", span, [&] { hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, span / 64, 16u, sink); });
  run("g128", span, [&] { hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, span / 128, 32u, sink); });
  run("w8", kBytes, [&] { hipLaunchKernelGGL((k_write<uint2>), dim3(grid), dim3(256), 0, 0, (uint2*)buf, kBytes / 8); });
  run("w4", kBytes, [&] { hipLaunchKernelGGL((k_write<uint32_t>), dim3(grid), dim3(256), 0, 0, (uint32_t*)buf, n4); });
  run("w4r", kBytes, [&] { hipLaunchKernelGGL(k_write_scatter, dim3(grid), dim3(256), 0, 0, (uint32_t*)buf, n4); });
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}

// bw.hip — the streaming-copy peak SURVEY §8(d) asks every bench line to carry beside its roofline
// fractions: what this box's HBM actually streams, measured in the same run as the kernels whose
// fractions are quoted (hj3d_stream_copy). Not on the join path; replaces nothing of the reference.
#include <algorithm>

#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

constexpr int kCopyBlock = 256;
constexpr int kCopyUnroll = 4;  // 16-B vectors per thread and step: 16 KB per workgroup step
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// Grid-stride copy of n16 16-B vectors; NT: non-temporal loads and stores (no L2 allocation).
template <bool NT>
__global__ __launch_bounds__(kCopyBlock) void k_stream_copy(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                            uint64_t n16) {
  const uint64_t step = uint64_t(gridDim.x) * kCopyBlock * kCopyUnroll;
  for (uint64_t base = uint64_t(blockIdx.x) * kCopyBlock * kCopyUnroll + threadIdx.x; base < n16; base += step) {
    v4u v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint64_t i = base + uint64_t(u) * kCopyBlock;
      if (i < n16) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint64_t i = base + uint64_t(u) * kCopyBlock;
      if (i < n16) {
        if (NT) __builtin_nontemporal_store(v[u], dst + i);
        else dst[i] = v[u];
      }
    }
  }
}

}  // namespace
}  // namespace hj3d

using namespace hj3d;

// Synchronous. Copies `bytes` (multiple of 16) from src to dst `reps` times per variant (plain and
// non-temporal vectors; grids of 4, 8 and 16 workgroups per CU) on the context stream, each launch
// timed by HIP events; out[0] = the best rate in GB/s counting read + write bytes, out[1] = the
// median launch's rate of the best variant, out[2] = that variant's id (grid factor, + 100 when
// non-temporal).
extern "C" hj3d_status hj3d_stream_copy(hj3d_ctx* ctx, void* dst, const void* src, uint64_t bytes, uint32_t reps,
                                        double out[3]) {
  if (!ctx || !dst || !src || !out || bytes < 16 || (bytes & 15) || reps == 0) return HJ3D_EINVAL;
  const uint64_t n16 = bytes / 16;
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess) return HJ3D_EDEVICE;
  if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); return HJ3D_EDEVICE; }
  double best = 0.0, best_med = 0.0, best_id = 0.0;
  hj3d_status st = HJ3D_OK;
  for (int nt = 0; nt < 2 && st == HJ3D_OK; ++nt) {
    for (int f : {4, 8, 16}) {
      const uint64_t need = (n16 + kCopyBlock * kCopyUnroll - 1) / (kCopyBlock * kCopyUnroll);
      const unsigned grid = unsigned(need < uint64_t(ctx->num_cus) * f ? need : uint64_t(ctx->num_cus) * f);
      std::vector<double> rate;
      for (uint32_t r = 0; r <= reps; ++r) {  // launch 0 warms up
        (void)hipEventRecord(a, ctx->stream);
        if (nt) hipLaunchKernelGGL(k_stream_copy<true>, dim3(grid), dim3(kCopyBlock), 0, ctx->stream,
                                   static_cast<const v4u*>(src), static_cast<v4u*>(dst), n16);
        else hipLaunchKernelGGL(k_stream_copy<false>, dim3(grid), dim3(kCopyBlock), 0, ctx->stream,
                                static_cast<const v4u*>(src), static_cast<v4u*>(dst), n16);
        (void)hipEventRecord(b, ctx->stream);
        if (hipEventSynchronize(b) != hipSuccess) { st = HJ3D_EDEVICE; break; }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r > 0 && ms > 0.f) rate.push_back(2.0 * double(bytes) / (double(ms) * 1e-3) / 1e9);
      }
      if (st != HJ3D_OK || rate.empty()) break;
      std::sort(rate.begin(), rate.end());
      if (rate.back() > best) {
        best = rate.back();
        best_med = rate[rate.size() / 2];
        best_id = f + (nt ? 100 : 0);
      }
    }
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (hipGetLastError() != hipSuccess && st == HJ3D_OK) st = HJ3D_EDEVICE;
  out[0] = best;
  out[1] = best_med;
  out[2] = best_id;
  return st;
}

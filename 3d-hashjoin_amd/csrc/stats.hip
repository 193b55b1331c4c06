// stats.hip — HtStatistics on the device (makeStatistics: ht_chaining.hh:260-292,
// ht_nested.hh:450-482). Chain length of a bucket = entries (chaining, dir slot included) or
// main nodes = distinct keys (nested); cc0 aggregates over all buckets, cc1 over non-empty ones.
// Off the timed path; synchronous.
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

// out: {empty, cc0_min, cc0_max, cc0_sum, cc1_min, cc1_max}; cc1_sum == cc0_sum
__global__ __launch_bounds__(kBlock) void k_chain_lengths(const uint32_t* __restrict__ off, uint32_t nbl,
                                                          uint64_t* __restrict__ out) {
  uint64_t empty = 0, mn0 = ~0ull, mx0 = 0, sum = 0, mn1 = ~0ull, mx1 = 0;
  for (uint64_t b = uint64_t(blockIdx.x) * kBlock + threadIdx.x; b < nbl; b += uint64_t(gridDim.x) * kBlock) {
    const uint64_t len = off[b + 1] - off[b];
    empty += len == 0;
    mn0 = len < mn0 ? len : mn0;
    mx0 = len > mx0 ? len : mx0;
    sum += len;
    if (len) {
      mn1 = len < mn1 ? len : mn1;
      mx1 = len > mx1 ? len : mx1;
    }
  }
  empty = wave_sum(empty);
  sum = wave_sum(sum);
  mn0 = wave_min(mn0);
  mx0 = wave_max(mx0);
  mn1 = wave_min(mn1);
  mx1 = wave_max(mx1);
  if ((threadIdx.x & 63) == 0) {
    auto* o = reinterpret_cast<unsigned long long*>(out);
    if (empty) atomicAdd(o + 0, empty);
    atomicMin(o + 1, mn0);
    atomicMax(o + 2, mx0);
    if (sum) atomicAdd(o + 3, sum);
    atomicMin(o + 4, mn1);
    atomicMax(o + 5, mx1);
  }
}

__global__ __launch_bounds__(kBlock) void k_ent_hashes(const uint2* __restrict__ ent, uint64_t n,
                                                       uint32_t* __restrict__ k, uint32_t* __restrict__ v) {
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock) {
    k[i] = ent[i].x;
    v[i] = 0;
  }
}

__global__ __launch_bounds__(kBlock) void k_count_heads(const uint32_t* __restrict__ k, uint64_t n,
                                                        uint64_t* __restrict__ out) {
  uint64_t c = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock)
    c += (i == 0 || k[i] != k[i - 1]);
  uint64_t v[1] = {c};
  block_flush<1, 0>(v, out);
}

}  // namespace

hipError_t table_stats(hj3d_ctx* ctx, const hj3d_table* t, hj3d_stats* st, hipStream_t s) {
  hipError_t e;
  const uint32_t nbl = t->nb_local;
  if ((e = ctx->misc.ensure(16 * sizeof(uint64_t))) != hipSuccess) return e;
  uint64_t* d = ctx->misc.as<uint64_t>();
  const uint64_t init[8] = {0, ~0ull, 0, 0, ~0ull, 0, 0, 0};
  if ((e = hipMemcpyAsync(d, init, sizeof(init), hipMemcpyHostToDevice, s)) != hipSuccess) return e;
  if (nbl) {
    const unsigned g = grid_for(ctx, nbl, kBlock * 4);
    hipLaunchKernelGGL(k_chain_lengths, dim3(g), dim3(kBlock), 0, s, t->off.as<const uint32_t>(), nbl, d);
  }
  uint32_t total = 0;
  if ((e = hipMemcpyAsync(&total, t->off.as<const uint32_t>() + nbl, sizeof(uint32_t), hipMemcpyDeviceToHost, s)) !=
      hipSuccess)
    return e;
  uint64_t h[8];
  if ((e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  st->nb = nbl;
  st->empty = h[0];
  st->cc0_min = h[1];
  st->cc0_max = h[2];
  st->cc0_sum = h[3];
  st->cc0_cnt = nbl;
  st->cc1_min = h[4];
  st->cc1_max = h[5];
  st->cc1_sum = h[3];
  st->cc1_cnt = nbl - h[0];
  if (t->desc.kind == HJ3D_NESTED) {
    uint64_t c[2];
    if ((e = hipMemcpyAsync(c, t->counts.as<const uint64_t>(), sizeof(c), hipMemcpyDeviceToHost, s)) != hipSuccess)
      return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    st->entries = c[0];
    st->distinct = total;  // one main record per distinct key
    return hipSuccess;
  }
  st->entries = total;
  st->distinct = 0;
  if (total) {  // distinct hash values (== distinct keys, murmur32 is a bijection): sort + heads
    if ((e = ctx->scratch[kScrSortK].ensure(4ull * total * sizeof(uint32_t))) != hipSuccess) return e;
    uint32_t* k0 = ctx->scratch[kScrSortK].as<uint32_t>();
    uint32_t *v0 = k0 + total, *k1 = v0 + total, *v1 = k1 + total;
    const unsigned g = grid_for(ctx, total, kBlock * 4);
    hipLaunchKernelGGL(k_ent_hashes, dim3(g), dim3(kBlock), 0, s, t->ent.as<const uint2>(), uint64_t(total), k0, v0);
    if ((e = radix_sort_pairs(ctx, k0, v0, k1, v1, total, 32, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(d + 8, 0, sizeof(uint64_t), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_count_heads, dim3(g), dim3(kBlock), 0, s, k0, uint64_t(total), d + 8);
    if ((e = hipMemcpyAsync(&st->distinct, d + 8, sizeof(uint64_t), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  }
  return hipGetLastError();
}

}  // namespace hj3d

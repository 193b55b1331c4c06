// sort.hip — stable LSD radix sort of (u32 key, u32 value) pairs, 8-bit digits, only as many
// passes as the keys have significant bits.
//
// Used by the nested (3D) build to group the duplicates of every key: sorting the
// (hash, row) pairs by hash makes each distinct key one contiguous run with its rows in
// input order. Sorting is insensitive to skew (a Zipf hot key is just a long run), which
// atomics-per-key builds are not.
//
// Per pass (digit = 8 bits): (1) per-tile digit histograms (LDS atomics), digit-major in
// HBM; (2) exclusive scan of the 256 x tiles histogram (scan.hip); (3) stable scatter through
// an LDS-staged tile (k_rs_scatter).
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

constexpr int kSBlock = 512;                // 8 waves
constexpr int kRounds = 16;
constexpr int kTile = kSBlock * kRounds;     // 8192 pairs per tile
constexpr int kRadix = 256;
constexpr int kWaves = kSBlock / kWave;

__global__ __launch_bounds__(kSBlock) void k_rs_hist(const uint32_t* __restrict__ keys, uint64_t n, int shift,
                                                     uint32_t ntiles, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kRadix];
  if (threadIdx.x < kRadix) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = uint64_t(blockIdx.x) * kTile;
  uint32_t k[kRounds];
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const uint64_t i = base + uint64_t(j) * kSBlock + threadIdx.x;
    k[j] = i < n ? keys[i] : 0u;
  }
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const uint64_t i = base + uint64_t(j) * kSBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[(k[j] >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kRadix) hist[uint64_t(threadIdx.x) * ntiles + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter of one tile. Ranks: per round of 512 elements (element order = round, wave,
// lane) each wave finds its same-digit peers with 8 ballots; waves are ordered by per-digit
// LDS counters and rounds by running digit counts. The ranked tile is staged in LDS in digit
// order and then written so that consecutive threads store consecutive addresses of one
// digit's run (coalesced), instead of one scattered 4-B store per element and array.
__global__ __launch_bounds__(kSBlock) void k_rs_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                        uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                        uint64_t n, int shift, uint32_t ntiles,
                                                        const uint32_t* __restrict__ offs) {
  __shared__ uint2 stage[kTile];             // 64 KB
  __shared__ uint32_t run[kRadix];           // tile-local start of each digit, advanced per round
  __shared__ uint32_t lstart[kRadix];        // tile-local start of each digit
  __shared__ uint32_t tbase[kRadix];         // global start of each digit for this tile
  __shared__ uint32_t wcnt[kWaves][kRadix];  // per-wave digit counts of the current round
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t base = uint64_t(blockIdx.x) * kTile;
  uint32_t k[kRounds], v[kRounds];
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const uint64_t i = base + uint64_t(j) * kSBlock + threadIdx.x;
    k[j] = i < n ? kin[i] : 0u;
    v[j] = i < n ? vin[i] : 0u;
  }
  if (threadIdx.x < kRadix) {
    run[threadIdx.x] = 0;
    tbase[threadIdx.x] = offs[uint64_t(threadIdx.x) * ntiles + blockIdx.x];
  }
  // tile-local digit histogram -> exclusive scan (digits 0..255 by the first 256 threads)
  for (int w = 0; w < kWaves; ++w)
    if (threadIdx.x < kRadix) wcnt[w][threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const uint64_t i = base + uint64_t(j) * kSBlock + threadIdx.x;
    if (i < n) atomicAdd(&wcnt[0][(k[j] >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kWave) {  // one wave scans 256 counts (4 per lane)
    uint32_t c[4], t = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      c[q] = wcnt[0][lane * 4 + q];
      t += c[q];
    }
    uint32_t tot;
    uint32_t pre = wave_excl_scan(t, &tot);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      lstart[lane * 4 + q] = pre;
      run[lane * 4 + q] = pre;
      pre += c[q];
    }
  }
  __syncthreads();
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    if (threadIdx.x < kRadix) {
#pragma unroll
      for (int w = 0; w < kWaves; ++w) wcnt[w][threadIdx.x] = 0;
    }
    __syncthreads();
    const uint64_t i = base + uint64_t(j) * kSBlock + threadIdx.x;
    const bool valid = i < n;
    const uint32_t d = (k[j] >> shift) & 255u;
    uint64_t peer = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const bool set = (d >> bit) & 1u;
      const uint64_t bb = __ballot(set);
      peer &= set ? bb : ~bb;
    }
    const uint32_t wrank = uint32_t(__popcll(peer & lt));
    if (valid && wrank == 0) wcnt[wid][d] = uint32_t(__popcll(peer));
    __syncthreads();
    if (valid) {
      uint32_t pos = run[d] + wrank;
      for (int w = 0; w < wid; ++w) pos += wcnt[w][d];
      stage[pos] = make_uint2(k[j], v[j]);
    }
    __syncthreads();
    if (threadIdx.x < kRadix) {
      uint32_t add = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) add += wcnt[w][threadIdx.x];
      run[threadIdx.x] += add;
    }
  }
  __syncthreads();
  const uint32_t m = uint32_t(n - base < uint64_t(kTile) ? n - base : uint64_t(kTile));
  for (uint32_t p = threadIdx.x; p < m; p += kSBlock) {
    const uint2 e = stage[p];
    const uint32_t d = (e.x >> shift) & 255u;
    const uint64_t o = uint64_t(tbase[d]) + (p - lstart[d]);
    kout[o] = e.x;
    vout[o] = e.y;
  }
}

}  // namespace

hipError_t radix_sort_pairs(hj3d_ctx* ctx, uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint64_t n,
                            int bits, hipStream_t s, bool* in_alt) {
  if (in_alt) *in_alt = false;
  if (n <= 1) return hipSuccess;
  const uint64_t ntiles = (n + kTile - 1) / kTile;
  hipError_t e = ctx->scratch[kScrD].ensure((uint64_t(kRadix) * ntiles + 1) * sizeof(uint32_t));
  if (e != hipSuccess) return e;
  uint32_t* hist = ctx->scratch[kScrD].as<uint32_t>();
  uint32_t *ki = k0, *vi = v0, *ko = k1, *vo = v1;
  int passes = 0;
  for (int shift = 0; shift < bits; shift += 8, ++passes) {
    hipLaunchKernelGGL(k_rs_hist, dim3(unsigned(ntiles)), dim3(kSBlock), 0, s, ki, n, shift, uint32_t(ntiles), hist);
    if ((e = exclusive_scan_u32(ctx, hist, hist, uint64_t(kRadix) * ntiles, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_rs_scatter, dim3(unsigned(ntiles)), dim3(kSBlock), 0, s, ki, vi, ko, vo, n, shift,
                       uint32_t(ntiles), hist);
    uint32_t* t;
    t = ki; ki = ko; ko = t;
    t = vi; vi = vo; vo = t;
  }
  if ((passes & 1) && in_alt) {
    *in_alt = true;  // the caller reads the result from (k1, v1)
  } else if (passes & 1) {  // result is in (k1, v1): copy back so it lands in (k0, v0)
    if ((e = hipMemcpyAsync(k0, k1, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(v0, v1, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
  }
  return hipGetLastError();
}

}  // namespace hj3d

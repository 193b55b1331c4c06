// scan.hip — exclusive prefix sums (CSR directory offsets, partition histograms, output offsets).
//
// u32: one launch, single pass with decoupled look-back over 4096-element tiles: a workgroup
// takes the next tile by ticket, publishes the tile's sum, adds up its predecessors' published
// sums (or the first inclusive prefix it meets) and publishes its own inclusive prefix. Status
// words carry a per-call epoch, so nothing is cleared between calls; the last tile resets the
// ticket. HBM traffic: 1 read + 1 write of the array.
// u64: reduce-then-scan in three launches (per-tile sums, one workgroup scanning the tile sums,
// per-tile scan: 2 reads + 1 write). A single-pass look-back form as for u32 measured slower
// (config C probe + unnest 0.820-0.827 against 0.813 ms, r04p: the look-back chain across XCDs
// costs more than the two extra launches) and was removed.
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

constexpr int kScanItems = 16;
constexpr int kTile = kBlock * kScanItems;  // 4096

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* lds) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  T r = 0;
  for (int w = 0; w < kBlock / kWave; ++w) r += lds[w];
  return r;
}

// Block-wide exclusive scan of one value per thread; returns the exclusive prefix and the total.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* lds, T* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  T wpre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    const T s = lds[w];
    if (w < wid) wpre += s;
    tot += s;
  }
  *total = tot;
  return wpre + x - v;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_tile_sums(const T* __restrict__ in, uint64_t n, T* __restrict__ sums) {
  __shared__ T lds[kBlock / kWave];
  const uint64_t base = uint64_t(blockIdx.x) * kTile;
  T acc = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
    if (i < n) acc += in[i];
  }
  const T s = block_sum(acc, lds);
  if (threadIdx.x == 0) sums[blockIdx.x] = s;
}

// One workgroup (1024 threads) scans `m` tile sums in place (exclusive); sums[m] = total.
template <typename T>
__global__ __launch_bounds__(1024) void k_scan_sums(T* sums, uint64_t m) {
  __shared__ T lds[1024 / kWave];
  __shared__ T carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (uint64_t base = 0; base < m; base += 1024) {
    const uint64_t i = base + threadIdx.x;
    const T v = i < m ? sums[i] : T(0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const T y = __shfl_up(x, o, kWave);
      if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    T wpre = 0, tot = 0;
    for (int w = 0; w < 1024 / kWave; ++w) {
      const T s = lds[w];
      if (w < wid) wpre += s;
      tot += s;
    }
    const T carry = carry_s;
    if (i < m) sums[i] = carry + wpre + x - v;
    __syncthreads();
    if (threadIdx.x == 0) carry_s = carry + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[m] = carry_s;
}

// Per-tile exclusive scan. The tile is loaded and stored coalesced (lane-strided) and
// transposed through LDS so that thread t scans the kScanItems consecutive elements
// [t*kScanItems, ...) of the tile; one pad word per kScanItems keeps the transposed LDS
// accesses free of bank conflicts.
constexpr int kScanPad = kTile + kTile / kScanItems;
__device__ __forceinline__ uint32_t scan_slot(uint32_t i) { return i + i / kScanItems; }

template <typename T>
__global__ __launch_bounds__(kBlock) void k_scan_tiles(const T* in, T* out, uint64_t n, const T* __restrict__ sums) {
  __shared__ T lds[kBlock / kWave];
  __shared__ T tile[kScanPad];
  const uint64_t base = uint64_t(blockIdx.x) * kTile;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    const uint32_t k = uint32_t(j) * kBlock + threadIdx.x;
    tile[scan_slot(k)] = base + k < n ? in[base + k] : T(0);
  }
  __syncthreads();
  T v[kScanItems];
  T local = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = tile[scan_slot(threadIdx.x * kScanItems + j)];
    local += v[j];
  }
  T total;
  T pre = block_excl_scan(local, lds, &total) + sums[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    tile[scan_slot(threadIdx.x * kScanItems + j)] = pre;
    pre += v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    const uint32_t k = uint32_t(j) * kBlock + threadIdx.x;
    if (base + k < n) out[base + k] = tile[scan_slot(k)];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kBlock - 1) out[n] = sums[gridDim.x];
}

__global__ __launch_bounds__(kBlock) void k_scan_lb(const uint32_t* in, uint32_t* out, uint64_t n,
                                                    uint64_t* __restrict__ status, uint32_t* __restrict__ ticket,
                                                    uint32_t epoch, uint32_t ntiles) {
  __shared__ uint32_t lds[kBlock / kWave];
  __shared__ uint32_t tile[kScanPad];
  __shared__ uint32_t tid_s, pre_s;
  if (threadIdx.x == 0) tid_s = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t t = tid_s;
  const uint64_t base = uint64_t(t) * kTile;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    const uint32_t k = uint32_t(j) * kBlock + threadIdx.x;
    tile[scan_slot(k)] = base + k < n ? in[base + k] : 0u;
  }
  __syncthreads();
  uint32_t v[kScanItems];
  uint32_t local = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = tile[scan_slot(threadIdx.x * kScanItems + j)];
    local += v[j];
  }
  uint32_t total;
  uint32_t pre = block_excl_scan(local, lds, &total);
  const int wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) lb_publish(status, t, epoch, t == 0 ? kLbInc : kLbAgg, total);
  if (wid == 0 && t > 0) {  // the first wave looks back over the tiles taken before this one
    const uint32_t excl = lb_exclusive(status, t, epoch);
    if (threadIdx.x == 0) {
      lb_publish(status, t, epoch, kLbInc, excl + total);
      pre_s = excl;
    }
  } else if (threadIdx.x == 0) {
    pre_s = 0;
  }
  if (threadIdx.x == 0 && t == ntiles - 1) {
    out[n] = pre_s + total;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // every ticket is taken
  }
  __syncthreads();
  pre += pre_s;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    tile[scan_slot(threadIdx.x * kScanItems + j)] = pre;
    pre += v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    const uint32_t k = uint32_t(j) * kBlock + threadIdx.x;
    if (base + k < n) out[base + k] = tile[scan_slot(k)];
  }
}

template <typename T>
hipError_t excl_scan(hj3d_ctx* ctx, const T* in, T* out, uint64_t n, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(out, 0, sizeof(T), s);
  const uint64_t tiles = (n + kTile - 1) / kTile;
  hipError_t e = ctx->scratch[kScrScan].ensure((tiles + 1) * sizeof(T));
  if (e != hipSuccess) return e;
  T* sums = ctx->scratch[kScrScan].as<T>();
  hipLaunchKernelGGL(k_tile_sums<T>, dim3(unsigned(tiles)), dim3(kBlock), 0, s, in, n, sums);
  hipLaunchKernelGGL(k_scan_sums<T>, dim3(1), dim3(1024), 0, s, sums, tiles);
  hipLaunchKernelGGL(k_scan_tiles<T>, dim3(unsigned(tiles)), dim3(kBlock), 0, s, in, out, n, sums);
  return hipGetLastError();
}

// Column sums of per-block partials (NF u64 fields per row, xor for the last NXOR): every
// thread folds whole rows (coalesced 8*NF-byte reads), then one block reduction per field.
template <int NF, int NXOR>
__global__ __launch_bounds__(1024) void k_reduce_partials(const uint64_t* __restrict__ part, uint32_t nblocks,
                                                          uint64_t* __restrict__ res, uint64_t set0,
                                                          const uint64_t* __restrict__ base0) {
  __shared__ uint64_t red[16][NF];
  uint64_t acc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f] = 0;
  for (uint32_t b = threadIdx.x; b < nblocks; b += 1024) {
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const uint64_t v = part[uint64_t(b) * NF + f];
      acc[f] = f >= NF - NXOR ? (acc[f] ^ v) : (acc[f] + v);
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    uint64_t a = acc[f];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t w = __shfl_xor(a, o, kWave);
      a = f >= NF - NXOR ? (a ^ w) : (a + w);
    }
    if (lane == 0) red[wid][f] = a;
  }
  __syncthreads();
  const int f = int(threadIdx.x);
  if (f < NF) {
    const bool x = f >= NF - NXOR;
    uint64_t a = 0;
    for (int w = 0; w < 16; ++w) a = x ? (a ^ red[w][f]) : (a + red[w][f]);
    if (f == 0 && set0 != ~0ull) res[0] = set0 + (base0 ? *base0 : 0ull);
    else res[f] = x ? (res[f] ^ a) : (res[f] + a);
  }
}

}  // namespace

hipError_t reduce_partials(const uint64_t* partials, uint32_t nblocks, int nf, int nxor, uint64_t* res, hipStream_t s,
                           uint64_t set0, const uint64_t* base0) {
  if (nf != kProbeFields || nxor != 1) return hipErrorInvalidValue;  // the one shape in use
  hipLaunchKernelGGL((k_reduce_partials<kProbeFields, 1>), dim3(1), dim3(1024), 0, s, partials, nblocks, res, set0,
                     base0);
  return hipGetLastError();
}

hipError_t exclusive_scan_u32(hj3d_ctx* ctx, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(out, 0, sizeof(uint32_t), s);
  const uint64_t tiles = (n + kTile - 1) / kTile;
  if (tiles >= (1ull << 31)) return excl_scan<uint32_t>(ctx, in, out, n, s);
  DevBuf& st = ctx->scan_status;
  const size_t before = st.bytes;
  hipError_t e = st.ensure(tiles * sizeof(uint64_t));
  // fresh memory could hold a word that looks published for this epoch (stale u32 data of a
  // freed buffer often does): clear it whenever the buffer was reallocated. The test is on the
  // size, not the address: the allocator readily returns the freed block's address again.
  if (e == hipSuccess && st.bytes != before) e = hipMemsetAsync(st.p, 0, st.bytes, s);
  if (e == hipSuccess) e = ctx->ensure_ctl();
  if (e != hipSuccess) return e;
  // the ticket: a control word kept zero between calls (the last tile resets it)
  uint32_t* ticket = reinterpret_cast<uint32_t*>(ctx->ctl.as<uint64_t>() + kCtlScanTicket);
  ctx->scan_epoch = (ctx->scan_epoch + 1) & ((1u << 28) - 1);  // below the u64 form's flag bits
  if (ctx->scan_epoch == 0) {
    // wrapped: words published 2^28 calls ago carry epochs the next calls will use again, so the
    // buffer starts over from cleared memory (epoch 0) before epoch 1 is reused
    ctx->scan_epoch = 1;
    if ((e = hipMemsetAsync(st.p, 0, st.bytes, s)) != hipSuccess) return e;
  }
  const uint32_t epoch = ctx->scan_epoch;
  hipLaunchKernelGGL(k_scan_lb, dim3(unsigned(tiles)), dim3(kBlock), 0, s, in, out, n,
                     st.as<uint64_t>(), ticket, epoch, uint32_t(tiles));
  return hipGetLastError();
}
hipError_t exclusive_scan_u64(hj3d_ctx* ctx, const uint64_t* in, uint64_t* out, uint64_t n, hipStream_t s) {
  return excl_scan<uint64_t>(ctx, in, out, n, s);
}

namespace {
__global__ __launch_bounds__(256) void k_zero_words(ZeroList z) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
    for (uint32_t i = threadIdx.x; i < z.n[k]; i += 256) z.p[k][i] = 0;
}
}  // namespace

hipError_t zero_words(const ZeroList& z, hipStream_t s) {
  hipLaunchKernelGGL(k_zero_words, dim3(1), dim3(256), 0, s, z);
  return hipGetLastError();
}

}  // namespace hj3d

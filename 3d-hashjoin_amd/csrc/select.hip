// select.hip — selection pushdown: AlgSelection / AlgDynSelection (reference algebra.hh:278-358)
// evaluated on the device over a whole relation instead of one host predicate call per tuple.
//
// The reference's selection sits between AlgScan and a join operator and forwards the tuples
// whose predicate holds, in scan order (algebra.hh:295-300). Here the predicate is a
// conjunction of up to HJ3D_SEL_MAX comparisons of a u32 tuple word against constants, and the
// forwarded tuples become a stable, compacted (key, row) pair column: row = the tuple's row id in
// the scanned relation, so the join downstream (hj3d_build / hj3d_probe with row_off = 4) sees
// exactly the reference's input order and reports the reference's row identities.
//
// Two streaming passes over tiles of kSelTile tuples: count the passing tuples per tile, scan the
// tile counts, then re-evaluate and write every passing tuple at its tile offset + rank within
// the tile (wave ballots, one LDS exchange per tile). Algorithmic bytes: the predicate and key
// words read (8 B/tuple, 12-B AoS rows are read in full lines) + 8 B per passing tuple written.
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

constexpr int kSelItems = 16;                     // tuples per thread per tile
constexpr uint32_t kSelTile = kBlock * kSelItems;  // 4096

// Passing tuples per tile: one bitmask per thread (item j = tile + j*kBlock + thread).
__device__ __forceinline__ uint32_t sel_tile_mask(const RelView& r, const SelArgs& a, uint64_t tile0) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < kSelItems; ++j) {
    const uint64_t i = tile0 + uint64_t(j) * kBlock + threadIdx.x;
    if (i < r.n && sel_eval(r, a, i)) m |= 1u << j;
  }
  return m;
}

__global__ __launch_bounds__(kBlock) void k_sel_count(RelView r, SelArgs a, uint32_t* __restrict__ tile_cnt) {
  __shared__ uint32_t wsum[kBlock / kWave];
  const uint32_t m = sel_tile_mask(r, a, uint64_t(blockIdx.x) * kSelTile);
  uint32_t c = __popc(m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kBlock / kWave; ++w) t += wsum[w];
    tile_cnt[blockIdx.x] = t;
  }
}

// tile_off[0..ntiles] = exclusive scan of the tile counts (tile_off[ntiles] = total).
__global__ __launch_bounds__(kBlock) void k_sel_write(RelView r, SelArgs a, const uint32_t* __restrict__ tile_off,
                                                      uint32_t ntiles, uint2* __restrict__ out,
                                                      uint64_t* __restrict__ count) {
  constexpr int kW = kBlock / kWave;
  __shared__ uint32_t cnt[kSelItems][kW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t tile0 = uint64_t(blockIdx.x) * kSelTile;
  const uint32_t m = sel_tile_mask(r, a, tile0);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t rank[kSelItems];
#pragma unroll
  for (int j = 0; j < kSelItems; ++j) {
    const uint64_t b = __ballot((m >> j) & 1u);
    rank[j] = __popcll(b & below);
    if (lane == 0) cnt[j][wid] = __popcll(b);
  }
  __syncthreads();
  // position of (j, wave) in the tile: all of items < j first, then the lower waves at item j
  uint32_t base = tile_off[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kSelItems; ++j) {
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kW; ++w) {
      const uint32_t c = cnt[j][w];
      before += (w < wid) ? c : 0u;
      all += c;
    }
    if ((m >> j) & 1u) {
      const uint64_t i = tile0 + uint64_t(j) * kBlock + threadIdx.x;
      out[base + before + rank[j]] = make_uint2(r.key(i), r.row(i));
    }
    base += all;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *count = tile_off[ntiles];
}

}  // namespace

hipError_t select_pairs(hj3d_ctx* ctx, const hj3d_rel& rel, const hj3d_sel_pred* preds, uint32_t npred, void* out,
                        void* count, hipStream_t s) {
  if (rel.n == 0) return hipMemsetAsync(count, 0, sizeof(uint64_t), s);
  const SelArgs a = sel_args(preds, npred);
  const RelView r = view_of(rel);
  const uint64_t ntiles = (rel.n + kSelTile - 1) / kSelTile;
  hipError_t e = ctx->scratch[kScrD].ensure((ntiles + 1) * sizeof(uint32_t));
  if (e != hipSuccess) return e;
  uint32_t* tiles = ctx->scratch[kScrD].as<uint32_t>();
  hipLaunchKernelGGL(k_sel_count, dim3(unsigned(ntiles)), dim3(kBlock), 0, s, r, a, tiles);
  if ((e = exclusive_scan_u32(ctx, tiles, tiles, ntiles, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_sel_write, dim3(unsigned(ntiles)), dim3(kBlock), 0, s, r, a, tiles, uint32_t(ntiles),
                     static_cast<uint2*>(out), static_cast<uint64_t*>(count));
  return hipGetLastError();
}

}  // namespace hj3d

// radix.hip — radix-partitioned build and probe of the chaining table (the hot path).
//
// Why: a probe of the CSR table costs two dependent random reads (directory, entries). On
// MI355X such small random reads are served at ~55 G/s from the Infinity Cache (~250 G/s from
// L2), so a 1e8-probe strand against a 1e7 table is bound by random-access throughput at
// ~4 ms while streaming S itself takes 0.17 ms (micro/micro_probe.hip). The fix is the classic
// radix join, sized for CDNA4's 160 KB LDS:
//   partition: stream the tuples once to count, once to scatter (hash, row) pairs into P
//              partitions by bucket range (partition p owns local buckets [p*W, (p+1)*W));
//   probe:     one 1024-thread workgroup per partition copies its table slice (off + entries,
//              <= 144 KB, coalesced) into LDS and probes all of the partition's pairs against
//              LDS; results are written densely in partition order.
//   build:     same partitioning of R, then one workgroup per partition counts, scans and
//              scatters its slice of the global CSR directory in LDS: the table is the plain
//              CSR layout of chain.hip (probe-side partitioning is independent of the build).
// Bucket ranges keep the reference's per-bucket semantics (chain order, comparison counts,
// statistics) untouched: every counter is computed per bucket exactly as in chain.hip.
#include <cmath>

#include "radix_seg.hpp"

namespace hj3d {
namespace {

constexpr int kPBlock = 1024;                    // partition kernels: 16 waves
constexpr int kPRounds = 16;
constexpr int kPTile = kPBlock * kPRounds;       // 16384 tuples per partition tile
constexpr int kPRoundsR = 8;                     // k_rp_part1r: 8192-tuple tiles
constexpr int kPSeg = 16;                        // k_rp_part1r: 128-B region segments
constexpr double kProbeWFrac = 0.8;              // partitioned probes: slice width at this share of the LDS
// Build kernels load and store through the caches (non-temporal forms measured worse: R is read
// twice, the pairs re-read by the build and the table by the probe, all from the Infinity Cache).
__device__ __forceinline__ void put(uint2* p, uint2 e) { *p = e; }
__device__ __forceinline__ void put(uint32_t* p, uint32_t v) { *p = v; }
static_assert(kPTile == 1 << 14, "k_rp_scatter packs (partition, rank) as p << 14 | rank");
constexpr uint32_t kMaxParts = 2048;             // fan-out limit of one partition pass
constexpr uint32_t kBuildSlice = 16384;          // buckets per build partition (64 KB of LDS counters)
constexpr uint32_t kSortedMax = 32;             // buckets up to this size are kept sorted by row

struct FastDiv {  // exact floor(a / d) for u32 a, 1 <= d < 2^32
  uint64_t m;
  static FastDiv make(uint32_t d) {
    FastDiv f;
    f.m = ~uint64_t(0) / d + 1;
    return f;
  }
  __device__ __forceinline__ uint32_t div(uint32_t a) const { return d1 ? a : uint32_t(__umul64hi(m, uint64_t(a))); }
  bool d1 = false;
};
inline FastDiv make_div(uint32_t d) {
  FastDiv f = FastDiv::make(d);
  f.d1 = d == 1;
  return f;
}

// The tuples of one relation, or of two back to back (hj3d_build_many's two tables of one geometry,
// experiment 4's S and T: one partition pass for both): relation 1's tiles follow relation 0's
// (nt0 of them), its partitions follow at P + p and its pairs after relation 0's.
struct RelTiles {
  RelView r0, r1;
  uint32_t nt0;  // tiles of r0
  uint32_t P;    // partitions per relation
  uint32_t tsz = kPTile;  // tuples per tile
  __device__ __forceinline__ bool second(uint32_t tile) const { return tile >= nt0; }
  __device__ __forceinline__ const RelView& rel(uint32_t tile) const { return tile >= nt0 ? r1 : r0; }
  __device__ __forceinline__ uint64_t base(uint32_t tile) const {
    return uint64_t(tile >= nt0 ? tile - nt0 : tile) * tsz;
  }
  __device__ __forceinline__ uint32_t pofs(uint32_t tile) const { return tile >= nt0 ? P : 0u; }
};

// Partition sizes per scatter workgroup: workgroup g of the G = gridDim.x persistent workgroups
// counts the tiles g, g + G, ... that k_rp_scatter's workgroup g will write, then claims its run
// inside every partition with one atomic on the partition's cursor (cur[p] ends as the partition's
// size) and keeps the run's offset in its row hist[g * P + p]. The order of the workgroups' runs
// inside a partition is the atomics' order: no counter depends on it (build3 places rows by rank,
// the nested builds aggregate), and no scan over the P x G counts is needed.
template <int ROUNDS>
__global__ __launch_bounds__(kPBlock) void k_rp_hist(RelTiles rt, FastMod fm, uint32_t lo, uint32_t nbl, FastDiv fw,
                                                     uint32_t P, uint32_t ntiles, uint32_t* __restrict__ hist,
                                                     uint32_t* __restrict__ cur) {
  __shared__ uint32_t cnt[kMaxParts];
  for (uint32_t p = threadIdx.x; p < P; p += kPBlock) cnt[p] = 0;
  __syncthreads();
  uint32_t key[ROUNDS];
  auto load = [&](uint32_t tile) __attribute__((always_inline)) {
    const RelView& r = rt.rel(tile);
    const uint64_t b = rt.base(tile);
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {  // all loads of the tile in flight together
      const uint64_t i = b + uint64_t(j) * kPBlock + threadIdx.x;
      key[j] = tile < ntiles && i < r.n ? r.key(i) : 0u;
    }
  };
  load(blockIdx.x);
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const RelView& r = rt.rel(tile);
    const uint64_t b = rt.base(tile);
    const uint32_t pofs = rt.pofs(tile);
    uint32_t bl[ROUNDS];
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      const uint64_t i = b + uint64_t(j) * kPBlock + threadIdx.x;
      bl[j] = i < r.n ? fm.mod(murmur32(key[j])) - lo : nbl;
    }
    load(tile + gridDim.x);  // next tile: loads in flight
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j)
      if (bl[j] < nbl) atomicAdd(&cnt[pofs + fw.div(bl[j])], 1u);
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < P; p += kPBlock) {
    const uint32_t c = cnt[p];
    hist[uint64_t(blockIdx.x) * P + p] = c ? atomicAdd(&cur[p], c) : 0u;
  }
}

template <int BLOCK = kJBlock>
__device__ uint32_t lds_excl_scan(uint32_t* a, uint32_t n, uint32_t* wsum);

// Scatter (hash, row) pairs to their partitions. The tile is first ranked per partition with
// LDS atomics (order inside a partition is irrelevant to every counter), staged in LDS in
// partition order (128 KB), then written out so that consecutive lanes store consecutive
// addresses of one partition's run: ~16 elements = one 128-B line per partition and tile at
// the probe's fan-out, instead of one scattered 8-B store per tuple.
// Persistent over tiles (one workgroup per CU, LDS-bound): the next tile's keys are loaded
// before the current tile's write-out, so the CU's reads and writes overlap.
// Partition starts: an LDS scan of the P partition sizes (k_rp_hist's cursors) in every workgroup;
// workgroup 0 writes them to ps[0..P] and clears the other cursor set for the next call.
template <int ROUNDS>
__global__ __launch_bounds__(kPBlock) void k_rp_scatter(RelTiles rt, FastMod fm, uint32_t lo, uint32_t nbl, FastDiv fw,
                                                        uint32_t P, uint32_t ntiles, const uint32_t* __restrict__ offs,
                                                        const uint32_t* __restrict__ cur, uint32_t* __restrict__ cur_next,
                                                        uint32_t* __restrict__ ps, uint2* __restrict__ out) {
  constexpr int kTile = kPBlock * ROUNDS;
  __shared__ uint2 stage[kTile];
  __shared__ uint32_t loc[kMaxParts];   // local counts, then local run starts
  __shared__ uint32_t gb[kMaxParts];    // global run start of each partition for this tile
  // the scans' wave sums live in the stage: every scan runs while the stage holds nothing (before
  // the tile is staged; the previous tile's write-out ended at a barrier)
  uint32_t* wsum = reinterpret_cast<uint32_t*>(stage);
  // explicit row ids are loaded with the keys, a tile ahead (loading them at the stage write after
  // the ranking phase waited for every load separately: one round trip per tuple and round)
  // (relation 0's mode; a relation 1 of the other mode is still right: its rows come from r.row(i)
  // at the stage write when relation 0 is implicit, and r.row(i) resolves implicit rows otherwise)
  const bool explicit_rows = rt.r0.row_off != 0xFFFFFFFFu;
  uint32_t h[ROUNDS], rw[ROUNDS];
  auto load = [&](uint32_t tile) __attribute__((always_inline)) {
    const RelView& r = rt.rel(tile);
    const uint64_t b = rt.base(tile);
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      const uint64_t i = b + uint64_t(j) * kPBlock + threadIdx.x;
      const bool ok = tile < ntiles && i < r.n;
      h[j] = ok ? r.key(i) : 0u;
      rw[j] = explicit_rows && ok ? r.row(i) : 0u;
    }
  };
  load(blockIdx.x);
  // this workgroup's write cursor per partition: partition start + its run's offset (k_rp_hist)
  for (uint32_t p = threadIdx.x; p < P; p += kPBlock) gb[p] = cur[p];
  __syncthreads();
  const uint32_t total = lds_excl_scan<kPBlock>(gb, P, wsum);
  for (uint32_t p = threadIdx.x; p < P; p += kPBlock) {
    if (blockIdx.x == 0) ps[p] = gb[p];
    gb[p] += offs[uint64_t(blockIdx.x) * P + p];
  }
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) ps[P] = total;
    for (uint32_t p = threadIdx.x; p <= kMaxParts; p += kPBlock) cur_next[p] = 0;
  }
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    for (uint32_t p = threadIdx.x; p < P; p += kPBlock) loc[p] = 0;
    const RelView& r = rt.rel(tile);
    const uint64_t base = rt.base(tile);
    const uint32_t pofs = rt.pofs(tile);
    uint32_t rk[ROUNDS];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      const uint64_t i = base + uint64_t(j) * kPBlock + threadIdx.x;
      h[j] = murmur32(h[j]);
      const uint32_t bl = fm.mod(h[j]) - lo;
      if (i < r.n && bl < nbl) {  // rk = partition << 14 | rank in the tile's run (kPTile = 2^14)
        const uint32_t part = pofs + fw.div(bl);
        rk[j] = (part << 14) | atomicAdd(&loc[part], 1u);
      } else {
        rk[j] = kInvalid;
      }
    }
    __syncthreads();
    const uint32_t m = lds_excl_scan(loc, P, wsum);  // staged tuples of this tile
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      if (rk[j] == kInvalid) continue;
      const uint64_t i = base + uint64_t(j) * kPBlock + threadIdx.x;
      stage[loc[rk[j] >> 14] + (rk[j] & (kTile - 1))] = make_uint2(h[j], explicit_rows ? rw[j] : r.row(i));
    }
    __syncthreads();
    load(tile + gridDim.x);  // next tile: loads in flight
    for (uint32_t k = threadIdx.x; k < m; k += kPBlock) {
      const uint2 e = stage[k];
      const uint32_t p = pofs + fw.div(fm.mod(e.x) - lo);
      put(out + gb[p] + (k - loc[p]), e);
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < P; p += kPBlock)  // advance the cursors by the tile's runs
      gb[p] += (p + 1 < P ? loc[p + 1] : m) - loc[p];
    __syncthreads();
  }
}

// One launch for both passes of small inputs (k_rp_hist + k_rp_scatter fused; implicit rows): every
// workgroup takes at most TMAX tiles (g, g + G, ...), issues all their key loads at once, keeps the
// hashes in registers while it counts them per partition and claims its runs on the partition
// cursors, then waits at a grid barrier for every workgroup's claims (the partition sizes), scans
// the sizes in LDS and scatters the tiles from its registers as k_rp_scatter does. R is read once,
// not twice, and one launch boundary goes. The G workgroups are persistent (one per CU, the host
// checks the occupancy); the barrier is a monotonic arrival counter (target = the running sum of
// the grids launched on it), so it is never reset. A barrier that does not complete in ~0.2 s sets
// the timeout word and lets the workgroup go on (results wrong, flagged) instead of hanging.
// Phase 2 stages kFzGroup tiles per pass. One relation only (hj3d_build; hj3d_build_many's two
// relations keep the two launches: at config E, 4 tiles per workgroup, the fused form measured
// 66.9 against 19.4 + 43.8 us, at config B, 5 tiles, 87.0 against 26.4 + 67.5 us).
// (Phase 2 with one tile per staging pass: 0.1378 / 0.1386 against 0.1344 / 0.1346 ms build at
// config B, r05y_B; HJ3D_OPT_RP_UNFUSED keeps the two-launch form for A/B and its parity test.)
constexpr int kFzRounds = 8;
constexpr int kFzGroup = 2;  // tiles staged per pass of phase 2
constexpr int kFzTMax = 6;  // tiles per workgroup held in registers (48 hashes per thread)
// On a timeout the workgroup sets the context's word bar[1] (read with the probe results) and writes
// the launch's tag (the context's fused-launch sequence number) into the table's flag word `tflag`
// (its counts word 3, unused by chaining tables): the table getters compare that word with the tag
// the table was built under, so a later build's timeout never marks this table and this one's is
// never lost. `ticks`: the timeout in 100 MHz ticks; `skip0`: workgroup 0 does not arrive
// (diagnostic HJ3D_OPT_DIAG_GBAR: the barrier cannot complete, every workgroup times out).
struct FzBar {
  uint64_t* bar;
  uint64_t target;
  uint64_t* tflag;
  uint64_t tag;
  uint64_t ticks;
  uint32_t skip0;
};
__device__ __forceinline__ void grid_barrier(const FzBar& b) {
  __syncthreads();
  if (threadIdx.x == 0) {
    if (!(b.skip0 && blockIdx.x == 0)) __hip_atomic_fetch_add(b.bar, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(b.bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < b.target) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > b.ticks) {  // default 0.2 s at 100 MHz
        __hip_atomic_store(b.bar + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(b.tflag, b.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// 32-bit index math and branch-free 32-bit divisions (FastDiv32) keep the held hashes in registers:
// the bucket is h - (h / NB) NB - lo, the partition bucket / W.
struct FzGeom {
  FastDiv32 dnb, dw;
  uint32_t nb, lo, nbl, P;
  __device__ __forceinline__ uint32_t bucket(uint32_t h) const { return h - dnb.div(h) * nb - lo; }
};
template <int TMAX>
__global__ __launch_bounds__(kPBlock) void k_rp_fused(RelTiles rt, FzGeom fz, uint32_t ntiles, uint32_t* __restrict__ cur,
                                                      uint32_t* __restrict__ cur_next, uint32_t* __restrict__ ps,
                                                      uint2* __restrict__ out, FzBar fb) {
  constexpr int R = kFzRounds;
  constexpr int kTile = kPBlock * R;
  __shared__ uint2 stage[kTile * kFzGroup];
  __shared__ uint32_t loc[kMaxParts];  // phase 1: counts; then the partition starts; per tile: local runs
  __shared__ uint32_t gb[kMaxParts];   // this workgroup's write cursor per partition
  uint32_t* wsum = reinterpret_cast<uint32_t*>(stage);
  const uint32_t G = gridDim.x, P = fz.P, me = threadIdx.x;
  uint32_t hv[TMAX][R];
  for (uint32_t p = me; p < P; p += kPBlock) loc[p] = 0;
  // tuples of tile t left to this thread's item j: i = tile base + j * 1024 + me < n (32-bit counts)
  const auto nleft = [&](uint32_t tile) __attribute__((always_inline)) {
    const RelView& r = rt.rel(tile);
    const uint64_t b = rt.base(tile);
    return tile < ntiles && r.n > b ? uint32_t(min(r.n - b, uint64_t(kTile))) : 0u;
  };
  // every key load of the workgroup's tiles in flight together
#pragma unroll
  for (int t = 0; t < TMAX; ++t) {
    const uint32_t tile = blockIdx.x + uint32_t(t) * G;
    const RelView& r = rt.rel(tile);
    const uint32_t nl = nleft(tile);
    const char* tb = r.base + rt.base(tile) * r.stride + r.key_off;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t li = uint32_t(j) * kPBlock + me;
      hv[t][j] = li < nl ? (*reinterpret_cast<const uint32_t*>(tb + li * r.stride))
                         : 0u;
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < TMAX; ++t) {
    const uint32_t tile = blockIdx.x + uint32_t(t) * G;
    const uint32_t nl = nleft(tile), pofs = rt.pofs(tile);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      hv[t][j] = murmur32(hv[t][j]);
      const uint32_t bl = fz.bucket(hv[t][j]);
      if (uint32_t(j) * kPBlock + me < nl && bl < fz.nbl) atomicAdd(&loc[pofs + fz.dw.div(bl)], 1u);
    }
  }
  __syncthreads();
  for (uint32_t p = me; p < P; p += kPBlock) {
    const uint32_t c = loc[p];
    gb[p] = c ? atomicAdd(&cur[p], c) : 0u;  // this workgroup's run inside partition p
  }
  grid_barrier(fb);
  // partition sizes are final: starts by an LDS scan (the cursors read at L2, past this CU's cache)
  for (uint32_t p = me; p < P; p += kPBlock) loc[p] = __hip_atomic_load(cur + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint32_t total = lds_excl_scan<kPBlock>(loc, P, wsum);
  for (uint32_t p = me; p < P; p += kPBlock) {
    if (blockIdx.x == 0) ps[p] = loc[p];
    gb[p] += loc[p];
  }
  if (blockIdx.x == 0) {
    if (me == 0) ps[P] = total;
    for (uint32_t p = me; p <= kMaxParts; p += kPBlock) cur_next[p] = 0;
  }
  // phase 2: kFzGroup tiles per staging pass (fewer barriers and scans than one pass per tile)
#pragma unroll
  for (int t0 = 0; t0 < TMAX; t0 += kFzGroup) {
    if (blockIdx.x + uint32_t(t0) * G >= ntiles) break;
    __syncthreads();  // (the starts / the previous pass's cursor advance are read below)
    for (uint32_t p = me; p < P; p += kPBlock) loc[p] = 0;
    uint32_t rk[kFzGroup][R];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kFzGroup; ++u) {
      const int t = t0 + u < TMAX ? t0 + u : TMAX - 1;
      const uint32_t nl = t0 + u < TMAX ? nleft(blockIdx.x + uint32_t(t) * G) : 0u;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        // (opaque to the compiler: phase 1's buckets are not kept live across the barrier for reuse
        // here, which would hold a second register per item)
        asm volatile("" : "+v"(hv[t][j]));
        const uint32_t bl = fz.bucket(hv[t][j]);
        rk[u][j] = kInvalid;
        if (uint32_t(j) * kPBlock + me < nl && bl < fz.nbl) {
          const uint32_t part = fz.dw.div(bl);
          rk[u][j] = (part << 15) | atomicAdd(&loc[part], 1u);
        }
      }
    }
    __syncthreads();
    const uint32_t m = lds_excl_scan<kPBlock>(loc, P, wsum);
#pragma unroll
    for (int u = 0; u < kFzGroup; ++u) {
      const int t = t0 + u < TMAX ? t0 + u : TMAX - 1;
      const uint32_t rb = uint32_t(rt.r0.row_base + rt.base(blockIdx.x + uint32_t(t) * G));  // implicit rows
#pragma unroll
      for (int j = 0; j < R; ++j) {
        if (rk[u][j] == kInvalid) continue;
        stage[loc[rk[u][j] >> 15] + (rk[u][j] & 0x7FFFu)] = make_uint2(hv[t][j], rb + uint32_t(j) * kPBlock + me);
      }
    }
    __syncthreads();
    for (uint32_t k = me; k < m; k += kPBlock) {
      const uint2 e = stage[k];
      const uint32_t p = fz.dw.div(fz.bucket(e.x));
      put(out + gb[p] + (k - loc[p]), e);
    }
    __syncthreads();
    for (uint32_t p = me; p < P; p += kPBlock) gb[p] += (p + 1 < P ? loc[p + 1] : m) - loc[p];
  }
}

// The same scatter with WHOLE-SEGMENT write-out into the exact runs k_rp_hist claimed.
// k_rp_scatter writes each tile's run of a partition as it comes: at ~8 pairs per partition and
// tile nearly every run starts and ends inside a 64/128-B segment, and the two halves of such a
// segment reach the L2 from tiles written microseconds apart (the first half evicted by then):
// partial-line writes, 2.7 TB/s at config C. Here thread p owns partition p (and p + 1024 with
// PPT = 2): the pairs of a run that do not complete an aligned SEG-pair segment stay in its
// registers (the carry) and ride in front of the partition's next run, so every store the tiles
// issue covers a whole segment; only the first segment of the workgroup's run (which starts at the
// run's exact position: phantom lanes in front of it are skipped) and the last (flushed at the end)
// are partial -- the lines shared with the neighbouring workgroups' runs. This is k_pk_part's
// write-out (chain_pk.hip) on exact runs instead of fixed-capacity regions: skewed keys cannot
// overflow anything, and the output is one contiguous range per partition, as k_rp_scatter's.
// Tuples: the tiles of k_rp_hist (kPTile = 16384), as two 8192-tuple halves.
// PPT = 1: P <= 1024, 128-B segments; PPT = 2: P <= 2048, 64-B segments (a smaller carry).
// The build-side partition writes whole segments (k_rp_wscatter) from kRpWsMin tiles per
// partitioning workgroup on; below that the plain scatter (k_rp_scatter) on kRpSmallRounds x 1024-tuple
// tiles, one workgroup per CU (its ~100 VGPRs leave room for one).
constexpr uint32_t kRpWsMin = 4;
constexpr int kRpSmallRounds = 8;
constexpr int kWsRounds = 8;
constexpr int kWsSub = kPBlock * kWsRounds;  // 8192 tuples per half tile
template <int PPT>
struct WsGeom {
  static constexpr uint32_t kSeg = PPT == 1 ? 16u : 8u;
  static constexpr uint32_t kStage = PPT == 1 ? 17408u : 15360u;  // the half tile + carries (pairs)
};
template <int PPT, bool EXPL>
__global__ __launch_bounds__(kPBlock) void k_rp_wscatter(RelTiles rt, FastMod fm, uint32_t lo, uint32_t nbl, FastDiv fw,
                                                         uint32_t P, uint32_t ntiles, const uint32_t* __restrict__ offs,
                                                         const uint32_t* __restrict__ cur, uint32_t* __restrict__ cur_next,
                                                         uint32_t* __restrict__ ps, uint2* __restrict__ out) {
  constexpr uint32_t SEG = WsGeom<PPT>::kSeg, STAGE = WsGeom<PPT>::kStage;
  __shared__ uint2 stage[STAGE];
  __shared__ uint32_t loc[kPBlock * PPT];    // per partition: rank counter of the half tile
  __shared__ uint32_t sbase[kPBlock * PPT];  // per partition: stage slot of the half tile's first pair
  __shared__ uint2 seginfo[STAGE / SEG];     // whole segment: {output index, stage start | skip << 16}
  __shared__ uint32_t wsum[kPBlock / kWave];
  const uint32_t me = threadIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // partition starts (scan of the sizes k_rp_hist left in cur), published by workgroup 0
  for (uint32_t p = me; p < P; p += kPBlock) loc[p] = cur[p];
  __syncthreads();
  const uint32_t total = lds_excl_scan<kPBlock>(loc, P, wsum);
  if (blockIdx.x == 0) {
    for (uint32_t p = me; p < P; p += kPBlock) ps[p] = loc[p];
    if (me == 0) ps[P] = total;
    for (uint32_t p = me; p <= kMaxParts; p += kPBlock) cur_next[p] = 0;
  }
  // per owned partition: output cursor (segment-aligned after the first segment), carried pairs
  // (the first `skip` of them phantoms standing for the run's unaligned start)
  uint32_t my_cur[PPT], my_kc[PPT], my_skip[PPT];
  uint2 creg[PPT][SEG - 1];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const uint32_t p = me + k * kPBlock;
    const uint32_t st = p < P ? loc[p] + offs[uint64_t(blockIdx.x) * P + p] : 0u;
    my_skip[k] = st % SEG;
    my_cur[k] = st - my_skip[k];
    my_kc[k] = my_skip[k];
#pragma unroll
    for (int j = 0; j < int(SEG) - 1; ++j) creg[k][j] = make_uint2(0, 0);
  }
  __syncthreads();
  for (uint32_t p = me; p < kPBlock * PPT; p += kPBlock) loc[p] = 0;
  __syncthreads();  // (the first half tile's rank atomics)
  uint32_t h[kWsRounds], rw[EXPL ? kWsRounds : 1];
  // half `hf` of tile `tile`
  auto load = [&](uint32_t tile, uint32_t hf) __attribute__((always_inline)) {
    const RelView& r = rt.rel(tile);
    const uint64_t base = rt.base(tile) + uint64_t(hf) * kWsSub;
#pragma unroll
    for (int j = 0; j < kWsRounds; ++j) {
      const uint64_t i = base + uint64_t(j) * kPBlock + me;
      h[j] = i < r.n ? r.key(i) : 0u;
      if constexpr (EXPL) rw[j] = i < r.n ? r.row(i) : 0u;
    }
  };
  auto flush_carry = [&]() __attribute__((always_inline)) {  // the partial segments at the cursors
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
#pragma unroll
      for (int j = 0; j < int(SEG) - 1; ++j)
        if (uint32_t(j) < my_kc[k] && uint32_t(j) >= my_skip[k]) out[my_cur[k] + j] = creg[k][j];
      my_cur[k] += my_kc[k];
      my_kc[k] = 0;
      my_skip[k] = 0;
    }
  };
  auto scan = [&](uint32_t v, uint32_t* tot) __attribute__((always_inline)) {
    uint32_t wt;
    const uint32_t pre = wave_excl_scan(v, &wt);
    if (lane == 0) wsum[wid] = wt;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kPBlock / kWave; ++w) {
      const uint32_t t = wsum[w];
      base += w < wid ? t : 0u;
      all += t;
    }
    __syncthreads();
    *tot = all;
    return base + pre;
  };
  // half `hf` of tile `tile`; the next half tile's keys (ntile, nhf; ntile >= ntiles: none) are
  // loaded once this one is staged, so the loads overlap the write-out
  auto process = [&](uint32_t tile, uint32_t hf, uint32_t ntile, uint32_t nhf) __attribute__((always_inline)) {
    const RelView& r = rt.rel(tile);
    const uint64_t base = rt.base(tile) + uint64_t(hf) * kWsSub;
    const uint32_t pofs = rt.pofs(tile);
    uint32_t rk[kWsRounds];  // partition << 13 | rank in the half tile
#pragma unroll
    for (int j = 0; j < kWsRounds; ++j) {
      const uint64_t i = base + uint64_t(j) * kPBlock + me;
      h[j] = murmur32(h[j]);
      const uint32_t bl = fm.mod(h[j]) - lo;
      rk[j] = kInvalid;
      if (i < r.n && bl < nbl) {
        const uint32_t p = pofs + fw.div(bl);
        rk[j] = (p << 13) | atomicAdd(&loc[p], 1u);
      }
    }
    __syncthreads();
    uint32_t c[PPT], L[PPT], pack = 0;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const uint32_t p = me + k * kPBlock;
      c[k] = p < P ? loc[p] : 0u;
      loc[p] = 0;  // read once per half tile; the next writes come after the next ranking barrier
      L[k] = my_kc[k] + c[k];
      pack += (L[k] << 16) | (L[k] / SEG);
    }
    uint32_t tot;
    uint32_t pre = scan(pack, &tot);
    if ((tot >> 16) > STAGE) {  // the carries and the half tile exceed the stage: carries out first (rare)
      flush_carry();
      pack = 0;
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        L[k] = c[k];
        pack += (L[k] << 16) | (L[k] / SEG);
      }
      pre = scan(pack, &tot);
    }
    const uint32_t nfull = tot & 0xFFFFu;
    uint32_t at = pre >> 16, fseg = pre & 0xFFFFu;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const uint32_t p = me + k * kPBlock;
      if (p < P) {
        sbase[p] = at + my_kc[k];
#pragma unroll
        for (int j = 0; j < int(SEG) - 1; ++j)
          if (uint32_t(j) < my_kc[k]) stage[at + j] = creg[k][j];
        for (uint32_t sg = 0; sg < L[k] / SEG; ++sg)
          seginfo[fseg + sg] = make_uint2(my_cur[k] + sg * SEG, (at + sg * SEG) | ((sg == 0 ? my_skip[k] : 0u) << 16));
      }
      at += L[k];
      fseg += L[k] / SEG;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kWsRounds; ++j) {
      if (rk[j] == kInvalid) continue;
      const uint64_t i = base + uint64_t(j) * kPBlock + me;
      uint32_t row;
      if constexpr (EXPL) row = rw[j];
      else row = uint32_t(r.row_base + i);
      stage[sbase[rk[j] >> 13] + (rk[j] & (kWsSub - 1))] = make_uint2(h[j], row);
    }
    if (ntile < ntiles) load(ntile, nhf);
    __syncthreads();
    for (uint32_t kk = me; kk < nfull * SEG; kk += kPBlock) {
      const uint2 si = seginfo[kk / SEG];
      const uint32_t j = kk % SEG;
      const uint2 e = stage[(si.y & 0xFFFFu) + j];
      if (j >= (si.y >> 16)) put(out + si.x + j, e);
    }
    // each run's tail (< one segment) becomes the partition's carry. (The next half tile's first
    // stage / seginfo writes follow its ranking barrier, which every thread reaches only after
    // these reads: no barrier here.)
    at = pre >> 16;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const uint32_t F = L[k] - L[k] % SEG;
#pragma unroll
      for (int j = 0; j < int(SEG) - 1; ++j)
        if (uint32_t(j) < L[k] - F) creg[k][j] = stage[at + F + j];
      if (F) my_skip[k] = 0;
      my_cur[k] += F;
      my_kc[k] = L[k] - F;
      at += L[k];
    }
  };
  if (blockIdx.x < ntiles) load(blockIdx.x, 0);
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    process(tile, 0, tile, 1);
    process(tile, 1, tile + gridDim.x, 0);
  }
  flush_carry();
}

// Block-wide exclusive scan of a[0..n) in LDS (in place); returns the total. BLOCK threads.
template <int BLOCK>
__device__ uint32_t lds_excl_scan(uint32_t* a, uint32_t n, uint32_t* wsum) {
  const uint32_t per = (n + BLOCK - 1) / BLOCK;
  const uint32_t beg = threadIdx.x * per;
  const uint32_t end = min(beg + per, n);
  uint32_t local = 0;
  for (uint32_t k = beg; k < end; ++k) local += a[k];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t wpre = 0, tot = 0;
  for (int w = 0; w < BLOCK / kWave; ++w) {
    const uint32_t v = wsum[w];
    if (w < wid) wpre += v;
    tot += v;
  }
  uint32_t run = wpre + x - local;
  for (uint32_t k = beg; k < end; ++k) {
    const uint32_t v = a[k];
    a[k] = run;
    run += v;
  }
  __syncthreads();
  return tot;
}

// One workgroup per build partition: local count -> scan -> scatter of the CSR slice.
__global__ __launch_bounds__(kJBlock) void k_rp_build(const uint2* __restrict__ pairs, const uint32_t* __restrict__ ps,
                                                      FastMod fm, uint32_t lo, uint32_t nbl, uint32_t W,
                                                      uint32_t* __restrict__ off, uint2* __restrict__ ent) {
  __shared__ uint32_t cnt[kBuildSlice];
  __shared__ uint32_t wsum[kJBlock / kWave];
  const uint32_t p = blockIdx.x;
  const uint32_t b0 = p * W;
  const uint32_t nbs = min(W, nbl - b0);
  const uint32_t s0 = ps[p], s1 = ps[p + 1];
  for (uint32_t k = threadIdx.x; k < nbs; k += kJBlock) cnt[k] = 0;
  __syncthreads();
  for (uint32_t i = s0 + threadIdx.x; i < s1; i += kJBlock) atomicAdd(&cnt[fm.mod(pairs[i].x) - lo - b0], 1u);
  __syncthreads();
  lds_excl_scan(cnt, nbs, wsum);
  for (uint32_t k = threadIdx.x; k < nbs; k += kJBlock) off[b0 + k] = s0 + cnt[k];
  if (b0 + nbs == nbl && threadIdx.x == 0) off[nbl] = s1;
  __syncthreads();
  for (uint32_t i = s0 + threadIdx.x; i < s1; i += kJBlock) {
    const uint2 e = pairs[i];
    const uint32_t pos = atomicAdd(&cnt[fm.mod(e.x) - lo - b0], 1u);
    ent[s0 + pos] = e;
  }
}

// Staged build partitions: kBuildSlice2 buckets, at most kBuildStage pairs through LDS.
constexpr uint32_t kBuildSlice2 = 8192;
constexpr uint32_t kBuildSlice2Max = 10240;  // wider slices keep the partition count <= 1024 (k_rp_wscatter<1>)
constexpr uint32_t kBuildStage = 14400;

// The staged build as a persistent kernel (one 1024-thread workgroup per CU takes partitions
// blockIdx.x, blockIdx.x + gridDim.x, ...): the next partition's pairs are loaded into registers
// while the current one is built, so a CU never idles on a partition's first loads. Per partition
// of <= kB3Per * 1024 pairs: count per bucket with LDS atomics (each pair keeps its arrival rank),
// scan to bucket starts (-> the directory slice), stage every pair at start + arrival rank, then
// every staged pair takes its final slot = bucket start + the rank of its row among the bucket's
// rows (buckets of 2..kSortedMax entries come out sorted by row, with no sort pass; longer ones
// stay in arrival order) and is written to the CSR. Larger partitions (skewed keys) scatter
// through HBM instead (sorting their small buckets there).
constexpr int kB3Per = 12;  // pairs per thread held in registers: partitions up to 12 * BLOCK pairs
// One 1024-thread workgroup per CU, slices up to WMAX buckets, STAGE pairs of LDS stage. (Two
// 512-thread workgroups per CU on half-width slices measured slower: build 0.191 against 0.164 ms.)
template <int BLOCK, uint32_t WMAX, uint32_t STAGE>
__global__ __launch_bounds__(BLOCK) void k_rp_build3(const uint2* __restrict__ pairs, const uint32_t* __restrict__ ps,
                                                     FastMod fm, uint32_t lo, uint32_t nbl, uint32_t W, uint32_t P,
                                                     uint32_t* __restrict__ off, uint2* __restrict__ ent) {
  __shared__ uint32_t cnt[WMAX + 1];
  __shared__ uint2 stage[STAGE];
  __shared__ uint32_t wsum[BLOCK / kWave];
  constexpr uint32_t kCap = kB3Per * BLOCK;
  static_assert(kCap <= STAGE, "a register-held partition must fit the stage");
  uint2 ea[kB3Per], eb[kB3Per];
  auto load = [&](uint2 (&e)[kB3Per], uint32_t p) __attribute__((always_inline)) {
    if (p >= P) return;
    const uint32_t s0 = ps[p], s1 = ps[p + 1];
    if (s1 - s0 > kCap) return;
#pragma unroll
    for (int u = 0; u < kB3Per; ++u) {
      const uint32_t i = s0 + u * BLOCK + threadIdx.x;
      e[u] = i < s1 ? pairs[i] : make_uint2(0, 0);
    }
  };
  auto build = [&](uint2 (&e)[kB3Per], uint32_t p) __attribute__((always_inline)) {
    const uint32_t b0 = p * W;
    const uint32_t nbs = min(W, nbl - b0);
    const uint32_t s0 = ps[p], s1 = ps[p + 1], m = s1 - s0;
    for (uint32_t k = threadIdx.x; k < nbs; k += BLOCK) cnt[k] = 0;
    __syncthreads();
    if (m > kCap) {  // skewed partition: scatter through HBM, sort the small buckets there
      for (uint32_t i = s0 + threadIdx.x; i < s1; i += BLOCK) atomicAdd(&cnt[fm.mod(pairs[i].x) - lo - b0], 1u);
      __syncthreads();
      lds_excl_scan<BLOCK>(cnt, nbs, wsum);
      for (uint32_t k = threadIdx.x; k < nbs; k += BLOCK) off[b0 + k] = s0 + cnt[k];
      if (b0 + nbs == nbl && threadIdx.x == 0) off[nbl] = s1;
      __syncthreads();
      for (uint32_t i = s0 + threadIdx.x; i < s1; i += BLOCK) {
        const uint2 x = pairs[i];
        ent[s0 + atomicAdd(&cnt[fm.mod(x.x) - lo - b0], 1u)] = x;
      }
      __syncthreads();
      for (uint32_t k = threadIdx.x; k < nbs; k += BLOCK) {
        const uint32_t bs = k ? cnt[k - 1] : 0u, n = cnt[k] - bs;
        if (n < 2 || n > kSortedMax) continue;
        uint2* E = ent + s0 + bs;
        for (uint32_t q = 1; q < n; ++q) {
          const uint2 x = E[q];
          uint32_t j = q;
          while (j > 0 && E[j - 1].y > x.y) {
            E[j] = E[j - 1];
            --j;
          }
          E[j] = x;
        }
      }
      __syncthreads();
      return;
    }
    uint32_t rk[kB3Per];  // bucket << 16 | arrival rank (W <= 2^16, ranks < 2^16)
#pragma unroll
    for (int u = 0; u < kB3Per; ++u) {
      const bool v = u * BLOCK + threadIdx.x < m;
      const uint32_t b = v ? fm.mod(e[u].x) - lo - b0 : 0u;
      rk[u] = v ? (b << 16) | atomicAdd(&cnt[b], 1u) : kInvalid;
    }
    __syncthreads();
    lds_excl_scan<BLOCK>(cnt, nbs, wsum);
    if (threadIdx.x == 0) cnt[nbs] = m;
    for (uint32_t k = threadIdx.x; k < nbs; k += BLOCK) put(off + b0 + k, s0 + cnt[k]);
    if (b0 + nbs == nbl && threadIdx.x == 0) off[nbl] = s1;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kB3Per; ++u)
      if (rk[u] != kInvalid) stage[cnt[rk[u] >> 16] + (rk[u] & 0xFFFFu)] = e[u];
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < m; q += BLOCK) {
      const uint2 x = stage[q];
      const uint32_t b = fm.mod(x.x) - lo - b0;
      const uint32_t bs = cnt[b], n = cnt[b + 1] - bs;
      uint32_t pos = q;
      if (n >= 2 && n <= kSortedMax) {
        uint32_t r = 0;
        for (uint32_t k = bs; k < bs + n; ++k) r += stage[k].y < x.y;
        pos = bs + r;
      }
      put(ent + s0 + pos, x);
    }
    __syncthreads();
  };
  load(ea, blockIdx.x);
  for (uint32_t p = blockIdx.x; p < P; p += 2 * gridDim.x) {
    load(eb, p + gridDim.x);
    build(ea, p);
    if (p + gridDim.x >= P) break;
    load(ea, p + 2 * gridDim.x);
    build(eb, p + gridDim.x);
  }
}

enum Mode { kAgg = 0, kDense = 1, kCount = 2, kWrite = 3 };

// Reference comparison count and match of one probe against bucket entries [s, s+n) of `E`
// (LDS or global). Buckets of <= kSortedMax entries are sorted by row (k_sort_small_buckets), so
// the reference's walk [first insert, newest, ..., second insert] is sorted index 0, n-1, ..., 1
// and the unique form stops at its first match like the reference (a wave runs the longest
// match position of its lanes, not the longest bucket). Longer buckets use the order-free
// two-pass form of chain.hip. CK: fold output checksums.
template <bool UNIQUE, int MODE, bool CK, typename EntT>
__device__ __forceinline__ void probe_bucket(uint32_t h, uint32_t pr, const EntT* E, uint32_t s, uint32_t n,
                                             uint64_t (&acc)[kProbeFields], uint64_t i, uint2* __restrict__ out,
                                             uint64_t out_cap, uint64_t* __restrict__ cnt) {
  if (MODE != kWrite) acc[0] += 1;
  if (UNIQUE) {
    uint32_t match = kInvalid, cmps = 0;
    if (n <= kSortedMax) {
      // the reference's walk itself, stopping at the first match: sorted index 0, n-1, ..., 1
      cmps = n;
      for (uint32_t c = 0; c < n; ++c) {
        const uint2 e = E[s + (c == 0 ? 0u : n - c)];
        if (e.x == h) {
          cmps = c + 1;
          match = e.y;
          break;
        }
      }
    } else {
      uint32_t minrow = kInvalid, lo_m = kInvalid, hi_m = 0, nm = 0;
      for (uint32_t k = s; k < s + n; ++k) {
        const uint2 e = E[k];
        minrow = min(minrow, e.y);
        if (e.x == h) {
          ++nm;
          lo_m = min(lo_m, e.y);
          hi_m = max(hi_m, e.y);
        }
      }
      if (nm == 0) {
        cmps = n;
      } else if (lo_m == minrow) {
        cmps = 1;
        match = lo_m;
      } else {
        uint32_t gt = 0;
        for (uint32_t k = s; k < s + n; ++k) gt += E[k].y > hi_m;
        cmps = 2 + gt;
        match = hi_m;
      }
    }
    if (MODE != kWrite) acc[3] += cmps;
    if (MODE == kDense) {
      if (i < out_cap)
        __builtin_nontemporal_store((uint64_t(match) << 32) | pr, reinterpret_cast<uint64_t*>(out + i));
    }
    if (match != kInvalid) {
      if (MODE == kWrite) {
        const uint64_t o = cnt[i];
        if (o < out_cap) out[o] = make_uint2(pr, match);
      } else {
        acc[1] += 1;
        acc[2] += 1;
        if (CK) {
          acc[4] += pr;
          acc[5] += match;
          const uint64_t ph = pair_hash(pr, match);
          acc[7] += ph;
          acc[8] ^= ph;
        }
      }
    }
    if (MODE == kCount) cnt[i] = match != kInvalid;
  } else {
    if (MODE != kWrite) acc[3] += n;
    uint64_t o = (MODE == kWrite) ? cnt[i] : 0;
    uint32_t nout = 0;
    for (uint32_t k = s; k < s + n; ++k) {
      const uint2 e = E[k];
      if (e.x != h) continue;
      ++nout;
      if (MODE == kWrite) {
        if (o < out_cap) out[o] = make_uint2(pr, e.y);
        ++o;
      } else if (CK) {
        acc[4] += pr;
        acc[5] += e.y;
        const uint64_t ph = pair_hash(pr, e.y);
        acc[7] += ph;
        acc[8] ^= ph;
      }
    }
    if (MODE != kWrite) {
      acc[1] += nout != 0;
      acc[2] += nout;
    }
    if (MODE == kCount) cnt[i] = nout;
  }
}

// probe_bucket for the kSegItems pairs of one lane at once (unique probe against an LDS slice,
// the hot path of config B): the directory words of all items are read together, then walk
// position c = 0, 1, 2 of every item still unmatched (sorted index 0, n-1, n-2) as one batch of
// independent LDS reads per position, so a chunk costs a few LDS latencies instead of one
// dependent chain per item. Positions >= 3 (buckets of >= 4 entries) and unsorted long buckets
// (> kSortedMax) finish per item. Counters identical to probe_bucket<true, MODE, CK>.
template <int MODE, bool CK, int NG>
__device__ __forceinline__ void probe_group_unique(const uint64_t (&v)[kSegItems], const uint64_t (&slot)[kSegItems],
                                                   uint32_t valid, int g, const uint32_t* loff, const uint2* lent,
                                                   FastMod fm, uint32_t lob0, uint64_t (&acc)[kProbeFields],
                                                   uint2* __restrict__ out, uint64_t out_cap) {
  static_assert(MODE == kDense || MODE == kAgg, "unique dense / aggregate forms only");
  // branch-free: every lane reads LDS (absent items read word 0) and selects afterwards
  uint32_t d[NG], match[NG], cmps[NG];
  bool live[NG];
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    const bool ok = (valid >> (g + j)) & 1u;
    const uint32_t w = loff[ok ? fm.mod(uint32_t(v[g + j])) - lob0 : 0u];
    d[j] = ok ? w : 0u;
  }
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    const uint32_t n = d[j] & 0xFFFFu;
    match[j] = kInvalid;
    cmps[j] = n;
    live[j] = n != 0 && n <= kSortedMax;
  }
#pragma unroll
  for (uint32_t c = 0; c < 3; ++c) {
    uint2 e[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const uint32_t n = d[j] & 0xFFFFu;
      const bool ok = live[j] && c < n;
      e[j] = lent[ok ? (d[j] >> 16) + (c == 0 ? 0u : n - c) : 0u];
      const bool hit = ok && e[j].x == uint32_t(v[g + j]);
      match[j] = hit ? e[j].y : match[j];
      cmps[j] = hit ? c + 1 : cmps[j];
      live[j] = live[j] && !hit;
    }
  }
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    const uint32_t h = uint32_t(v[g + j]), n = d[j] & 0xFFFFu, s = d[j] >> 16;
    if (live[j] && n > 3) {
      for (uint32_t c = 3; c < n; ++c) {
        const uint2 e = lent[s + n - c];
        if (e.x == h) {
          cmps[j] = c + 1;
          match[j] = e.y;
          break;
        }
      }
    } else if (n > kSortedMax) {  // order-free form of probe_bucket
      uint32_t minrow = kInvalid, lo_m = kInvalid, hi_m = 0, nm = 0;
      for (uint32_t k = s; k < s + n; ++k) {
        const uint2 e = lent[k];
        minrow = min(minrow, e.y);
        if (e.x == h) {
          ++nm;
          lo_m = min(lo_m, e.y);
          hi_m = max(hi_m, e.y);
        }
      }
      if (nm != 0 && lo_m == minrow) {
        cmps[j] = 1;
        match[j] = lo_m;
      } else if (nm != 0) {
        uint32_t gt = 0;
        for (uint32_t k = s; k < s + n; ++k) gt += lent[k].y > hi_m;
        cmps[j] = 2 + gt;
        match[j] = hi_m;
      }
    }
  }
  uint32_t nv = 0, nm = 0, sc = 0;  // per-group sums, folded into the u64 accumulators once
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    const bool ok = (valid >> (g + j)) & 1u;
    const uint32_t pr = uint32_t(v[g + j] >> 32);
    nv += ok;
    sc += cmps[j];  // 0 for absent items (d = 0)
    const bool m = match[j] != kInvalid;
    nm += m;
    if (MODE == kDense && ok && slot[g + j] < out_cap)
      __builtin_nontemporal_store((uint64_t(match[j]) << 32) | pr, reinterpret_cast<uint64_t*>(out + slot[g + j]));
    if (CK && m) {
      acc[4] += pr;
      acc[5] += match[j];
      const uint64_t ph = pair_hash(pr, match[j]);
      acc[7] += ph;
      acc[8] ^= ph;
    }
  }
  acc[0] += nv;
  acc[1] += nm;
  acc[2] += nm;
  acc[3] += sc;
}

// Items are taken in groups of NG (register pressure: 4 independent lookups per LDS round).
template <int MODE, bool CK, int NG = 4>
__device__ __forceinline__ void probe_chunk_unique(const uint64_t (&v)[kSegItems], const uint64_t (&slot)[kSegItems],
                                                   uint32_t valid, const uint32_t* loff, const uint2* lent,
                                                   FastMod fm, uint32_t lob0, uint64_t (&acc)[kProbeFields],
                                                   uint2* __restrict__ out, uint64_t out_cap) {
  static_assert(kSegItems % NG == 0, "groups of NG items");
#pragma unroll
  for (int g = 0; g < kSegItems; g += NG)
    probe_group_unique<MODE, CK, NG>(v, slot, valid, g, loff, lent, fm, lob0, acc, out, out_cap);
}
// Copy the table slice of buckets [b0, b0 + nbs) into LDS: directory word k = (start of bucket k
// relative to the slice) << 16 | (its entry count) (both < 2^16: a slice holds < 18432 entries),
// then the entries. Every load of a batch of kStage rounds (directory AND entries: a whole
// typical slice) is issued before the first LDS write, so staging costs one memory latency
// rather than one per round.
__device__ __forceinline__ void stage_slice(const uint32_t* __restrict__ off, const uint2* __restrict__ ent, uint32_t b0,
                                            uint32_t nbs, uint32_t e0, uint32_t ne, uint32_t* ldir, uint2* lent) {
  constexpr int kStage = 12;
  const uint64_t* src = reinterpret_cast<const uint64_t*>(ent + e0);
  uint64_t* dst = reinterpret_cast<uint64_t*>(lent);
  const uint32_t nmax = max(nbs, ne);
  for (uint32_t k0 = threadIdx.x; k0 < nmax; k0 += kJBlock * kStage) {
    uint32_t v[kStage], w[kStage];
    uint64_t x[kStage];
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const uint32_t k = k0 + u * kJBlock;
      v[u] = k < nbs ? off[b0 + k] : 0u;
      w[u] = k < nbs ? off[b0 + k + 1] : 0u;
      x[u] = k < ne ? src[k] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const uint32_t k = k0 + u * kJBlock;
      if (k < nbs) ldir[k] = ((v[u] - e0) << 16) | (w[u] - v[u]);
      if (k < ne) dst[k] = x[u];
    }
  }
}

// ---- single-pass probe-side partitioning (no histogram pass) ----
// Persistent workgroup g owns, for every partition p, a private region of `cap` pairs
// (region[(g * P + p) * cap ...]) and its fill cursor in LDS. Per tile: rank per partition (LDS
// atomics), stage in partition order (LDS), write each partition's run at the cursor. A run that
// does not fit (skewed probe keys) goes to the overflow list, probed by k_probe_ovf. S is read
// once instead of twice (histogram + scatter). IMPLICIT (row id = row_base + index): the stage
// holds {hash, partition << 16 | tile index} so the write-out needs no second modulo/division.
template <int BLOCK, int ROUNDS, int MAXP, bool IMPLICIT>
__global__ __launch_bounds__(BLOCK) void k_rp_part1(RelView r, FastMod fm, uint32_t lo, uint32_t nbl, FastDiv fw,
                                                    uint32_t P, uint32_t ntiles, uint32_t cap,
                                                    uint2* __restrict__ region, uint32_t* __restrict__ counts,
                                                    uint2* __restrict__ ovf, unsigned long long* __restrict__ novf) {
  constexpr int TILE = BLOCK * ROUNDS;
  constexpr int TBITS = __builtin_ctz(TILE);
  static_assert((TILE & (TILE - 1)) == 0 && TILE <= (1 << 16), "tile must be a power of two");
  static_assert(MAXP < (1 << 16), "partition ids are packed into 16 bits");
  __shared__ uint2 stage[TILE];
  __shared__ uint32_t loc[MAXP + 1];  // tile counts, then tile-local run starts (loc[P] = tile size)
  __shared__ uint32_t cur[MAXP];      // region fill of each partition
  __shared__ uint32_t wsum[BLOCK / kWave];
  const uint64_t gbase = uint64_t(blockIdx.x) * P;
  for (uint32_t p = threadIdx.x; p < P; p += BLOCK) cur[p] = 0;
  uint32_t h[ROUNDS];
  uint32_t rw[IMPLICIT ? 1 : ROUNDS];  // explicit row ids, loaded with the keys a tile ahead
#pragma unroll
  for (int j = 0; j < ROUNDS; ++j) {
    const uint64_t i = uint64_t(blockIdx.x) * TILE + uint64_t(j) * BLOCK + threadIdx.x;
    h[j] = i < r.n ? r.key(i) : 0u;
    if constexpr (!IMPLICIT) rw[j] = i < r.n ? r.row(i) : 0u;
  }
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    for (uint32_t p = threadIdx.x; p < P; p += BLOCK) loc[p] = 0;
    const uint64_t base = uint64_t(tile) * TILE;
    uint32_t rk[ROUNDS];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      const uint64_t i = base + uint64_t(j) * BLOCK + threadIdx.x;
      h[j] = murmur32(h[j]);
      const uint32_t bl = fm.mod(h[j]) - lo;
      if (i < r.n && bl < nbl) {
        const uint32_t part = fw.div(bl);
        rk[j] = (part << TBITS) | atomicAdd(&loc[part], 1u);
      } else {
        rk[j] = kInvalid;
      }
    }
    __syncthreads();
    const uint32_t m = lds_excl_scan<BLOCK>(loc, P, wsum);
    if (threadIdx.x == 0) loc[P] = m;
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      if (rk[j] == kInvalid) continue;
      const uint32_t li = uint32_t(j) * BLOCK + threadIdx.x;
      uint32_t y = ((rk[j] >> TBITS) << 16) | li;
      if constexpr (!IMPLICIT) y = rw[j];
      stage[loc[rk[j] >> TBITS] + (rk[j] & (TILE - 1))] = make_uint2(h[j], y);
    }
    __syncthreads();
    const uint64_t nbase = uint64_t(tile + gridDim.x) * TILE;  // next tile: loads in flight
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      const uint64_t i = nbase + uint64_t(j) * BLOCK + threadIdx.x;
      h[j] = i < r.n ? r.key(i) : 0u;
      if constexpr (!IMPLICIT) rw[j] = i < r.n ? r.row(i) : 0u;
    }
    // kOutU staged pairs per thread and step: their LDS reads and stores are independent, so the
    // step exposes kOutU-way parallelism instead of one dependent LDS -> LDS -> store chain
    constexpr int kOutU = 4;
    for (uint32_t k0 = 0; k0 < m; k0 += kOutU * BLOCK) {
      uint2 e[kOutU];
      uint32_t o[kOutU], p[kOutU];
#pragma unroll
      for (int u = 0; u < kOutU; ++u) {
        const uint32_t k = k0 + u * BLOCK + threadIdx.x;
        e[u] = k < m ? stage[k] : make_uint2(0, 0);
      }
#pragma unroll
      for (int u = 0; u < kOutU; ++u) {
        const uint32_t k = k0 + u * BLOCK + threadIdx.x;
        if (IMPLICIT) {
          p[u] = e[u].y >> 16;
          e[u].y = uint32_t(r.row_base + base) + (e[u].y & 0xFFFFu);
        } else {
          p[u] = fw.div(fm.mod(e[u].x) - lo);
        }
        o[u] = k < m ? cur[p[u]] + (k - loc[p[u]]) : 0u;
      }
#pragma unroll
      for (int u = 0; u < kOutU; ++u) {
        const uint32_t k = k0 + u * BLOCK + threadIdx.x;
        const bool v = k < m;
        if (v && o[u] < cap) region[region_idx(blockIdx.x, p[u], gridDim.x, P) * cap + o[u]] = e[u];  // plain stores: L2 merges a run's partial lines
        const uint64_t spill = __ballot(v && o[u] >= cap);
        if (spill) {  // wave-aggregated append to the overflow list
          const int leader = __ffsll((unsigned long long)spill) - 1;
          unsigned long long b0 = 0;
          if (lane == leader) b0 = atomicAdd(novf, (unsigned long long)__popcll(spill));
          b0 = __shfl(b0, leader, kWave);
          if (v && o[u] >= cap) ovf[b0 + __popcll(spill & lt)] = e[u];
        }
      }
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < P; p += BLOCK) cur[p] += loc[p + 1] - loc[p];
    __syncthreads();
  }
  for (uint32_t p = threadIdx.x; p < P; p += BLOCK) counts[gbase + p] = min(cur[p], cap);
}

// Wave-aggregated append of the lanes with spill_me set to the overflow list.
__device__ __forceinline__ void ovf_append(bool spill_me, uint2 e, uint2* __restrict__ ovf,
                                           unsigned long long* __restrict__ novf) {
  const uint64_t spill = __ballot(spill_me);
  if (!spill) return;
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int leader = __ffsll((unsigned long long)spill) - 1;
  unsigned long long b0 = 0;
  if (lane == leader) b0 = atomicAdd(novf, (unsigned long long)__popcll(spill));
  b0 = __shfl(b0, leader, kWave);
  if (spill_me) ovf[b0 + __popcll(spill & lt)] = e;
}

// k_rp_part1 that writes every region in whole, aligned SEG-pair segments (SEG = 16: 128 B), each
// by one store instruction. A tile's run of partition p is short (tile / P pairs), so with plain
// write-out nearly every run starts and ends inside a segment, and the two halves of such a
// segment reach the L2 from different tiles microseconds apart: the S stream has evicted the
// first half by then and the segment goes to HBM as partial writes. Here the pairs of a run
// that do not complete a segment are CARRIED: thread p keeps partition p's <= SEG-1 leftover
// pairs in registers and puts them in front of p's next run in the LDS stage. The whole
// segments of the tile are listed (segfull: stage start | partition << 16) and enumerated SEG
// lanes per segment, so one wave-instruction stores 64 / SEG complete segments; the stage itself
// needs no alignment (runs are packed). One partition per thread: P <= BLOCK. The carries are
// flushed at the end. A tile whose runs plus carries exceed the stage first flushes the carries.
// SEL: a one-word selection (AlgSelection in front of the probe) fused in, as an inclusive range
// test on the word (SelRange): tuples failing it are dropped like tuples of unowned buckets;
// npass += the passing tuples.
template <int BLOCK, int ROUNDS, int SEG, bool IMPLICIT, bool SEL = false>
__global__ __launch_bounds__(BLOCK) void k_rp_part1r(RelView r, FastMod fm, uint32_t lo, uint32_t nbl, FastDiv fw,
                                                     uint32_t P, uint32_t ntiles, uint32_t cap,
                                                     uint2* __restrict__ region, uint32_t* __restrict__ counts,
                                                     uint2* __restrict__ ovf, unsigned long long* __restrict__ novf,
                                                     SelRange sel = SelRange{}, unsigned long long* __restrict__ npass = nullptr) {
  constexpr int TILE = BLOCK * ROUNDS;
  constexpr int TBITS = __builtin_ctz(TILE);
  constexpr uint32_t kSeg = SEG;
  // stage capacity (pairs): the tile + the carries (expected (SEG-1)/2 per partition)
  constexpr uint32_t SCAP = 2 * TILE + (SEG > 8 ? 1024u : 0u);
  static_assert((TILE & (TILE - 1)) == 0 && TILE <= (1 << 15), "tile must be a power of two");
  static_assert(SCAP + BLOCK * (SEG - 1) < (1u << 16), "stage starts are packed into 16 bits");
  __shared__ uint2 stage[SCAP];
  __shared__ uint32_t loc[BLOCK];      // tile counts (rank atomics)
  __shared__ uint32_t sbase[BLOCK];    // stage index of the run's first new pair (start + carry)
  __shared__ uint2 pinfo[BLOCK];       // per run: {region offset - stage index, sbase}
  __shared__ uint32_t segfull[SCAP / kSeg];  // the whole segments to write: stage start | partition << 16
  __shared__ uint32_t wsum[BLOCK / kWave];
  const uint32_t me = threadIdx.x;  // the partition this thread carries for (me < P)
  const uint64_t gbase = uint64_t(blockIdx.x) * P;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint2 creg[kSeg - 1];
  uint32_t my_kc = 0, my_cur = 0;
#pragma unroll
  for (int j = 0; j < int(kSeg) - 1; ++j) creg[j] = make_uint2(0, 0);
  uint32_t h[ROUNDS];
  uint32_t pw[SEL ? ROUNDS : 1];  // the predicate word of the tile in flight
  uint32_t rw[IMPLICIT ? 1 : ROUNDS];  // explicit row ids, loaded with the keys a tile ahead
  uint32_t npassed = 0;
  auto load_pw = [&](int j, uint64_t i) {
    if constexpr (SEL) pw[j] = i < r.n ? *reinterpret_cast<const uint32_t*>(r.base + i * r.stride + sel.word_off) : 0u;
    if constexpr (!IMPLICIT) rw[j] = i < r.n ? r.row(i) : 0u;
  };
#pragma unroll
  for (int j = 0; j < ROUNDS; ++j) {
    const uint64_t i = uint64_t(blockIdx.x) * TILE + uint64_t(j) * BLOCK + threadIdx.x;
    h[j] = i < r.n ? r.key(i) : 0u;
    load_pw(j, i);
  }
  auto flush_carry = [&]() {  // thread me writes its carry at its cursor (a partial segment)
#pragma unroll
    for (int j = 0; j < int(kSeg) - 1; ++j) {
      const bool v = me < P && uint32_t(j) < my_kc;
      const uint32_t o = my_cur + j;
      if (v && o < cap) region[region_idx(blockIdx.x, me, gridDim.x, P) * cap + o] = creg[j];
      ovf_append(v && o >= cap, creg[j], ovf, novf);
    }
    my_cur += my_kc;
    my_kc = 0;
  };
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    if (me < P) loc[me] = 0;
    const uint64_t base = uint64_t(tile) * TILE;
    uint32_t rk[ROUNDS];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      const uint64_t i = base + uint64_t(j) * BLOCK + threadIdx.x;
      h[j] = murmur32(h[j]);
      const uint32_t bl = fm.mod(h[j]) - lo;
      bool pass = true;
      if constexpr (SEL) {
        pass = sel.test(pw[j]);
        npassed += (i < r.n && pass);
      }
      if (i < r.n && bl < nbl && pass) {
        const uint32_t part = fw.div(bl);
        rk[j] = (part << TBITS) | atomicAdd(&loc[part], 1u);
      } else {
        rk[j] = kInvalid;
      }
    }
    __syncthreads();
    const uint32_t my_c = me < P ? loc[me] : 0u;
    // run lengths -> exclusive scan over the threads (one partition per thread)
    auto scan = [&](uint32_t v, uint32_t* total) {
      uint32_t x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, kWave);
        if (lane >= o) x += y;
      }
      if (lane == 63) wsum[wid] = x;
      __syncthreads();
      uint32_t pre = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < BLOCK / kWave; ++w) {
        const uint32_t t = wsum[w];
        if (w < wid) pre += t;
        tot += t;
      }
      __syncthreads();
      *total = tot;
      return pre + x - v;
    };
    // one scan for both: run length (carry + new) << 16 | whole segments (both sums < 2^16)
    auto seg_counts = [&]() {
      const uint32_t L = my_kc + my_c;
      return (L << 16) | (L / kSeg);
    };
    uint32_t tot;
    uint32_t pre = scan(seg_counts(), &tot);
    if ((tot >> 16) > SCAP) {  // too many carried pairs: flush them (the tile alone then fits)
      flush_carry();
      pre = scan(seg_counts(), &tot);
    }
    const uint32_t my_loc = pre >> 16, my_fseg = pre & 0xFFFFu, nfull = tot & 0xFFFFu;
    const uint32_t my_len = my_kc + my_c;
    if (me < P) {
      sbase[me] = my_loc + my_kc;
      pinfo[me] = make_uint2(my_cur - my_loc, my_loc + my_kc);
#pragma unroll
      for (int j = 0; j < int(kSeg) - 1; ++j)
        if (uint32_t(j) < my_kc) stage[my_loc + j] = creg[j];
      for (uint32_t sg = 0; sg < my_len / kSeg; ++sg) segfull[my_fseg + sg] = (my_loc + sg * kSeg) | (me << 16);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      if (rk[j] == kInvalid) continue;
      const uint32_t part = rk[j] >> TBITS;
      const uint32_t li = uint32_t(j) * BLOCK + threadIdx.x;
      uint32_t y = li;
      if constexpr (!IMPLICIT) y = rw[j];
      stage[sbase[part] + (rk[j] & (TILE - 1))] = make_uint2(h[j], y);
    }
    const uint64_t nbase = uint64_t(tile + gridDim.x) * TILE;  // next tile: loads in flight
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      const uint64_t i = nbase + uint64_t(j) * BLOCK + threadIdx.x;
      h[j] = i < r.n ? r.key(i) : 0u;
      load_pw(j, i);
    }
    __syncthreads();
    // the whole segments: stage index k of run p -> region offset k + pinfo[p].x (each run's
    // tail, the next carry, is not visited)
    const uint32_t rb = uint32_t(r.row_base + base);
    for (uint32_t kk = threadIdx.x; kk < nfull * kSeg; kk += BLOCK) {
      const uint32_t sf = segfull[kk / kSeg];
      const uint32_t p = sf >> 16, k = (sf & 0xFFFFu) + (kk % kSeg);
      const uint2 pi = pinfo[p];
      uint2 e = stage[k];
      if (IMPLICIT && k >= pi.y) e.y = rb + e.y;
      const uint32_t o = k + pi.x;
      if (o < cap) region[region_idx(blockIdx.x, p, gridDim.x, P) * cap + o] = e;
      ovf_append(o >= cap, e, ovf, novf);
    }
    // the run's tail (< one segment) becomes the partition's carry
    if (me < P) {
      const uint32_t F = my_len - my_len % kSeg;
#pragma unroll
      for (int j = 0; j < int(kSeg) - 1; ++j) {
        if (uint32_t(j) < my_len - F) {
          uint2 e = stage[my_loc + F + j];
          if (IMPLICIT && F + j >= my_kc) e.y = rb + e.y;
          creg[j] = e;
        }
      }
      my_cur += F;
      my_kc = my_len - F;
    }
    __syncthreads();
  }
  flush_carry();
  if (me < P) counts[gbase + me] = min(my_cur, cap);
  if constexpr (SEL) {
    uint32_t c = npassed;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
    if (lane == 0 && c) atomicAdd(npass, (unsigned long long)c);
  }
}

// cnt_pm[p * G + g] = counts[g * P + p]: partition-major order for the output-slot scan.
__global__ void k_transpose_counts(const uint32_t* __restrict__ counts, uint32_t G, uint32_t P,
                                   uint32_t* __restrict__ cnt_pm) {
  const uint64_t n = uint64_t(G) * P;
  for (uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < n; q += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t p = uint32_t(q / G), g = uint32_t(q % G);
    cnt_pm[q] = counts[uint64_t(g) * P + p];
  }
}

// Probe of one partition's regions (seg_walk, radix_seg.hpp) against its table slice in LDS.
// The output slot of a pair is seg[p * G + g] + its position in the region (dense over all
// regions, partition-major). FITS: the kernel handles only the partitions whose slice fits LDS
// (the common case, a tight loop over LDS), or only the others (reads the slice through L2);
// both are launched.
template <bool UNIQUE, int MODE, bool CK, bool FITS>
__global__ __launch_bounds__(kJBlock) void k_rp_probe_seg(const uint2* __restrict__ region,
                                                          const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ seg, uint32_t G, uint32_t cap,
                                                          const uint32_t* __restrict__ off, const uint2* __restrict__ ent,
                                                          FastMod fm, uint32_t lo, uint32_t nbl, uint32_t W, uint32_t P,
                                                          uint32_t splits, bool flat, uint2* __restrict__ out,
                                                          uint64_t out_cap, uint64_t* __restrict__ cnt,
                                                          uint64_t* __restrict__ partials) {
  __shared__ uint32_t lds[kProbeLdsWords];
  const uint32_t p = blockIdx.x / splits, sp = blockIdx.x % splits;
  const uint32_t b0 = p * W;
  const uint32_t nbs = min(W, nbl - b0);
  const uint32_t e0 = off[b0], e1 = off[b0 + nbs];
  const uint32_t ne = e1 - e0;
  const bool fits = (nbs + 1) + 2ull * ne + 1 <= kProbeLdsWords;
  if (fits != FITS) {  // the other kernel takes this partition; keep this block's partial row zero
    if (FITS && MODE != kWrite && threadIdx.x < kProbeFields)
      partials[uint64_t(blockIdx.x) * kProbeFields + threadIdx.x] = 0;
    return;
  }
  uint32_t* loff = lds;
  uint2* lent = reinterpret_cast<uint2*>(lds + ((nbs + 2) & ~1u));
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (FITS && UNIQUE && (MODE == kDense || MODE == kAgg)) {  // batched LDS lookups
    seg_walk<true>(region, counts, seg, G, cap, P, p, splits, sp, flat,
                   [&] { stage_slice(off, ent, b0, nbs, e0, ne, loff, lent); },
                   [&](const uint64_t (&v)[kSegItems], const uint64_t (&sl)[kSegItems], uint32_t valid) {
                     probe_chunk_unique<MODE, CK>(v, sl, valid, loff, lent, fm, lo + b0, acc, out, out_cap);
                   });
    block_store<kProbeFields, 1>(acc, partials + uint64_t(blockIdx.x) * kProbeFields);
    return;
  }
  seg_walk(region, counts, seg, G, cap, P, p, splits, sp, flat,
           [&] { if (FITS) stage_slice(off, ent, b0, nbs, e0, ne, loff, lent); },
           [&](uint32_t hv, uint32_t row, uint64_t i) {
             const uint32_t bl = fm.mod(hv) - lo - b0;
             if (FITS) {
               const uint32_t d = loff[bl];
               probe_bucket<UNIQUE, MODE, CK>(hv, row, lent, d >> 16, d & 0xFFFFu, acc, i, out, out_cap, cnt);
             } else {
               const uint32_t s = off[b0 + bl];
               probe_bucket<UNIQUE, MODE, CK>(hv, row, ent, s, off[b0 + bl + 1] - s, acc, i, out, out_cap, cnt);
             }
           });
  if (MODE != kWrite) {
    if (FITS) block_store<kProbeFields, 1>(acc, partials + uint64_t(blockIdx.x) * kProbeFields);
    else block_flush<kProbeFields, 1>(acc, partials + uint64_t(gridDim.x) * kProbeFields);  // extra row (atomics)
  }
}

// Overflow pairs (runs that did not fit their region): probed against the table in HBM; output
// slots follow the regions' (base = seg[P * G]).
template <bool UNIQUE, int MODE, bool CK>
__global__ __launch_bounds__(kBlock) void k_probe_ovf(const uint2* __restrict__ ovf,
                                                      const unsigned long long* __restrict__ novf,
                                                      const uint32_t* __restrict__ base_slot,
                                                      const uint32_t* __restrict__ off, const uint2* __restrict__ ent,
                                                      FastMod fm, uint32_t lo, uint2* __restrict__ out,
                                                      uint64_t out_cap, uint64_t* __restrict__ cnt,
                                                      uint64_t* __restrict__ res) {
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t n = *novf, b = *base_slot;
  for (uint64_t j = uint64_t(blockIdx.x) * kBlock + threadIdx.x; j < n; j += uint64_t(gridDim.x) * kBlock) {
    const uint2 e = ovf[j];
    const uint32_t bl = fm.mod(e.x) - lo;
    const uint32_t s = off[bl];
    probe_bucket<UNIQUE, MODE, CK>(e.x, e.y, ent, s, off[bl + 1] - s, acc, b + j, out, out_cap, cnt);
  }
  if (MODE != kWrite) block_flush<kProbeFields, 1>(acc, res);
}

struct Plan {
  uint32_t W = 1, P = 1, ntiles = 0;
  FastDiv fw;
};

Plan plan_for(uint32_t nbl, uint32_t W, uint64_t n) {
  Plan pl;
  pl.W = W < 1 ? 1 : W;
  pl.P = uint32_t((uint64_t(nbl) + pl.W - 1) / pl.W);
  if (pl.P == 0) pl.P = 1;
  pl.ntiles = uint32_t((n + kPTile - 1) / kPTile);
  pl.fw = make_div(pl.W);
  return pl;
}

// Partition `r` into (hash, row) pairs by bucket range; ps[0..P] = partition starts. Two launches:
// k_rp_hist (sizes, runs claimed on the partition cursors) and k_rp_scatter (starts, pairs).
// t_hist / t_scatter: timer phases of the two streaming kernels (-1: untimed).
hipError_t partition_pairs(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, const Plan& pl, uint2* out,
                           uint32_t* ps, hipStream_t s, int t_hist = -1, int t_scatter = -1,
                           const hj3d_rel* r1 = nullptr) {
  hipError_t e;
  // r1: a second relation of the same table geometry, partitioned in the same two launches (its
  // partitions follow at P .. 2P - 1, its pairs after r's)
  const uint32_t PT = r1 ? 2 * pl.P : pl.P;
  const uint32_t cus = uint32_t(ctx->num_cus);
  // whole segments (16384-tuple tiles, k_rp_wscatter) once a workgroup takes several tiles (their
  // carries ride into later tiles): config C (24 tiles per workgroup) 0.735 -> 0.543 ms; with 1-2.4
  // tiles each (configs E and B) most runs are flushed partial anyway and the plain write-out
  // measured faster (E, both tables in one pass: 51.8 against 2 x 20 us; B: 70.4 against 67.4 us).
  // Small inputs take the plain scatter on kRpSmallRounds x 1024-tuple tiles instead (more,
  // evenly spread tiles: config B's 611 tiles of 16384 gave 157 workgroups 2 and 99 of them 3),
  // one workgroup per CU.
  const uint32_t nt16 = uint32_t((r.n + kPTile - 1) / kPTile) + (r1 ? uint32_t((r1->n + kPTile - 1) / kPTile) : 0u);
  const bool ws = nt16 >= kRpWsMin * (nt16 < cus ? nt16 : cus);
  const uint32_t rounds = ws ? uint32_t(kPRounds) : uint32_t(kRpSmallRounds);
  const uint32_t tsz = kPBlock * rounds;
  const uint32_t nt0 = uint32_t((r.n + tsz - 1) / tsz), nt1 = r1 ? uint32_t((r1->n + tsz - 1) / tsz) : 0u;
  const uint32_t ntiles = nt0 + nt1;
  if (ntiles == 0) return hipMemsetAsync(ps, 0, (uint64_t(PT) + 1) * sizeof(uint32_t), s);
  if (PT > kMaxParts) return hipErrorNotSupported;
  // G persistent workgroups in both passes, one row of run offsets per workgroup
  const uint32_t gmax = cus;
  const uint32_t g = ntiles < gmax ? ntiles : gmax;
  if ((e = ctx->scratch[kScrPHist].ensure(uint64_t(PT) * g * sizeof(uint32_t))) != hipSuccess) return e;
  uint32_t* hist = ctx->scratch[kScrPHist].as<uint32_t>();
  if (!ctx->part_cur.p) {
    if ((e = ctx->part_cur.ensure(2 * (kMaxParts + 1) * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = hipMemsetAsync(ctx->part_cur.p, 0, ctx->part_cur.bytes, s)) != hipSuccess) return e;
  }
  uint32_t* cur = ctx->part_cur.as<uint32_t>() + (ctx->part_parity & 1u) * (kMaxParts + 1);
  uint32_t* cur_next = ctx->part_cur.as<uint32_t>() + ((ctx->part_parity + 1) & 1u) * (kMaxParts + 1);
  ctx->part_parity ^= 1u;
  RelTiles rt;
  rt.r0 = view_of(r);
  rt.r1 = r1 ? view_of(*r1) : rt.r0;
  rt.nt0 = nt0;
  rt.P = pl.P;
  rt.tsz = tsz;
  const uint32_t lo = uint32_t(t->desc.bucket_lo);
  // small implicit-row inputs: one fused launch (k_rp_fused) when every workgroup's tiles fit its
  // registers and the G workgroups are co-resident (the grid barrier needs all of them at once)
  const bool implicit = r.row_off == HJ3D_ROW_IMPLICIT && (!r1 || r1->row_off == HJ3D_ROW_IMPLICIT);
  const uint32_t tpw = (ntiles + g - 1) / g;
  if (!ctx->rp_unfused && !r1 && !ws && rounds == uint32_t(kFzRounds) && implicit && tpw <= uint32_t(kFzTMax) &&
      t->desc.num_buckets >= 2 && t->desc.num_buckets < (1ull << 32) && pl.W >= 2) {
    const void* kf = tpw <= 2   ? reinterpret_cast<const void*>(&k_rp_fused<2>)
                     : tpw == 3 ? reinterpret_cast<const void*>(&k_rp_fused<3>)
                     : tpw == 4 ? reinterpret_cast<const void*>(&k_rp_fused<4>)
                     : tpw == 5 ? reinterpret_cast<const void*>(&k_rp_fused<5>)
                                : reinterpret_cast<const void*>(&k_rp_fused<6>);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, kPBlock, 0) == hipSuccess &&
        uint64_t(per_cu) * cus >= g) {
      if (!ctx->gbar.p) {
        if ((e = ctx->gbar.ensure(2 * sizeof(uint64_t))) != hipSuccess) return e;
        if ((e = hipMemsetAsync(ctx->gbar.p, 0, ctx->gbar.bytes, s)) != hipSuccess) return e;
      }
      // the target counts this launch's arrivals; the context's running sum moves only once the
      // launch is accepted (a failed launch adds no arrivals, so every later barrier would time out)
      FzBar fb;
      fb.bar = ctx->gbar.as<uint64_t>();
      fb.skip0 = ctx->diag_gbar ? 1u : 0u;
      fb.target = ctx->gbar_target + g;
      fb.tflag = const_cast<hj3d_table*>(t)->counts.as<uint64_t>() + 3;
      fb.tag = ctx->gbar_seq + 1;
      fb.ticks = ctx->diag_gbar ? ctx->diag_gbar : 20000000ull;
      PhaseTimer tm(ctx, t_scatter);
      FzGeom fz;
      fz.dnb = FastDiv32::make(uint32_t(t->desc.num_buckets));
      fz.dw = FastDiv32::make(pl.W);
      fz.nb = uint32_t(t->desc.num_buckets);
      fz.lo = lo;
      fz.nbl = t->nb_local;
      fz.P = PT;
#define HJ3D_FZ_LAUNCH(T)                                                                                             \
  hipLaunchKernelGGL(k_rp_fused<T>, dim3(g), dim3(kPBlock), 0, s, rt, fz, ntiles, cur, cur_next, ps, out, fb)
      switch (tpw <= 2 ? 2 : tpw) {
        case 2: HJ3D_FZ_LAUNCH(2); break;
        case 3: HJ3D_FZ_LAUNCH(3); break;
        case 4: HJ3D_FZ_LAUNCH(4); break;
        case 5: HJ3D_FZ_LAUNCH(5); break;
        default: HJ3D_FZ_LAUNCH(6); break;
      }
#undef HJ3D_FZ_LAUNCH
      if ((e = hipGetLastError()) != hipSuccess) return e;
      ctx->gbar_target += g - fb.skip0;  // the arrivals this launch makes
      ctx->gbar_seq = fb.tag;
      const_cast<hj3d_table*>(t)->gbar_tag = fb.tag;  // the table's getters check its flag word
      return hipSuccess;
    }
  }
  {
    PhaseTimer tm(ctx, t_hist);
    if (rounds == kPRounds)
      hipLaunchKernelGGL(k_rp_hist<kPRounds>, dim3(g), dim3(kPBlock), 0, s, rt, t->fm, lo, t->nb_local, pl.fw, PT, ntiles,
                         hist, cur);
    else
      hipLaunchKernelGGL(k_rp_hist<kRpSmallRounds>, dim3(g), dim3(kPBlock), 0, s, rt, t->fm, lo, t->nb_local, pl.fw,
                         PT, ntiles, hist, cur);
  }
  {
    PhaseTimer tm(ctx, t_scatter);
    // explicit rows when either relation has them (RelView::row resolves implicit rows too): the
    // row mode of relation 0 alone would give relation 1's explicit rows as row_base + i
    const bool ex = r.row_off != HJ3D_ROW_IMPLICIT || (r1 && r1->row_off != HJ3D_ROW_IMPLICIT);
#define HJ3D_WS_LAUNCH(PPT, EX)                                                                                   \
  hipLaunchKernelGGL((k_rp_wscatter<PPT, EX>), dim3(g), dim3(kPBlock), 0, s, rt, t->fm, lo, t->nb_local, pl.fw, PT, \
                     ntiles, hist, cur, cur_next, ps, out)
    if (ws && PT <= kPBlock) {
      if (ex) HJ3D_WS_LAUNCH(1, true);
      else HJ3D_WS_LAUNCH(1, false);
    } else if (ws) {
      if (ex) HJ3D_WS_LAUNCH(2, true);
      else HJ3D_WS_LAUNCH(2, false);
    } else
#undef HJ3D_WS_LAUNCH
      hipLaunchKernelGGL(k_rp_scatter<kRpSmallRounds>, dim3(g), dim3(kPBlock), 0, s, rt, t->fm, lo, t->nb_local,
                         pl.fw, PT, ntiles, hist, cur, cur_next, ps, out);
  }
  return hipGetLastError();
}

// Sort every bucket of 2..kSortedMax entries by row (insertion sort, one thread per bucket; the
// bucket was just written and is L2-resident). Longer buckets stay in arrival order.
__global__ __launch_bounds__(256) void k_sort_small_buckets(const uint32_t* __restrict__ off, uint32_t nbl,
                                                            uint2* __restrict__ ent) {
  for (uint32_t b = blockIdx.x * 256 + threadIdx.x; b < nbl; b += gridDim.x * 256) {
    const uint32_t s = off[b], n = off[b + 1] - s;
    if (n < 2 || n > kSortedMax) continue;
    for (uint32_t k = 1; k < n; ++k) {
      const uint2 x = ent[s + k];
      uint32_t j = k;
      while (j > 0 && ent[s + j - 1].y > x.y) {
        ent[s + j] = ent[s + j - 1];
        --j;
      }
      ent[s + j] = x;
    }
  }
}

}  // namespace

hipError_t sort_small_buckets(hj3d_ctx* ctx, hj3d_table* t, hipStream_t s) {
  if (t->nb_local == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sort_small_buckets, dim3(grid_for(ctx, t->nb_local, 256 * 4)), dim3(256), 0, s,
                     t->off.as<const uint32_t>(), t->nb_local, t->ent.as<uint2>());
  return hipGetLastError();
}

bool radix_probe_applicable(const hj3d_ctx* ctx, const hj3d_table* t, uint64_t n_probe) {
  // worth the partition passes once the probe side is large (HJ3D_OPT_RADIX_MIN, default 2^20)
  return t->desc.kind == HJ3D_CHAIN && !ctx->force_direct && n_probe >= ctx->radix_min && n_probe > 0 &&
         t->nb_local >= 64 && n_probe < (1ull << 32);
}

hipError_t radix_partition_pairs(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t W, uint2* out,
                                 uint32_t* ps, uint32_t* nparts, hipStream_t s, const hj3d_rel* r1) {
  const Plan pl = plan_for(t->nb_local, W, r.n);
  if (pl.P * (r1 ? 2u : 1u) > kMaxParts) return hipErrorNotSupported;
  *nparts = pl.P;
  return partition_pairs(ctx, t, r, pl, out, ps, s, -1, -1, r1);
}

hipError_t radix_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s, bool* rows_sorted) {
  hipError_t e;
  const uint32_t nbl = t->nb_local;
  if (rows_sorted) *rows_sorted = false;
  if ((e = t->off.ensure((uint64_t(nbl) + 1) * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = t->ent.ensure((r.n ? r.n : 1) * sizeof(uint2))) != hipSuccess) return e;
  // staged build (8192-bucket slices, small buckets sorted in LDS) while the fill leaves room in
  // the stage; else the 16384-bucket counting build; beyond 2048 slices the direct build
  const double fill = nbl ? double(r.n) / nbl : 0.0;
  // staged slices: 8192 buckets, or up to kBuildSlice2Max where that brings the partition count to
  // 1024 (one partition per partitioner thread: 128-B segments in k_rp_wscatter, and whole waves
  // of k_rp_build3's persistent workgroups; config B: 1221 -> 1024 partitions of 9766 buckets)
  uint32_t W2 = kBuildSlice2;
  const uint32_t Wk = uint32_t((uint64_t(nbl) + kPBlock - 1) / kPBlock);
  if (Wk > W2 && Wk <= kBuildSlice2Max && fill * Wk * 1.25 <= kBuildStage) W2 = Wk;
  bool staged = fill * W2 * 1.25 <= kBuildStage && (uint64_t(nbl) + W2 - 1) / W2 <= kMaxParts;
  const Plan pl = plan_for(nbl, staged ? W2 : kBuildSlice, r.n);
  if (pl.P > kMaxParts) return hipErrorNotSupported;  // > 2048 x 16384 buckets: the direct build
  if ((e = ctx->scratch[kScrPairs].ensure((r.n ? r.n : 1) * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrPStart].ensure((uint64_t(pl.P) + 1) * sizeof(uint32_t))) != hipSuccess) return e;
  uint2* pairs = ctx->scratch[kScrPairs].as<uint2>();
  uint32_t* ps = ctx->scratch[kScrPStart].as<uint32_t>();
  if ((e = partition_pairs(ctx, t, r, pl, pairs, ps, s)) != hipSuccess) return e;
  if (nbl && staged) {
    const uint32_t cus = uint32_t(ctx->num_cus);
    const uint32_t g = pl.P < cus ? pl.P : cus;
    hipLaunchKernelGGL((k_rp_build3<kJBlock, kBuildSlice2Max, kBuildStage>), dim3(g), dim3(kJBlock), 0, s, pairs, ps,
                         t->fm, uint32_t(t->desc.bucket_lo), nbl, pl.W, pl.P, t->off.as<uint32_t>(), t->ent.as<uint2>());
    if (rows_sorted) *rows_sorted = true;
  } else if (nbl) {
    hipLaunchKernelGGL(k_rp_build, dim3(pl.P), dim3(kJBlock), 0, s, pairs, ps, t->fm, uint32_t(t->desc.bucket_lo), nbl,
                       pl.W, t->off.as<uint32_t>(), t->ent.as<uint2>());
  } else {
    if ((e = hipMemsetAsync(t->off.p, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
  }
  t->n_build = r.n;
  return hipGetLastError();
}

namespace {

struct SegLaunch {
  const hj3d_table* t;
  Plan pl;
  uint32_t G, cap, splits;
  bool flat;
  const uint2* region;
  const uint32_t* counts;
  const uint32_t* seg;
  const uint2* ovf;
  const unsigned long long* novf;
  int ovf_grid;
};

template <bool UNIQUE, int MODE, bool CK>
void launch_seg(const SegLaunch& L, uint2* out, uint64_t cap, uint64_t* cnt, uint64_t* partials, uint64_t* res,
                hipStream_t s) {
  const hj3d_table* t = L.t;
  hipLaunchKernelGGL((k_rp_probe_seg<UNIQUE, MODE, CK, true>), dim3(L.pl.P * L.splits), dim3(kJBlock), 0, s, L.region,
                     L.counts, L.seg, L.G, L.cap, t->off.as<const uint32_t>(), t->ent.as<const uint2>(), t->fm,
                     uint32_t(t->desc.bucket_lo), t->nb_local, L.pl.W, L.pl.P, L.splits, L.flat, out, cap, cnt,
                     partials);
  hipLaunchKernelGGL((k_rp_probe_seg<UNIQUE, MODE, CK, false>), dim3(L.pl.P * L.splits), dim3(kJBlock), 0, s,
                     L.region, L.counts, L.seg, L.G, L.cap, t->off.as<const uint32_t>(), t->ent.as<const uint2>(),
                     t->fm, uint32_t(t->desc.bucket_lo), t->nb_local, L.pl.W, L.pl.P, L.splits, L.flat, out, cap,
                     cnt, partials);
  hipLaunchKernelGGL((k_probe_ovf<UNIQUE, MODE, CK>), dim3(L.ovf_grid), dim3(kBlock), 0, s, L.ovf, L.novf,
                     L.seg + uint64_t(L.G) * L.pl.P, t->off.as<const uint32_t>(), t->ent.as<const uint2>(), t->fm,
                     uint32_t(t->desc.bucket_lo), out, cap, cnt, res);
}

template <int MODE>
void launch_seg_any(const SegLaunch& L, bool unique, bool ck, uint2* out, uint64_t cap, uint64_t* cnt,
                    uint64_t* partials, uint64_t* res, hipStream_t s) {
  if (unique) {
    if (ck) launch_seg<true, MODE, true>(L, out, cap, cnt, partials, res, s);
    else launch_seg<true, MODE, false>(L, out, cap, cnt, partials, res, s);
  } else {
    if (ck) launch_seg<false, MODE, true>(L, out, cap, cnt, partials, res, s);
    else launch_seg<false, MODE, false>(L, out, cap, cnt, partials, res, s);
  }
}

}  // namespace

hipError_t pk_probe_slices(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t W, ProbeParts* pp,
                           PkGeom* pk, hipStream_t s) {
  hipError_t e;
  PkSlices sl;
  if ((e = pk_slices(ctx, t, r, W, &sl, s, false)) != hipSuccess) return e;
  const uint64_t nreg = uint64_t(sl.S2) * sl.P;
  // (kScrB: free during a probe; the nested probe's slot arrays use kScrA / kScrC)
  if ((e = ctx->scratch[kScrB].ensure((nreg + 1) * sizeof(uint32_t))) != hipSuccess) return e;
  uint32_t* seg = ctx->scratch[kScrB].as<uint32_t>();
  hipLaunchKernelGGL(k_transpose_counts, dim3(grid_for(ctx, nreg, 256)), dim3(256), 0, s, sl.fcnt, sl.S2, sl.P, seg);
  if ((e = exclusive_scan_u32(ctx, seg, seg, nreg, s)) != hipSuccess) return e;
  pp->W = sl.pk.W;
  pp->P = sl.P;
  pp->G = sl.S2;
  pp->cap = sl.cap2;
  pp->splits = 1;
  pp->flat = double(r.n) / double(nreg) < 256.0;
  pp->region = sl.fine;
  pp->counts = sl.fcnt;
  pp->seg = seg;
  pp->ovf = sl.ovf;
  pp->novf = sl.novf;
  *pk = sl.pk;
  return hipGetLastError();
}

hipError_t radix_partition_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t W, ProbeParts* pp,
                                 hipStream_t s, const SelArgs* sel, unsigned long long** npass, bool slots,
                                 const ZeroList* also) {
  hipError_t e;
  const uint32_t nbl = t->nb_local;
  if (W < 64) W = 64;
  // more than kMaxParts slices: wider slices that no longer fit LDS (probed through L2 by the
  // non-fitting kernel, still one bucket range per workgroup)
  if ((uint64_t(nbl) + W - 1) / W > kMaxParts) W = uint32_t((uint64_t(nbl) + kMaxParts - 1) / kMaxParts);
  {
    // the probe runs one LDS-bound workgroup per CU and slice: round the slice count up to whole
    // waves of workgroups (narrower slices), so no last wave of a few slices costs a full one
    // (config C: 1302 slices = 5.1 waves -> 1536 = 6). Not past the whole-segment partitioner's
    // 1024 slices nor the plain one's 2048.
    const uint32_t G = uint32_t(ctx->num_cus);
    const uint32_t P0 = uint32_t((uint64_t(nbl) + W - 1) / W);
    uint32_t P1 = (P0 + G - 1) / G * G;
    if (P0 <= 1024 && P1 > 1024) P1 = 1024;
    if (P0 >= G && P1 <= kMaxParts && P1 > P0) {
      const uint32_t W1 = uint32_t((uint64_t(nbl) + P1 - 1) / P1);
      if (W1 >= 64) W = W1;
    }
  }
  Plan pl = plan_for(nbl, W, r.n);
  const uint32_t P = pl.P;
  if (P > kMaxParts) return hipErrorNotSupported;
  // up to one partition per thread: the whole-segment partitioner and its 8192-tuple tiles
  const bool seg_writes = P <= uint32_t(kPBlock);
  SelRange sr{};
  if (sel && (!seg_writes || !SelRange::from(*sel, &sr))) return hipErrorNotSupported;  // fused: part1r, one word
  const uint32_t tile = seg_writes ? uint32_t(kPBlock * kPRoundsR) : uint32_t(kPTile);
  pl.ntiles = uint32_t((r.n + tile - 1) / tile);
  const uint32_t G = pl.ntiles < uint32_t(ctx->num_cus) ? pl.ntiles : uint32_t(ctx->num_cus);
  // region capacity: expected pairs per (workgroup, partition) + 8 sigma + slack, 128-B multiple
  const uint64_t per_g = uint64_t((pl.ntiles + G - 1) / G) * tile;
  const double ex = double(per_g < r.n ? per_g : r.n) / P;
  uint64_t cap = uint64_t(ex + 8.0 * std::sqrt(ex) + 32.0);
  cap = (cap + 15) & ~uint64_t(15);
  const uint64_t nreg = uint64_t(G) * P;
  if ((e = ctx->scratch[kScrPairs].ensure(nreg * cap * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrPHist].ensure((3 * nreg + 2) * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrSortV].ensure(r.n * sizeof(uint2) + 64)) != hipSuccess) return e;
  uint2* region = ctx->scratch[kScrPairs].as<uint2>();
  uint32_t* counts = ctx->scratch[kScrPHist].as<uint32_t>();
  uint32_t* seg = counts + nreg;  // nreg + 1 (transposed counts, scanned in place)
  unsigned long long* novf = ctx->scratch[kScrSortV].as<unsigned long long>();
  uint2* ovf = reinterpret_cast<uint2*>(ctx->scratch[kScrSortV].as<char>() + 64);
  if (also) {  // novf, npass and the caller's words in one launch
    ZeroList z = *also;
    if (!z.add(reinterpret_cast<uint64_t*>(novf), 2)) return hipErrorInvalidValue;
    if ((e = zero_words(z, s)) != hipSuccess) return e;
  } else if ((e = hipMemsetAsync(novf, 0, 2 * sizeof(unsigned long long), s)) != hipSuccess) {  // novf, npass
    return e;
  }
  if (npass) *npass = novf + 1;
  const RelView v = view_of(r);
  {
    PhaseTimer tm(ctx, HJ3D_T_SCATTER);
    const uint32_t lo = uint32_t(t->desc.bucket_lo);
    const bool imp = r.row_off == HJ3D_ROW_IMPLICIT;
    if (sel) {
      if (imp)
        hipLaunchKernelGGL((k_rp_part1r<kPBlock, kPRoundsR, kPSeg, true, true>), dim3(G), dim3(kPBlock), 0, s, v, t->fm, lo,
                           nbl, pl.fw, P, pl.ntiles, uint32_t(cap), region, counts, ovf, novf, sr, novf + 1);
      else
        hipLaunchKernelGGL((k_rp_part1r<kPBlock, kPRoundsR, kPSeg, false, true>), dim3(G), dim3(kPBlock), 0, s, v, t->fm,
                           lo, nbl, pl.fw, P, pl.ntiles, uint32_t(cap), region, counts, ovf, novf, sr, novf + 1);
    } else if (seg_writes) {
      if (imp)
        hipLaunchKernelGGL((k_rp_part1r<kPBlock, kPRoundsR, kPSeg, true>), dim3(G), dim3(kPBlock), 0, s, v, t->fm, lo, nbl,
                           pl.fw, P, pl.ntiles, uint32_t(cap), region, counts, ovf, novf);
      else
        hipLaunchKernelGGL((k_rp_part1r<kPBlock, kPRoundsR, kPSeg, false>), dim3(G), dim3(kPBlock), 0, s, v, t->fm, lo, nbl,
                           pl.fw, P, pl.ntiles, uint32_t(cap), region, counts, ovf, novf);
    } else if (imp) {
      hipLaunchKernelGGL((k_rp_part1<kPBlock, kPRounds, kMaxParts, true>), dim3(G), dim3(kPBlock), 0, s, v, t->fm, lo,
                         nbl, pl.fw, P, pl.ntiles, uint32_t(cap), region, counts, ovf, novf);
    } else {
      hipLaunchKernelGGL((k_rp_part1<kPBlock, kPRounds, kMaxParts, false>), dim3(G), dim3(kPBlock), 0, s, v, t->fm, lo,
                         nbl, pl.fw, P, pl.ntiles, uint32_t(cap), region, counts, ovf, novf);
    }
  }
  if (slots) {
    hipLaunchKernelGGL(k_transpose_counts, dim3(grid_for(ctx, nreg, 256)), dim3(256), 0, s, counts, G, P, seg);
    if ((e = exclusive_scan_u32(ctx, seg, seg, nreg, s)) != hipSuccess) return e;
  }
  pp->W = pl.W;
  pp->P = P;
  pp->G = G;
  pp->cap = uint32_t(cap);
  // two probe workgroups per CU's worth of partitions at least: small P splits its regions
  const uint32_t want_blocks = uint32_t(ctx->num_cus) * 2;
  pp->splits = P < want_blocks ? (want_blocks + P - 1) / P : 1u;
  if (pp->splits > G) pp->splits = G;
  pp->flat = double(r.n) / double(nreg) < 256.0;
  pp->region = region;
  pp->counts = counts;
  pp->seg = seg;
  pp->ovf = ovf;
  pp->novf = novf;
  return hipGetLastError();
}

hipError_t radix_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                       uint64_t out_cap, uint64_t* res, hipStream_t s, const SelArgs* sel) {
  hipError_t e;
  // slice width: 80% of the LDS slice budget at the table's mean bucket fill
  const double fill = t->n_build ? double(t->n_build) / double(t->nb_local) : 0.0;
  ProbeParts pp;
  unsigned long long* npass = nullptr;
  if ((e = radix_partition_probe(ctx, t, r, uint32_t(kProbeWFrac * kProbeLdsWords / (1.0 + 2.0 * fill)), &pp, s, sel,
                                 sel ? &npass : nullptr)) != hipSuccess)
    return e;
  SegLaunch L;
  L.t = t;
  L.pl.W = pp.W;
  L.pl.P = pp.P;
  L.G = pp.G;
  L.cap = pp.cap;
  L.splits = pp.splits;
  L.flat = pp.flat;
  L.region = pp.region;
  L.counts = pp.counts;
  L.seg = pp.seg;
  L.ovf = pp.ovf;
  L.novf = pp.novf;
  L.ovf_grid = ctx->num_cus;
  const uint32_t nblocks = pp.P * pp.splits;
  // one row per probe workgroup + one extra row accumulated with atomics by the non-fitting kernel
  if ((e = ctx->scratch[kScrPartial].ensure(uint64_t(nblocks + 2) * kProbeFields * sizeof(uint64_t))) != hipSuccess)
    return e;
  uint64_t* partials = ctx->scratch[kScrPartial].as<uint64_t>();
  if ((e = hipMemsetAsync(partials + uint64_t(nblocks) * kProbeFields, 0, kProbeFields * sizeof(uint64_t), s)) !=
      hipSuccess)
    return e;
  // n_probe of earlier accumulated probes (the reduction below sets res[0] = that + r.n)
  uint64_t* base0 = partials + uint64_t(nblocks + 1) * kProbeFields;
  // (with a fused selection: n_probe = the passing tuples, counted by the partitioner)
  if ((e = hipMemcpyAsync(base0, sel ? static_cast<void*>(npass) : static_cast<void*>(res), sizeof(uint64_t),
                          hipMemcpyDeviceToDevice, s)) != hipSuccess)
    return e;
  const bool unique = flags & HJ3D_PROBE_UNIQUE;
  const bool emit = (flags & HJ3D_PROBE_EMIT) && out;
  const bool ck = flags & HJ3D_PROBE_CHECKSUM;
  uint2* o = static_cast<uint2*>(out);
  PhaseTimer tk(ctx, HJ3D_T_PROBE_KERNEL);  // for the non-unique EMIT form this includes the offset scan
  if (!emit) {
    launch_seg_any<kAgg>(L, unique, ck, nullptr, 0, nullptr, partials, res, s);
  } else if (unique) {
    launch_seg_any<kDense>(L, true, ck, o, out_cap, nullptr, partials, res, s);
  } else {
    if ((e = ctx->scratch[kScrA].ensure((r.n + 1) * sizeof(uint64_t))) != hipSuccess) return e;
    uint64_t* cnt = ctx->scratch[kScrA].as<uint64_t>();
    if ((e = hipMemsetAsync(cnt, 0, (r.n + 1) * sizeof(uint64_t), s)) != hipSuccess) return e;
    launch_seg_any<kCount>(L, false, ck, nullptr, 0, cnt, partials, res, s);
    // slots of unowned tuples (dropped by the partition) stay 0
    if ((e = exclusive_scan_u64(ctx, cnt, cnt, r.n, s)) != hipSuccess) return e;
    launch_seg_any<kWrite>(L, false, ck, o, out_cap, cnt, nullptr, res, s);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // n_probe counts every scanned tuple, also those of unowned buckets (dropped by the partition)
  return reduce_partials(partials, nblocks + 1, kProbeFields, 1, res, s, sel ? 0ull : r.n, base0);
}

}  // namespace hj3d

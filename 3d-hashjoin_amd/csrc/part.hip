// part.hip — multi-GPU exchange helpers and on-device synthetic relations.
//
// Bucket-range partition: owner(bucket) = bucket * P / NB, so every GPU owns a
// contiguous range of the global directory and its statistics / comparison counts are those of
// the single-table reference. Tuples leave as 8-B (key, global row) pairs, grouped by owner,
// stable (input order kept within an owner). Same tile/ballot machinery as sort.hip.
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

constexpr int kRounds = 16;
constexpr int kTile = kBlock * kRounds;
constexpr int kWaves = kBlock / kWave;
constexpr int kMaxParts = 256;

__device__ __forceinline__ uint32_t owner_of(uint32_t key, FastMod fm, uint64_t nb, uint32_t parts) {
  const uint64_t b = fm.mod(murmur32(key));
  return uint32_t((b * parts) / nb);
}

// sel: a selection (AlgSelection below the exchange) evaluated where the tuples are read; tuples
// failing it are not shipped (npred = 0: none).
__global__ __launch_bounds__(kBlock) void k_part_hist(RelView r, FastMod fm, uint64_t nb, uint32_t parts,
                                                      uint32_t ntiles, uint32_t* __restrict__ hist, SelArgs sel) {
  __shared__ uint32_t h[kMaxParts];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = uint64_t(blockIdx.x) * kTile;
  for (int j = 0; j < kRounds; ++j) {
    const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
    if (i < r.n && (sel.npred == 0 || sel_eval(r, sel, i))) atomicAdd(&h[owner_of(r.key(i), fm, nb, parts)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < parts) hist[uint64_t(threadIdx.x) * ntiles + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(kBlock) void k_part_scatter(RelView r, FastMod fm, uint64_t nb, uint32_t parts,
                                                         uint32_t ntiles, const uint32_t* __restrict__ offs,
                                                         uint2* __restrict__ out, SelArgs sel) {
  __shared__ uint32_t run[kMaxParts];
  __shared__ uint32_t wcnt[kWaves][kMaxParts];
  __shared__ uint32_t tbase[kMaxParts];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  run[threadIdx.x] = 0;
  tbase[threadIdx.x] = threadIdx.x < parts ? offs[uint64_t(threadIdx.x) * ntiles + blockIdx.x] : 0u;
  const uint64_t base = uint64_t(blockIdx.x) * kTile;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int j = 0; j < kRounds; ++j) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) wcnt[w][threadIdx.x] = 0;
    __syncthreads();
    const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
    const bool valid = i < r.n && (sel.npred == 0 || sel_eval(r, sel, i));
    const uint32_t key = valid ? r.key(i) : 0u;
    const uint32_t row = valid ? r.row(i) : 0u;
    const uint32_t d = valid ? owner_of(key, fm, nb, parts) : 0u;
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
      out[uint64_t(tbase[d]) + pos] = make_uint2(key, row);
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) add += wcnt[w][threadIdx.x];
    run[threadIdx.x] += add;
  }
}

__global__ void k_part_counts(const uint32_t* __restrict__ offs, uint32_t ntiles, uint32_t parts,
                              uint64_t* __restrict__ counts) {
  const uint32_t p = threadIdx.x;
  if (p < parts) counts[p] = uint64_t(offs[uint64_t(p + 1) * ntiles]) - offs[uint64_t(p) * ntiles];
}

// ---- single-pass exchange partitioner (the probe side: order inside a destination not kept) ----
// The probe's counters are per tuple, so its pairs need no stable order, and the two passes above
// (histogram, then scatter: the relation read twice) become one. Destination p's pairs go to
// out[p * stride ...]: a persistent workgroup (one per CU) takes 8192-tuple tiles; per tile it ranks
// the tuples by destination (wave multi-split: one ballot per destination bit, one LDS atomic per
// destination and wave), claims each destination's run with one device atomic on counts[p] (the
// run's place in p's area), stages the tile destination-major in LDS and writes the runs out with
// consecutive lanes on consecutive pairs. The next tile's keys load while this one is written.
// Per tuple: the tuple read once (12 B at the headline layout) + one 8-B pair written.
// Two 512-thread workgroups per CU (4096-tuple tiles): one workgroup's barrier-separated phases
// overlap the other's memory waits. 1e9 tuples into 8 destinations, same box: one 1024-thread
// workgroup per CU 4.81 / 4.80 ms, two of 512 threads 4.20 / 4.19 ms, three 4.80 / 4.76 ms
// (profiles/r04c_ab_xpart.log).
constexpr int kXpBlock = 512;  // threads per workgroup
constexpr int kXpWgs = 2;      // persistent workgroups per CU
constexpr int kXpRounds = 8;   // tuples per thread and tile (4096-tuple tiles); pairs stored non-temporal
constexpr int kXpTile = kXpBlock * kXpRounds;  // rank inside the tile: < 2^16
constexpr int kXpMaxParts = 256;

template <bool SEL, bool IMPLICIT>
__global__ __launch_bounds__(kXpBlock) void k_xpart(RelView r, FastMod fm, uint64_t nb, uint32_t parts, uint32_t pbits,
                                                    uint32_t magic, uint64_t ntiles, uint64_t stride,
                                                    uint2* __restrict__ out, unsigned long long* __restrict__ counts,
                                                    uint2* __restrict__ sink, SelArgs sel) {
  __shared__ uint2 stage[kXpTile];
  __shared__ uint8_t sown[kXpTile];
  __shared__ uint32_t loc[kXpMaxParts], sbase[kXpMaxParts], bnd[kXpMaxParts + 1];
  __shared__ unsigned long long gbase[kXpMaxParts];
  __shared__ uint32_t ntot;
  const uint32_t me = threadIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  // bnd[p] = first bucket of destination p (hj3d_part_range): owner(b) = max p with bnd[p] <= b
  for (uint32_t p = me; p <= parts; p += kXpBlock)
    bnd[p] = p == parts ? uint32_t(nb) : uint32_t((uint64_t(p) * nb + parts - 1) / parts);
  for (uint32_t p = me; p < kXpMaxParts; p += kXpBlock) loc[p] = 0;
  __syncthreads();
  // Memory ordering: vmcnt counts loads and stores together, in issue order. The per-tile memory
  // instruction counts are therefore fixed (clamped loads; kXpRounds stores, a lane without a pair
  // storing to its own sink slot), so the wait for the next tile's keys leaves this tile's stores in
  // flight (a store behind a branch would make the compiler wait for every older store).
  uint32_t h[kXpRounds], rw[IMPLICIT ? 1 : kXpRounds];
  const auto tile_len = [&](uint64_t tile) __attribute__((always_inline)) {
    const uint64_t base = tile * kXpTile;
    return base >= r.n ? 0u : uint32_t(r.n - base < kXpTile ? r.n - base : kXpTile);
  };
  // a wave-uniform 64-bit tile pointer + 32-bit lane offsets; past the end: the tile's (or the
  // relation's) last tuple again, unconditionally
  auto load = [&](uint64_t tile) __attribute__((always_inline)) {
    const uint64_t t = tile < ntiles ? tile : ntiles - 1;
    const uint32_t lim = tile_len(t) - 1;
    const char* tp = r.base + t * kXpTile * r.stride;
#pragma unroll
    for (int j = 0; j < kXpRounds; ++j) {
      const uint32_t o = min(uint32_t(j) * kXpBlock + me, lim) * r.stride;
      h[j] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(tp + o + r.key_off));
      if constexpr (!IMPLICIT) rw[j] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(tp + o + r.row_off));
    }
  };
  // the loop starts one (empty) tile early, so the first tile's keys are loaded by the same code
  // as every later tile's: the waits at the loop head then see one issue order only
  for (int64_t tile = int64_t(blockIdx.x) - int64_t(gridDim.x); tile < int64_t(ntiles); tile += gridDim.x) {
    const uint64_t base = tile < 0 ? 0 : uint64_t(tile) * kXpTile;
    const uint32_t len = tile < 0 ? 0u : tile_len(uint64_t(tile));
    uint32_t rk[kXpRounds];  // destination << 16 | rank inside the tile's run, or kInvalid
#pragma unroll
    for (int j = 0; j < kXpRounds; ++j) {
      const uint32_t li = uint32_t(j) * kXpBlock + me;
      bool valid = li < len;
      if constexpr (SEL) valid = valid && sel_eval(r, sel, base + li);
      uint32_t d = 0;
      if (valid) {
        const uint32_t b = fm.mod(murmur32(h[j]));
        d = __umulhi(b, magic);  // <= owner(b), at most one or two below it
        while (d + 1 < parts && b >= bnd[d + 1]) ++d;
      }
      uint64_t peer = __ballot(valid);
      for (uint32_t bit = 0; bit < pbits; ++bit) {
        const bool set = (d >> bit) & 1u;
        const uint64_t bb = __ballot(set);
        peer &= set ? bb : ~bb;
      }
      const uint32_t wr = uint32_t(__popcll(peer & lt));
      uint32_t bs = 0;
      if (valid && wr == 0) bs = atomicAdd(&loc[d], uint32_t(__popcll(peer)));
      bs = uint32_t(__shfl(int(bs), valid ? __ffsll((unsigned long long)peer) - 1 : lane, kWave));
      rk[j] = valid ? (d << 16) | (bs + wr) : kInvalid;
    }
    __syncthreads();
    constexpr int kPer = kXpMaxParts / kWave;  // wave 0: destinations lane, lane + 64, ...
    unsigned long long g[kPer];
    if (wid == 0) {  // run starts in the stage, and each run's place in its destination's area
      uint32_t c[kPer];
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const uint32_t p = uint32_t(lane) + k * kWave;
        c[k] = p < parts ? loc[p] : 0u;
        if (p < parts) loc[p] = 0;
      }
#pragma unroll
      for (int k = 0; k < kPer; ++k)  // the claims issued together; their values are needed last
        g[k] = c[k] ? atomicAdd(counts + lane + k * kWave, (unsigned long long)c[k]) : 0ull;
      // stage order: destination-major, p = lane + k * 64 -> (k, lane) scan order is p order
      uint32_t run = 0;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        uint32_t wt;
        const uint32_t pre = wave_excl_scan(c[k], &wt);
        const uint32_t p = uint32_t(lane) + k * kWave;
        if (p < parts) sbase[p] = run + pre;
        run += wt;
      }
      if (lane == 0) ntot = run;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kXpRounds; ++j) {
      if (rk[j] == kInvalid) continue;
      const uint32_t d = rk[j] >> 16, s = sbase[d] + (rk[j] & 0xFFFFu);
      stage[s] = make_uint2(h[j], IMPLICIT ? uint32_t(r.row_base + base) + uint32_t(j) * kXpBlock + me : rw[j]);
      sown[s] = uint8_t(d);
    }
    load(uint64_t(tile + gridDim.x));  // the next tile's keys in flight while this one is written
    if (wid == 0) {
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const uint32_t p = uint32_t(lane) + k * kWave;
        if (p < parts) gbase[p] = g[k];
      }
    }
    __syncthreads();
    const uint32_t nt = ntot;
#pragma unroll
    for (int it = 0; it < kXpRounds; ++it) {
      const uint32_t kk = uint32_t(it) * kXpBlock + me;
      const uint32_t d = sown[kk];
      const uint64_t pos = gbase[d] + (kk - sbase[d]);
      const uint2 e = stage[kk];
      uint2* dst = kk < nt && pos < stride ? out + d * stride + pos : sink + me;
      __builtin_nontemporal_store((uint64_t(e.y) << 32) | e.x, reinterpret_cast<uint64_t*>(dst));
    }
  }
}

// Bijective permutation of [0, n): 4-round Feistel network on the smallest even-bit domain
// >= n, with cycle walking back into [0, n).
struct Feistel {
  uint64_t n, seed;
  uint32_t half;
  uint64_t mask;
  __host__ __device__ static Feistel make(uint64_t n, uint64_t seed) {
    Feistel f;
    f.n = n;
    f.seed = seed;
    uint32_t bits = 0;
    while (bits < 64 && (1ull << bits) < n) ++bits;
    f.half = (bits + 1) / 2;
    if (f.half == 0) f.half = 1;
    f.mask = (1ull << f.half) - 1;
    return f;
  }
  __host__ __device__ uint64_t round_fn(uint64_t x, int k) const {
    return mix64(x ^ (seed + 0x9e3779b97f4a7c15ull * uint64_t(k + 1))) & mask;
  }
  __host__ __device__ uint64_t enc1(uint64_t x) const {
    uint64_t L = x >> half, R = x & mask;
    for (int k = 0; k < 4; ++k) {
      const uint64_t t = L ^ round_fn(R, k);
      L = R;
      R = t;
    }
    return (L << half) | R;
  }
  __host__ __device__ uint64_t dec1(uint64_t x) const {
    uint64_t L = x >> half, R = x & mask;
    for (int k = 3; k >= 0; --k) {
      const uint64_t t = R ^ round_fn(L, k);
      R = L;
      L = t;
    }
    return (L << half) | R;
  }
  __host__ __device__ uint64_t perm(uint64_t x) const {
    if (n <= 1) return 0;
    uint64_t y = enc1(x);
    while (y >= n) y = enc1(y);
    return y;
  }
  __host__ __device__ uint64_t inv(uint64_t y) const {
    if (n <= 1) return 0;
    uint64_t x = dec1(y);
    while (x >= n) x = dec1(x);
    return x;
  }
};

__global__ __launch_bounds__(kBlock) void k_gen_keys(char* __restrict__ t, uint64_t n, uint32_t stride,
                                                     uint32_t key_off, uint64_t row_base, Feistel f, bool identity) {
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock) {
    const uint64_t g = row_base + i;
    *reinterpret_cast<uint32_t*>(t + i * stride + key_off) = uint32_t(identity ? g : f.perm(g));
  }
}

__global__ __launch_bounds__(kBlock) void k_gen_fk(char* __restrict__ t, uint64_t n, uint32_t stride,
                                                   uint32_t key_off, uint64_t row_base, uint32_t fk_max,
                                                   uint64_t seed) {
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock) {
    const uint64_t x = mix64((row_base + i) ^ seed);
    *reinterpret_cast<uint32_t*>(t + i * stride + key_off) = uint32_t(((x >> 32) * uint64_t(fk_max)) >> 32);
  }
}

// Zipf(theta) over {1..n} by rejection-inversion (Hoermann & Derflinger 1996, the method of the
// reference's util/zipf_distribution.hh), driven by a counter-based RNG of the global row so
// every row's value is independent of the launch geometry. Not the reference's sequential
// mt19937 stream: full-size runs check parity through the key/FK pair identity instead.
struct ZipfRI {
  double q, n, hx1, hn, s;
  __host__ __device__ static double helper1(double x) {
    return fabs(x) > 1e-8 ? log1p(x) / x : 1.0 - x * (0.5 - x * (1.0 / 3.0 - 0.25 * x));
  }
  __host__ __device__ static double helper2(double x) {
    return fabs(x) > 1e-8 ? expm1(x) / x : 1.0 + x * 0.5 * (1.0 + x * (1.0 / 3.0) * (1.0 + 0.25 * x));
  }
  __host__ __device__ double h(double x) const { return exp(-q * log(x)); }
  __host__ __device__ double H(double x) const {
    const double lx = log(x);
    return helper2((1.0 - q) * lx) * lx;
  }
  __host__ __device__ double Hinv(double x) const {
    double t = x * (1.0 - q);
    if (t < -1.0) t = -1.0;
    return exp(helper1(t) * x);
  }
  static ZipfRI make(uint32_t n, double theta) {
    ZipfRI z;
    z.q = theta;
    z.n = double(n);
    z.hx1 = z.H(1.5) - 1.0;
    z.hn = z.H(z.n + 0.5);
    z.s = 2.0 - z.Hinv(z.H(2.5) - z.h(2.0));
    return z;
  }
  __device__ uint32_t sample(uint64_t key) const {
    for (uint64_t c = 0;; ++c) {
      const double u01 = double(mix64(key ^ (c * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull)) >> 11) * 0x1.0p-53;
      const double u = hn + u01 * (hx1 - hn);
      const double x = Hinv(u);
      double k = floor(x + 0.5);
      k = k < 1.0 ? 1.0 : (k > n ? n : k);
      if (k - x <= s || u >= H(k + 0.5) - h(k)) return uint32_t(k);
    }
  }
};

__global__ __launch_bounds__(kBlock) void k_gen_zipf(char* __restrict__ t, uint64_t n, uint32_t stride,
                                                     uint32_t key_off, uint64_t row_base, ZipfRI z, uint64_t seed) {
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock)
    *reinterpret_cast<uint32_t*>(t + i * stride + key_off) = z.sample(mix64((row_base + i) ^ seed)) - 1u;
}

__global__ __launch_bounds__(kBlock) void k_inv(RelView b, uint64_t n_keys, uint32_t* __restrict__ inv) {
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < b.n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t k = b.key(i);
    if (k < n_keys) inv[k] = b.row(i);
  }
}

__global__ __launch_bounds__(kBlock) void k_expect(RelView p, uint64_t n_keys, const uint32_t* __restrict__ inv,
                                                   bool swap, uint64_t* __restrict__ res) {
  uint64_t a[5] = {0, 0, 0, 0, 0};
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < p.n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t k = p.key(i);
    if (k >= n_keys) continue;
    const uint32_t x = swap ? inv[k] : p.row(i), y = swap ? p.row(i) : inv[k];
    const uint64_t h = pair_hash(x, y);
    a[0] += 1;
    a[1] += x;
    a[2] += y;
    a[3] += h;
    a[4] ^= h;
  }
  block_flush<5, 1>(a, res);
}

// Expected key/FK pairs when the build keys came from k_gen_keys(n_keys, seed): the partner
// of FK k is the build row perm^-1(k) (no table, no inverse array: works per rank).
__global__ __launch_bounds__(kBlock) void k_expect_gen(RelView p, Feistel f, bool swap, uint64_t* __restrict__ res) {
  uint64_t a[5] = {0, 0, 0, 0, 0};
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < p.n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t k = p.key(i);
    if (k >= f.n) continue;
    const uint32_t br = uint32_t(f.inv(k)), pr = p.row(i);
    const uint32_t x = swap ? br : pr, y = swap ? pr : br;
    const uint64_t h = pair_hash(x, y);
    a[0] += 1;
    a[1] += x;
    a[2] += y;
    a[3] += h;
    a[4] ^= h;
  }
  block_flush<5, 1>(a, res);
}

// ---- #dv pre-pass: the reference counts the distinct FK values of S.a with
// an unordered_set (main_experiment1.cc:453-454) to size the Crs / Nrs / NrsNU tables. Across
// GPUs: every rank sets the bits of its keys in a bitmap over the key domain, the ranks exchange
// bitmap slices (all-to-all: rank r receives slice r of every bitmap), OR + popcount their slice,
// and sum the counts. ----

// bit k of bm for every key k < domain; keys >= domain are counted in *outside (u64).
__global__ __launch_bounds__(kBlock) void k_key_bitmap(RelView r, uint64_t domain, uint32_t* __restrict__ bm,
                                                       unsigned long long* __restrict__ outside) {
  uint32_t nout = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < r.n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t k = r.key(i);
    if (k < domain) {
      const uint32_t bit = 1u << (k & 31);
      uint32_t* w = bm + (k >> 5);
      if (!(*w & bit)) atomicOr(w, bit);  // skip the atomic when the bit is already visible
    } else {
      ++nout;
    }
  }
  const uint64_t t = wave_sum(uint64_t(nout));
  if (outside && (threadIdx.x & 63) == 0 && t) atomicAdd(outside, (unsigned long long)t);
}

// The same bitmap without a device atomic per key (large inputs): the key domain is cut into NS =
// 2^lg slices of whole 32-bit words, word w in slice w & (NS - 1) at slice word w >> lg, each slice
// small enough for an LDS bitmap (<= kDvSliceWords words; interleaved by word, so a key range that
// is dense in one part of the domain still spreads over every slice).
//  pass 1 k_dv_part: one 1024-thread workgroup per 8192-tuple tile reads the keys (12-B tuples as
//    three 16-B loads per 4 tuples), ranks them by slice with LDS atomics (no order kept) and writes
//    the tile back slice-major as bit positions inside the slice (u32), with its NS + 1 run bounds
//    (u16) per tile; keys >= domain are counted in *outside.
//  pass 2 k_dv_bits: workgroup (s, g) sets the bits of slice s's runs in tiles [g·T/G2, (g+1)·T/G2)
//    in an LDS bitmap (an LDS read first: a bit already set costs no atomic) and stores it as partial
//    row g of slice s.
//  pass 3 k_dv_merge: bm[w] |= OR over the G2 partial rows of slice w & (NS-1), word w >> lg.
// Per key: the tuple read once + 4 B written and read back; the partial rows are G2 × the bitmap.
constexpr int kDvBlock = 1024;
constexpr int kDvPer = 8;
constexpr int kDvTile = kDvBlock * kDvPer;  // run bounds fit u16
constexpr uint32_t kDvMaxSlices = 1024;
constexpr uint32_t kDvSliceWords = 20480;  // 80 KB: two pass-2 workgroups per CU
constexpr uint32_t kDvSkip = 0xFFFFFFFFu;  // a tuple past the end or a key outside the domain

// KO = key word inside a 12-B tuple (0..2) for the vector load form; -1: any layout (RelView::key)
template <int KO>
__global__ __launch_bounds__(kDvBlock) void k_dv_part(RelView r, uint64_t domain, uint32_t lg,
                                                      uint32_t* __restrict__ pos_out, uint16_t* __restrict__ bounds,
                                                      unsigned long long* __restrict__ outside) {
  __shared__ uint32_t stage[kDvTile];
  __shared__ uint32_t cnt[kDvMaxSlices];
  __shared__ uint32_t wtot[kDvBlock / kWave];
  const uint32_t me = threadIdx.x, ns = 1u << lg;
  const int lane = me & 63, wid = me >> 6;
  const uint64_t base = uint64_t(blockIdx.x) * kDvTile;
  for (uint32_t s = me; s < ns; s += kDvBlock) cnt[s] = 0;
  uint32_t k[kDvPer];
  if constexpr (KO >= 0) {
    // thread me: tuples base + h·4096 + 4·me .. +3 for h = 0, 1
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t i0 = base + uint64_t(h) * (kDvTile / 2) + 4ull * me;
      if (i0 + 4 <= r.n) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* p = reinterpret_cast<const u32x4*>(r.base + i0 * 12);
        const u32x4 a = __builtin_nontemporal_load(p), b = __builtin_nontemporal_load(p + 1),
                    c = __builtin_nontemporal_load(p + 2);
        const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) k[h * 4 + q] = w[3 * q + KO];
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) k[h * 4 + q] = i0 + q < r.n ? r.key(i0 + q) : kDvSkip;
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < kDvPer; ++q) {
      const uint64_t i = base + uint64_t(q) * kDvBlock + me;
      k[q] = i < r.n ? r.key(i) : kDvSkip;
    }
  }
  // tuples past the end drop out; keys outside the domain are counted
  uint32_t nout = 0, valid = 0;
#pragma unroll
  for (int q = 0; q < kDvPer; ++q) {
    const uint64_t i = KO >= 0 ? base + uint64_t(q >> 2) * (kDvTile / 2) + 4ull * me + (q & 3)
                               : base + uint64_t(q) * kDvBlock + me;
    if (i < r.n) {
      if (uint64_t(k[q]) < domain) valid |= 1u << q;
      else ++nout;
    }
  }
  __syncthreads();  // cnt cleared
  uint32_t slot[kDvPer];
#pragma unroll
  for (int q = 0; q < kDvPer; ++q)
    if (valid >> q & 1u) slot[q] = atomicAdd(&cnt[(k[q] >> 5) & (ns - 1)], 1u);
  __syncthreads();
  // exclusive scan of the slice counts (ns <= 1024 = one per thread)
  const uint32_t c = me < ns ? cnt[me] : 0u;
  uint32_t wt;
  const uint32_t ex = wave_excl_scan(c, &wt);
  if (lane == 0) wtot[wid] = wt;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kDvBlock / kWave; ++w) {
    const uint32_t x = wtot[w];
    before += w < wid ? x : 0u;
    total += x;
  }
  __syncthreads();  // every thread has read its slice count
  uint16_t* bd = bounds + uint64_t(blockIdx.x) * (ns + 1);
  if (me < ns) {
    cnt[me] = before + ex;
    bd[me] = uint16_t(before + ex);
  }
  if (me == 0) bd[ns] = uint16_t(total);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kDvPer; ++q)
    if (valid >> q & 1u) {
      const uint32_t w = k[q] >> 5;
      stage[cnt[w & (ns - 1)] + slot[q]] = ((w >> lg) << 5) | (k[q] & 31u);
    }
  __syncthreads();
  for (uint32_t x = me; x < total; x += kDvBlock) __builtin_nontemporal_store(stage[x], pos_out + base + x);
  const uint64_t t = wave_sum(uint64_t(nout));
  if (outside && lane == 0 && t) atomicAdd(outside, (unsigned long long)t);
}

// workgroup (s, g) = blockIdx.x = s * g2 + g; tiles [g·ntiles/g2, (g+1)·ntiles/g2), wave w takes
// every 16th of them
__global__ __launch_bounds__(kDvBlock) void k_dv_bits(const uint32_t* __restrict__ pos, const uint16_t* __restrict__ bounds,
                                                      uint32_t lg, uint64_t ntiles, uint32_t g2, uint32_t wps,
                                                      uint32_t* __restrict__ part) {
  extern __shared__ uint32_t bm[];
  const uint32_t me = threadIdx.x, ns = 1u << lg;
  const uint32_t s = blockIdx.x / g2, g = blockIdx.x % g2;
  const int lane = me & 63, wid = me >> 6;
  for (uint32_t j = me; j < wps; j += kDvBlock) bm[j] = 0;
  __syncthreads();
  constexpr int kU = 8;  // keys per lane and run loaded in one batch (the next run's batch in flight)
  constexpr uint32_t kWaves = kDvBlock / kWave;
  const uint64_t t0 = ntiles * g / g2, t1 = ntiles * (g + 1) / g2;
  const uint64_t ntw = t0 + wid < t1 ? (t1 - t0 - wid + kWaves - 1) / kWaves : 0;  // this wave's tiles
  const auto set_bit = [&](uint32_t v) __attribute__((always_inline)) {
    const uint32_t bit = 1u << (v & 31u);
    if (!(bm[v >> 5] & bit)) atomicOr(&bm[v >> 5], bit);
  };
  for (uint64_t c0 = 0; c0 < ntw; c0 += kWave) {
    // lane k: run bounds of the wave's tile c0 + k (tile t0 + wid + 16 (c0 + k))
    uint32_t blo = 0, bhi = 0;
    if (c0 + lane < ntw) {
      const uint16_t* bd = bounds + (t0 + wid + kWaves * (c0 + lane)) * (ns + 1) + s;
      blo = bd[0];
      bhi = bd[1];
    }
    const uint32_t m = uint32_t(ntw - c0 < kWave ? ntw - c0 : kWave);
    // runs taken kD at a time, the next kD runs' batches in flight
    constexpr int kD = 2;
    uint32_t v[kD][kU], nv[kD][kU];
    const auto load = [&](uint32_t (&dst)[kD][kU], uint32_t i0) __attribute__((always_inline)) {
#pragma unroll
      for (int d = 0; d < kD; ++d) {
        const uint32_t i = i0 + d < m ? i0 + d : m - 1;
        const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(blo), int(i)));
        const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(bhi), int(i)));
        const uint32_t* p = pos + (t0 + wid + kWaves * (c0 + i)) * kDvTile;
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const uint32_t x = lo + lane + u * kWave;
          dst[d][u] = __builtin_nontemporal_load(p + (x < hi ? x : 0u));  // unconditional (slot 0 past the run)
        }
      }
    };
    load(v, 0);
    for (uint32_t i0 = 0; i0 < m; i0 += kD) {
      load(nv, i0 + kD < m ? i0 + kD : i0);
#pragma unroll
      for (int d = 0; d < kD; ++d) {
        const uint32_t i = i0 + d;
        if (i >= m) break;
        const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(blo), int(i)));
        const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(bhi), int(i)));
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (lo + lane + u * kWave < hi) set_bit(v[d][u]);
        if (lo + kU * kWave < hi) {  // a run longer than one batch
          const uint32_t* p = pos + (t0 + wid + kWaves * (c0 + i)) * kDvTile;
          for (uint32_t x = lo + kU * kWave + lane; x < hi; x += kWave) set_bit(__builtin_nontemporal_load(p + x));
        }
      }
#pragma unroll
      for (int d = 0; d < kD; ++d)
#pragma unroll
        for (int u = 0; u < kU; ++u) v[d][u] = nv[d][u];
    }
  }
  __syncthreads();
  uint32_t* row = part + (uint64_t(s) * g2 + g) * wps;
  for (uint32_t j = me; j < wps; j += kDvBlock) row[j] = bm[j];
}

// thread (s, j), j fastest: bm[j·NS + s] |= OR over g of part[(s·g2 + g)·wps + j]
__global__ __launch_bounds__(kBlock) void k_dv_merge(const uint32_t* __restrict__ part, uint32_t lg, uint32_t g2,
                                                     uint32_t wps, uint64_t words, uint32_t* __restrict__ bm) {
  const uint64_t n = uint64_t(wps) << lg;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t s = uint32_t(i / wps), j = uint32_t(i % wps);
    const uint64_t w = (uint64_t(j) << lg) | s;
    if (w >= words) continue;
    const uint32_t* src = part + uint64_t(s) * g2 * wps + j;
    uint32_t x = 0;
    uint32_t g = 0;
    for (; g + 8 <= g2; g += 8) {  // eight independent loads in flight
      uint32_t y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) y[u] = src[uint64_t(g + u) * wps];
#pragma unroll
      for (int u = 0; u < 8; ++u) x |= y[u];
    }
    for (; g < g2; ++g) x |= src[uint64_t(g) * wps];
    if (x) bm[w] |= x;
  }
}

// *count += popcount(OR over rows of bm[row * words + w]) over w < words.
__global__ __launch_bounds__(kBlock) void k_or_popcount(const uint32_t* __restrict__ bm, uint32_t rows, uint64_t words,
                                                        unsigned long long* __restrict__ count) {
  uint64_t c = 0;
  for (uint64_t w = uint64_t(blockIdx.x) * kBlock + threadIdx.x; w < words; w += uint64_t(gridDim.x) * kBlock) {
    uint32_t x = 0;
    for (uint32_t q = 0; q < rows; ++q) x |= bm[uint64_t(q) * words + w];
    c += __popc(x);
  }
  const uint64_t t = wave_sum(c);
  if ((threadIdx.x & 63) == 0 && t) atomicAdd(count, (unsigned long long)t);
}

}  // namespace

hipError_t expected_fk_join_gen(hj3d_ctx* ctx, const hj3d_rel& probe, uint64_t n_keys, uint64_t seed, bool swap,
                                void* res, hipStream_t s) {
  if (probe.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_expect_gen, dim3(grid_for(ctx, probe.n, kBlock * 4)), dim3(kBlock), 0, s, view_of(probe),
                     Feistel::make(n_keys, seed), swap, static_cast<uint64_t*>(res));
  return hipGetLastError();
}

hipError_t partition(hj3d_ctx* ctx, const hj3d_rel& r, uint64_t nb, uint32_t parts, void* out_pairs, void* counts,
                     hipStream_t s, const SelArgs* sel) {
  if (parts == 0 || parts > kMaxParts || nb == 0 || nb >= (1ull << 32)) return hipErrorInvalidValue;
  hipError_t e;
  const uint64_t ntiles = (r.n + kTile - 1) / kTile;
  if (r.n == 0) return hipMemsetAsync(counts, 0, parts * sizeof(uint64_t), s);
  if ((e = ctx->scratch[kScrD].ensure((uint64_t(parts) * ntiles + 1) * sizeof(uint32_t))) != hipSuccess) return e;
  uint32_t* hist = ctx->scratch[kScrD].as<uint32_t>();
  const FastMod fm = FastMod::make(uint32_t(nb));
  const RelView v = view_of(r);
  const SelArgs sa = sel ? *sel : SelArgs{};
  hipLaunchKernelGGL(k_part_hist, dim3(unsigned(ntiles)), dim3(kBlock), 0, s, v, fm, nb, parts, uint32_t(ntiles), hist,
                     sa);
  if ((e = exclusive_scan_u32(ctx, hist, hist, uint64_t(parts) * ntiles, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_part_scatter, dim3(unsigned(ntiles)), dim3(kBlock), 0, s, v, fm, nb, parts, uint32_t(ntiles),
                     hist, static_cast<uint2*>(out_pairs), sa);
  hipLaunchKernelGGL(k_part_counts, dim3(1), dim3(kMaxParts), 0, s, hist, uint32_t(ntiles), parts,
                     static_cast<uint64_t*>(counts));
  return hipGetLastError();
}

hipError_t partition_strided(hj3d_ctx* ctx, const hj3d_rel& r, uint64_t nb, uint32_t parts, void* out_pairs,
                             uint64_t stride, void* counts, hipStream_t s, const SelArgs* sel) {
  if (parts == 0 || parts > kXpMaxParts || nb == 0 || nb >= (1ull << 32) || (stride == 0 && r.n)) return hipErrorInvalidValue;
  hipError_t e;
  if ((e = hipMemsetAsync(counts, 0, parts * sizeof(uint64_t), s)) != hipSuccess) return e;
  if (r.n == 0) return hipSuccess;
  const uint64_t ntiles = (r.n + kXpTile - 1) / kXpTile;
  const uint64_t want = uint64_t(ctx->num_cus) * kXpWgs;  // persistent: kXpWgs workgroups per CU
  const unsigned grid = unsigned(ntiles < want ? ntiles : want);
  uint32_t pbits = 0;
  while ((1u << pbits) < parts) ++pbits;
  const uint64_t m = (uint64_t(parts) << 32) / nb;  // owner(b) >= mulhi(b, m) >= owner(b) - 2
  const uint32_t magic = m > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(m);
  const FastMod fm = FastMod::make(uint32_t(nb));
  const RelView v = view_of(r);
  auto* cnt = static_cast<unsigned long long*>(counts);
  auto* out = static_cast<uint2*>(out_pairs);
  const bool implicit = v.row_off == 0xFFFFFFFFu;
  uint2* sink;  // garbage stores of lanes without a pair
  if ((e = store_sink(ctx, &sink)) != hipSuccess) return e;
  const SelArgs sa = sel ? *sel : SelArgs{};
  if (sa.npred)
    hipLaunchKernelGGL((implicit ? k_xpart<true, true> : k_xpart<true, false>), dim3(grid), dim3(kXpBlock), 0, s, v, fm,
                       nb, parts, pbits, magic, ntiles, stride, out, cnt, sink, sa);
  else
    hipLaunchKernelGGL((implicit ? k_xpart<false, true> : k_xpart<false, false>), dim3(grid), dim3(kXpBlock), 0, s, v,
                       fm, nb, parts, pbits, magic, ntiles, stride, out, cnt, sink, sa);
  return hipGetLastError();
}

hipError_t gen_keys(void* tuples, uint64_t n, uint32_t stride, uint32_t key_off, uint64_t row_base, uint64_t n_keys,
                    uint64_t seed, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const Feistel f = Feistel::make(n_keys, seed);
  const unsigned g = unsigned(n / kBlock + 1 < 4096 ? n / kBlock + 1 : 4096);
  hipLaunchKernelGGL(k_gen_keys, dim3(g), dim3(kBlock), 0, s, static_cast<char*>(tuples), n, stride, key_off, row_base,
                     f, n_keys == 0);
  return hipGetLastError();
}

hipError_t gen_fk(void* tuples, uint64_t n, uint32_t stride, uint32_t key_off, uint64_t row_base, uint32_t fk_max,
                  uint64_t seed, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const unsigned g = unsigned(n / kBlock + 1 < 4096 ? n / kBlock + 1 : 4096);
  hipLaunchKernelGGL(k_gen_fk, dim3(g), dim3(kBlock), 0, s, static_cast<char*>(tuples), n, stride, key_off, row_base,
                     fk_max, seed);
  return hipGetLastError();
}

hipError_t gen_zipf(void* tuples, uint64_t n, uint32_t stride, uint32_t key_off, uint64_t row_base, uint32_t fk_max,
                    double theta, uint64_t seed, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const ZipfRI z = ZipfRI::make(fk_max, theta);
  const unsigned g = unsigned(n / kBlock + 1 < 4096 ? n / kBlock + 1 : 4096);
  hipLaunchKernelGGL(k_gen_zipf, dim3(g), dim3(kBlock), 0, s, static_cast<char*>(tuples), n, stride, key_off,
                     row_base, z, seed);
  return hipGetLastError();
}

hipError_t expected_fk_join(hj3d_ctx* ctx, const hj3d_rel& build, const hj3d_rel& probe, uint64_t n_keys, bool swap,
                            void* res, hipStream_t s) {
  hipError_t e = ctx->scratch[kScrD].ensure((n_keys ? n_keys : 1) * sizeof(uint32_t));
  if (e != hipSuccess) return e;
  uint32_t* inv = ctx->scratch[kScrD].as<uint32_t>();
  if ((e = hipMemsetAsync(inv, 0xFF, (n_keys ? n_keys : 1) * sizeof(uint32_t), s)) != hipSuccess) return e;
  const RelView b = view_of(build), p = view_of(probe);
  if (build.n)
    hipLaunchKernelGGL(k_inv, dim3(grid_for(ctx, build.n, kBlock * 4)), dim3(kBlock), 0, s, b, n_keys, inv);
  if (probe.n)
    hipLaunchKernelGGL(k_expect, dim3(grid_for(ctx, probe.n, kBlock * 4)), dim3(kBlock), 0, s, p, n_keys, inv,
                       swap, static_cast<uint64_t*>(res));
  return hipGetLastError();
}

hipError_t key_bitmap(hj3d_ctx* ctx, const hj3d_rel& r, uint64_t domain, void* bitmap, void* outside, hipStream_t s) {
  if (r.n == 0) return hipSuccess;
  const uint64_t words = (domain + 31) / 32;
  uint32_t lg = 0;
  while ((words >> lg) > kDvSliceWords) ++lg;
  if ((words + (1ull << lg) - 1) >> lg > kDvSliceWords) ++lg;  // ceil(words / NS) <= kDvSliceWords
  static const bool direct = [] {
    const char* e = getenv("HJ3D_OPT_DV_DIRECT");
    return e && *e && *e != '0';
  }();
  if (!direct && r.n >= (1u << 20) && domain > 0 && (1u << lg) <= kDvMaxSlices && r.stride >= 4) {
    const uint32_t ns = 1u << lg, wps = uint32_t((words + ns - 1) >> lg);
    const uint64_t ntiles = (r.n + kDvTile - 1) / kDvTile;
    uint32_t g2 = uint32_t(2 * ctx->num_cus) / ns;  // two 80-KB workgroups per CU
    if (g2 < 1) g2 = 1;
    if (g2 > ntiles) g2 = uint32_t(ntiles);
    hipError_t e;
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dv_bits),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    if ((e = ctx->scratch[kScrSortK].ensure(ntiles * kDvTile * sizeof(uint32_t))) != hipSuccess ||
        (e = ctx->scratch[kScrPHist].ensure(ntiles * (ns + 1) * sizeof(uint16_t))) != hipSuccess ||
        (e = ctx->scratch[kScrSortV].ensure(uint64_t(ns) * g2 * wps * sizeof(uint32_t))) != hipSuccess)
      return e;
    uint32_t* pos = ctx->scratch[kScrSortK].as<uint32_t>();
    uint16_t* bounds = ctx->scratch[kScrPHist].as<uint16_t>();
    uint32_t* part = ctx->scratch[kScrSortV].as<uint32_t>();
    const RelView v = view_of(r);
    auto* outs = static_cast<unsigned long long*>(outside);
    const bool v12 = r.stride == 12 && (reinterpret_cast<uintptr_t>(r.base) & 15) == 0 && r.key_off % 4 == 0;
    auto pk = v12 ? (r.key_off == 0 ? k_dv_part<0> : r.key_off == 4 ? k_dv_part<1> : k_dv_part<2>) : k_dv_part<-1>;
    hipLaunchKernelGGL(pk, dim3(unsigned(ntiles)), dim3(kDvBlock), 0, s, v, domain, lg, pos, bounds, outs);
    hipLaunchKernelGGL(k_dv_bits, dim3(ns * g2), dim3(kDvBlock), wps * sizeof(uint32_t), s, pos, bounds, lg, ntiles,
                       g2, wps, part);
    hipLaunchKernelGGL(k_dv_merge, dim3(grid_for(ctx, uint64_t(wps) << lg, kBlock * 4)), dim3(kBlock), 0, s, part, lg,
                       g2, wps, words, static_cast<uint32_t*>(bitmap));
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_key_bitmap, dim3(grid_for(ctx, r.n, kBlock * 4)), dim3(kBlock), 0, s, view_of(r), domain,
                     static_cast<uint32_t*>(bitmap), static_cast<unsigned long long*>(outside));
  return hipGetLastError();
}

hipError_t bitmap_or_popcount(hj3d_ctx* ctx, const void* bitmaps, uint32_t rows, uint64_t words, void* count,
                              hipStream_t s) {
  if (words == 0 || rows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_or_popcount, dim3(grid_for(ctx, words, kBlock * 4)), dim3(kBlock), 0, s,
                     static_cast<const uint32_t*>(bitmaps), rows, words, static_cast<unsigned long long*>(count));
  return hipGetLastError();
}

}  // namespace hj3d

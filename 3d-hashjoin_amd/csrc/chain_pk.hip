// chain_pk.hip — the unique chaining probe on PACKED pairs: the config-B hot path
// (AlgHashJoinProbe<..., IsBuildKeyUnique = true>::step, algebra.hh:625-659, over a whole scanned
// relation). Two launches per probe strand, nothing else on the stream:
//
//   k_pk_part   one persistent 1024-thread workgroup per CU streams the probe relation once:
//               hash (murmur3 fmix32), bucket b = h % NB and the slice p of b (slices of W
//               buckets, sized so that a slice of the table fits LDS), and writes the pair
//               {v, row} with v = (b - p*W) << qbits | h / NB to the workgroup's region of slice p.
//               The bucket and the quotient determine h (h = (h / NB) * NB + b), so the probe needs
//               neither a modulo nor a division per tuple. Regions are written in whole 128-B
//               segments (runs shorter than a segment ride in registers to the next tile).
//   k_pk_probe  one 1024-thread workgroup per slice (or share of its regions): stages the slice
//               (directory + entries, entry hashes turned into quotients) in LDS, reserves its
//               output range with one atomic, probes every pair against LDS in the reference's
//               walk order with the unique early exit, writes {row, partner} densely; then the
//               pairs that overflowed a region (skewed probe keys) are taken in chunks by whichever
//               workgroups finish first, against the table in HBM; the last workgroup to finish
//               folds every workgroup's counters into the result slot and resets the control words.
// The control words (overflow count, output cursor, ticket, ...) are zero between probes: the last
// workgroup of k_pk_probe restores them, so no fill runs on the stream.
// Counters are those of radix.hip's probe: c_htProbeCmp from the sorted-bucket walk
// [index 0, n-1, ..., 1] with early exit (buckets <= 32 entries), the order-free form beyond.
#include <cmath>

#include "radix_seg.hpp"

namespace hj3d {
namespace {

constexpr int kPkBlock = 1024;
// Tunables, fixed by the sweeps recorded in DESIGN.md 4.1 (the losing variants are gone from the
// source): 8192-tuple tiles (4096: 0.556 ms, 8192: 0.466 ms for k_pk_part at config B), the next tile's
// keys loaded once the stage is built (two tiles ahead spilled), 128-B region segments (64-B: slower in
// both kernels), non-temporal key loads (0.447 -> 0.436 ms) and region stores (0.452 -> 0.447 ms),
// five barriers per tile, guarded key loads and rank atomics (the clamped form was not faster).
constexpr int kPkRounds = 8;
constexpr int kPkTile = kPkBlock * kPkRounds;
constexpr int kPkTBits = 32 - __builtin_clz(uint32_t(kPkTile - 1));  // bits of a rank inside the tile
constexpr uint32_t kPkSeg = 16;                                     // pairs per region segment (128 B)
constexpr uint32_t kPkStage = 17408;  // LDS stage (pairs): the tile + the carried pairs (< kPkSeg per slice)
static_assert(kPkTile <= kPkStage && kPkStage < 65536, "the tile alone fits the stage; stage offsets in 16 bits");
// the stage of the two-slices-per-thread form (64-B segments: carries of < 8 pairs, ~3.5 on average per
// slice, so the tile and ~7 K carried pairs; with its 16 KB of slice words and 15.5 KB of segment
// words it fills the LDS)
constexpr uint32_t kPkStage2 = 15872;
constexpr uint32_t kPkMaxP1 = 2 * kPkBlock;  // slices one partition level takes (two per thread)
constexpr uint32_t kSortedMaxPk = 32;
constexpr uint32_t kOvfFlag = 0x80000000u;

// control words (u64) of one probe strand
enum { kCtlNovf = 0, kCtlOut = 1, kCtlTicket = 2, kCtlOvfCursor = 3, kCtlNprobe = 4, kCtlWords = 8 };


// Wave-aggregated append to the overflow list: pairs {h, row} (counted in ctl[kCtlNovf]).
__device__ __forceinline__ void pk_ovf_append(bool me, uint2 e, uint2* __restrict__ ovf, uint64_t* ctl) {
  const uint64_t m = __ballot(me);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint64_t b = 0;
  if (lane == leader) b = atomicAdd(reinterpret_cast<unsigned long long*>(ctl + kCtlNovf), (unsigned long long)__popcll(m));
  b = __shfl(b, leader, kWave);
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  if (me) ovf[b + __popcll(m & lt)] = e;
}

// ---- k_pk_part: the probe relation -> packed pairs in per-(workgroup, slice) regions ----
// Regions: region[(g * P + p) * cap + k], counts[g * P + p] pairs. PPT slices per thread (P <= 1024
// PPT): thread t carries slices t + k * 1024's leftover pairs (< one segment each) in registers. PPT = 1:
// 128-B segments; PPT = 2 (1024 < P <= 2048, one partition level instead of two: config D's
// 2.5e7-bucket rank at 4 GPUs): 64-B segments, a smaller carry and stage. SEL: a one-word selection
// fused in.
// Memory ordering: vmcnt counts loads and stores together, in issue order, so a load can only be
// waited for together with every older store. The next tile's keys are loaded right after this tile's
// stage is built (loading two tiles ahead, so that the wait would never cover this tile's region
// stores, spilled registers and measured slower).
template <int PPT>
struct PkPartGeom {
  static constexpr uint32_t kSeg = kPkSeg / PPT;                          // pairs per region segment
  static constexpr uint32_t kStage = PPT == 1 ? kPkStage : kPkStage2;      // LDS stage (pairs)
};
template <bool IMPLICIT, bool SEL, int PPT>
__global__ __launch_bounds__(kPkBlock) void k_pk_part(RelView r, PkGeom pk, uint32_t ntiles, uint32_t cap,
                                                      uint2* __restrict__ region, uint32_t* __restrict__ counts,
                                                      uint2* __restrict__ ovf, uint64_t* __restrict__ ctl,
                                                      SelRange sel, uint32_t stage_lim) {
  constexpr uint32_t SEG = PkPartGeom<PPT>::kSeg, STAGE = PkPartGeom<PPT>::kStage;
  __shared__ uint2 stage[STAGE];
  __shared__ uint32_t loc[kPkBlock * PPT];
  __shared__ uint32_t sbase[kPkBlock * PPT];
  __shared__ uint2 seginfo[STAGE / SEG];  // whole segment: {region index | kOvfFlag + slice, stage start}
  __shared__ uint32_t wsum[kPkBlock / kWave];
  const uint32_t me = threadIdx.x, P = pk.P, n = uint32_t(r.n);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // this thread's slices sl(k) = me + k * 1024 and their regions (host: G * P * cap < 2^31)
  const auto sl = [&](int k) __attribute__((always_inline)) { return me + uint32_t(k) * kPkBlock; };
  uint32_t my_reg[PPT];
  uint2 creg[PPT][SEG - 1];
  // my_cur: pairs taken by the slice's region so far; my_end: where its region stopped taking pairs
  // (cap, or the start of the first segment that did not fit: after a mid-stream carry flush the
  // cursor is no longer segment-aligned, so a segment may straddle the region's end)
  uint32_t my_kc[PPT], my_cur[PPT], my_end[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    my_reg[k] = (blockIdx.x * P + sl(k)) * cap;
    my_kc[k] = 0;
    my_cur[k] = 0;
    my_end[k] = cap;
#pragma unroll
    for (int j = 0; j < int(SEG) - 1; ++j) creg[k][j] = make_uint2(0, 0);
  }
  uint32_t ha[kPkRounds], pa[SEL ? kPkRounds : 1];
  // explicit rows: loaded with the key at tile prefetch and kept in registers (the row word shares
  // the key's line; loading it again after the ranking phase fetched that line twice: 15.4 B per
  // 8-B received pair, round 3).
  uint32_t wa[IMPLICIT ? 1 : kPkRounds];
  // {key, row} pairs: two 4-B loads issued back to back (the second hits the line the first brought
  // in) measured faster than one 8-B load: 1e8 received pairs, same box, 0.505 / 0.505 against
  // 0.597 / 0.593 ms (profiles/r04f_ab_pairs.log).
  auto load = [&](uint32_t (&h)[kPkRounds], uint32_t (&pw)[SEL ? kPkRounds : 1],
                  uint32_t (&rw)[IMPLICIT ? 1 : kPkRounds], uint32_t tile) __attribute__((always_inline)) {
    const uint32_t base = tile * kPkTile;
#pragma unroll
    for (int j = 0; j < kPkRounds; ++j) {
      const uint32_t i = base + uint32_t(j) * kPkBlock + me;
      const char* t = r.base + uint64_t(i) * r.stride;
      h[j] = i < n ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(t + r.key_off)) : 0u;
      if constexpr (!IMPLICIT)
        rw[j] = i < n ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(t + r.row_off)) : 0u;
      if constexpr (SEL) pw[j] = i < n ? *reinterpret_cast<const uint32_t*>(t + sel.word_off) : 0u;
    }
  };
  auto to_ovf = [&](uint2 e, uint32_t p, bool me_) __attribute__((always_inline)) {  // packed pair of slice p -> {h, row}
    pk_ovf_append(me_, make_uint2(pk.hash_of(e.x, p), e.y), ovf, ctl);
  };
  auto flush_carry = [&]() __attribute__((always_inline)) {  // partial segments at the cursors
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
#pragma unroll
      for (int j = 0; j < int(SEG) - 1; ++j) {
        const bool v = sl(k) < P && uint32_t(j) < my_kc[k];
        const uint32_t o = my_cur[k] + j;
        if (v && o < my_end[k]) region[my_reg[k] + o] = creg[k][j];
        to_ovf(creg[k][j], sl(k), v && o >= my_end[k]);
      }
      my_cur[k] += my_kc[k];
      my_kc[k] = 0;
    }
  };
  // exclusive scan of one value per thread
  auto scan = [&](uint32_t v, uint32_t* total) __attribute__((always_inline)) {
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
    for (int w = 0; w < kPkBlock / kWave; ++w) {
      const uint32_t t = wsum[w];
      if (w < wid) pre += t;
      tot += t;
    }
    __syncthreads();
    *total = tot;
    return pre + x - v;
  };
  uint32_t npassed = 0;
  auto process = [&](uint32_t tile, uint32_t (&h)[kPkRounds], uint32_t (&pw)[SEL ? kPkRounds : 1],
                     uint32_t (&rw)[IMPLICIT ? 1 : kPkRounds]) __attribute__((always_inline)) {
    // a slice counter is cleared right after its count is read (nothing touches it again in the tile)
    // and no barrier ends the tile: the next tile's first LDS writes (stage, seginfo, sbase) come after
    // its ranking barrier, which every thread reaches only when done reading
    const uint32_t base = tile * kPkTile;
    uint32_t rk[kPkRounds];
    // hash, bucket, slice, rank: the LDS atomics are unconditional (invalid tuples add 0 to slot 0)
#pragma unroll
    for (int j = 0; j < kPkRounds; ++j) {
      const uint32_t i = base + uint32_t(j) * kPkBlock + me;
      const uint32_t hv = murmur32(h[j]);
      const uint32_t q = pk.dnb.div(hv);
      const uint32_t bl = hv - q * pk.nb - pk.lo;
      bool pass = i < n;
      if constexpr (SEL) {
        pass = pass && sel.test(pw[j]);
        npassed += pass;
      }
      const bool ok = pass && bl < pk.nbl;
      rk[j] = kInvalid;
      if (ok) {
        const uint32_t p = pk.dw.div(bl);
        h[j] = ((bl - p * pk.W) << pk.qbits) | q;  // the packed pair's first word
        rk[j] = (p << kPkTBits) | atomicAdd(&loc[p], 1u);
      }
    }
    __syncthreads();
    uint32_t my_c[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      my_c[k] = sl(k) < P ? loc[sl(k)] : 0u;
      loc[sl(k)] = 0;
    }
    // per slice (L << 16) | L / SEG, L = its carry + this tile's pairs; the thread's slices in a row
    const auto seg_counts = [&](int k) __attribute__((always_inline)) {
      const uint32_t L = my_kc[k] + my_c[k];
      return (L << 16) | (L / SEG);
    };
    const auto seg_sum = [&]() __attribute__((always_inline)) {
      uint32_t t = 0;
#pragma unroll
      for (int k = 0; k < PPT; ++k) t += seg_counts(k);
      return t;
    };
    uint32_t tot;
    uint32_t pre = scan(seg_sum(), &tot);
    if ((tot >> 16) > stage_lim) {  // too many carried pairs: write them out; the tile alone fits
      flush_carry();
      pre = scan(seg_sum(), &tot);
    }
    const uint32_t nfull = tot & 0xFFFFu;
    uint32_t my_loc[PPT], my_len[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      my_loc[k] = pre >> 16;
      const uint32_t my_fseg = pre & 0xFFFFu;
      pre += seg_counts(k);
      my_len[k] = my_kc[k] + my_c[k];
      if (sl(k) < P) {
        sbase[sl(k)] = my_loc[k] + my_kc[k];
#pragma unroll
        for (int j = 0; j < int(SEG) - 1; ++j)
          if (uint32_t(j) < my_kc[k]) stage[my_loc[k] + j] = creg[k][j];
        for (uint32_t sg = 0; sg < my_len[k] / SEG; ++sg) {
          // segment-aligned (cap is a multiple of SEG) unless a mid-stream flush moved the cursor:
          // a segment goes to the region only whole, else (all of it) to the overflow list
          const uint32_t o = my_cur[k] + sg * SEG;
          const bool fit = o + SEG <= my_end[k];
          if (!fit && o < my_end[k]) my_end[k] = o;
          seginfo[my_fseg + sg] = make_uint2(fit ? my_reg[k] + o : (kOvfFlag | sl(k)), my_loc[k] + sg * SEG);
        }
      }
    }
    __syncthreads();
    const uint32_t rb = IMPLICIT ? uint32_t(r.row_base) + base : 0u;
#pragma unroll
    for (int j = 0; j < kPkRounds; ++j) {
      if (rk[j] == kInvalid) continue;
      const uint32_t li = uint32_t(j) * kPkBlock + me;
      uint32_t row;
      if constexpr (IMPLICIT) row = rb + li;
      else row = rw[j];
      stage[sbase[rk[j] >> kPkTBits] + (rk[j] & ((1u << kPkTBits) - 1))] = make_uint2(h[j], row);
    }
    load(h, pw, rw, tile + gridDim.x);  // the next tile (keys past the end load nothing)
    __syncthreads();
    // whole segments: SEG consecutive lanes store one segment
    for (uint32_t kk = me; kk < nfull * SEG; kk += kPkBlock) {
      const uint2 si = seginfo[kk / SEG];
      const uint32_t j = kk % SEG;
      const uint2 e = stage[si.y + j];
      const bool spill = si.x & kOvfFlag;
      if (!spill)
        __builtin_nontemporal_store((uint64_t(e.y) << 32) | e.x, reinterpret_cast<uint64_t*>(region + si.x + j));
      to_ovf(e, si.x & ~kOvfFlag, spill);
    }
    // the run's tail (< one segment) becomes the slice's carry
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      if (sl(k) < P) {
        const uint32_t F = my_len[k] - my_len[k] % SEG;
#pragma unroll
        for (int j = 0; j < int(SEG) - 1; ++j)
          if (uint32_t(j) < my_len[k] - F) creg[k][j] = stage[my_loc[k] + F + j];
        my_cur[k] += F;
        my_kc[k] = my_len[k] - F;
      }
    }
  };
#pragma unroll
  for (int k = 0; k < PPT; ++k) loc[sl(k)] = 0;
  __syncthreads();
  load(ha, pa, wa, blockIdx.x);
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) process(tile, ha, pa, wa);
  flush_carry();
#pragma unroll
  for (int k = 0; k < PPT; ++k)
    if (sl(k) < P) counts[blockIdx.x * P + sl(k)] = min(my_cur[k], my_end[k]);
  // n_probe: every scanned tuple (the reference's probe count), or the selection's passing tuples
  if constexpr (SEL) {
    uint32_t c = npassed;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
    if (lane == 0 && c) atomicAdd(reinterpret_cast<unsigned long long*>(ctl + kCtlNprobe), (unsigned long long)c);
  } else {
    if (blockIdx.x == 0 && me == 0) atomicAdd(reinterpret_cast<unsigned long long*>(ctl + kCtlNprobe), (unsigned long long)n);
  }
}

// ---- k_pk_split: the second partition level (more than 1024 slices) ----
// k_pk_part then partitions by coarse ranges of C slices (its packed word holds the bucket inside
// the coarse range); workgroup (p1, s) takes the pass-1 regions g in [G1 s / S2, G1 (s + 1) / S2) of
// coarse range p1 as one stream, re-packs every pair for its slice p = p1 C + c (bucket inside the
// slice) and writes it to the fine region (s, p) at fine[(s * P + p) * cap2], counts2[s * P + p]
// pairs: exactly the region layout k_pk_probe walks (G = S2 regions per slice). Per 8192-pair tile:
// rank by slice with a wave-level multi-split (one ballot per bit of c, one LDS atomic per slice and
// wave), stage the tile slice-major in LDS, write each slice's run out with consecutive lanes on
// consecutive pairs. Pairs past a fine region's capacity go to the overflow list as {h, row}.
// workgroup size: several per CU (1024: 4.21 ms, 512: 3.50, 256: 3.39 at config D); the next tile's
// pairs are loaded while this one is split (3.51 ms without)
constexpr int kSpBlock = 256;
constexpr int kSpRounds = 8;
constexpr int kSpTile = kSpBlock * kSpRounds;
constexpr uint32_t kSpMaxC = 64;
__global__ __launch_bounds__(kSpBlock) void k_pk_split(const uint2* __restrict__ reg1,
                                                       const uint32_t* __restrict__ cnt1, uint32_t G1, uint32_t P1,
                                                       uint32_t cap1, uint32_t S2, PkGeom pk, uint32_t C,
                                                       uint32_t cbits, uint32_t cap2, uint2* __restrict__ reg2,
                                                       uint32_t* __restrict__ cnt2, uint2* __restrict__ ovf,
                                                       uint64_t* __restrict__ ctl) {
  __shared__ uint2 stage[kSpTile];
  __shared__ uint8_t cof[kSpTile];
  __shared__ uint32_t rstart[66];
  __shared__ uint32_t tcnt[2][kSpMaxC];
  __shared__ uint32_t tstart[kSpMaxC];
  __shared__ uint2 dlim[kSpMaxC];  // {fine index of stage position 0 of the slice's run, region end}
  __shared__ uint32_t cur[kSpMaxC];
  const uint32_t me = threadIdx.x;
  const int lane = threadIdx.x & 63;
  const uint32_t p1 = blockIdx.x / S2, s = blockIdx.x % S2;
  const uint32_t g_lo = uint32_t(uint64_t(G1) * s / S2), g_hi = uint32_t(uint64_t(G1) * (s + 1) / S2);
  const uint32_t nr = g_hi - g_lo;  // <= 64 (host: G1 <= 64 * S2)
  const uint32_t pbase = p1 * C;    // first fine slice of the coarse range
  if (me < 64) {
    const uint32_t len = uint32_t(lane) < nr ? cnt1[uint64_t(g_lo + lane) * P1 + p1] : 0u;
    uint32_t tot;
    const uint32_t pre = wave_excl_scan(len, &tot);
    if (uint32_t(lane) < nr) rstart[lane] = pre;
    if (lane == 0) {
      rstart[nr] = tot;
      rstart[nr + 1] = tot;
    }
  }
  if (me < kSpMaxC) {
    tcnt[0][me] = 0;
    tcnt[1][me] = 0;
    cur[me] = 0;
  }
  __syncthreads();
  const uint32_t total = rstart[nr];
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  // per-lane stream cursor: region cr holds stream positions [rstart[cr], nst)
  uint32_t cr = 0, nst = rstart[1];
  const uint2* rsrc = reg1 + (uint64_t(g_lo) * P1 + p1) * cap1;
  auto load = [&](uint2 (&v)[kSpRounds], uint32_t t0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kSpRounds; ++j) {
      const uint32_t f = t0 + uint32_t(j) * kSpBlock + me;
      v[j] = make_uint2(0, 0);
      if (f < total) {
        while (f >= nst) {
          ++cr;
          nst = rstart[cr + 1];
          rsrc = reg1 + (uint64_t(g_lo + cr) * P1 + p1) * cap1;
        }
        v[j] = rsrc[f - rstart[cr]];
      }
    }
  };
  uint2 cv[kSpRounds];
  load(cv, 0);
  uint32_t par = 0;
  for (uint32_t t0 = 0; t0 < total; t0 += kSpTile, par ^= 1u) {
    uint2 nv[kSpRounds];
    load(nv, t0 + kSpTile);
    uint32_t cc[kSpRounds], rk[kSpRounds];
#pragma unroll
    for (int j = 0; j < kSpRounds; ++j) {
      const bool valid = t0 + uint32_t(j) * kSpBlock + me < total;
      const uint32_t bic = cv[j].x >> pk.qbits;  // bucket inside the coarse range
      const uint32_t c = valid ? pk.dw.div(bic) : 0u;
      cv[j].x = ((bic - c * pk.W) << pk.qbits) | (cv[j].x & pk.qmask);
      cc[j] = c;
      // lanes of this wave with the same slice: one ballot per bit of c
      uint64_t m = __ballot(valid);
      for (uint32_t b = 0; b < cbits; ++b) {
        const uint64_t mb = __ballot(valid && ((c >> b) & 1u));
        m &= ((c >> b) & 1u) ? mb : ~mb;
      }
      const bool leader = (m & lt) == 0;
      uint32_t base = 0;
      if (valid && leader) base = atomicAdd(&tcnt[par][c], uint32_t(__popcll(m)));
      base = __shfl(base, valid ? __ffsll((unsigned long long)m) - 1 : lane, kWave);
      rk[j] = valid ? base + uint32_t(__popcll(m & lt)) : kInvalid;
    }
    __syncthreads();
    if (me < 64) {  // slice runs of the tile: starts in the stage, destinations, cursors
      uint32_t run_pre = 0;
      for (uint32_t c0 = 0; c0 < C; c0 += 64) {
        const uint32_t c = c0 + lane;
        const uint32_t n = c < C ? tcnt[par][c] : 0u;
        uint32_t tot;
        const uint32_t pre = wave_excl_scan(n, &tot) + run_pre;
        if (c < C) {
          const uint32_t fb = (s * pk.P + pbase + c) * cap2;
          tstart[c] = pre;
          dlim[c] = make_uint2(fb + cur[c] - pre, fb + cap2);
          cur[c] += n;
          tcnt[par ^ 1u][c] = 0;
        }
        run_pre += tot;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSpRounds; ++j) {
      if (rk[j] == kInvalid) continue;
      const uint32_t k = tstart[cc[j]] + rk[j];
      stage[k] = cv[j];
      cof[k] = uint8_t(cc[j]);
    }
    __syncthreads();
    const uint32_t tn = min(uint32_t(kSpTile), total - t0);
    for (uint32_t k = me; k < tn; k += kSpBlock) {
      const uint32_t c = cof[k];
      const uint2 dl = dlim[c];
      const uint2 e = stage[k];
      const uint32_t d = dl.x + k;
      const bool fit = d < dl.y;
      if (fit) reg2[d] = e;
      pk_ovf_append(!fit, make_uint2(pk.hash_of(e.x, pbase + c), e.y), ovf, ctl);
    }
#pragma unroll
    for (int j = 0; j < kSpRounds; ++j) cv[j] = nv[j];
  }
  __syncthreads();
  if (me < C && pbase + me < pk.P) cnt2[uint64_t(s) * pk.P + pbase + me] = min(cur[me], cap2);
}

// ---- k_pk_probe ----
constexpr uint32_t kLdsWords = kPkLdsWords;
// packed pairs in and output pairs out as one non-temporal 8-B access each (two 4-B accesses: no gain)
__device__ __forceinline__ void pair_st(uint2* p, uint32_t lo, uint32_t hi) {
  __builtin_nontemporal_store((uint64_t(hi) << 32) | lo, reinterpret_cast<uint64_t*>(p));
}
__device__ __forceinline__ uint64_t pair_ld(const uint2* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p));
}
// K = pairs per lane and chunk (the next chunk in flight), chosen per probe from the expected
// region length (pk_items): a region of L pairs costs ceil(L / 64K) chunks of 64K item slots, so
// K = 7 walks config B's ~384-pair regions in one 448-slot chunk where K = 8 spends 512 slots.
// All K items of a chunk have their LDS lookups batched.
constexpr int kItemsMin = 5, kItemsMax = 8;

// Unique probe of one lane's items against the LDS slice: directory word (start << 16 | count),
// entries {q, row} sorted by row inside buckets of <= 32. Walk position c = 0, 1, 2 (sorted index
// 0, n-1, n-2) batched over K items, the rest per item.
template <int K, int MODE, bool CK>
__device__ __forceinline__ void pk_probe_items(const uint64_t (&v)[K], uint32_t valid, uint64_t slot0,
                                               const uint32_t* ldir, const uint2* lent, const PkGeom& pk,
                                               uint64_t (&acc)[kProbeFields], uint2* __restrict__ out,
                                               uint64_t out_cap) {
  uint32_t nm = 0, sc = 0, nv = 0;
#pragma unroll
  for (int g = 0; g < K; g += K) {
    uint32_t d[K], match[K], cmps[K], q[K];
    bool live[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const bool ok = (valid >> (g + j)) & 1u;
      const uint32_t x = uint32_t(v[g + j]);
      q[j] = x & pk.qmask;
      const uint32_t w = ldir[ok ? x >> pk.qbits : 0u];
      d[j] = ok ? w : 0u;
      match[j] = kInvalid;
      cmps[j] = d[j] & 0xFFFFu;
      live[j] = cmps[j] != 0 && cmps[j] <= kSortedMaxPk;
    }
#pragma unroll
    for (uint32_t c = 0; c < 3; ++c) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint32_t nn = d[j] & 0xFFFFu;
        const bool ok = live[j] && c < nn;
        const uint2 e = lent[ok ? (d[j] >> 16) + (c == 0 ? 0u : nn - c) : 0u];
        const bool hit = ok && e.x == q[j];
        match[j] = hit ? e.y : match[j];
        cmps[j] = hit ? c + 1 : cmps[j];
        live[j] = live[j] && !hit;
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t nn = d[j] & 0xFFFFu, s = d[j] >> 16;
      if (live[j] && nn > 3) {
        for (uint32_t c = 3; c < nn; ++c) {
          const uint2 e = lent[s + nn - c];
          if (e.x == q[j]) {
            cmps[j] = c + 1;
            match[j] = e.y;
            break;
          }
        }
      } else if (nn > kSortedMaxPk) {  // long bucket in arrival order: order-free form
        uint32_t minrow = kInvalid, lo_m = kInvalid, hi_m = 0, cnt = 0;
        for (uint32_t k = s; k < s + nn; ++k) {
          const uint2 e = lent[k];
          minrow = min(minrow, e.y);
          if (e.x == q[j]) {
            ++cnt;
            lo_m = min(lo_m, e.y);
            hi_m = max(hi_m, e.y);
          }
        }
        if (cnt != 0 && lo_m == minrow) {
          cmps[j] = 1;
          match[j] = lo_m;
        } else if (cnt != 0) {
          uint32_t gt = 0;
          for (uint32_t k = s; k < s + nn; ++k) gt += lent[k].y > hi_m;
          cmps[j] = 2 + gt;
          match[j] = hi_m;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const bool ok = (valid >> (g + j)) & 1u;
      const uint32_t row = uint32_t(v[g + j] >> 32);
      const bool m = match[j] != kInvalid;
      nv += ok;
      nm += m;
      sc += cmps[j];
      if (MODE == 1) {
        const uint64_t slot = slot0 + uint32_t((g + j) * 64);
        if (ok && slot < out_cap) pair_st(out + slot, row, match[j]);
      }
      if (CK && m) {
        acc[4] += row;
        acc[5] += match[j];
        const uint64_t ph = pair_hash(row, match[j]);
        acc[7] += ph;
        acc[8] ^= ph;
      }
    }
  }
  acc[1] += nm;
  acc[2] += nm;
  acc[3] += sc;
  (void)nv;
}

// The same unique probe of one {h, row} pair against buckets in HBM (off / ent, entries {h, row}):
// slices that do not fit LDS (heavy skew) and the overflow pairs.
template <int MODE, bool CK>
__device__ __forceinline__ void pk_probe_hbm(uint32_t h, uint32_t row, uint32_t s, uint32_t nn,
                                             const uint2* __restrict__ ent, uint64_t slot,
                                             uint64_t (&acc)[kProbeFields], uint2* __restrict__ out,
                                             uint64_t out_cap) {
  uint32_t match = kInvalid, cmps = nn;
  if (nn <= kSortedMaxPk) {
    for (uint32_t c = 0; c < nn; ++c) {
      const uint2 e = ent[s + (c == 0 ? 0u : nn - c)];
      if (e.x == h) {
        cmps = c + 1;
        match = e.y;
        break;
      }
    }
  } else {
    uint32_t minrow = kInvalid, lo_m = kInvalid, hi_m = 0, cnt = 0;
    for (uint32_t k = s; k < s + nn; ++k) {
      const uint2 e = ent[k];
      minrow = min(minrow, e.y);
      if (e.x == h) {
        ++cnt;
        lo_m = min(lo_m, e.y);
        hi_m = max(hi_m, e.y);
      }
    }
    if (cnt != 0 && lo_m == minrow) {
      cmps = 1;
      match = lo_m;
    } else if (cnt != 0) {
      uint32_t gt = 0;
      for (uint32_t k = s; k < s + nn; ++k) gt += ent[k].y > hi_m;
      cmps = 2 + gt;
      match = hi_m;
    }
  }
  acc[3] += cmps;
  if (match != kInvalid) {
    acc[1] += 1;
    acc[2] += 1;
    if (CK) {
      acc[4] += row;
      acc[5] += match;
      const uint64_t ph = pair_hash(row, match);
      acc[7] += ph;
      acc[8] ^= ph;
    }
  }
  if (MODE == 1 && slot < out_cap)
    __builtin_nontemporal_store((uint64_t(match) << 32) | row, reinterpret_cast<uint64_t*>(out + slot));
}

// Slice of buckets [b0, b0 + nbs) into LDS: directory words (start - e0) << 16 | count, then the
// entries with their hash replaced by the quotient h / NB (the bucket is implied by the slot).
// All loads of a round batch are issued before the first LDS write.
__device__ __forceinline__ void pk_stage(const uint32_t* __restrict__ off, const uint2* __restrict__ ent, uint32_t b0,
                                         uint32_t nbs, uint32_t e0, uint32_t ne, const FastDiv32& dnb, uint32_t* ldir,
                                         uint2* lent) {
  constexpr int kStage = 12;
  const uint32_t nmax = max(nbs, ne);
  for (uint32_t k0 = threadIdx.x; k0 < nmax; k0 += kPkBlock * kStage) {
    uint32_t a[kStage], b[kStage];
    uint2 x[kStage];
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const uint32_t k = k0 + u * kPkBlock;
      a[u] = k < nbs ? off[b0 + k] : 0u;
      b[u] = k < nbs ? off[b0 + k + 1] : 0u;
      x[u] = k < ne ? ent[e0 + k] : make_uint2(0, 0);
    }
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const uint32_t k = k0 + u * kPkBlock;
      if (k < nbs) ldir[k] = ((a[u] - e0) << 16) | (b[u] - a[u]);
      if (k < ne) lent[k] = make_uint2(dnb.div(x[u].x), x[u].y);
    }
  }
}

template <int K, int MODE, bool CK>
__global__ __launch_bounds__(kPkBlock) void k_pk_probe(const uint2* __restrict__ region,
                                                       const uint32_t* __restrict__ counts, uint32_t G, uint32_t cap,
                                                       uint32_t splits, bool flat, const uint32_t* __restrict__ off,
                                                       const uint2* __restrict__ ent, PkGeom pk, FastMod fm,
                                                       uint2* __restrict__ out, uint64_t out_cap,
                                                       const uint2* __restrict__ ovf, uint64_t* __restrict__ ctl,
                                                       uint64_t* __restrict__ partials, uint64_t* __restrict__ res,
                                                       int accumulate) {
  constexpr int BLOCK = kPkBlock;
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint32_t wtot[BLOCK / kWave];
  __shared__ uint32_t rpre[BLOCK / kWave][65];
  __shared__ uint64_t bbase;
  __shared__ uint64_t red[BLOCK / kWave][kProbeFields];
  __shared__ uint32_t flag;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kWaves = BLOCK / kWave;
  const uint32_t P = pk.P;
  const uint32_t p = blockIdx.x / splits, sp = blockIdx.x % splits;
  const uint32_t b0 = p * pk.W;
  const uint32_t nbs = min(pk.W, pk.nbl - b0);
  const uint32_t e0 = off[b0], e1 = off[b0 + nbs], ne = e1 - e0;
  const bool fits = (nbs + 2) + 2ull * ne <= kLdsWords;
  uint32_t* ldir = lds;
  uint2* lent = reinterpret_cast<uint2*>(lds + ((nbs + 2) & ~1u));
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};

  // this block's regions: wave w takes g = g_lo + w + 16 k (lane k holds region k's count)
  const uint32_t g_lo = uint32_t(uint64_t(G) * sp / splits), g_hi = uint32_t(uint64_t(G) * (sp + 1) / splits);
  const uint32_t nr = g_hi > g_lo + wid ? (g_hi - g_lo - wid + kWaves - 1) / kWaves : 0u;  // <= 64
  uint32_t my_len = 0;
  if (uint32_t(lane) < nr) my_len = counts[(g_lo + wid + kWaves * lane) * P + p];
  uint32_t wtotal;
  const uint32_t my_pre = wave_excl_scan(my_len, &wtotal);  // wave-local stream offset of region `lane`
  if (lane == 0) wtot[wid] = wtotal;
  rpre[wid][lane] = uint32_t(lane) < nr ? my_pre : ~0u;  // region starts of the wave's stream
  if (lane == 0) rpre[wid][64] = ~0u;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kWaves; ++w) t += wtot[w];
    bbase = (MODE == 1 && t) ? atomicAdd(reinterpret_cast<unsigned long long*>(ctl + kCtlOut), (unsigned long long)t) : 0ull;
  }
  uint32_t wpre = 0;
  for (int w = 0; w < wid; ++w) wpre += wtot[w];
  auto pre_at = [&](uint32_t k) __attribute__((always_inline)) { return uint32_t(__builtin_amdgcn_readlane(int(my_pre), int(k))); };
  auto len_at = [&](uint32_t k) __attribute__((always_inline)) { return uint32_t(__builtin_amdgcn_readlane(int(my_len), int(k))); };
  auto src_of = [&](uint32_t k) __attribute__((always_inline)) { return region + (g_lo + wid + kWaves * k) * P * cap + p * cap; };

  // one chunk = K x 64 consecutive items of the wave's stream (flat: regions concatenated;
  // otherwise a chunk stays inside one region). Loads of the steady-state loops are unconditional
  // (clamped addresses). (Stores of absent items to a sink, for a fixed store count per chunk, were
  // tried and not kept.)
  // flat: each lane keeps its own cursor, region cr holding stream positions [its start, nst), and
  // steps it forward (positions only grow, the region starts come from rpre): a compare per item
  const auto src_off = [&](uint32_t k) __attribute__((always_inline)) {
    return int64_t((uint64_t(g_lo + wid + kWaves * k) * P + p) * cap);
  };
  uint32_t cr = 0, nst = rpre[wid][1];
  int64_t cbase = src_off(0);  // region cr's first pair - its stream start
  auto load_flat = [&](uint64_t (&v)[K], uint32_t f0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t f = min(f0 + j * 64 + lane, wtotal - 1);  // clamped (the last prefetch re-reads)
      while (f >= nst) {
        ++cr;
        cbase = src_off(cr) - int64_t(nst);
        nst = rpre[wid][cr + 1];
      }
      v[j] = pair_ld(region + (cbase + int64_t(f)));
    }
  };
  // non-flat cursor: region r, offset qq
  uint32_t r = 0, qq = 0, len = nr ? len_at(0) : 0u;
  while (r < nr && len == 0) {
    ++r;
    len = r < nr ? len_at(r) : 0u;
  }
  auto load_reg = [&](uint64_t (&v)[K], uint32_t rr, uint32_t q0, uint32_t ll) __attribute__((always_inline)) {
    const uint2* src = rr < nr ? src_of(rr) : region;
    const uint32_t last = ll ? ll - 1 : 0u;
#pragma unroll
    for (int j = 0; j < K; ++j)
      v[j] = pair_ld(src + min(q0 + j * 64 + lane, last));
  };
  auto probe_hbm_chunk = [&](const uint64_t (&v)[K], uint32_t valid, uint64_t slot0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (!((valid >> j) & 1u)) continue;
      const uint32_t x = uint32_t(v[j]), bl = b0 + (x >> pk.qbits);
      const uint32_t s = off[bl];
      pk_probe_hbm<MODE, CK>(pk.hash_of(x, p), uint32_t(v[j] >> 32), s, off[bl + 1] - s, ent, slot0 + j * 64, acc,
                             out, out_cap);
    }
  };
  // the walk: probe(v, valid mask, wave-local stream offset of the lane's item 0); stage() runs
  // (followed by a barrier) once the first chunk's loads are issued, so their latency overlaps it
  auto walk = [&](auto&& stage, auto&& probe) __attribute__((always_inline)) {
    constexpr uint32_t kChunk = 64 * K;
    uint64_t cur[K];
    if (flat) {
      if (wtotal) load_flat(cur, 0);
      stage();
      __syncthreads();
      if (wtotal == 0) return;
      for (uint32_t f0 = 0; f0 < wtotal; f0 += kChunk) {
        uint64_t nxt[K];
        load_flat(nxt, min(f0 + kChunk, (wtotal - 1) / kChunk * kChunk));
        uint32_t vm = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) vm |= uint32_t(f0 + j * 64 + lane < wtotal) << j;
        probe(cur, vm, f0 + lane);
#pragma unroll
        for (int j = 0; j < K; ++j) cur[j] = nxt[j];
      }
    } else {
      load_reg(cur, r, qq, len);
      stage();
      __syncthreads();
      while (r < nr) {
        uint32_t nr_ = r, nq = qq + kChunk, nl = len;
        while (nr_ < nr && nq >= nl) {
          ++nr_;
          nq = 0;
          nl = nr_ < nr ? len_at(nr_) : 0u;
        }
        uint64_t nxt[K];
        load_reg(nxt, nr_, nq, nl);
        uint32_t vm = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) vm |= uint32_t(qq + j * 64 + lane < len) << j;
        probe(cur, vm, pre_at(r) + qq + lane);
        r = nr_;
        qq = nq;
        len = nl;
#pragma unroll
        for (int j = 0; j < K; ++j) cur[j] = nxt[j];
      }
    }
  };
  if (fits) {
    walk([&]() __attribute__((always_inline)) { pk_stage(off, ent, b0, nbs, e0, ne, pk.dnb, ldir, lent); },
         [&](const uint64_t (&v)[K], uint32_t valid, uint32_t srel) __attribute__((always_inline)) {
           pk_probe_items<K, MODE, CK>(v, valid, bbase + wpre + srel, ldir, lent, pk, acc, out, out_cap);
         });
  } else {
    walk([&]() __attribute__((always_inline)) {},
         [&](const uint64_t (&v)[K], uint32_t valid, uint32_t srel) __attribute__((always_inline)) {
           probe_hbm_chunk(v, valid, bbase + wpre + srel);
         });
  }
  // overflow pairs {h, row} (runs that did not fit their region): chunks of 1024 claimed by any
  // workgroup that is done with its own slice; output slots from the same cursor
  const uint64_t novf = __hip_atomic_load(ctl + kCtlNovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (novf) {
    for (;;) {
      __syncthreads();
      if (threadIdx.x == 0) {
        const uint64_t c = atomicAdd(reinterpret_cast<unsigned long long*>(ctl + kCtlOvfCursor), (unsigned long long)BLOCK);
        const uint64_t take = c < novf ? min(uint64_t(BLOCK), novf - c) : 0ull;
        bbase = c;
        flag = uint32_t(take);
        if (MODE == 1 && take)
          red[0][0] = atomicAdd(reinterpret_cast<unsigned long long*>(ctl + kCtlOut), (unsigned long long)take);
      }
      __syncthreads();
      const uint32_t take = flag;
      if (!take) break;
      const uint64_t c = bbase, ob = MODE == 1 ? red[0][0] : 0ull;
      if (threadIdx.x < take) {
        const uint2 e = ovf[c + threadIdx.x];
        const uint32_t bl = fm.mod(e.x) - pk.lo;
        const uint32_t s = off[bl];
        pk_probe_hbm<MODE, CK>(e.x, e.y, s, off[bl + 1] - s, ent, ob + threadIdx.x, acc, out, out_cap);
      }
    }
  }
  // this block's counters -> partials row (write-through stores), then the ticket; the last block
  // folds every row into the result slot (loads that bypass the CU's L1) and resets the control words.
  // Ordering: the hand-off is the gfx950 form "8-B agent atomics both sides" of MI355X_MICROARCH.md
  // (inter-workgroup visibility): every partial is an 8-B relaxed agent-scope store made by wave 0,
  // which waits for them (vmcnt(0)) before its lane 0 takes the ticket with an agent-scope atomic;
  // the block whose ticket came last reads the partials with 8-B relaxed agent-scope loads after a
  // barrier. A release on the ticket (an L2 write-back per block) is not needed for that form; a
  // target that counts stores apart from loads (vscnt) would need one here.
  __syncthreads();
#pragma unroll
  for (int f = 1; f < kProbeFields; ++f) {
    const uint64_t w = f == kProbeFields - 1 ? wave_xor(acc[f]) : wave_sum(acc[f]);
    if (lane == 0) red[wid][f] = w;
  }
  __syncthreads();
  if (threadIdx.x < kProbeFields) {
    const int f = threadIdx.x;
    uint64_t a = 0;
    for (int w = 0; w < kWaves; ++w) a = f == kProbeFields - 1 ? (a ^ red[w][f]) : (a + red[w][f]);
    __hip_atomic_store(partials + uint64_t(blockIdx.x) * kProbeFields + f, f == 0 ? 0ull : a, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (wid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) {
      const uint64_t t = __hip_atomic_fetch_add(ctl + kCtlTicket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag = t == gridDim.x - 1;
    }
  }
  __syncthreads();
  if (!flag) return;
  // the last block: column sums over every block's row
  uint64_t sum[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t b = threadIdx.x; b < gridDim.x; b += BLOCK) {
#pragma unroll
    for (int f = 1; f < kProbeFields; ++f) {
      const uint64_t x = __hip_atomic_load(partials + uint64_t(b) * kProbeFields + f, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      sum[f] = f == kProbeFields - 1 ? (sum[f] ^ x) : (sum[f] + x);
    }
  }
  __syncthreads();
#pragma unroll
  for (int f = 1; f < kProbeFields; ++f) {
    const uint64_t w = f == kProbeFields - 1 ? wave_xor(sum[f]) : wave_sum(sum[f]);
    if (lane == 0) red[wid][f] = w;
  }
  __syncthreads();
  if (threadIdx.x < kProbeFields) {
    const int f = threadIdx.x;
    uint64_t a = 0;
    if (f == 0) {
      a = __hip_atomic_load(ctl + kCtlNprobe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      for (int w = 0; w < kWaves; ++w) a = f == kProbeFields - 1 ? (a ^ red[w][f]) : (a + red[w][f]);
    }
    if (accumulate) a = f == kProbeFields - 1 ? (res[f] ^ a) : (res[f] + a);
    res[f] = a;
  }
  if (!accumulate && threadIdx.x >= kProbeFields && threadIdx.x < 16) res[threadIdx.x] = 0;
  if (threadIdx.x < kCtlWords) __hip_atomic_store(ctl + threadIdx.x, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- the chaining build of tables beyond the radix build's range (config D: 1e8 buckets) ----
// R is partitioned like a probe side: k_pk_part into coarse ranges, k_pk_split into slices of
// kPbW buckets (S2 fine regions per slice). k_pk_slice_sums totals each slice's regions (then an
// exclusive scan gives its CSR base ps[p]); k_pk_build, one persistent 1024-thread workgroup per
// CU, builds slice after slice as k_rp_build3 does (radix.hip): the slice's pairs gathered into
// registers (the next slice's loads in flight while the current one is built), counted per bucket
// with LDS atomics (each pair keeps its arrival rank), bucket starts by an LDS scan, the pairs
// staged in bucket order, then each written to its row rank inside its bucket (the reference's
// chain order is arithmetic in row order: buckets of <= 32 entries sorted by row). Larger slices
// (skewed keys) go through HBM in the same kernel. Region overflows are not built here: the host
// checks the overflow count and falls back to the direct build (chain.hip).
constexpr uint32_t kPbW = 8192;       // buckets per build slice (bucket << 16 | rank packing: < 2^16)
constexpr int kPbPer = 11;            // pairs per lane in registers: fine regions of <= 704 pairs
constexpr uint32_t kPbStage = 12288;  // LDS stage of a slice's pairs
static_assert(kPbPer * kPkBlock <= int(kPbStage), "a register-held slice fits the stage");

__global__ __launch_bounds__(256) void k_pk_slice_sums(const uint32_t* __restrict__ cnt2, uint32_t S2, uint32_t P,
                                                       uint32_t* __restrict__ tot) {
  const uint32_t p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  uint32_t t = 0;
  for (uint32_t s = 0; s < S2; ++s) t += cnt2[uint64_t(s) * P + p];
  tot[p] = t;
}

// exclusive scan of n <= kPbW + 1 LDS words by one 1024-thread workgroup
__device__ __forceinline__ void pb_lds_scan(uint32_t* a, uint32_t n, uint32_t* wsum) {
  constexpr int kPer = (kPbW + kPkBlock) / kPkBlock;  // 9 words per thread
  const uint32_t t0 = threadIdx.x * kPer;
  uint32_t v[kPer], loc = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    v[k] = t0 + k < n ? a[t0 + k] : 0u;
    loc += v[k];
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t wt;
  const uint32_t pre = wave_excl_scan(loc, &wt);
  if (lane == 0) wsum[wid] = wt;
  __syncthreads();
  uint32_t base = 0;
  for (int w = 0; w < wid; ++w) base += wsum[w];
  uint32_t run = base + pre;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    if (t0 + k < n) a[t0 + k] = run;
    run += v[k];
  }
  __syncthreads();
}

__global__ __launch_bounds__(kPkBlock) void k_pk_build(const uint2* __restrict__ fine, const uint32_t* __restrict__ cnt2,
                                                       uint32_t S2, uint32_t cap2, const uint32_t* __restrict__ ps,
                                                       PkGeom pk, uint32_t* __restrict__ off, uint2* __restrict__ ent) {
  __shared__ uint32_t cnt[kPbW + 1];
  __shared__ uint2 stage[kPbStage];
  __shared__ uint32_t wsum[kPkBlock / kWave];
  constexpr uint32_t kCap = kPbPer * kPkBlock;
  const uint32_t P = pk.P, nbl = pk.nbl, W = pk.W;
  // pair i of slice p: fine[i + delta] with the delta of the last region starting at or before i
  auto gather = [&](uint32_t p, uint32_t i) __attribute__((always_inline)) {
    uint32_t run = 0;
    int64_t d = int64_t(uint64_t(p) * cap2);
    for (uint32_t sg = 0; sg < S2; ++sg) {
      if (i >= run) d = int64_t((uint64_t(sg) * P + p) * cap2) - int64_t(run);
      run += cnt2[uint64_t(sg) * P + p];
    }
    return fine[int64_t(i) + d];
  };
  // fast form: wave w holds fine region (w, p) (<= kPbPer * 64 pairs; S2 <= 16 regions per slice)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  auto fits = [&](uint32_t p) __attribute__((always_inline)) {
    bool ok = true;
    for (uint32_t sg = 0; sg < S2; ++sg) ok = ok && cnt2[uint64_t(sg) * P + p] <= uint32_t(kPbPer) * 64u;
    return ok;
  };
  uint2 ea[kPbPer], eb[kPbPer];
  auto load = [&](uint2 (&e)[kPbPer], uint32_t p) __attribute__((always_inline)) {
    if (p >= P || !fits(p)) return;
    const uint32_t c = uint32_t(wid) < S2 ? cnt2[uint64_t(wid) * P + p] : 0u;
    const uint2* src = fine + (uint64_t(wid) * P + p) * cap2;
#pragma unroll
    for (int u = 0; u < kPbPer; ++u) {
      const uint32_t i = uint32_t(u) * 64u + lane;
      e[u] = i < c ? src[i] : make_uint2(0, 0);
    }
  };
  auto build = [&](uint2 (&e)[kPbPer], uint32_t p) __attribute__((always_inline)) {
    const uint32_t b0 = p * W;
    const uint32_t nbs = min(W, nbl - b0);
    const uint32_t s0 = ps[p], m = ps[p + 1] - s0;
    for (uint32_t k = threadIdx.x; k < nbs; k += kPkBlock) cnt[k] = 0;
    __syncthreads();
    if (!fits(p) || m > kCap) {  // skewed slice: scatter through HBM, sort the small buckets there
      for (uint32_t i = threadIdx.x; i < m; i += kPkBlock) atomicAdd(&cnt[gather(p, i).x >> pk.qbits], 1u);
      __syncthreads();
      pb_lds_scan(cnt, nbs, wsum);
      for (uint32_t k = threadIdx.x; k < nbs; k += kPkBlock) off[b0 + k] = s0 + cnt[k];
      if (b0 + nbs == nbl && threadIdx.x == 0) off[nbl] = s0 + m;
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < m; i += kPkBlock) {
        const uint2 x = gather(p, i);
        ent[s0 + atomicAdd(&cnt[x.x >> pk.qbits], 1u)] = make_uint2(pk.hash_of(x.x, p), x.y);
      }
      __syncthreads();
      for (uint32_t k = threadIdx.x; k < nbs; k += kPkBlock) {
        const uint32_t bs = k ? cnt[k - 1] : 0u, n = cnt[k] - bs;
        if (n < 2 || n > kSortedMaxPk) continue;
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
    uint32_t rk[kPbPer];  // bucket << 16 | arrival rank
    const uint32_t c = uint32_t(wid) < S2 ? cnt2[uint64_t(wid) * P + p] : 0u;
#pragma unroll
    for (int u = 0; u < kPbPer; ++u) {
      const bool v = uint32_t(u) * 64u + lane < c;
      const uint32_t b = v ? e[u].x >> pk.qbits : 0u;
      rk[u] = v ? (b << 16) | atomicAdd(&cnt[b], 1u) : kInvalid;
    }
    __syncthreads();
    pb_lds_scan(cnt, nbs, wsum);
    if (threadIdx.x == 0) cnt[nbs] = m;
    for (uint32_t k = threadIdx.x; k < nbs; k += kPkBlock) off[b0 + k] = s0 + cnt[k];
    if (b0 + nbs == nbl && threadIdx.x == 0) off[nbl] = s0 + m;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPbPer; ++u)
      if (rk[u] != kInvalid) stage[cnt[rk[u] >> 16] + (rk[u] & 0xFFFFu)] = e[u];
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < m; q += kPkBlock) {
      const uint2 x = stage[q];
      const uint32_t b = x.x >> pk.qbits;
      const uint32_t bs = cnt[b], n = cnt[b + 1] - bs;
      uint32_t pos = q;
      if (n >= 2 && n <= kSortedMaxPk) {
        uint32_t rr = 0;
        for (uint32_t k = bs; k < bs + n; ++k) rr += stage[k].y < x.y;
        pos = bs + rr;
      }
      ent[s0 + pos] = make_uint2(pk.hash_of(x.x, p), x.y);
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

}  // namespace

// Pairs per lane and chunk for the region walk: the K in [kItemsMin, kItemsMax] with the fewest
// expected item slots per region, region lengths ~ N(L, L) (a region gets each of L * (#regions)
// tuples with probability 1 / #regions); ties go to the larger K (fewer chunks).
static int pk_items(double L) {
  int best = kItemsMax;
  double best_slots = 0.0;
  const double sd = std::sqrt(L > 1.0 ? L : 1.0);
  for (int K = kItemsMax; K >= kItemsMin; --K) {
    const double c = 64.0 * K;
    double slots = 0.0, wsum = 0.0;
    for (int z = -40; z <= 40; ++z) {  // normal quadrature over +-4 sigma
      const double x = L + 0.1 * z * sd, w = std::exp(-0.005 * z * z);
      slots += w * std::ceil((x < 1.0 ? 1.0 : x) / c) * c;
      wsum += w;
    }
    slots /= wsum;
    if (K == kItemsMax || slots < best_slots * 0.999) {
      best = K;
      best_slots = slots;
    }
  }
  return best;
}

bool pk_probe_applicable(const hj3d_ctx* ctx, const hj3d_table* t, uint64_t n_probe, uint32_t flags) {
  return t->desc.kind == HJ3D_CHAIN && (flags & HJ3D_PROBE_UNIQUE) && !ctx->force_direct && !ctx->pk_off &&
         n_probe >= ctx->radix_min && n_probe > 0 && t->nb_local >= 64 && t->desc.num_buckets >= 2 &&
         n_probe < (1ull << 32) && t->built;
}

// The largest slice width W (buckets) whose LDS image (W directory words, two words per entry,
// ~W * fill entries) fits kPkLdsWords with 6 sigma of headroom on the entry count.
static uint32_t pk_slice_width(double fill) {
  double W = double(kPkLdsWords) / (1.0 + 2.0 * fill);
  for (int i = 0; i < 6; ++i) W = (double(kPkLdsWords) - 2.0 - 12.0 * std::sqrt(W * fill)) / (1.0 + 2.0 * fill);
  return W < 64.0 ? 64u : uint32_t(W);
}

PkPlan pk_plan(const hj3d_ctx* ctx, uint32_t nbl, uint64_t n_build) {
  PkPlan pl;
  const double fill = n_build ? double(n_build) / double(nbl) : 0.0;
  uint32_t W = pk_slice_width(fill);
  if (ctx->pk_slice_max && W > ctx->pk_slice_max) W = ctx->pk_slice_max;
  if (W > nbl) W = nbl;
  uint32_t P = (nbl + W - 1) / W;
  // whole waves of probe workgroups (one per CU): the slice count rounded up to a multiple of the
  // CUs, staying at one partition level when that is possible
  const uint32_t ncu = uint32_t(ctx->num_cus);
  if (P >= ncu / 2) {
    uint32_t Pq = (P + ncu - 1) / ncu * ncu;
    if (P <= kPkMaxP1 && Pq > kPkMaxP1) Pq = kPkMaxP1;
    P = Pq;
    W = (nbl + P - 1) / P;
    P = (nbl + W - 1) / W;
  }
  pl.W = W;
  pl.P = P;
  // slices per coarse range of the first level: one level up to kPkMaxP1 slices (k_pk_part's two
  // slices per thread beyond 1024: config D's 2.5e7-bucket rank at 4 GPUs, 2048 slices, without the
  // k_pk_split pass); beyond, coarse ranges of 1024 slices' worth
  pl.C = P <= kPkMaxP1 ? 1u : (P + kPkBlock - 1) / kPkBlock;
  pl.W1 = W * pl.C;
  pl.P1 = (nbl + pl.W1 - 1) / pl.W1;
  return pl;
}

hipError_t pk_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out, uint64_t out_cap,
                    uint64_t* res, hipStream_t s, const SelArgs* sel) {
  hipError_t e;
  const uint32_t nbl = t->nb_local, nb = uint32_t(t->desc.num_buckets);
  const PkPlan pl = pk_plan(ctx, nbl, t->n_build);
  const bool two = pl.C > 1;
  if (pl.C > kSpMaxC) return hipErrorNotSupported;
  // the packed word: bucket in the (first-level) slice and the quotient h / NB (bits of its max)
  auto bits = [](uint64_t x) { uint32_t b = 0; while (x) { ++b; x >>= 1; } return b; };
  const uint32_t qbits = bits(0xFFFFFFFFull / nb), wbits = bits(pl.W1 - 1);
  if (qbits + wbits > 32) return hipErrorNotSupported;
  SelRange sr{};
  if (sel && !SelRange::from(*sel, &sr)) return hipErrorNotSupported;
  const uint32_t ntiles = uint32_t((r.n + kPkTile - 1) / kPkTile);
  const uint32_t G = ntiles < uint32_t(ctx->num_cus) ? ntiles : uint32_t(ctx->num_cus);
  // region capacity: expected pairs per (workgroup, slice) + 8 sigma + slack, whole segments
  auto capacity = [](double ex) {
    uint64_t c = uint64_t(ex + 8.0 * std::sqrt(ex) + 32.0);
    return (c + kPkSeg - 1) / kPkSeg * kPkSeg;
  };
  const uint64_t per_g = uint64_t((ntiles + G - 1) / G) * kPkTile;
  const uint64_t cap = capacity(double(per_g < r.n ? per_g : r.n) / pl.P1);
  const uint64_t nreg = uint64_t(G) * pl.P1;
  if (nreg * cap >= (1ull << 31)) return hipErrorNotSupported;
  // second level: S2 workgroups per coarse range, each writing one fine region per slice
  const uint32_t S2 = two ? (G < 16u ? G : 16u) : 0u;
  // a fine region gathers the pass-1 regions of ceil(G / S2) workgroups at most (G need not be a
  // multiple of S2): its expected pairs are that many workgroups' share of the slice
  const double per_gp = double(per_g < r.n ? per_g : r.n) / pl.P;
  const uint64_t cap2 = two ? capacity(per_gp * double((G + S2 - 1) / S2)) : 0;
  const uint64_t nreg2 = uint64_t(S2) * pl.P;
  if (two && nreg2 * cap2 >= (1ull << 31)) return hipErrorNotSupported;
  if ((e = ctx->scratch[kScrPairs].ensure(nreg * cap * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrPHist].ensure(nreg * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrSortV].ensure(r.n * sizeof(uint2))) != hipSuccess) return e;
  if (two) {
    if ((e = ctx->scratch[kScrPk2].ensure(nreg2 * cap2 * sizeof(uint2))) != hipSuccess) return e;
    if ((e = ctx->scratch[kScrPk2Cnt].ensure(nreg2 * sizeof(uint32_t))) != hipSuccess) return e;
  }
  const uint32_t want_blocks = uint32_t(ctx->num_cus) * 2;
  const uint32_t Gp = two ? S2 : G;  // regions per slice that the probe walks
  uint32_t splits = pl.P < want_blocks ? (want_blocks + pl.P - 1) / pl.P : 1u;
  if (splits > Gp) splits = Gp;
  const uint32_t nblocks = pl.P * splits;
  if ((e = ctx->scratch[kScrPartial].ensure(uint64_t(nblocks) * kProbeFields * sizeof(uint64_t))) != hipSuccess)
    return e;
  if ((e = ctx->ensure_ctl()) != hipSuccess) return e;
  auto geom = [&](uint32_t W, uint32_t P) {
    PkGeom g;
    g.dnb = FastDiv32::make(nb);
    g.dw = W >= 2 ? FastDiv32::make(W) : FastDiv32{};
    g.nb = nb;
    g.lo = uint32_t(t->desc.bucket_lo);
    g.nbl = nbl;
    g.W = W;
    g.P = P;
    g.qbits = qbits;
    g.qmask = qbits >= 32 ? 0xFFFFFFFFu : ((1u << qbits) - 1);
    return g;
  };
  const PkGeom pk1 = geom(pl.W1, pl.P1), pk = geom(pl.W, pl.P);
  uint2* region = ctx->scratch[kScrPairs].as<uint2>();
  uint32_t* counts = ctx->scratch[kScrPHist].as<uint32_t>();
  uint2* ovf = ctx->scratch[kScrSortV].as<uint2>();
  uint64_t* ctl = ctx->ctl.as<uint64_t>();
  const RelView v = view_of(r);
  const bool imp = r.row_off == HJ3D_ROW_IMPLICIT;
  const uint32_t slim = ctx->pk_stage ? (ctx->pk_stage < kPkStage ? ctx->pk_stage : kPkStage) : kPkStage;
  {
    KernelSpan tm(ctx, HJ3D_T_SCATTER);
    const uint32_t c32 = uint32_t(cap);
    // (one level beyond 1024 slices: two slices per partitioning thread)
    const uint32_t slim2 = slim < kPkStage2 ? slim : kPkStage2;
#define HJ3D_PKP_LAUNCH(IMP, SEL)                                                                                   \
  if (pl.P1 > uint32_t(kPkBlock))                                                                                   \
    tm.launch(k_pk_part<IMP, SEL, 2>, dim3(G), dim3(kPkBlock), s, v, pk1, ntiles, c32, region, counts, ovf, ctl, sr, \
              slim2);                                                                                               \
  else                                                                                                              \
    tm.launch(k_pk_part<IMP, SEL, 1>, dim3(G), dim3(kPkBlock), s, v, pk1, ntiles, c32, region, counts, ovf, ctl, sr, slim);
    if (sel) {
      if (imp) HJ3D_PKP_LAUNCH(true, true)
      else HJ3D_PKP_LAUNCH(false, true)
    } else {
      if (imp) HJ3D_PKP_LAUNCH(true, false)
      else HJ3D_PKP_LAUNCH(false, false)
    }
#undef HJ3D_PKP_LAUNCH
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const uint2* pregion = region;
  const uint32_t* pcounts = counts;
  uint32_t pcap = uint32_t(cap);
  if (two) {
    uint2* fine = ctx->scratch[kScrPk2].as<uint2>();
    uint32_t* fcnt = ctx->scratch[kScrPk2Cnt].as<uint32_t>();
    KernelSpan ts(ctx, HJ3D_T_HIST);
    ts.launch(k_pk_split, dim3(pl.P1 * S2), dim3(kSpBlock), s, static_cast<const uint2*>(region),
              static_cast<const uint32_t*>(counts), G, pl.P1, uint32_t(cap), S2, pk, pl.C, bits(pl.C - 1),
              uint32_t(cap2), fine, fcnt, ovf, ctl);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    pregion = fine;
    pcounts = fcnt;
    pcap = uint32_t(cap2);
  }
  const bool emit = (flags & HJ3D_PROBE_EMIT) && out;
  const bool ck = flags & HJ3D_PROBE_CHECKSUM;
  const int acc = (flags & HJ3D_PROBE_ACCUMULATE) ? 1 : 0;
  const uint64_t preg = uint64_t(Gp) * pl.P;
  // short regions (< 256 pairs expected) are walked as one flattened stream per wave (always-flat
  // walks measured slower at config B's ~384-pair regions)
  const bool flat = double(r.n) / double(preg) < 256.0;
  const int items = ctx->pk_items ? ctx->pk_items : flat ? kItemsMax : pk_items(double(r.n) / double(preg));
  uint2* o = static_cast<uint2*>(out);
  uint64_t* partials = ctx->scratch[kScrPartial].as<uint64_t>();
  {
    KernelSpan tk(ctx, HJ3D_T_PROBE_KERNEL);
#define HJ3D_PK_LAUNCH(K, MODE, CK)                                                                                  \
  tk.launch(k_pk_probe<K, MODE, CK>, dim3(nblocks), dim3(kPkBlock), s, pregion, pcounts, Gp, pcap,              \
                     splits, flat, t->off.as<const uint32_t>(), t->ent.as<const uint2>(), pk, t->fm, o, out_cap, ovf, \
                     ctl, partials, res, acc)
#define HJ3D_PK_LAUNCH_K(MODE, CK)               \
  switch (items) {                               \
    case 5: HJ3D_PK_LAUNCH(5, MODE, CK); break;  \
    case 6: HJ3D_PK_LAUNCH(6, MODE, CK); break;  \
    case 7: HJ3D_PK_LAUNCH(7, MODE, CK); break;  \
    default: HJ3D_PK_LAUNCH(8, MODE, CK); break; \
  }
    if (emit) {
      if (ck) HJ3D_PK_LAUNCH_K(1, true)
      else HJ3D_PK_LAUNCH_K(1, false)
    } else {
      if (ck) HJ3D_PK_LAUNCH_K(0, true)
      else HJ3D_PK_LAUNCH_K(0, false)
    }
#undef HJ3D_PK_LAUNCH_K
#undef HJ3D_PK_LAUNCH
  }
  return hipGetLastError();
}


hipError_t pk_slices(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t W, PkSlices* o, hipStream_t s,
                     bool sums) {
  hipError_t e;
  const uint32_t nbl = t->nb_local, nb = uint32_t(t->desc.num_buckets);
  if (nbl < 64 || r.n == 0 || r.n >= (1ull << 31) || W < 2) return hipErrorNotSupported;
  const uint32_t P = (nbl + W - 1) / W;
  const uint32_t C = (P + kPkBlock - 1) / kPkBlock;
  if (C > kSpMaxC) return hipErrorNotSupported;
  const uint32_t W1 = W * C, P1 = (nbl + W1 - 1) / W1;
  auto bits = [](uint64_t x) { uint32_t b = 0; while (x) { ++b; x >>= 1; } return b; };
  const uint32_t qbits = bits(0xFFFFFFFFull / nb);
  // the packed word holds the bucket inside the coarse range (and, after the split, inside the
  // slice, whose width W must also fit, for the nested build's empty marker W << qbits)
  if (qbits + bits(W1 - 1) > 32 || qbits + bits(W) > 32) return hipErrorNotSupported;
  const uint32_t ntiles = uint32_t((r.n + kPkTile - 1) / kPkTile);
  const uint32_t G = ntiles < uint32_t(ctx->num_cus) ? ntiles : uint32_t(ctx->num_cus);
  auto capacity = [](double ex) {
    uint64_t c = uint64_t(ex + 8.0 * std::sqrt(ex) + 32.0);
    return (c + kPkSeg - 1) / kPkSeg * kPkSeg;
  };
  const uint64_t per_g = uint64_t((ntiles + G - 1) / G) * kPkTile;
  const uint64_t cap = capacity(double(per_g < r.n ? per_g : r.n) / P1);
  const uint64_t nreg = uint64_t(G) * P1;
  const uint32_t S2 = G < 16u ? G : 16u;
  // a fine region gathers the pass-1 regions of ceil(G / S2) workgroups at most (G need not be a
  // multiple of S2): its expected pairs are that many workgroups' share of the slice
  const double per_gp = double(per_g < r.n ? per_g : r.n) / P;
  const uint64_t cap2 = capacity(per_gp * double((G + S2 - 1) / S2));
  const uint64_t nreg2 = uint64_t(S2) * P;
  if (nreg * cap >= (1ull << 31) || nreg2 * cap2 >= (1ull << 31)) return hipErrorNotSupported;
  if ((e = ctx->scratch[kScrPairs].ensure(nreg * cap * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrPHist].ensure(nreg * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrSortV].ensure(r.n * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrPk2].ensure(nreg2 * cap2 * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrPk2Cnt].ensure(nreg2 * sizeof(uint32_t))) != hipSuccess) return e;
  if (sums && (e = ctx->scratch[kScrPStart].ensure((uint64_t(P) + 1) * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = ctx->ensure_ctl()) != hipSuccess) return e;
  auto geom = [&](uint32_t w, uint32_t p) {
    PkGeom g;
    g.dnb = FastDiv32::make(nb);
    g.dw = FastDiv32::make(w);
    g.nb = nb;
    g.lo = uint32_t(t->desc.bucket_lo);
    g.nbl = nbl;
    g.W = w;
    g.P = p;
    g.qbits = qbits;
    g.qmask = qbits >= 32 ? 0xFFFFFFFFu : ((1u << qbits) - 1);
    return g;
  };
  const PkGeom pk1 = geom(W1, P1), pk = geom(W, P);
  uint2* region = ctx->scratch[kScrPairs].as<uint2>();
  uint32_t* counts = ctx->scratch[kScrPHist].as<uint32_t>();
  uint2* ovf = ctx->scratch[kScrSortV].as<uint2>();
  uint2* fine = ctx->scratch[kScrPk2].as<uint2>();
  uint32_t* fcnt = ctx->scratch[kScrPk2Cnt].as<uint32_t>();
  uint32_t* ps = sums ? ctx->scratch[kScrPStart].as<uint32_t>() : nullptr;
  uint64_t* ctl = ctx->ctl.as<uint64_t>();
  const RelView v = view_of(r);
  SelRange sr{};
  if (r.row_off == HJ3D_ROW_IMPLICIT)
    hipLaunchKernelGGL((k_pk_part<true, false, 1>), dim3(G), dim3(kPkBlock), 0, s, v, pk1, ntiles, uint32_t(cap), region,
                       counts, ovf, ctl, sr, kPkStage);
  else
    hipLaunchKernelGGL((k_pk_part<false, false, 1>), dim3(G), dim3(kPkBlock), 0, s, v, pk1, ntiles, uint32_t(cap), region,
                       counts, ovf, ctl, sr, kPkStage);
  // (C = 1: the split only regroups each slice's G regions into S2)
  hipLaunchKernelGGL(k_pk_split, dim3(P1 * S2), dim3(kSpBlock), 0, s, static_cast<const uint2*>(region),
                     static_cast<const uint32_t*>(counts), G, P1, uint32_t(cap), S2, pk, C, bits(C - 1), uint32_t(cap2),
                     fine, fcnt, ovf, ctl);
  if (sums) {
    hipLaunchKernelGGL(k_pk_slice_sums, dim3((P + 255) / 256), dim3(256), 0, s, static_cast<const uint32_t*>(fcnt), S2, P, ps);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = exclusive_scan_u32(ctx, ps, ps, P, s)) != hipSuccess) return e;
  }
  o->pk = pk;
  o->P = P;
  o->S2 = S2;
  o->cap2 = uint32_t(cap2);
  o->fine = fine;
  o->fcnt = fcnt;
  o->ps = ps;
  o->ovf = ovf;
  o->novf = reinterpret_cast<const unsigned long long*>(ctl + kCtlNovf);
  return hipGetLastError();
}

hipError_t pk_ctl_reset(hj3d_ctx* ctx, hipStream_t s) {
  return hipMemsetAsync(ctx->ctl.p, 0, kCtlWords * sizeof(uint64_t), s);
}

hipError_t pk_overflow_check(hj3d_ctx* ctx, hipStream_t s, uint64_t* novf) {
  hipError_t e;
  uint64_t* ctl = ctx->ctl.as<uint64_t>();
  *novf = 0;
  if ((e = hipMemcpyAsync(novf, ctl + kCtlNovf, sizeof(*novf), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(ctl, 0, kCtlWords * sizeof(uint64_t), s)) != hipSuccess) return e;
  return hipStreamSynchronize(s);
}

hipError_t pk_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s) {
  hipError_t e;
  const uint32_t nbl = t->nb_local;
  if (ctx->force_direct || nbl < 64 || r.n == 0 || r.n >= (1ull << 31)) return hipErrorNotSupported;
  const uint32_t W = kPbW, P = (nbl + W - 1) / W;
  const uint32_t C = (P + kPkBlock - 1) / kPkBlock;
  if ((C < 2 && !ctx->pk_build) || C > kSpMaxC) return hipErrorNotSupported;  // one level: the radix build's range
  if ((e = t->off.ensure((uint64_t(nbl) + 1) * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = t->ent.ensure(r.n * sizeof(uint2))) != hipSuccess) return e;
  PkSlices sl;
  if ((e = pk_slices(ctx, t, r, W, &sl, s)) != hipSuccess) return e;
  const uint32_t g2 = P < uint32_t(ctx->num_cus) ? P : uint32_t(ctx->num_cus);
  hipLaunchKernelGGL(k_pk_build, dim3(g2), dim3(kPkBlock), 0, s, sl.fine, sl.fcnt, sl.S2, sl.cap2, sl.ps, sl.pk,
                     t->off.as<uint32_t>(), t->ent.as<uint2>());
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // pairs past a region's capacity (skewed keys) are not in the slices: then the direct build
  // runs instead. The control words go back to zero (the probes' invariant) either way.
  uint64_t novf = 0;
  if ((e = pk_overflow_check(ctx, s, &novf)) != hipSuccess) return e;
  if (novf) return hipErrorNotSupported;
  t->n_build = r.n;
  return hipSuccess;
}

}  // namespace hj3d

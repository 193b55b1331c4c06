// nested_agg.hip — build of the nested ("3D") table by bucket-range partition + per-partition
// aggregation in LDS (the default nested build for large inputs).
//
// The nested table (nested.hip) needs, per bucket, one main record per distinct key {hash,
// first_row, sub_off, sub_len} and every key's rows contiguous in `sub` (HtNested1: a main node
// per distinct key with its duplicates in a sub-chain, ht_nested.hh:287-311, 386-436). Neither the
// order of the mains inside a bucket nor the order of the rows inside a key matters: the probe
// derives the reference's comparison count from first-row ranks and unnest output is order-free.
// So instead of sorting all tuples by key (3 LSD passes at 16 B/tuple each, nested.hip):
//   1. partition the build tuples into (hash, row) pairs by ranges of W <= kAggW buckets
//      (radix_partition_pairs: one histogram pass, one LDS-staged scatter pass);
//   2. one workgroup per partition inserts the partition's keys into an LDS hash table (count +
//      min row per key; a hot key's lanes are aggregated per wave first, so Zipf skew costs one
//      LDS atomic per wave, not per tuple), assigns every key its main slot (bucket order) and
//      sub range, then reads the pairs again and scatters every row into its key's sub range.
//      A range whose distinct keys do not fit the table is retried in halves (many keys per
//      bucket), so the table never overflows; below kAggMinSpan buckets per round the build
//      gives up (hipErrorNotSupported) and the sort-based build runs instead;
//   3. the partitions' main records are compacted and the directory offsets rebased (scan of
//      the per-partition key counts).
// Traffic: 12 B read (tuple) x 2 + 8 B write + 2 x 8 B read (pairs) + 4 B write (sub) per tuple,
// + 16 B per distinct key (twice) + 4 B per bucket.
// Tables of more than 2048 partitions (config D's 1e8-bucket Nrs table on one GPU, 2.5e7 and 5e7
// buckets per rank at 4 and 2 GPUs) take step 1 from the packed partitioner's two levels instead
// (pk_slices, chain_pk.hip: k_pk_part + k_pk_split, 12 + 8 + 8 + 8 B per tuple): each slice's pairs
// lie in S2 = 16 fine regions, read as one stream, and the LDS table's key is the packed word
// {bucket in the slice, h / NB} itself (unique per hash inside the slice: no modulo per pair). Pairs
// that overflowed a region (skewed keys) set the give-up flag: the sort build then runs.
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

// max buckets per partition (one LDS table round at fill <= ~1.3)
constexpr uint32_t kAggW = 6144;
// LDS hash table slots (prime, sized per build: ~1.5 slots per bucket of the partition + the insert
// slack; at most 10223): with double hashing every probe step visits all slots (double hashing
// measured 2.25 -> 1.94 ms against linear probing for uniform keys at load ~0.6). The table lives in
// dynamic LDS, so small partitions (configs D, E) run two 512-thread workgroups per CU.
constexpr uint32_t kAggCapMax = 10223;
constexpr uint32_t kAggRounds = 1;  // initial rounds per partition (2, 3: slower under Zipf, pairs re-read)
constexpr uint32_t kAggMinSpan = 384;  // smallest bucket range per round before giving up
constexpr int kAggU = 8;  // pairs per thread and step (the next step's in flight; 4 / 16: slower)
// the small-partition form: two 512-thread workgroups per CU (256 threads, four per CU: slower)
constexpr int kSmallBlock = 512;
constexpr int kSmallSlots = 6144 / kSmallBlock;  // table slots per thread (cap <= 6144)
constexpr size_t kSmallLds = 81920, kBigLds = 160 * 1024;  // dynamic LDS of the two forms (two / one per CU)
constexpr double kSmallCapF = 1.5;  // small form: table slots per bucket of the partition (+ the insert slack)
constexpr uint32_t kPartsPerCu = 2;  // target partitions per CU (4: config E 0.27 -> 0.34 ms)
// buckets per partition on the packed slices. Uniform keys, 1e9 tuples / 1e8 buckets: 26.1 ms (5,357
// buckets, one 1024-thread workgroup per CU) -> 19.9 ms (2,048) -> 18.5 ms (1,536; two 512-thread
// workgroups per CU, a quarter of the sub-row window); 1,024 exceeds the 65,536 slices
// (profiles/r04n_ab_pkw.log)
constexpr uint32_t kPkW = 1536;
// the register form k_nagg_reg: mean partitions of at most kRegFill of its capacity, tables of at most
// kRegSlots x 1024 slots (6, which takes config E's 5,701: 0.27 -> 0.29 ms)
constexpr double kRegFill = 0.85;
constexpr uint32_t kRegSlots = 4;
// the streaming form's hot-key wave leader election: in partitions above 5/4 of the mean size (in
// every partition: measured slower; duplicates inside a wave are rare elsewhere)
#ifndef HJ3D_NAGG_CLK
#define HJ3D_NAGG_CLK 0  // diagnostic: per-workgroup phase clocks of k_nagg (read by hj3d_diag_nagg_clk)
#endif
[[maybe_unused]] constexpr uint32_t kClkParts = 16384, kClkPts = 8;
#if HJ3D_NAGG_CLK
__device__ uint64_t g_nagg_clk[kClkParts * kClkPts];
#endif
// point k of partition gp's timeline: 100 MHz wall clock (point 7: the end of the last round's pass-B
// sweep, before the image goes out, or with the look-back finish the finish's end)
__device__ __forceinline__ void nagg_clk(uint32_t gp, int k) {
#if HJ3D_NAGG_CLK
  if (threadIdx.x == 0 && gp < kClkParts) {
    g_nagg_clk[gp * kClkPts + k] = k == 7 ? blockIdx.x : wall_clock64();
    // point 6: where the workgroup runs, {XCC_ID, HW_ID} (CU, SH, SE of wave 0)
    if (k == 0)
      g_nagg_clk[gp * kClkPts + 6] = (uint64_t(__builtin_amdgcn_s_getreg((31 << 11) | 20)) << 32) |
                                     uint32_t(__builtin_amdgcn_s_getreg((31 << 11) | 4));
  }
#else
  (void)gp;
  (void)k;
#endif
}

__device__ __forceinline__ uint32_t slot_of(uint32_t h, uint32_t cap) { return __umulhi(h * 0x9E3779B1u, cap); }
// per-key probe step in [1, cap) (double hashing: no primary clusters, so the longest probe
// sequence among a wave's 64 lanes, which the whole wave waits for, stays short)
__device__ __forceinline__ uint32_t step_of(uint32_t h, uint32_t cap) { return 1u + __umulhi(h * 0x85EBCA6Bu, cap - 1); }
__device__ __forceinline__ uint32_t next_slot(uint32_t s, uint32_t st, uint32_t cap) {
  s += st;
  return s >= cap ? s - cap : s;
}

// Slot of key h, inserting it if absent; k: the key its home slot held when the caller read it (a
// stale empty is fine: slots only ever go from empty to a key, and the CAS sees the truth). Returns
// kInvalid after kMaxProbe slots without a place (a table too full for the round: the caller flags
// it as overflowing and retries a narrower range). A key at its home slot costs the caller's batched
// read only; a new key whose home slot was empty one CAS (no re-read, no key counter).
constexpr uint32_t kMaxProbe = 64;
__device__ __forceinline__ uint32_t tab_insert_k(uint32_t* tkey, uint32_t h, uint32_t k, uint32_t empty,
                                                 uint32_t cap) {
  uint32_t s = slot_of(h, cap);
  const uint32_t st = step_of(h, cap);
#pragma unroll 1
  for (uint32_t n = 0; n < kMaxProbe; ++n) {
    if (k == h) return s;
    if (k == empty) {
      const uint32_t old = atomicCAS(&tkey[s], empty, h);
      if (old == empty || old == h) return s;
    }
    s = next_slot(s, st, cap);
    k = tkey[s];
  }
  return kInvalid;
}
__device__ __forceinline__ uint32_t tab_insert(uint32_t* tkey, uint32_t h, uint32_t empty, uint32_t cap) {
  return tab_insert_k(tkey, h, tkey[slot_of(h, cap)], empty, cap);
}

__device__ __forceinline__ uint32_t tab_find(const uint32_t* tkey, uint32_t h, uint32_t cap) {
  uint32_t s = slot_of(h, cap);
  const uint32_t st = step_of(h, cap);
  while (tkey[s] != h) s = next_slot(s, st, cap);
  return s;
}
// the same for a key known not to sit in its home slot (the caller's batched read): from the next slot
__device__ __forceinline__ uint32_t tab_find_away(const uint32_t* tkey, uint32_t h, uint32_t cap) {
  const uint32_t st = step_of(h, cap);
  uint32_t s = next_slot(slot_of(h, cap), st, cap);
  while (tkey[s] != h) s = next_slot(s, st, cap);
  return s;
}

// min over the wave's 64 lanes (all active), for every lane: DPP butterflies inside each row of 16
// lanes (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then the four row minima by
// readlane. (__shfl_xor compiled to six ds_bpermute rounds, each waiting on LDS.)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_min_step(uint32_t v) {
  return min(v, uint32_t(__builtin_amdgcn_update_dpp(int(kInvalid), int(v), CTRL, 0xF, 0xF, false)));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = dpp_min_step<0xB1>(v);
  v = dpp_min_step<0x4E>(v);
  v = dpp_min_step<0x141>(v);
  v = dpp_min_step<0x140>(v);
  const uint32_t a = uint32_t(__builtin_amdgcn_readlane(int(v), 0)), b = uint32_t(__builtin_amdgcn_readlane(int(v), 16));
  const uint32_t c = uint32_t(__builtin_amdgcn_readlane(int(v), 32)), d = uint32_t(__builtin_amdgcn_readlane(int(v), 48));
  return min(min(a, b), min(c, d));
}

// Exclusive scan of a[0..n) in LDS by BLOCK threads (contiguous chunks per thread); returns
// the total. All threads must call it.
template <int BLOCK>
__device__ uint32_t block_scan_lds(uint32_t* a, uint32_t n, uint32_t* wsum) {
  constexpr int kWavesA = BLOCK / kWave;
  const uint32_t per = (n + BLOCK - 1) / BLOCK;
  const uint32_t b = threadIdx.x * per, e = min(n, b + per);
  uint32_t t = 0;
  for (uint32_t i = b; i < e; ++i) t += a[i];
  uint32_t wt;
  const uint32_t wpre = wave_excl_scan(t, &wt);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 63) wsum[wid] = wpre + t;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWavesA; ++w) {
    const uint32_t x = wsum[w];
    if (w < wid) pre += x;
    tot += x;
  }
  pre += wpre;
  for (uint32_t i = b; i < e; ++i) {
    const uint32_t x = a[i];
    a[i] = pre;
    pre += x;
  }
  __syncthreads();
  return tot;
}

// One workgroup per partition p (local buckets [b0, b0 + nbs), pairs [ps[p], ps[p+1])).
// Writes: off[b0 + k] = partition-local main offset of bucket k; mtmp[ps[p] + i] the partition's
// main records in bucket order (i < its key count, with sub_off global); sub rows; dcount[p].
// Dynamic LDS (agg_lds_bytes): tkey | tcnt | tmin [cap each] | (pad to 8 B) | bcnt [max(W, 2 kAggQ per
// wave)] | wsum | (unused), ovf | region starts | hot-key words. bcnt doubles as pass A's per-wave miss
// queues (kAggQ pairs per wave): its counts live only from the end of pass A to pass B.
// SLOTS >= cap / BLOCK: table slots per thread in the per-slot loops.
constexpr uint32_t kAggMaxS2 = 16;  // fine regions per slice (pk_slices)
constexpr uint32_t kAggQ = 128;     // pass A's miss queue: pairs per wave (a ring, flushed 64 at a time)
__host__ __device__ constexpr uint32_t agg_bcnt_words(uint32_t W, int block) {
  return W > 2u * kAggQ * uint32_t(block / 64) ? W : 2u * kAggQ * uint32_t(block / 64);
}
// fixed words: tkey, tcnt [cap each] | wsum (waves + 2: block-scan sums, ovf) | region starts
// (kAggMaxS2 + 2) | hot-key words (2 waves + 2), rounded to 8 B; then the region R: in pass A tmin [cap]
// | bcnt [agg_bcnt_words] (8-B aligned: the miss queues), in pass B the sub-row image (every word of the
// allocation past the fixed ones)
__host__ __device__ constexpr uint32_t agg_fixed_words(uint32_t cap, int block) {
  return (2 * cap + uint32_t(block / 64) + 2 + kAggMaxS2 + 2 + 2 * uint32_t(block / 64) + 2 + 1) & ~1u;
}
__host__ __device__ constexpr uint32_t agg_lds_words(uint32_t cap, uint32_t W, int block) {
  return agg_fixed_words(cap, block) + cap + (cap & 1u) + agg_bcnt_words(W, block);
}
// PK: the partition's pairs are slice p's fine regions (pk_slices), packed words as keys.
struct NaggSrc {
  const uint2* fine = nullptr;
  const uint32_t* fcnt = nullptr;
  uint32_t S2 = 0, cap2 = 0;
  PkGeom pk{};
};
// The tables one launch builds: one, or two of one geometry (experiment 4's S and T share NB): the
// partitions of table 1 follow table 0's (global partition index P.. 2P - 1), its pairs follow
// table 0's at pbase[1]; per table its directory, main records, sub rows and counts words.
struct NaggTabs {
  uint32_t P = 0, nt = 1;
  uint32_t pbase[2] = {0, 0};
  uint32_t* off[2] = {nullptr, nullptr};
  uint32_t* sub[2] = {nullptr, nullptr};
  uint4* main[2] = {nullptr, nullptr};
  uint64_t* counts[2] = {nullptr, nullptr};  // word 2: longest key, word 3: give-up flag
  uint64_t* hc[2] = {nullptr, nullptr};      // the tables' pinned host mirrors of the counts words (or none)
  uint32_t* sink = nullptr;  // pass B's stores of items without a row (the context's store-sink words)
  uint32_t ldsw = 0;         // k_nagg's dynamic LDS words (>= agg_lds_words): the image takes the rest
  // partitions the register form leaves to k_nagg_defer (more pairs than its registers hold, or more
  // keys than its table): defer[0] the count (zeroed by k_nagg_order / k_nagg_pk_ovf), then the indices
  uint32_t* defer = nullptr;
  uint32_t elect_min = 0;    // partitions of at least this many pairs elect a wave leader per hot key
  // Hot keys split off heavy partitions (k_nagg_hot, one-level partitions only): per partition kHotW
  // words {flag, key, rows (cursor), min row, other pairs (cursor)}; the other pairs compacted into
  // hpairs[ps[gp] ..]; the key's rows already in the suffix of the partition's sub range
  uint32_t* hot = nullptr;
  uint2* hpairs = nullptr;
  // slice path: decoupled look-back instead of the scan / rebase / mains launches (nested_agg_finish)
  uint64_t* lbw = nullptr;  // [0] partition ticket, [1] finished workgroups, then the status words
  uint32_t lb_epoch = 0;
  uint32_t lb_skip0 = 0;             // HJ3D_OPT_DIAG_LOOKBACK: partition 0 never publishes (tests)
  uint64_t lb_ticks = 20000000ull;   // a look-back's wait limit (100 MHz ticks: 0.2 s)
};
constexpr uint32_t kHotW = 8;
// one partition (global index gp) of k_nagg
template <int BLOCK, int SLOTS, bool PK>
__device__ __forceinline__ uint32_t nagg_one(uint32_t gp, const uint2* __restrict__ pairs, const uint32_t* __restrict__ ps,
                                         FastMod fm, uint32_t lo, uint32_t nbl, uint32_t nb_global, uint32_t W,
                                         uint4* __restrict__ mtmp, uint32_t* __restrict__ dcount, uint32_t cap,
                                         const NaggSrc& src, const NaggTabs& tabs, uint32_t* agg_lds,
                                         bool lb = false) {
  constexpr uint32_t kNw = BLOCK / kWave;
  uint32_t* tkey = agg_lds;
  uint32_t* tcnt = tkey + cap;  // count, then the rows before the key in the round (pass B: its cursor)
  uint32_t* wsum = tcnt + cap;
  uint32_t& ovf = wsum[kNw + 1];
  uint32_t* rstart = wsum + kNw + 2;  // PK: stream start of every fine region (+ 2 sentinels)
  // hot key of a heavy partition: per-wave hot rows (then their exclusive prefix) and min rows, the
  // key's slot and its rows' total
  uint32_t* hotw = rstart + kAggMaxS2 + 2;
  uint32_t* hotm = hotw + kNw;
  uint32_t& hslot = hotm[kNw];
  uint32_t& hrows = hotm[kNw + 1];
  uint32_t* tmin = agg_lds + agg_fixed_words(cap, BLOCK);  // min row, until the main records are written
  // keys per bucket of the round, then their main offsets (8-B aligned: pass A's miss queues)
  uint32_t* bcnt = tmin + cap + (cap & 1u);
  uint32_t* img = tmin;  // pass B: the window's sub rows, assembled
  const uint32_t imgw = tabs.ldsw - agg_fixed_words(cap, BLOCK);
  const uint32_t ti = tabs.nt > 1 && gp >= tabs.P ? 1u : 0u;
  const uint32_t p = gp - ti * tabs.P;                      // partition inside table ti
  uint32_t* __restrict__ off = tabs.off[ti];
  uint32_t* __restrict__ sub = tabs.sub[ti];
  auto* maxlen = reinterpret_cast<unsigned long long*>(tabs.counts[ti] + 2);
  auto* fail = reinterpret_cast<uint32_t*>(tabs.counts[ti] + 3);
  const uint32_t b0 = p * W, nbs = min(W, nbl - b0);
  // (table ti's sub rows are numbered from its first pair: ps[ti * P])
  const uint32_t e0 = ps[gp], e1 = ps[gp + 1], tb = ps[ti * tabs.P];
  uint32_t total = e1 - e0;
  // a hot key split off by k_nagg_hot: its rows are in place (the suffix of the partition's sub range),
  // the stream is the partition's other pairs, compacted
  const uint32_t* hw = tabs.hot ? tabs.hot + uint64_t(gp) * kHotW : nullptr;
  const bool ext = hw && hw[0];
  if (ext) {
    pairs = tabs.hpairs;
    total = hw[4];
  }
  const bool elect = total >= tabs.elect_min;  // (uniform per workgroup)
  nagg_clk(gp, 0);
  nagg_clk(gp, 7);
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  if constexpr (PK) {
    if (threadIdx.x < 64) {
      const uint32_t len = uint32_t(lane) < src.S2 ? src.fcnt[uint64_t(lane) * src.pk.P + p] : 0u;
      uint32_t tot;
      const uint32_t pre = wave_excl_scan(len, &tot);
      if (uint32_t(lane) < src.S2) rstart[lane] = pre;
      if (lane == 0) {
        rstart[src.S2] = tot;
        rstart[src.S2 + 1] = tot;
      }
    }
    // (the first barrier below orders these writes before any read)
  }
  // bucket of a table key inside the partition, and the hash its main record carries
  const auto lbk = [&](uint32_t x) __attribute__((always_inline)) {
    if constexpr (PK) return x >> src.pk.qbits;
    else return fm.mod(x) - lo - b0;
  };
  const auto hash_of = [&](uint32_t x) __attribute__((always_inline)) {
    if constexpr (PK) return src.pk.hash_of(x, p);
    else return x;
  };
  uint32_t cr = 0, nst = 0;  // (contiguous PK form: the lane's region cursor)
  const uint2* rsrc = nullptr;
  // The passes stream the partition's pairs in steps of kAggU items per lane, the next step's loads
  // in flight. Every step issues exactly kAggU loads per lane (indices clamped to the last pair), so
  // the compiler waits for the batch in flight with a counted s_waitcnt at its use, not vmcnt(0) right
  // after issuing it (a data-dependent number of loads, or of stores in pass B, made every step wait
  // for the next step's loads). Contiguous form: item i0 + u * BLOCK + tid of the partition.
  // Slices (PK): wave w walks the fine regions w, w + waves, ... one after another,
  // a step being kAggU x 64 consecutive items of one region, so no item searches for its region.
  // body(v, valid): v the step's pairs, valid the bit mask of the lane's real items.
  const uint32_t wid = threadIdx.x / kWave;
  const auto stream = [&](auto&& body) __attribute__((always_inline)) {
    uint2 v[kAggU], nv[kAggU];
    if constexpr (PK) {
      const auto rlen = [&](uint32_t r) __attribute__((always_inline)) { return rstart[r + 1] - rstart[r]; };
      const auto skip = [&](uint32_t r) __attribute__((always_inline)) {  // the next non-empty region from r
        while (r < src.S2 && rlen(r) == 0) r += kNw;
        return r;
      };
      const auto wload = [&](uint32_t r, uint32_t q, uint2 (&x)[kAggU]) __attribute__((always_inline)) {
        if (r >= src.S2) return;
        const uint2* b = src.fine + (uint64_t(r) * src.pk.P + p) * src.cap2;
        const uint32_t last = rlen(r) - 1;
#pragma unroll
        for (int u = 0; u < kAggU; ++u) x[u] = b[min(q + uint32_t(u) * kWave + uint32_t(lane), last)];
      };
      uint32_t r = skip(wid), q = 0;
      wload(r, q, nv);
      while (r < src.S2) {
#pragma unroll
        for (int u = 0; u < kAggU; ++u) v[u] = nv[u];
        const uint32_t len = rlen(r);
        uint32_t valid = 0;
#pragma unroll
        for (int u = 0; u < kAggU; ++u) valid |= uint32_t(q + uint32_t(u) * kWave + uint32_t(lane) < len) << u;
        q += kAggU * kWave;
        if (q >= len) {
          r = skip(r + kNw);
          q = 0;
        }
        wload(r, q, nv);  // next step in flight
        body(v, valid);
      }
    } else {
      const auto load = [&](uint32_t f0, uint2 (&x)[kAggU]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < kAggU; ++u) {
          const uint32_t f = min(f0 + u * BLOCK + threadIdx.x, total - 1);
          if constexpr (PK) {
            while (f >= nst) {  // per-lane cursor over the fine regions (indices only grow in a pass)
              ++cr;
              nst = rstart[cr + 1];
              rsrc = src.fine + (uint64_t(cr) * src.pk.P + p) * src.cap2;
            }
            x[u] = rsrc[f - rstart[cr]];
          } else {
            x[u] = pairs[e0 + f];
          }
        }
      };
      if constexpr (PK) {
        cr = 0;
        nst = rstart[1];
        rsrc = src.fine + uint64_t(p) * src.cap2;
      }
      if (total) load(0, nv);
      for (uint32_t i0 = 0; i0 < total; i0 += BLOCK * kAggU) {
#pragma unroll
        for (int u = 0; u < kAggU; ++u) v[u] = nv[u];
        load(i0 + BLOCK * kAggU, nv);  // next batch in flight
        uint32_t valid = 0;
#pragma unroll
        for (int u = 0; u < kAggU; ++u) valid |= uint32_t(i0 + u * BLOCK + threadIdx.x < total) << u;
        body(v, valid);
      }
    }
  };
  uint2* wq = reinterpret_cast<uint2*>(bcnt) + wid * kAggQ;  // pass A's miss queue of this wave
  uint32_t mrun = 0, srun = 0, mxlen = 0;  // keys and rows of the finished rounds
  uint32_t c0 = 0, span = (nbs + kAggRounds - 1) / kAggRounds;
  const uint32_t wid_ = threadIdx.x / kWave;
  while (c0 < nbs) {
    const uint32_t c1 = min(nbs, c0 + span);
    const bool whole = c0 == 0 && c1 == nbs;
    // a key that no key of this round is: its bucket lies outside [b0 + c0, b0 + c1)
    const uint32_t empty = PK ? (c1 << src.pk.qbits) : uint32_t((uint64_t(lo) + b0 + c1) % nb_global);
    // Hot key (heavy partitions, one round over the whole range): a Zipf key holding
    // most of a partition's rows (config C: 829 K of ~880 K) made its workgroup the launch's
    // critical path (1.2 of 1.34 ms), each of its rows paying the wave-leader election in both
    // passes. The key is found from BLOCK pairs sampled evenly over the partition (each wave votes for
    // its lane 0's key; taken when its votes reach a quarter of the samples); its rows then take a
    // register path: pass A counts them and their min row per lane (one table update per wave at the
    // end), pass B places them at the key's range start + the wave's prefix (from pass A's per-wave
    // counts: both passes walk the stream in one order) + a running ballot count: no LDS atomic.
    // (split off: the key is this round's when its bucket is)
    uint32_t H = ext && (whole || lbk(hw[1]) - c0 < c1 - c0) ? hw[1] : empty;
    if (!ext && elect && whole && total >= 4u * BLOCK) {
      if constexpr (PK) __syncthreads();  // (the region starts written above)
      const uint32_t f = uint32_t(uint64_t(total) * threadIdx.x / BLOCK);
      uint32_t key;
      if constexpr (PK) {
        uint32_t r = 0;
        while (r + 1 < src.S2 && f >= rstart[r + 1]) ++r;
        key = src.fine[(uint64_t(r) * src.pk.P + p) * src.cap2 + (f - rstart[r])].x;
      } else {
        key = pairs[e0 + f].x;
      }
      const uint32_t cand = uint32_t(__builtin_amdgcn_readlane(int(key), 0));
      const uint32_t votes = uint32_t(__popcll(__ballot(key == cand)));
      if (lane == 0) {
        hotw[wid_] = cand;
        hotm[wid_] = votes;
      }
      __syncthreads();
      uint32_t best = 0;
#pragma unroll 1
      for (int w = 0; w < BLOCK / kWave; ++w) {
        uint32_t sc = 0;
#pragma unroll 1
        for (int w2 = 0; w2 < BLOCK / kWave; ++w2) sc += hotw[w2] == hotw[w] ? hotm[w2] : 0u;
        if (sc > best) {
          best = sc;
          H = hotw[w];
        }
      }
      if (best < BLOCK / 4) H = empty;
      __syncthreads();  // (the scratch words are rewritten below)
    }
    const bool hot = H != empty;  // (uniform)
    for (uint32_t s = threadIdx.x; s < cap; s += BLOCK) {
      tkey[s] = empty;
      tcnt[s] = 0;
      tmin[s] = kInvalid;
    }
    // bcnt past the miss queues (each wave clears its own queue's words after its last flush)
    for (uint32_t k = kNw * 2 * kAggQ + threadIdx.x; k < c1 - c0; k += BLOCK) bcnt[k] = 0;
    if (threadIdx.x == 0) ovf = 0;
    __syncthreads();
    nagg_clk(gp, 1);
    // ---- pass A: count and min row per key ----
    uint32_t hc = 0, hm = kInvalid;  // hot rows and their min row (this lane)
    // Items whose key is not in its home slot (new keys, keys placed further along their probe
    // sequence: ~1 in 4 at config D) go to the wave's miss queue instead of walking the probe
    // sequence in place: in place, nearly every item had a few such lanes, so the wave ran a divergent
    // probe loop per item; the queue is walked with every lane busy once it holds 64 items.
    uint32_t qh = 0, qt = 0;  // (wave-uniform) ring head and tail, pairs
    const auto qtake = [&](bool take) __attribute__((always_inline)) {  // this lane's pair at the head
      __builtin_amdgcn_wave_barrier();
      if (take) {
        const uint2 e = wq[(qh + uint32_t(lane)) & (kAggQ - 1)];
        const uint32_t s = tab_insert(tkey, e.x, empty, cap);
        if (s == kInvalid) {
          ovf = 1;
        } else {
          atomicAdd(&tcnt[s], 1u);
          atomicMin(&tmin[s], e.y);
        }
      }
      __builtin_amdgcn_wave_barrier();
    };
    stream([&](const uint2 (&v)[kAggU], uint32_t valid) __attribute__((always_inline)) {
      // home slots of all items read together (one LDS latency for the batch); only items whose
      // key is not in its home slot walk the probe sequence; active items as one bit mask
      uint32_t actm = 0;
      uint32_t k0[kAggU];
#pragma unroll
      for (int u = 0; u < kAggU; ++u) {
        // one round over the whole range (the common case): every pair of the partition is in it,
        // so no bucket (a 64-bit multiply-high per pair on the modulo path) is computed
        bool inr = true;
        if (!whole) {
          const uint32_t lb = lbk(v[u].x);
          inr = lb >= c0 && lb < c1;
        }
        const bool a = ((valid >> u) & 1u) && inr;
        actm |= uint32_t(a) << u;
        k0[u] = tkey[a ? slot_of(v[u].x, cap) : 0u];
      }
#pragma unroll
      for (int u = 0; u < kAggU; ++u) {
        bool a = (actm >> u) & 1u;
        if (hot) {
          const bool h = a && v[u].x == H;
          hc += h;
          hm = h ? min(hm, v[u].y) : hm;
          a = a && !h;
        }
        const uint64_t am = elect ? __ballot(a) : 0ull;
        if (am) {  // the wave's first active key, if several lanes hold it (a Zipf hot key)
          const int leader = __ffsll((unsigned long long)am) - 1;
          const uint32_t hl = uint32_t(__builtin_amdgcn_readlane(int(v[u].x), leader));
          const bool mine = a && v[u].x == hl;
          const uint64_t same = __ballot(mine);
          if (__popcll(same) > 1) {
            const uint32_t rmin = wave_min_u32(mine ? v[u].y : kInvalid);
            if (lane == leader) {
              const uint32_t s = tab_insert(tkey, hl, empty, cap);
              if (s == kInvalid) {
                ovf = 1;
              } else {
                atomicAdd(&tcnt[s], uint32_t(__popcll(same)));
                atomicMin(&tmin[s], rmin);
              }
            }
            a = a && !mine;
          }
        }
        const bool miss = a && k0[u] != v[u].x;
        if (a && !miss) {
          const uint32_t s = slot_of(v[u].x, cap);
          atomicAdd(&tcnt[s], 1u);
          atomicMin(&tmin[s], v[u].y);
        }
        const uint64_t mb = __ballot(miss);
        if (miss) wq[(qt + uint32_t(__popcll(mb & lt))) & (kAggQ - 1)] = v[u];
        qt += uint32_t(__popcll(mb));
        if (qt - qh >= kWave) {  // 64 pairs: one with every lane
          qtake(true);
          qh += kWave;
        }
      }
    });
    qtake(uint32_t(lane) < qt - qh);
    {  // this wave's queue words back to bucket counts (zero) for the main slots below
      uint32_t* qw = reinterpret_cast<uint32_t*>(wq);
      for (uint32_t k = uint32_t(lane); k < 2 * kAggQ; k += kWave)
        if (wid_ * 2 * kAggQ + k < c1 - c0) qw[k] = 0;
    }
    if (hot) {  // the hot key into the table: per-wave totals, then one insert
      uint32_t c = hc;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
      const uint32_t m = wave_min_u32(hm);
      if (lane == 0) {
        hotw[wid_] = c;
        hotm[wid_] = m;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t tot = 0, mn = kInvalid;
        for (int w = 0; w < BLOCK / kWave; ++w) {  // -> the waves' exclusive prefix
          const uint32_t x = hotw[w];
          hotw[w] = tot;
          tot += x;
          mn = min(mn, hotm[w]);
        }
        if (ext) {  // (the stream held none of its rows)
          tot = hw[2];
          mn = hw[3];
        }
        const uint32_t sl = tot ? tab_insert(tkey, H, empty, cap) : kInvalid;
        if (tot && sl == kInvalid) {
          ovf = 1;
        } else if (tot) {
          tcnt[sl] += tot;
          tmin[sl] = min(tmin[sl], mn);
        }
        hslot = sl;
        hrows = tot;
      }
    }
    __syncthreads();
    nagg_clk(gp, 2);
    if (ovf) {  // too many distinct keys for one round: retry the first half of the range
      if (c1 - c0 <= kAggMinSpan) {  // > ~24 keys per bucket: the sort-based build instead
        if (threadIdx.x == 0) atomicOr(fail, 1u);
        return 0;
      }
      span = (c1 - c0 + 1) / 2;
      __syncthreads();
      continue;
    }
    // ---- main slots: rank of every key inside its bucket (registers), bucket offsets ----
    // (empty slots: tkey = empty, tcnt = 0, tmin = kInvalid)
    uint32_t rank[SLOTS];
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const uint32_t s = j * BLOCK + threadIdx.x;
      rank[j] = s < cap && tcnt[s] ? atomicAdd(&bcnt[lbk(tkey[s]) - c0], 1u) : 0u;
    }
    __syncthreads();
    const uint32_t nk = block_scan_lds<BLOCK>(bcnt, c1 - c0, wsum);  // bcnt[k] = first main of bucket c0 + k
    // slice path's look-back: the partition's key count is final after its last round's pass A, so it is
    // published here, long before the workgroup looks back (after pass B); waiting for predecessors'
    // counts at the end of their pass B stalled every workgroup behind the slowest (D shape 39 ms)
    if (lb && c1 == nbs && threadIdx.x == 0 && !(tabs.lb_skip0 && gp == 0))
      __hip_atomic_store(tabs.lbw + 2 + gp, (uint64_t(tabs.lb_epoch & 0x3FFFFFFFu) << 34) | (1ull << 32) | (mrun + nk),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // sub ranges: exclusive scan of the counts in slot order; tcnt becomes the sub cursor
    uint32_t cnt[SLOTS];
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const uint32_t s = j * BLOCK + threadIdx.x;
      cnt[j] = s < cap ? tcnt[s] : 0u;
      if (ext && hot && s == hslot) tcnt[s] = 0;  // (its range: after every other row)
    }
    __syncthreads();
    const uint32_t nrows = block_scan_lds<BLOCK>(tcnt, cap, wsum);
    // main records (partition-local slots, global sub offsets) and the round's directory words
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const uint32_t s = j * BLOCK + threadIdx.x;
      if (cnt[j]) {
        const uint32_t h = tkey[s];
        const uint32_t m = mrun + bcnt[lbk(h) - c0] + rank[j];
        // (table ti's sub rows; a split-off hot key's: past the partition's other rows, of every round)
        const uint32_t so = e0 - tb + (ext && hot && s == hslot ? total : srun + tcnt[s]);
        mtmp[e0 + m] = make_uint4(hash_of(h), tmin[s], so, cnt[j]);
        mxlen = max(mxlen, cnt[j]);
      }
    }
    for (uint32_t k = threadIdx.x; k < c1 - c0; k += BLOCK) off[b0 + c0 + k] = mrun + bcnt[k];
    __syncthreads();
    nagg_clk(gp, 3);
    // ---- pass B: rows into their keys' sub ranges ----
    // The round's first imgw rows are assembled in LDS (the image) and go out as whole lines; rows past
    // it (a partition with more rows than the image holds) and a hot key's rows (per-wave runs) go to
    // HBM directly. 4-B row stores scattered over a partition's whole sub range left the L2 with partial
    // lines (config C: 2.2 GB written for 0.55 GB of sub rows and main records; build 2.06 -> 1.62 ms
    // with no row stores at all). Tried: more sweeps over the pairs, one per image-sized slot range of
    // keys (C: 3 sweeps, 2.36 ms against 1.87 ms for one sweep; config D's shape gained nothing).
    uint32_t* __restrict__ gsub = sub + (e0 - tb + srun);  // the round's sub rows
    const bool hk = hot && !ext && hslot != kInvalid;  // (uniform) rows of the hot key: to HBM, per wave
    // (hot key: its range start + this wave's prefix)
    uint32_t hcur = hk ? tcnt[hslot] + hotw[wid_] : 0u;
    const uint32_t hstart = hk ? tcnt[hslot] : 0u, hlen = hk ? hrows : 0u;  // (its cursor never moves)
    // DIRECT: rows also go to HBM (every item then stores once, to its row or the sink: a fixed store
    // count per step); otherwise pass B writes LDS only
    const auto passb = [&](auto direct_c) __attribute__((always_inline)) {
      constexpr bool DIRECT = decltype(direct_c)::value;
      stream([&](const uint2 (&v)[kAggU], uint32_t valid) __attribute__((always_inline)) {
        uint32_t actm = 0;
        uint32_t k0[kAggU];
#pragma unroll
        for (int u = 0; u < kAggU; ++u) {
          bool inr = true;
          if (!whole) {
            const uint32_t lb = lbk(v[u].x);
            inr = lb >= c0 && lb < c1;
          }
          const bool a = ((valid >> u) & 1u) && inr;
          actm |= uint32_t(a) << u;
          k0[u] = tkey[a ? slot_of(v[u].x, cap) : 0u];
        }
#pragma unroll
        for (int u = 0; u < kAggU; ++u) {
          bool a = (actm >> u) & 1u;
          uint32_t dl = kInvalid;  // the row's place in the round's sub range
          uint32_t* dst = tabs.sink;
          if (hk) {
            const bool h = a && v[u].x == H;
            if constexpr (DIRECT) {
              const uint64_t hm2 = __ballot(h);
              if (h) dst = gsub + hcur + uint32_t(__popcll(hm2 & lt));
              hcur += uint32_t(__popcll(hm2));
            }
            a = a && !h;
          }
          const uint64_t am = elect ? __ballot(a) : 0ull;
          if (am) {
            const int leader = __ffsll((unsigned long long)am) - 1;
            const uint32_t hl = uint32_t(__builtin_amdgcn_readlane(int(v[u].x), leader));
            const bool mine = a && v[u].x == hl;
            const uint64_t same = __ballot(mine);
            if (__popcll(same) > 1) {  // one cursor bump for the group, consecutive sub slots
              uint32_t base = 0;
              if (lane == leader) base = atomicAdd(&tcnt[tab_find(tkey, hl, cap)], uint32_t(__popcll(same)));
              base = uint32_t(__builtin_amdgcn_readlane(int(base), leader));
              if (mine) dl = base + uint32_t(__popcll(same & lt));
              a = a && !mine;
            }
          }
          if (a) {
            const uint32_t s = k0[u] == v[u].x ? slot_of(v[u].x, cap) : tab_find_away(tkey, v[u].x, cap);
            dl = atomicAdd(&tcnt[s], 1u);
          }
          if constexpr (DIRECT) {
            if (dl != kInvalid) {
              if (dl < imgw) img[dl] = v[u].y;
              else dst = gsub + dl;
            }
            *dst = v[u].y;  // (straight-line: one store per item and lane; non-temporal: C build 3.7 ms)
          } else {
            if (dl != kInvalid) img[dl] = v[u].y;
          }
        }
      });
    };
    if (hk || nrows > imgw) passb(std::true_type{});
    else passb(std::false_type{});
    __syncthreads();
#if HJ3D_NAGG_CLK
    if (!lb && threadIdx.x == 0 && gp < kClkParts) g_nagg_clk[gp * kClkPts + 7] = wall_clock64();  // (sweep end)
#endif
    // the image out as whole lines (the hot key's rows, already in place, skipped), non-temporal
    // (same box: D shape 16.57 -> 16.29 ms, E build 0.2598 -> 0.2581 ms, C within noise; r06z_ntw_*,
    // r06z_ntc_C_ab.jsonl)
    for (uint32_t k = threadIdx.x; k < min(nrows, imgw); k += BLOCK)
      if (k - hstart >= hlen) __builtin_nontemporal_store(img[k], gsub + k);
    __syncthreads();  // (the next round's table; the next partition's)
    nagg_clk(gp, 4);
    mrun += nk;
    srun += nrows;
    c0 = c1;
  }
  nagg_clk(gp, 5);
  if (threadIdx.x == 0) dcount[gp] = mrun;
  const uint64_t wm = wave_max(uint64_t(mxlen));
  if ((threadIdx.x & 63) == 0 && wm) atomicMax(maxlen, (unsigned long long)wm);
  return mrun;
}

// The slice path's finish inside k_nagg (one table; partitions taken in ticket order, so every
// partition before gp has a running or finished workgroup): publish the partition's key count, find
// its main-record base by a decoupled look-back over the status words (64 predecessors per step, one
// per lane of wave 0: the nearest inclusive prefix plus the aggregates after it), publish the
// inclusive prefix, move the main records to their final slots and rebase the partition's directory
// words; the last workgroup to finish writes the table's counts (and their host copy) and resets the
// ticket. Status word: epoch << 34 | flag << 32 | value (flag 1 aggregate, 2 inclusive prefix), each an
// 8-B relaxed agent-scope atomic (MI355X_MICROARCH.md, inter-workgroup hand-off: the word carries all
// the data; acquire / release forms write back or invalidate the XCD's L2 and, issued by every
// workgroup, slowed the whole launch 2x: D shape 16.4 -> 32 ms). A
// look-back that waits 0.2 s sets the table's give-up flag (the sort build replaces it) instead of
// hanging. Replaces exclusive_scan_u32 + k_nagg_rebase + k_nagg_mains (config D's Nrs table: ~1.2 ms).
__device__ __forceinline__ void nagg_lb_finish(uint32_t gp, uint32_t nk, uint32_t P, uint32_t W, uint32_t nbl,
                                               const uint4* __restrict__ mtmp, const uint32_t* __restrict__ ps,
                                               const NaggTabs& tabs, uint32_t* bw) {
  uint64_t* st = tabs.lbw + 2;
  const uint64_t ep = uint64_t(tabs.lb_epoch & 0x3FFFFFFFu);
  const auto pack = [&](uint64_t f, uint64_t v) __attribute__((always_inline)) { return (ep << 34) | (f << 32) | v; };
  uint64_t* counts = tabs.counts[0];
  // (the aggregate is usually out already, from the last round's pass A; a partition that gave up
  // publishes its 0 here)
  const bool publish = !(tabs.lb_skip0 && gp == 0);
  if (threadIdx.x == 0 && publish) __hip_atomic_store(st + gp, pack(1, nk), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    uint64_t prefix = 0;
    int64_t j = int64_t(gp) - 1;
    const uint64_t t0 = wall_clock64();
    while (j >= 0) {
      const uint64_t w = int64_t(lane) <= j
                             ? __hip_atomic_load(st + (j - lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : pack(2, 0);
      const bool ok = (w >> 34) == ep && ((w >> 32) & 3u) != 0;
      const uint64_t im = __ballot(ok && ((w >> 32) & 3u) == 2), bad = __ballot(!ok);
      const int fi = im ? __ffsll((unsigned long long)im) - 1 : 64;
      const uint64_t upto = fi >= 63 ? ~0ull : ((2ull << fi) - 1);
      if (bad & upto) {  // a predecessor has not published yet
        if (wall_clock64() - t0 > tabs.lb_ticks) {
          if (lane == 0) atomicOr(reinterpret_cast<uint32_t*>(counts + 3), 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      prefix += wave_sum(lane <= fi ? (w & 0xFFFFFFFFull) : 0ull);
      if (fi < 64) break;
      j -= kWave;
    }
    if (lane == 0) {
      if (publish) __hip_atomic_store(st + gp, pack(2, prefix + nk), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bw[0] = uint32_t(prefix);
    }
  }
  __syncthreads();
  const uint32_t base = bw[0];
  // (the partition's main records and directory words were written by this workgroup: L2-warm)
  uint4* __restrict__ mains = tabs.main[0];
  const uint32_t e0 = ps[gp];
  for (uint32_t i = threadIdx.x; i < nk; i += blockDim.x) mains[base + i] = mtmp[e0 + i];
  uint32_t* __restrict__ off = tabs.off[0];
  const uint32_t b0 = gp * W, nbs = min(W, nbl - b0);
  for (uint32_t k = threadIdx.x; k < nbs; k += blockDim.x) off[b0 + k] += base;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t done = __hip_atomic_fetch_add(tabs.lbw + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == P - 1) {  // the last workgroup: every other one has published and finished
      const bool failed = __hip_atomic_load(reinterpret_cast<uint32_t*>(counts + 3), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT) != 0;
      uint64_t c0 = 0, c1 = 0;
      if (!failed) {
        c0 = ps[P] - ps[0];
        c1 = __hip_atomic_load(st + (P - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xFFFFFFFFull;
        counts[0] = c0;
        counts[1] = c1;
        off[nbl] = uint32_t(c1);
      }
      if (uint64_t* h = tabs.hc[0]) {  // the host's copy
        h[0] = c0;
        h[1] = c1;
        h[2] = __hip_atomic_load(counts + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        h[3] = __hip_atomic_load(counts + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(tabs.lbw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(tabs.lbw + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One workgroup per partition: gp = blockIdx.x, or order[blockIdx.x] (heavy first), or a ticket (the
// slice path's look-back finish; one call site of nagg_one for both: two inlined copies spilled).
template <int BLOCK, int SLOTS, bool PK>
__global__ __launch_bounds__(BLOCK, 4) void k_nagg(const uint2* __restrict__ pairs, const uint32_t* __restrict__ ps,
                                                FastMod fm, uint32_t lo, uint32_t nbl, uint32_t nb_global, uint32_t W,
                                                uint4* __restrict__ mtmp, uint32_t* __restrict__ dcount,
                                                const uint32_t* __restrict__ order, uint32_t cap, NaggSrc src,
                                                NaggTabs tabs) {
  extern __shared__ uint32_t agg_lds[];
  const bool lb = PK && tabs.lbw;
  uint32_t* bw = agg_lds + 2 * cap;  // (the block-scan words: free before and after nagg_one)
  uint32_t gp;
  if (lb) {  // partitions in ticket order (the look-back waits only on earlier tickets)
    if (threadIdx.x == 0)
      bw[0] = uint32_t(__hip_atomic_fetch_add(tabs.lbw, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    __syncthreads();
    gp = bw[0];
    __syncthreads();
  } else {
    gp = PK || !order ? blockIdx.x : order[blockIdx.x];
  }
  const uint32_t nk = nagg_one<BLOCK, SLOTS, PK>(gp, pairs, ps, fm, lo, nbl, nb_global, W, mtmp, dcount, cap, src, tabs,
                                                 agg_lds, lb);
  if (!lb) return;
  __syncthreads();
  nagg_lb_finish(gp, nk, src.pk.P, W, nbl, mtmp, ps, tabs, bw);
#if HJ3D_NAGG_CLK
  if (threadIdx.x == 0 && gp < kClkParts) g_nagg_clk[gp * kClkPts + 7] = wall_clock64();  // (finish end)
#endif
}

// ---- k_nagg_reg: the partition held in registers, its sub rows assembled in LDS ----
// k_nagg streams every partition twice from HBM (pass A, pass B) and scatters each sub row with a
// 4-B store into the partition's sub window, whose lines the L2 evicts before they are complete
// (3.8x write amplification at config C). Here one persistent 1024-thread workgroup per CU takes
// partitions idx = blockIdx.x, + gridDim.x, ... (partition order[idx], heavy first, or idx itself):
// a partition of <= kRegCap pairs is loaded into registers ONCE (the next partition's loads are
// issued as soon as pass B has read them, and overlap the image write-out and the next table's
// initialisation), pass A and pass B run on the registers, pass B places every row into an LDS image
// of the partition's sub range, and the image goes out as whole lines. Per pair: 8 B read + 4 B
// written. A partition with more pairs than kRegCap (a Zipf hot key's) or more distinct keys than
// the table holds takes k_nagg's streaming form (nagg_one) in place, in the same workgroup.
constexpr int kRegBlock = 1024;
constexpr int kRegK = 16;                                      // pairs per lane (20, 24: spills)
constexpr uint32_t kRegCap = uint32_t(kRegK) * kRegBlock;      // pairs per partition (16384)
__host__ __device__ constexpr uint32_t reg_lds_words(uint32_t cap, uint32_t W) {
  return 3 * cap + W + kRegCap + kRegBlock / 64 + 2 + 2 * (kAggMaxS2 + 2);
}
template <bool PK, int SLOTS>
__global__ __launch_bounds__(kRegBlock) void k_nagg_reg(const uint2* __restrict__ pairs, const uint32_t* __restrict__ ps,
                                                        FastMod fm, uint32_t lo, uint32_t nbl, uint32_t nb_global,
                                                        uint32_t W, uint32_t PT, uint4* __restrict__ mtmp,
                                                        uint32_t* __restrict__ dcount, uint32_t cap, NaggSrc src,
                                                        NaggTabs tabs, const uint32_t* __restrict__ order) {
  extern __shared__ uint32_t agg_lds[];
  uint32_t* tkey = agg_lds;
  uint32_t* tcnt = tkey + cap;
  uint32_t* tmin = tcnt + cap;
  uint32_t* bcnt = tmin + cap;
  uint32_t* img = bcnt + W;
  uint32_t* wsum = img + kRegCap;
  uint32_t& ovf = wsum[kRegBlock / kWave + 1];
  uint32_t* rst = wsum + kRegBlock / kWave + 2;  // [2][kAggMaxS2 + 2]: region starts of the two slices in turn
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  uint32_t mxlen = 0;
  const auto part_of = [&](uint32_t idx) __attribute__((always_inline)) { return order ? order[idx] : idx; };
  // region starts of slice gp into rst[b] (PK: one table; wave 0)
  const auto starts = [&](uint32_t idx, uint32_t b) __attribute__((always_inline)) {
    if constexpr (PK) {
      if (wid == 0 && idx < PT) {
        const uint32_t gp = part_of(idx);
        const uint32_t len = uint32_t(lane) < src.S2 ? src.fcnt[uint64_t(lane) * src.pk.P + gp] : 0u;
        uint32_t tot;
        const uint32_t pre = wave_excl_scan(len, &tot);
        uint32_t* r = rst + b * (kAggMaxS2 + 2);
        if (uint32_t(lane) < src.S2) r[lane] = pre;
        if (lane == 0) {
          r[src.S2] = tot;
          r[src.S2 + 1] = tot;
        }
      }
    }
  };
  const auto count_of = [&](uint32_t gp, uint32_t b) __attribute__((always_inline)) {
    if constexpr (PK) return rst[b * (kAggMaxS2 + 2) + src.S2];
    else return ps[gp + 1] - ps[gp];
  };
  // kRegK loads per lane, always (indices clamped to the partition's last pair); a partition of more
  // than kRegCap pairs takes the streaming form, so its registers are never used
  uint2 v[kRegK];
  const auto load = [&](uint32_t idx, uint32_t b) __attribute__((always_inline)) {
    if (idx >= PT) return;  // (past the last partition: rst[b] was not written)
    const uint32_t gp = part_of(idx);
    const uint32_t m = count_of(gp, b);
    const uint32_t last = m ? m - 1 : 0u;
    if constexpr (PK) {
      const uint32_t* r = rst + b * (kAggMaxS2 + 2);
      uint32_t cr = 0;
#pragma unroll
      for (int u = 0; u < kRegK; ++u) {
        const uint32_t f = min(uint32_t(u) * kRegBlock + threadIdx.x, last);
        while (cr + 1 < src.S2 && f >= r[cr + 1]) ++cr;
        v[u] = src.fine[(uint64_t(cr) * src.pk.P + gp) * src.cap2 + (f - r[cr])];
      }
    } else {
      const uint32_t e0 = ps[gp];
#pragma unroll
      for (int u = 0; u < kRegK; ++u) v[u] = pairs[e0 + min(uint32_t(u) * kRegBlock + threadIdx.x, last)];
    }
  };
  const auto process = [&](uint32_t idx, uint32_t b) __attribute__((always_inline)) {
    const uint32_t gp = part_of(idx);
    const uint32_t ti = tabs.nt > 1 && gp >= tabs.P ? 1u : 0u;
    const uint32_t p = gp - ti * tabs.P;  // partition inside table ti
    uint32_t* __restrict__ off = tabs.off[ti];
    uint32_t* __restrict__ sub = tabs.sub[ti];
    const uint32_t b0 = p * W, nbs = min(W, nbl - b0);
    const uint32_t e0 = ps[gp], m = count_of(gp, b);
    const uint32_t empty = PK ? (nbs << src.pk.qbits) : uint32_t((uint64_t(lo) + b0 + nbs) % nb_global);
    const auto lbk = [&](uint32_t x) __attribute__((always_inline)) {
      if constexpr (PK) return x >> src.pk.qbits;
      else return fm.mod(x) - lo - b0;
    };
    // (a partition whose hot key k_nagg_hot split off: k_nagg's streaming form, which knows the split)
    const bool big = m > kRegCap || (tabs.hot && tabs.hot[uint64_t(gp) * kHotW]);
    if (!big) {
      for (uint32_t s = threadIdx.x; s < cap; s += kRegBlock) {
        tkey[s] = empty;
        tcnt[s] = 0;
        tmin[s] = kInvalid;
      }
      for (uint32_t k = threadIdx.x; k < nbs; k += kRegBlock) bcnt[k] = 0;
      if (threadIdx.x == 0) ovf = 0;
    }
    starts(idx + gridDim.x, b ^ 1u);  // the next partition's region starts (PK)
    __syncthreads();
    // ---- pass A: count and min row per key (registers) ----
    if (!big) {
#pragma unroll
      for (int u0 = 0; u0 < kRegK; u0 += 8) {
        uint32_t actm = 0, k0[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const bool a = uint32_t(u0 + u) * kRegBlock + threadIdx.x < m;
          actm |= uint32_t(a) << u;
          k0[u] = tkey[a ? slot_of(v[u0 + u].x, cap) : 0u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const uint2 e = v[u0 + u];
          bool a = (actm >> u) & 1u;
          const uint64_t am = __ballot(a);
          if (am) {  // the wave's first active key, if several lanes hold it (a hot key)
            const int leader = __ffsll((unsigned long long)am) - 1;
            const uint32_t hl = uint32_t(__builtin_amdgcn_readlane(int(e.x), leader));
            const bool mine = a && e.x == hl;
            const uint64_t same = __ballot(mine);
            if (__popcll(same) > 1) {
              const uint32_t rmin = wave_min_u32(mine ? e.y : kInvalid);
              if (lane == leader) {
                const uint32_t s = tab_insert(tkey, hl, empty, cap);
                if (s == kInvalid) {
                  ovf = 1;
                } else {
                  atomicAdd(&tcnt[s], uint32_t(__popcll(same)));
                  atomicMin(&tmin[s], rmin);
                }
              }
              a = a && !mine;
            }
          }
          if (a) {
            const uint32_t s = k0[u] == e.x ? slot_of(e.x, cap) : tab_insert_k(tkey, e.x, k0[u], empty, cap);
            if (s == kInvalid) {
              ovf = 1;
            } else {
              atomicAdd(&tcnt[s], 1u);
              atomicMin(&tmin[s], e.y);
            }
          }
        }
      }
      __syncthreads();
    }
    if (big || ovf) {
      // more pairs than the registers hold, or more keys than one table round: left to k_nagg's
      // streaming form (k_nagg_defer, the next launch; nothing of the partition is written yet). Run in
      // place it cost this kernel its registers: the inlined streaming code spilled the pair registers
      if (threadIdx.x == 0) tabs.defer[1 + atomicAdd(&tabs.defer[0], 1u)] = gp;
      load(idx + gridDim.x, b ^ 1u);
      return;
    }
    // ---- main slots: rank of every key inside its bucket, bucket offsets, sub ranges ----
    uint32_t rank[SLOTS], cnt[SLOTS];
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const uint32_t s = j * kRegBlock + threadIdx.x;
      rank[j] = s < cap && tcnt[s] ? atomicAdd(&bcnt[lbk(tkey[s])], 1u) : 0u;
    }
    __syncthreads();
    const uint32_t nk = block_scan_lds<kRegBlock>(bcnt, nbs, wsum);
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const uint32_t s = j * kRegBlock + threadIdx.x;
      cnt[j] = s < cap ? tcnt[s] : 0u;
    }
    __syncthreads();
    block_scan_lds<kRegBlock>(tcnt, cap, wsum);  // tcnt: the key's first slot in the image
    const uint32_t sb = e0 - ps[ti * tabs.P];     // the partition's sub range starts at its first pair
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const uint32_t s = j * kRegBlock + threadIdx.x;
      if (cnt[j]) {
        const uint32_t h = tkey[s];
        uint32_t hash;
        if constexpr (PK) hash = src.pk.hash_of(h, p);
        else hash = h;
        mtmp[e0 + bcnt[lbk(h)] + rank[j]] = make_uint4(hash, tmin[s], sb + tcnt[s], cnt[j]);
        mxlen = max(mxlen, cnt[j]);
      }
    }
    for (uint32_t k = threadIdx.x; k < nbs; k += kRegBlock) off[b0 + k] = bcnt[k];
    __syncthreads();
    // ---- pass B: every row to its key's next image slot ----
#pragma unroll
    for (int u = 0; u < kRegK; ++u) {
      const uint2 e = v[u];
      bool a = uint32_t(u) * kRegBlock + threadIdx.x < m;
      const uint64_t am = __ballot(a);
      if (am) {
        const int leader = __ffsll((unsigned long long)am) - 1;
        const uint32_t hl = uint32_t(__builtin_amdgcn_readlane(int(e.x), leader));
        const bool mine = a && e.x == hl;
        const uint64_t same = __ballot(mine);
        if (__popcll(same) > 1) {  // one cursor bump for the group, consecutive slots
          uint32_t base = 0;
          if (lane == leader) base = atomicAdd(&tcnt[tab_find(tkey, hl, cap)], uint32_t(__popcll(same)));
          base = uint32_t(__builtin_amdgcn_readlane(int(base), leader));
          if (mine) img[base + uint32_t(__popcll(same & lt))] = e.y;
          a = a && !mine;
        }
      }
      if (a) img[atomicAdd(&tcnt[tab_find(tkey, e.x, cap)], 1u)] = e.y;
    }
    __syncthreads();
    // the registers are free: the next partition's loads go out now and overlap the image
    // write-out and the next table's initialisation
    load(idx + gridDim.x, b ^ 1u);
    // ---- the image out: the partition's sub range as whole lines ----
    for (uint32_t k = threadIdx.x; k < m; k += kRegBlock) sub[sb + k] = img[k];
    if (threadIdx.x == 0) dcount[gp] = nk;
  };
  uint32_t idx = blockIdx.x;
  starts(idx, 0);
  __syncthreads();
  load(idx, 0);
  for (uint32_t it = 0; idx < PT; ++it, idx += gridDim.x) {
    process(idx, it & 1u);
    __syncthreads();
  }
  const uint64_t wm = wave_max(uint64_t(mxlen));
  for (uint32_t ti = 0; ti < tabs.nt; ++ti) {
    // (the longest key over both tables is an upper bound for each; the probe only sizes by it)
    auto* maxlen = reinterpret_cast<unsigned long long*>(tabs.counts[ti] + 2);
    if (lane == 0 && wm) atomicMax(maxlen, (unsigned long long)wm);
  }
}

// The partitions k_nagg_reg left (tabs.defer), k_nagg's streaming form: workgroup b takes the
// deferred partitions b, b + gridDim.x, ... (none: every workgroup exits at once).
template <int BLOCK, int SLOTS, bool PK>
__global__ __launch_bounds__(BLOCK, 4) void k_nagg_defer(const uint2* __restrict__ pairs, const uint32_t* __restrict__ ps,
                                                      FastMod fm, uint32_t lo, uint32_t nbl, uint32_t nb_global,
                                                      uint32_t W, uint4* __restrict__ mtmp, uint32_t* __restrict__ dcount,
                                                      uint32_t cap, NaggSrc src, NaggTabs tabs) {
  extern __shared__ uint32_t agg_lds[];
  const uint32_t n = tabs.defer[0];
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    nagg_one<BLOCK, SLOTS, PK>(tabs.defer[1 + i], pairs, ps, fm, lo, nbl, nb_global, W, mtmp, dcount, cap, src, tabs,
                               agg_lds);
    __syncthreads();  // (the next partition's table clear after every read of this one's)
  }
}

// order = the partitions by size class, heavy first (> 8x the mean pairs, then > 2x, then the
// rest), each class in index order: the aggregation takes its partitions in this order, so a Zipf hot
// key's partition starts in the first wave of workgroups instead of extending the tail. One
// workgroup, P <= 8192 (a stable three-way split by block scans; a full sort by size cost 27 us).
constexpr int kOrdPer = 8;  // partitions per thread
// Hot-key split (k_nagg_hot): partitions above 2x the mean are cut into chunks of kHotChunk pairs.
constexpr int kHotBlock = 1024, kHotK = 16;
constexpr uint32_t kHotChunk = uint32_t(kHotBlock) * kHotK;
// hinfo (with tabs.hot): [0] the heavy partitions (order[0 .. nheavy)), [1 + i] the first chunk of heavy
// partition i, [1 + nheavy] the chunk total; every partition's hot words cleared.
__global__ __launch_bounds__(1024) void k_nagg_order(const uint32_t* __restrict__ ps, uint32_t P,
                                                     uint32_t* __restrict__ order, NaggTabs tabs,
                                                     uint32_t* __restrict__ hinfo) {
  __shared__ uint32_t wsum[16], csum[16];
  __shared__ uint32_t base, cbase;
  if (threadIdx.x < 4 * tabs.nt) tabs.counts[threadIdx.x / 4][threadIdx.x % 4] = 0;  // (the build's counts words)
  if (threadIdx.x == 64 && tabs.defer) tabs.defer[0] = 0;
  const uint32_t mean = P ? (ps[P] - ps[0]) / P : 0u;
  uint32_t cls[kOrdPer], nch[kOrdPer];
#pragma unroll
  for (int k = 0; k < kOrdPer; ++k) {  // thread t holds partitions kOrdPer t + k
    const uint32_t p = kOrdPer * threadIdx.x + k;
    const uint32_t sz = p < P ? ps[p + 1] - ps[p] : 0u;
    cls[k] = p >= P ? 3u : sz > 8u * mean ? 0u : sz > 2u * mean ? 1u : 2u;
    nch[k] = (sz + kHotChunk - 1) / kHotChunk;
    if (tabs.hot && p < P) {
      uint32_t* hw = tabs.hot + uint64_t(p) * kHotW;
      hw[0] = 0;
      hw[2] = 0;
      hw[3] = kInvalid;
      hw[4] = 0;
    }
  }
  if (threadIdx.x == 0) base = cbase = 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint32_t c = 0; c < 3; ++c) {
    uint32_t t = 0, tc = 0;
#pragma unroll
    for (int k = 0; k < kOrdPer; ++k) {
      t += cls[k] == c;
      tc += cls[k] == c ? nch[k] : 0u;
    }
    uint32_t wt, wc;
    const uint32_t wpre = wave_excl_scan(t, &wt), cpre = wave_excl_scan(tc, &wc);
    if (lane == 0) {
      wsum[wid] = wt;
      csum[wid] = wc;
    }
    __syncthreads();
    uint32_t pre = 0, tot = 0, cp = 0, ctot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      pre += w < wid ? wsum[w] : 0u;
      tot += wsum[w];
      cp += w < wid ? csum[w] : 0u;
      ctot += csum[w];
    }
    uint32_t at = base + pre + wpre, ch = cbase + cp + cpre;
#pragma unroll
    for (int k = 0; k < kOrdPer; ++k)
      if (cls[k] == c) {
        if (hinfo && c < 2) hinfo[1 + at] = ch;  // (heavy: classes 0 and 1)
        ch += nch[k];
        order[at++] = kOrdPer * threadIdx.x + k;
      }
    __syncthreads();
    if (threadIdx.x == 0) {
      base += tot;
      cbase += ctot;
      if (hinfo && c == 1) {
        hinfo[0] = base;
        hinfo[1 + base] = cbase;
      }
    }
    __syncthreads();
  }
}

// Hot keys of the heavy partitions, split off before the aggregation. A Zipf key can hold most of a
// partition (config C: 829 K of its ~880 K pairs), and that partition's one workgroup then streamed it
// twice while the rest of the chip had finished (k_nagg 1.19 ms, of which the heavy workgroup 1.0 ms;
// the other partitions alone balance to ~0.7 ms). Here chunk c of the heavy partitions (kHotChunk pairs
// held in registers) goes to one workgroup: it finds the partition's hot key from kHotBlock pairs
// sampled evenly over the whole partition (every workgroup of the partition draws the same sample and
// agrees; a key with fewer than a quarter of the votes: nothing to do), counts the key's rows and their
// min row, claims its runs with one atomic per workgroup and writes the key's rows down from the end of
// the partition's sub range (rows of a key have no order) and the other pairs, compacted, to
// hpairs[ps[gp] ..]. nagg_one then streams only those (its `ext` mode) and gives the key the
// sub range's suffix.
__global__ __launch_bounds__(kHotBlock) void k_nagg_hot(const uint2* __restrict__ pairs, const uint32_t* __restrict__ ps,
                                                        const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ hinfo, NaggTabs tabs) {
  constexpr int kNw = kHotBlock / kWave;
  __shared__ uint32_t vk[kNw], vn[kNw], wh[kNw], wn[kNw], wm[kNw];
  __shared__ uint32_t sH, sok, hbase, nbase;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const uint32_t nheavy = hinfo[0], nchunks = hinfo[1 + nheavy];
  for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    uint32_t lo = 0, hi = nheavy;  // the heavy partition holding chunk c: largest i with hinfo[1 + i] <= c
    while (hi - lo > 1) {
      const uint32_t md = (lo + hi) >> 1;
      if (hinfo[1 + md] <= c) lo = md;
      else hi = md;
    }
    const uint32_t gp = order[lo], k = c - hinfo[1 + lo];
    const uint32_t e0 = ps[gp], total = ps[gp + 1] - e0;
    {  // the partition's hot key: each wave votes for its lane 0's sampled key
      const uint32_t key = pairs[e0 + uint32_t(uint64_t(total) * threadIdx.x / kHotBlock)].x;
      const uint32_t cand = uint32_t(__builtin_amdgcn_readlane(int(key), 0));
      const uint32_t votes = uint32_t(__popcll(__ballot(key == cand)));
      if (lane == 0) {
        vk[wid] = cand;
        vn[wid] = votes;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t best = 0, H = 0;
      for (int w = 0; w < kNw; ++w) {
        uint32_t sc = 0;
        for (int w2 = 0; w2 < kNw; ++w2) sc += vk[w2] == vk[w] ? vn[w2] : 0u;
        if (sc > best) {
          best = sc;
          H = vk[w];
        }
      }
      sH = H;
      sok = best >= kHotBlock / 4;
    }
    __syncthreads();
    if (!sok) continue;  // (uniform: every chunk of the partition skips it)
    const uint32_t H = sH;
    const uint32_t c0 = k * kHotChunk, m = min(kHotChunk, total - c0);
    uint2 v[kHotK];
#pragma unroll
    for (int u = 0; u < kHotK; ++u) v[u] = pairs[e0 + c0 + min(uint32_t(u) * kHotBlock + threadIdx.x, m - 1)];
    uint32_t mn = kInvalid, nh = 0, nn = 0;
#pragma unroll
    for (int u = 0; u < kHotK; ++u) {
      const bool valid = uint32_t(u) * kHotBlock + threadIdx.x < m, h = valid && v[u].x == H;
      mn = h ? min(mn, v[u].y) : mn;
      const uint64_t bh = __ballot(h), bv = __ballot(valid);
      nh += uint32_t(__popcll(bh));
      nn += uint32_t(__popcll(bv & ~bh));
    }
    mn = wave_min_u32(mn);
    if (lane == 0) {
      wh[wid] = nh;
      wn[wid] = nn;
      wm[wid] = mn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // the waves' exclusive prefixes, the workgroup's runs claimed
      uint32_t th = 0, tn = 0, tm = kInvalid;
      for (int w = 0; w < kNw; ++w) {
        const uint32_t x = wh[w], y = wn[w];
        wh[w] = th;
        wn[w] = tn;
        th += x;
        tn += y;
        tm = min(tm, wm[w]);
      }
      uint32_t* hw = tabs.hot + uint64_t(gp) * kHotW;
      hbase = th ? atomicAdd(&hw[2], th) : 0u;
      nbase = tn ? atomicAdd(&hw[4], tn) : 0u;
      if (th) atomicMin(&hw[3], tm);
      if (k == 0) {  // (the partition's other chunks agree on H)
        hw[1] = H;
        hw[0] = 1;
      }
    }
    __syncthreads();
    const uint32_t ti = tabs.nt > 1 && gp >= tabs.P ? 1u : 0u;
    uint32_t* __restrict__ sub = tabs.sub[ti];
    const uint32_t send = e0 - ps[ti * tabs.P] + total;  // one past the partition's last sub row
    uint32_t hc = hbase + wh[wid], nc = nbase + wn[wid];
#pragma unroll
    for (int u = 0; u < kHotK; ++u) {
      const bool valid = uint32_t(u) * kHotBlock + threadIdx.x < m, h = valid && v[u].x == H;
      const uint64_t bh = __ballot(h), bn = __ballot(valid) & ~bh;
      if (h) sub[send - 1 - (hc + uint32_t(__popcll(bh & lt)))] = v[u].y;
      else if (valid) tabs.hpairs[e0 + nc + uint32_t(__popcll(bn & lt))] = v[u];
      hc += uint32_t(__popcll(bh));
      nc += uint32_t(__popcll(bn));
    }
    __syncthreads();  // (the shared words of the next chunk)
  }
}

// off[b] += first main of b's partition; main records moved to their final slots.
// k_nagg_rebase / k_nagg_mains / k_nagg_counts run only when no partition gave up (`fail`: the
// sort build replaces the table then; the host checks the flag once, after the whole build).
__global__ __launch_bounds__(kBlock) void k_nagg_rebase(NaggTabs tabs, uint32_t nbl, FastDiv32 dw,
                                                        const uint32_t* __restrict__ mbase) {
  const uint32_t ti = blockIdx.y;  // one grid row per table
  if (reinterpret_cast<const uint32_t*>(tabs.counts[ti] + 3)[0]) return;  // fail flag
  uint32_t* __restrict__ off = tabs.off[ti];
  const uint32_t* mb = mbase + ti * tabs.P;
  const uint32_t m0 = mb[0];  // the table's first main record in the scan over every table
  for (uint32_t b = blockIdx.x * kBlock + threadIdx.x; b < nbl; b += gridDim.x * kBlock) off[b] += mb[dw.div(b)] - m0;
}

__global__ __launch_bounds__(kBlock) void k_nagg_mains(const uint4* __restrict__ mtmp, const uint32_t* __restrict__ ps,
                                                       const uint32_t* __restrict__ mbase, NaggTabs tabs, uint32_t nbl) {
  const uint32_t gp = blockIdx.x, ti = tabs.nt > 1 && gp >= tabs.P ? 1u : 0u;
  if (gp == 0 && threadIdx.x < tabs.nt) {  // every table's counts (entries, main records, off[nbl])
    const uint32_t tj = threadIdx.x;
    uint64_t* counts = tabs.counts[tj];
    uint64_t c0 = 0, c1 = 0;
    if (!reinterpret_cast<const uint32_t*>(counts + 3)[0]) {
      const uint32_t a = tj * tabs.P, b = (tj + 1) * tabs.P;
      c0 = ps[b] - ps[a];
      c1 = mbase[b] - mbase[a];
      counts[0] = c0;
      counts[1] = c1;
      tabs.off[tj][nbl] = uint32_t(c1);
    }
    // the host's copy, written here instead of by a device-to-host copy behind the build (words 2
    // and 3 were final when k_nagg ended); the host reads it after the build's event
    if (uint64_t* h = tabs.hc[tj]) {
      h[0] = c0;
      h[1] = c1;
      h[2] = counts[2];
      h[3] = counts[3];
    }
  }
  if (reinterpret_cast<const uint32_t*>(tabs.counts[ti] + 3)[0]) return;  // fail flag
  uint4* __restrict__ mains = tabs.main[ti];
  const uint32_t n = mbase[gp + 1] - mbase[gp], m0 = mbase[gp] - mbase[ti * tabs.P];
  for (uint32_t i = threadIdx.x; i < n; i += kBlock) mains[m0 + i] = mtmp[ps[gp] + i];
}

// The three launches above in one, for at most 2048 partitions (the one-level paths): workgroup gp
// takes its main-record base from the key counts of its table's partitions before it (a block sum
// over <= 2048 words read from L2, instead of a scan launch), adds it to its buckets' directory words,
// moves its main records to their final slots, and the first workgroup of each table writes the
// table's counts (and their host copy). Nothing for a table whose build gave up.
__global__ __launch_bounds__(kBlock) void k_nagg_fin(const uint4* __restrict__ mtmp, const uint32_t* __restrict__ ps,
                                                     const uint32_t* __restrict__ dcount, NaggTabs tabs, uint32_t nbl,
                                                     uint32_t W) {
  __shared__ uint64_t red[2][kBlock / kWave];
  const uint32_t gp = blockIdx.x, ti = tabs.nt > 1 && gp >= tabs.P ? 1u : 0u, p = gp - ti * tabs.P;
  const uint32_t t0 = ti * tabs.P;
  uint64_t* counts = tabs.counts[ti];
  const bool failed = reinterpret_cast<const uint32_t*>(counts + 3)[0] != 0;
  // keys of the table's partitions before gp, and of all of them
  uint64_t before = 0, all = 0;
  for (uint32_t k = t0 + threadIdx.x; k < t0 + tabs.P; k += kBlock) {
    const uint32_t c = dcount[k];
    before += k < gp ? c : 0u;
    all += c;
  }
  before = wave_sum(before);
  all = wave_sum(all);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = before;
    red[1][wid] = all;
  }
  __syncthreads();
  uint32_t base = 0;
  uint64_t tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    base += uint32_t(red[0][w]);
    tot += red[1][w];
  }
  if (p == 0 && threadIdx.x == 0) {
    uint64_t c0 = 0, c1 = 0;
    if (!failed) {
      c0 = ps[t0 + tabs.P] - ps[t0];
      c1 = tot;
      counts[0] = c0;
      counts[1] = c1;
      tabs.off[ti][nbl] = uint32_t(c1);
    }
    if (uint64_t* h = tabs.hc[ti]) {  // the host's copy (words 2 and 3 were final when k_nagg ended)
      h[0] = c0;
      h[1] = c1;
      h[2] = counts[2];
      h[3] = counts[3];
    }
  }
  if (failed) return;
  uint32_t* __restrict__ off = tabs.off[ti];
  const uint32_t b0 = p * W, nbs = min(W, nbl - b0);
  for (uint32_t k = threadIdx.x; k < nbs; k += kBlock) off[b0 + k] += base;
  uint4* __restrict__ mains = tabs.main[ti];
  const uint32_t n = dcount[gp], e0 = ps[gp];
  for (uint32_t i = threadIdx.x; i < n; i += kBlock) mains[base + i] = mtmp[e0 + i];
}

// pk_slices' region overflows -> the give-up flag (the sort build replaces the table); the packed
// partitioner's control words back to zero, the invariant of the probes that share them
__global__ void k_nagg_pk_ovf(uint64_t* __restrict__ ctl, uint64_t* __restrict__ counts, uint32_t* __restrict__ defer,
                              uint64_t* __restrict__ lbw) {
  if (threadIdx.x < 4) counts[threadIdx.x] = threadIdx.x == 3 && ctl[0] != 0 ? 1u : 0u;  // ctl[0]: the overflow count
  if (threadIdx.x == 4) defer[0] = 0;
  if (lbw && threadIdx.x >= 8 && threadIdx.x < 10) lbw[threadIdx.x - 8] = 0;  // the look-back's counters
  __syncthreads();
  if (threadIdx.x < 8) ctl[threadIdx.x] = 0;
}


}  // namespace

hipError_t nested_build_agg_many(hj3d_ctx* ctx, hj3d_table* const* tt, const hj3d_rel* rr, uint32_t nt, hipStream_t s,
                                 const char** path) {
  if (nt < 1 || nt > 2) return hipErrorNotSupported;
  hj3d_table* t = tt[0];
  const uint32_t nbl = t->nb_local;
  uint64_t n = 0;
  for (uint32_t k = 0; k < nt; ++k) {
    // every table of one launch has one geometry (the partitions of both follow one plan)
    if (tt[k]->nb_local != nbl || tt[k]->desc.bucket_lo != t->desc.bucket_lo ||
        tt[k]->desc.num_buckets != t->desc.num_buckets || tt[k]->desc.kind != HJ3D_NESTED)
      return hipErrorNotSupported;
    // small inputs and tables that one partition would cover (no free bucket for the LDS table's
    // empty marker) take the sort-based build
    if (rr[k].n < (ctx->radix_min >> 4) || rr[k].n == 0) return hipErrorNotSupported;
    n += rr[k].n;
  }
  if (ctx->force_direct || n >= (1ull << 31) || nbl <= 1024 || t->desc.num_buckets >= (1ull << 32))
    return hipErrorNotSupported;
  hipError_t e;
  for (uint32_t k = 0; k < nt; ++k) {
    if ((e = tt[k]->off.ensure((uint64_t(nbl) + 1) * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = tt[k]->main.ensure(rr[k].n * sizeof(uint4))) != hipSuccess) return e;
    if ((e = tt[k]->sub.ensure(rr[k].n * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = tt[k]->counts.ensure(4 * sizeof(uint64_t))) != hipSuccess) return e;
  }
  // (the counts words are zeroed by the first kernel after the partition: k_nagg_order / k_nagg_pk_ovf)
  // partition width: kAggW buckets, narrower when that would leave the chip with fewer than two
  // partitions per CU (config E: 2M buckets -> 512 partitions of 4K instead of 342 of 6K)
  // Then the count is rounded up to whole waves of workgroups (one k_nagg workgroup per CU at a
  // time, latency-bound, so a last wave of a few partitions costs as long as a full one): config C
  // 9.6M buckets -> 1792 partitions of 5357 (7 waves) instead of 1563 of 6144 (6.1 waves, run as 7).
  const uint32_t G = uint32_t(ctx->num_cus);
  uint32_t W = uint32_t((uint64_t(nbl) + kPartsPerCu * G - 1) / (kPartsPerCu * G));
  W = W < 1024 ? 1024 : W > kAggW ? kAggW : W;
  bool pk = false;  // more than 2048 partitions: the packed partitioner's slices (pk_slices)
  {
    const uint64_t P0 = (uint64_t(nbl) + W - 1) / W, P1 = (P0 + G - 1) / G * G;
    const uint64_t W1 = (uint64_t(nbl) + P1 - 1) / P1;
    if (P1 <= 2048 && W1 >= 1024) W = uint32_t(W1);
    if (P0 > 2048 || ctx->nested_pk) {
      pk = true;
      W = uint32_t(W1 >= 1024 ? W1 : W);
      // the slices take any partition count: kPkW buckets per partition,
      // narrow enough for the small form's two workgroups per CU and a small sub-row window
      // (at most 65536 slices: pk_slices' two levels of 1024 x 64)
      W = std::min<uint32_t>(W, std::max<uint32_t>(kPkW, (nbl + 65535) / 65536));
    }
  }
  const uint32_t P = (nbl + W - 1) / W;
  if (pk && nt > 1) return hipErrorNotSupported;  // one table at a time on the slices
  if (!pk && uint64_t(P) * nt > 2048u) return hipErrorNotSupported;  // k_nagg_order's limit
  const uint32_t PT = P * nt;  // partitions over every table
  if (path) *path = pk ? "nested_agg_slices" : "nested_agg";
  // scratch: pairs (n uint2; PK: the fine regions of pk_slices) | main records before compaction
  // (n uint4) | starts | key counts, order
  if (!pk && (e = ctx->scratch[kScrPairs].ensure(n * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrSortK].ensure(n * sizeof(uint4))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrSlot].ensure(((4 + kHotW) * uint64_t(PT) + 16) * sizeof(uint32_t))) != hipSuccess) return e;
  uint4* mtmp = ctx->scratch[kScrSortK].as<uint4>();
  uint32_t* dcount = ctx->scratch[kScrSlot].as<uint32_t>();  // PT + 1 (scanned in place into the main bases)
  uint32_t* order = dcount + PT + 1;
  uint32_t* defer = order + PT + 1;  // the register form's deferred partitions (count, PT indices)
  uint32_t* hinfo = defer + PT + 1;  // hot-key split: heavy partitions and their chunks (PT + 2)
  uint32_t* hotw = hinfo + PT + 2;   // hot-key split: kHotW words per partition
  if ((e = ctx->ensure_ctl()) != hipSuccess) return e;
  auto prime_at_least = [](uint32_t x) {
    for (;; ++x) {
      bool pr = x > 1;
      for (uint32_t d = 2; d * d <= x && pr; ++d) pr = x % d != 0;
      if (pr) return x;
    }
  };
  const uint32_t capr = prime_at_least(uint32_t(1.5 * W) + kRegBlock + 64);
  const bool reg = double(n) / PT <= kRegFill * kRegCap &&
                   capr <= kRegSlots * kRegBlock && reg_lds_words(capr, W) * 4 <= 160 * 1024;
  NaggTabs tabs;
  tabs.P = P;
  tabs.nt = nt;
  // the slice path's streaming aggregation finishes by decoupled look-back (no scan / rebase / mains)
  // (tried on the one-level paths too, when no partition is heavy: config E build 0.258-0.261 ->
  // 0.266 ms, `profiles/r06v_E_lookback_ab.jsonl`; k_nagg_fin kept there)
  uint64_t* lbw = nullptr;
  if (pk && !reg) {
    const size_t need = (uint64_t(PT) + 2) * sizeof(uint64_t);
    if (ctx->nagg_lb.bytes < need) {
      if ((e = ctx->nagg_lb.ensure(need)) != hipSuccess) return e;
      if ((e = hipMemsetAsync(ctx->nagg_lb.p, 0, ctx->nagg_lb.bytes, s)) != hipSuccess) return e;
    }
    lbw = ctx->nagg_lb.as<uint64_t>();
    tabs.lbw = lbw;
    tabs.lb_epoch = ++ctx->nagg_epoch;
    tabs.lb_skip0 = ctx->diag_lb ? 1u : 0u;
    if (ctx->diag_lb) tabs.lb_ticks = ctx->diag_lb;
  }
  tabs.sink = reinterpret_cast<uint32_t*>(ctx->ctl.as<uint64_t>() + 64);  // ctl words [64, 128): store sink
  tabs.defer = defer;
  // the hot-key election of the streaming form: in partitions above 5/4 of the mean only
  tabs.elect_min = uint32_t(std::min<uint64_t>(5 * n / (4 * uint64_t(PT)), 0xFFFFFFFFull));
  for (uint32_t k = 0; k < nt; ++k) {
    tabs.pbase[k] = k ? uint32_t(rr[0].n) : 0u;
    tabs.off[k] = tt[k]->off.as<uint32_t>();
    tabs.sub[k] = tt[k]->sub.as<uint32_t>();
    tabs.main[k] = tt[k]->main.as<uint4>();
    tabs.counts[k] = tt[k]->counts.as<uint64_t>();
    tabs.hc[k] = tt[k]->hc;  // (allocated by the caller: nested_host_counts)
  }
  const uint2* pairs = nullptr;
  const uint32_t* ps = nullptr;
  NaggSrc src;
  if (pk) {
    PkSlices sl;
    if ((e = pk_slices(ctx, t, rr[0], W, &sl, s)) != hipSuccess) return e;
    if (sl.P != P) return hipErrorNotSupported;
    src.fine = sl.fine;
    src.fcnt = sl.fcnt;
    src.S2 = sl.S2;
    src.cap2 = sl.cap2;
    src.pk = sl.pk;
    ps = sl.ps;
    // region overflows (skewed keys) -> the give-up flag; the control words back to zero
    hipLaunchKernelGGL(k_nagg_pk_ovf, dim3(1), dim3(64), 0, s, ctx->ctl.as<uint64_t>(), tabs.counts[0], tabs.defer,
                       lbw);
  } else {
    if ((e = ctx->scratch[kScrPStart].ensure((uint64_t(PT) + 2) * sizeof(uint32_t))) != hipSuccess) return e;
    uint32_t* pst = ctx->scratch[kScrPStart].as<uint32_t>();
    uint2* pw = ctx->scratch[kScrPairs].as<uint2>();
    // both tables' relations in one partition pass (two launches): table 1's partitions are P .. 2P-1
    uint32_t np = 0;
    if ((e = radix_partition_pairs(ctx, t, rr[0], W, pw, pst, &np, s, nt > 1 ? &rr[1] : nullptr)) != hipSuccess)
      return e;
    if (np != P) return hipErrorNotSupported;
    pairs = pw;
    ps = pst;
    // the hot-key split where the mean partition holds at least a chunk (heavier partitions then last
    // long enough to matter; config E's ~8 K pairs: no launch)
    const bool hs = double(n) / PT >= double(kHotChunk);
    if (hs) {  // the other pairs of heavy partitions, compacted (at most every pair)
      if ((e = ctx->scratch[kScrSortV].ensure(n * sizeof(uint2))) != hipSuccess) return e;
      tabs.hot = hotw;
      tabs.hpairs = ctx->scratch[kScrSortV].as<uint2>();
    }
    hipLaunchKernelGGL(k_nagg_order, dim3(1), dim3(1024), 0, s, ps, PT, order, tabs, hs ? hinfo : nullptr);
    if (hs) hipLaunchKernelGGL(k_nagg_hot, dim3(2 * G), dim3(kHotBlock), 0, s, pairs, ps, order, hinfo, tabs);
  }
  // table size: a prime >= 1.5 slots per bucket (about one key per bucket: NB = #dv / b) + the
  // insert slack; a partition with more keys retries its range in halves. Two 512-thread
  // workgroups per CU when the LDS fits twice (config E), else one 1024-thread one.
  static bool lds_attr = false;  // dynamic LDS above 64 KB
  if (!lds_attr) {
    for (const void* k : {reinterpret_cast<const void*>(&k_nagg_reg<true, 4>),
                          reinterpret_cast<const void*>(&k_nagg_reg<false, 4>),
                          reinterpret_cast<const void*>(&k_nagg_reg<true, 6>),
                          reinterpret_cast<const void*>(&k_nagg_reg<false, 6>),
                          reinterpret_cast<const void*>(&k_nagg<kSmallBlock, kSmallSlots, false>),
                          reinterpret_cast<const void*>(&k_nagg<kSmallBlock, kSmallSlots, true>),
                          reinterpret_cast<const void*>(&k_nagg<1024, 10, false>),
                          reinterpret_cast<const void*>(&k_nagg<1024, 10, true>),
                          reinterpret_cast<const void*>(&k_nagg_defer<kSmallBlock, kSmallSlots, false>),
                          reinterpret_cast<const void*>(&k_nagg_defer<kSmallBlock, kSmallSlots, true>),
                          reinterpret_cast<const void*>(&k_nagg_defer<1024, 10, false>),
                          reinterpret_cast<const void*>(&k_nagg_defer<1024, 10, true>)})
      if ((e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)) != hipSuccess) return e;
    lds_attr = true;
  }
  // the small form's table: ~1.5 slots per bucket, which leaves its pass-B image room for a config-D
  // slice's rows (15.4 K pairs; 2.5 slots per bucket left 11.6 K: D shape 17.7 -> 16.6 ms)
  const uint32_t cap512 = prime_at_least(std::max<uint32_t>(2048, uint32_t(kSmallCapF * W) + kSmallBlock + 64));
  const bool small = cap512 <= 6144 && agg_lds_words(cap512, W, kSmallBlock) * 4 <= kSmallLds;
  // the 1024-thread form's table (one workgroup per CU: the whole LDS, the image takes what the table leaves)
  // (a smaller table for a larger image measured slower at config C: 1.87 -> 1.90 ms at 1.2 slots per bucket)
  const uint32_t cap1024 = kAggCapMax;
  const uint32_t lo = uint32_t(t->desc.bucket_lo), nbg = uint32_t(t->desc.num_buckets);
  // the register form (k_nagg_reg) where the partitions' mean pair count fits its registers with room
  // (a larger partition takes k_nagg's streaming form inside it)
  if (reg) {
    const size_t lds = reg_lds_words(capr, W) * sizeof(uint32_t);
    const dim3 gr(std::min<uint32_t>(PT, G)), bl(kRegBlock);
    if (capr <= 4 * kRegBlock) {
      if (pk)
        hipLaunchKernelGGL((k_nagg_reg<true, 4>), gr, bl, lds, s, pairs, ps, t->fm, lo, nbl, nbg, W, PT, mtmp, dcount,
                           capr, src, tabs, nullptr);
      else
        hipLaunchKernelGGL((k_nagg_reg<false, 4>), gr, bl, lds, s, pairs, ps, t->fm, lo, nbl, nbg, W, PT, mtmp, dcount,
                           capr, src, tabs, order);
    } else {
      if (pk)
        hipLaunchKernelGGL((k_nagg_reg<true, 6>), gr, bl, lds, s, pairs, ps, t->fm, lo, nbl, nbg, W, PT, mtmp, dcount,
                           capr, src, tabs, nullptr);
      else
        hipLaunchKernelGGL((k_nagg_reg<false, 6>), gr, bl, lds, s, pairs, ps, t->fm, lo, nbl, nbg, W, PT, mtmp, dcount,
                           capr, src, tabs, order);
    }
    if (path) *path = pk ? "nested_agg_slices_reg" : "nested_agg_reg";
    // the partitions it left (usually none), in k_nagg's streaming form
    if (small) {
      tabs.ldsw = kSmallLds / 4;
      if (pk)
        hipLaunchKernelGGL((k_nagg_defer<kSmallBlock, kSmallSlots, true>), dim3(2 * G), dim3(kSmallBlock), kSmallLds, s,
                           pairs, ps, t->fm, lo, nbl, nbg, W, mtmp, dcount, cap512, src, tabs);
      else
        hipLaunchKernelGGL((k_nagg_defer<kSmallBlock, kSmallSlots, false>), dim3(2 * G), dim3(kSmallBlock), kSmallLds,
                           s, pairs, ps, t->fm, lo, nbl, nbg, W, mtmp, dcount, cap512, src, tabs);
    } else {
      tabs.ldsw = kBigLds / 4;
      if (pk)
        hipLaunchKernelGGL((k_nagg_defer<1024, 10, true>), dim3(G), dim3(1024), kBigLds, s, pairs, ps, t->fm, lo, nbl,
                           nbg, W, mtmp, dcount, cap1024, src, tabs);
      else
        hipLaunchKernelGGL((k_nagg_defer<1024, 10, false>), dim3(G), dim3(1024), kBigLds, s, pairs, ps, t->fm, lo, nbl,
                           nbg, W, mtmp, dcount, cap1024, src, tabs);
    }
  } else if (small) {
    tabs.ldsw = kSmallLds / 4;
    if (pk)
      hipLaunchKernelGGL((k_nagg<kSmallBlock, kSmallSlots, true>), dim3(PT), dim3(kSmallBlock), kSmallLds, s, pairs, ps,
                         t->fm, lo, nbl, nbg, W, mtmp, dcount, order, cap512, src, tabs);
    else
      hipLaunchKernelGGL((k_nagg<kSmallBlock, kSmallSlots, false>), dim3(PT), dim3(kSmallBlock), kSmallLds, s, pairs,
                         ps, t->fm, lo, nbl, nbg, W, mtmp, dcount, order, cap512, src, tabs);
  } else {
    tabs.ldsw = kBigLds / 4;
    if (pk)
      hipLaunchKernelGGL((k_nagg<1024, 10, true>), dim3(PT), dim3(1024), kBigLds, s, pairs, ps, t->fm, lo, nbl, nbg, W,
                         mtmp, dcount, order, cap1024, src, tabs);
    else
      hipLaunchKernelGGL((k_nagg<1024, 10, false>), dim3(PT), dim3(1024), kBigLds, s, pairs, ps, t->fm, lo, nbl, nbg, W,
                         mtmp, dcount, order, cap1024, src, tabs);
  }
  // no host wait here: if a partition gave up (fail, counts word 3), the kernels below do nothing
  // for its table and the caller, which reads the counts at the table's next use, runs the sort
  // build instead
  if (!pk) {  // (at most 2048 partitions)
    hipLaunchKernelGGL(k_nagg_fin, dim3(PT), dim3(kBlock), 0, s, mtmp, ps, dcount, tabs, nbl, W);
  } else if (!lbw) {
    if ((e = exclusive_scan_u32(ctx, dcount, dcount, PT, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_nagg_rebase, dim3(grid_for(ctx, nbl, kBlock), nt), dim3(kBlock), 0, s, tabs, nbl,
                       FastDiv32::make(W), dcount);
    hipLaunchKernelGGL(k_nagg_mains, dim3(PT), dim3(kBlock), 0, s, mtmp, ps, dcount, tabs, nbl);
  }
  for (uint32_t k = 0; k < nt; ++k) tt[k]->n_build = rr[k].n;
  return hipGetLastError();
}

hipError_t nested_build_agg(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s, const char** path) {
  return nested_build_agg_many(ctx, &t, &r, 1, s, path);
}

}  // namespace hj3d

// Diagnostic (builds with HJ3D_NAGG_CLK only; else HJ3D_EUNSUPPORTED): the last k_nagg launch's
// per-partition phase clocks, 8 words per partition (0 entry, 1 table cleared, 2 pass A done, 3 main
// records written, 4 pass B done, 5 exit: 100 MHz wall clock; 7 the workgroup's dispatch index).
extern "C" hj3d_status hj3d_diag_nagg_clk(uint64_t* host, uint32_t parts) {
#if HJ3D_NAGG_CLK
  if (!host || parts > hj3d::kClkParts) return HJ3D_EINVAL;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hj3d::g_nagg_clk), uint64_t(parts) * hj3d::kClkPts * sizeof(uint64_t)) ==
                 hipSuccess
             ? HJ3D_OK
             : HJ3D_EDEVICE;
#else
  (void)host;
  (void)parts;
  return HJ3D_EUNSUPPORTED;
#endif
}

// nested.hip — the nested ("3D") hash table (HtNested1, ht_nested.hh) on MI355X.
//
// Layout (replaces 32-B MainNodes + 16-B SubNodes chained by pointers):
//   off[b]   u32, b in [0, nb_local]: main records of bucket b are main[off[b] .. off[b+1])
//   main[m]  {u32 hash, u32 first_row, u32 sub_off, u32 sub_len}  one per distinct key (16 B)
//   sub[j]   u32 build rows, grouped per key: sub[sub_off .. sub_off+sub_len) (4 B / tuple)
// first_row is the key's first inserted tuple = MainNode::data() (ht_nested.hh:386-396).
// The reference keeps a bucket's main nodes in first-occurrence order (tail append,
// ht_nested.hh:299-308); the probe reproduces findMainNodeByOther's comparison count
// (ht_nested.hh:354-382) as 1 + #(mains of the bucket with a smaller first_row).
//
// Build: (hash,row) pairs -> stable radix sort by hash (sort.hip) -> run heads -> one main
// record per run (first row = segmented min) -> bucket CSR of the main records.
// Probe: as chaining, over main records. Unnest (AlgUnnestHt, algebra.hh:510-541): light
// matches (<= kInline rows) are expanded by the probing thread; heavy ones (Zipf hot keys)
// are queued and expanded by whole workgroups, so one hot key cannot serialize a thread.
#include "radix_seg.hpp"

namespace hj3d {
namespace {

constexpr int kItems = 4;
constexpr uint32_t kInline = 32;

__device__ __forceinline__ bool is_head(const uint32_t* hk, uint64_t e) { return e == 0 || hk[e] != hk[e - 1]; }

// (key, row) pairs in input order; counts[0] += owned tuples, counts[3] = max key (sort width)
__global__ __launch_bounds__(kBlock) void k_extract(RelView r, FastMod fm, uint32_t lo, uint32_t nbl,
                                                    uint32_t* __restrict__ hk, uint32_t* __restrict__ rv,
                                                    uint64_t* __restrict__ counts) {
  uint64_t owned = 0, mx = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < r.n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t k = r.key(i);
    hk[i] = k;
    rv[i] = r.row(i);
    owned += (fm.mod(murmur32(k)) - lo) < nbl;
    mx = k > mx ? k : mx;
  }
  uint64_t v[1] = {owned};
  block_flush<1, 0>(v, counts);  // counts[0] = stored tuples (HtStatistics::_numEntries)
  const uint64_t wm = wave_max(mx);
  if ((threadIdx.x & 63) == 0 && wm) atomicMax(reinterpret_cast<unsigned long long*>(counts + 3), wm);
}

__global__ __launch_bounds__(kBlock) void k_heads(const uint32_t* __restrict__ hk, uint64_t n, uint32_t* __restrict__ x) {
  for (uint64_t e = uint64_t(blockIdx.x) * kBlock + threadIdx.x; e < n; e += uint64_t(gridDim.x) * kBlock)
    x[e] = is_head(hk, e) ? 1u : 0u;
}

// One main record per run of equal keys: hash, run start and (rows ascending within the run,
// i.e. implicit row ids and a stable sort) first_row; else first_row is left to k_run_min.
__global__ __launch_bounds__(kBlock) void k_runs(const uint32_t* __restrict__ hk, uint64_t n,
                                                 const uint32_t* __restrict__ x, const uint32_t* __restrict__ rows,
                                                 bool rows_sorted, uint32_t* __restrict__ mh,
                                                 uint32_t* __restrict__ msub, uint32_t* __restrict__ mfirst) {
  for (uint64_t e = uint64_t(blockIdx.x) * kBlock + threadIdx.x; e < n; e += uint64_t(gridDim.x) * kBlock) {
    if (!is_head(hk, e)) continue;
    const uint32_t m = x[e];
    mh[m] = murmur32(hk[e]);
    msub[m] = uint32_t(e);
    mfirst[m] = rows_sorted ? rows[e] : kInvalid;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) msub[x[n]] = uint32_t(n);
}

// first_row of every run = min row id in the run (segmented wave min + one atomicMin per
// wave-segment; a hot key's long run costs one atomic per wave, not per tuple).
__global__ __launch_bounds__(kBlock) void k_run_min(const uint32_t* __restrict__ hk, const uint32_t* __restrict__ rv,
                                                    uint64_t n, const uint32_t* __restrict__ x,
                                                    uint32_t* __restrict__ mfirst) {
  const int lane = threadIdx.x & 63;
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t base = uint64_t(blockIdx.x) * kBlock; base < n; base += stride) {
    const uint64_t e = base + threadIdx.x;
    const bool valid = e < n;
    const uint32_t m = valid ? (is_head(hk, e) ? x[e] : x[e] - 1u) : kInvalid;
    uint32_t v = valid ? rv[e] : kInvalid;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_down(v, o, kWave);
      const uint32_t my = __shfl_down(m, o, kWave);
      if (lane + o < 64 && my == m) v = min(v, y);
    }
    const uint32_t mp = __shfl_up(m, 1, kWave);
    if (valid && (lane == 0 || mp != m)) atomicMin(&mfirst[m], v);
  }
}

__global__ __launch_bounds__(kBlock) void k_main_count(const uint32_t* __restrict__ mh, const uint32_t* __restrict__ x,
                                                       uint64_t n, FastMod fm, uint32_t lo, uint32_t nbl,
                                                       uint32_t* __restrict__ off, uint32_t* __restrict__ mslot) {
  const uint32_t d = x[n];
  for (uint64_t m = uint64_t(blockIdx.x) * kBlock + threadIdx.x; m < d; m += uint64_t(gridDim.x) * kBlock) {
    const uint32_t b = fm.mod(mh[m]) - lo;
    mslot[m] = b < nbl ? atomicAdd(&off[b], 1u) : kInvalid;
  }
}

__global__ __launch_bounds__(kBlock) void k_main_scatter(const uint32_t* __restrict__ mh,
                                                         const uint32_t* __restrict__ mfirst,
                                                         const uint32_t* __restrict__ msub,
                                                         const uint32_t* __restrict__ mslot,
                                                         const uint32_t* __restrict__ x, uint64_t n, FastMod fm,
                                                         uint32_t lo, const uint32_t* __restrict__ off,
                                                         uint4* __restrict__ mains, uint64_t* __restrict__ counts) {
  const uint32_t d = x[n];
  uint64_t nd = 0, mx = 0;
  for (uint64_t m = uint64_t(blockIdx.x) * kBlock + threadIdx.x; m < d; m += uint64_t(gridDim.x) * kBlock) {
    const uint32_t sl = mslot[m];
    if (sl == kInvalid) continue;
    const uint32_t b = fm.mod(mh[m]) - lo;
    const uint32_t len = msub[m + 1] - msub[m];
    mains[off[b] + sl] = make_uint4(mh[m], mfirst[m], msub[m], len);
    ++nd;
    mx = len > mx ? len : mx;
  }
  uint64_t v[1] = {nd};
  block_flush<1, 0>(v, counts + 1);  // distinct keys
  const uint64_t wm = wave_max(mx);
  if ((threadIdx.x & 63) == 0 && wm) atomicMax(reinterpret_cast<unsigned long long*>(counts + 2), wm);
}

enum NMode { kAggNU = 0, kDenseNU = 1, kAggUN = 2, kCountUN = 3 };

struct Heavy {
  uint32_t probe_row;
  uint32_t main_idx;
};

// Probe strand over the nested table. kAggNU / kDenseNU: AlgNestJoinProbe -> AlgTop (nested
// tuples). kAggUN: AlgNestJoinProbe -> AlgUnnestHt -> AlgTop. kCountUN: like kAggUN but
// records per probe tuple its output count (cnt) and matched main (mid) for a scan + expand.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_nested_probe(RelView r, FastMod fm, uint32_t lo, uint32_t nbl,
                                                         const uint32_t* __restrict__ off,
                                                         const uint4* __restrict__ mains,
                                                         const uint32_t* __restrict__ sub,
                                                         uint2* __restrict__ out, uint64_t out_cap,
                                                         uint64_t* __restrict__ cnt, uint32_t* __restrict__ mid,
                                                         Heavy* __restrict__ heavy, uint64_t* __restrict__ nheavy,
                                                         uint64_t* __restrict__ res) {
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t stride = uint64_t(gridDim.x) * kBlock * kItems;
  for (uint64_t base = uint64_t(blockIdx.x) * kBlock * kItems; base < r.n; base += stride) {
    uint32_t h[kItems], b[kItems], pr[kItems], s[kItems], e[kItems];
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
      const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
      const bool v = i < r.n;
      h[j] = murmur32(v ? r.key(i) : 0u);
      pr[j] = v ? r.row(i) : 0u;
      b[j] = v ? fm.mod(h[j]) - lo : kInvalid;
    }
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
      s[j] = 0;
      e[j] = 0;
      if (b[j] < nbl) {
        s[j] = off[b[j]];
        e[j] = off[b[j] + 1];
      }
    }
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
      const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
      if (i >= r.n) continue;
      acc[0] += 1;
      uint32_t found = kInvalid;
      uint4 M = make_uint4(0, 0, 0, 0);
      for (uint32_t k = s[j]; k < e[j]; ++k) {
        const uint4 c = mains[k];
        if (c.x == h[j]) {
          found = k;
          M = c;
          break;
        }
      }
      if (found == kInvalid) {
        acc[3] += e[j] - s[j];
      } else {
        uint32_t before = 0;  // mains of this bucket inserted before the matching one
        for (uint32_t k = s[j]; k < e[j]; ++k) before += mains[k].y < M.y;
        acc[3] += 1 + before;
        acc[1] += 1;
      }
      if (MODE == kAggNU || MODE == kDenseNU) {
        if (found != kInvalid) {
          acc[2] += 1;
          acc[4] += pr[j];
          acc[5] += M.y;
          const uint64_t ph = pair_hash(pr[j], M.y);
          acc[7] += ph;
          acc[8] ^= ph;
        }
        if (MODE == kDenseNU && i < out_cap) out[i] = make_uint2(pr[j], found == kInvalid ? kInvalid : M.y);
      } else if (MODE == kAggUN) {
        if (found != kInvalid) {
          acc[2] += M.w;
          if (M.w <= kInline) {
            for (uint32_t q = 0; q < M.w; ++q) {
              const uint32_t br = sub[M.z + q];
              acc[4] += pr[j];
              acc[5] += br;
              const uint64_t ph = pair_hash(pr[j], br);
              acc[7] += ph;
              acc[8] ^= ph;
            }
          } else {
            const uint64_t slot = atomicAdd(reinterpret_cast<unsigned long long*>(nheavy), 1ull);
            heavy[slot] = Heavy{pr[j], found};
          }
        }
      } else {  // kCountUN
        acc[2] += found != kInvalid ? M.w : 0u;
        cnt[i] = found != kInvalid ? M.w : 0u;
        mid[i] = found;
      }
    }
  }
  block_flush<kProbeFields, 1>(acc, res);
}

// Heavy matches (> kInline rows): every workgroup takes a share of every queued (probe row,
// main) pair, so one Zipf hot key is expanded by the whole chip, not by one workgroup.
__global__ __launch_bounds__(kBlock) void k_expand_heavy(const Heavy* __restrict__ heavy,
                                                         const uint64_t* __restrict__ nheavy,
                                                         const uint4* __restrict__ mains,
                                                         const uint32_t* __restrict__ sub, uint64_t* __restrict__ res) {
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t nh = *nheavy;
  for (uint64_t q = 0; q < nh; ++q) {
    const Heavy hv = heavy[q];
    const uint4 M = mains[hv.main_idx];
    for (uint32_t k = blockIdx.x * kBlock + threadIdx.x; k < M.w; k += gridDim.x * kBlock) {
      const uint32_t br = sub[M.z + k];
      acc[4] += hv.probe_row;
      acc[5] += br;
      const uint64_t ph = pair_hash(hv.probe_row, br);
      acc[7] += ph;
      acc[8] ^= ph;
    }
  }
  block_flush<kProbeFields, 1>(acc, res);
}

// Materialised unnest. Output slots of probe slot i are [ooff[i], ooff[i+1]) (exclusive scan of
// the per-slot output counts). A slot is a probe tuple (direct probe: its main mid[i], its row
// r.row(i)) or a partitioned pair (radix probe: sub_off zo[i] and probe row po[i] written by the
// probe, so the expansion reads no main record). One workgroup per 256 consecutive slots: their
// light outputs (<= kHeavyOut per slot) are enumerated p = 0..L-1 by consecutive threads, each
// finding its slot by a binary search over the 256 local offsets in LDS, so the stores of a
// workgroup form one (nearly) contiguous, coalesced range. Heavier slots are queued and written
// by k_expand_heavy_flat with all workgroups.
constexpr uint32_t kHeavyOut = 8192;
// Fixed by measurement: k_expand_light takes four outputs per thread and
// step (one: 0.829 against 0.813 ms at config C; eight: 0.805 against 0.794) and its slot blocks
// XCD-ordered (config D Nrs probe 6.14 -> 5.64 ms); a nested probe on slices wider than LDS shares
// each slice among kHbmSplits XCD-ordered workgroups (8 / 16 / 32: 8.43 / 8.24 / 9.12 ms at D); more
// than 2048 LDS slices go through the packed two-level partition; the materialised unnest stores a
// fixed count per chunk (0.813 -> 0.791 ms at C).
constexpr int kExpU = 4;
constexpr uint32_t kHbmSplits = 16;  // one region stream per wave at G = 256
static_assert(kBlock == 256, "k_expand_light's binary search covers 256 slots in 8 steps");

struct SlotSrc {
  RelView r;                   // direct: probe relation (row of slot i = r.row(i))
  const uint32_t* mid;         // direct: matched main of slot i
  const uint4* mains;
  const uint32_t* zo;          // radix: sub_off of slot i
  const uint32_t* po;          // radix: probe row of slot i
  template <bool SLOTS>
  __device__ __forceinline__ void get(uint64_t i, uint32_t& z, uint32_t& pr) const {
    if (SLOTS) {
      z = zo[i];
      pr = po[i];
    } else {
      z = mains[mid[i]].z;
      pr = r.row(i);
    }
  }
};

template <bool SLOTS, bool CK>
__global__ __launch_bounds__(kBlock) void k_expand_light(SlotSrc src, uint64_t nslots, const uint64_t* __restrict__ ooff,
                                                         const uint32_t* __restrict__ sub, uint2* __restrict__ out,
                                                         uint64_t out_cap, uint32_t* __restrict__ heavy,
                                                         uint32_t* __restrict__ nheavy, uint64_t* __restrict__ partials,
                                                         uint2* __restrict__ sink) {
  __shared__ uint32_t loff[kBlock + 1];
  __shared__ uint32_t lz[kBlock];
  __shared__ uint32_t lpr[kBlock];
  __shared__ uint64_t lpos[kBlock];
  __shared__ uint32_t wsum[kBlock / kWave];
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  // XCD-ordered blocks: workgroup b runs on XCD b % 8, so consecutive slot blocks
  // (probe tuples of one slice: their keys' sub rows lie in one window of `sub`) would read that
  // window into eight L2s; XCD x takes the x-th eighth of the blocks instead
  uint32_t bid = blockIdx.x;
  {
    const uint32_t per = gridDim.x / 8;
    if (bid < per * 8) bid = (bid % 8) * per + bid / 8;
  }
  const uint64_t i = uint64_t(bid) * kBlock + threadIdx.x;
  uint32_t c = 0, z = 0, pr = 0;
  uint64_t pos = 0;
  if (i < nslots) {
    pos = ooff[i];
    const uint64_t cc = ooff[i + 1] - pos;
    if (cc) {
      src.get<SLOTS>(i, z, pr);
      if (cc > kHeavyOut) heavy[atomicAdd(nheavy, 1u)] = uint32_t(i);
      else c = uint32_t(cc);
    }
  }
  // block exclusive scan of the light counts
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t wt;
  const uint32_t wx = wave_excl_scan(c, &wt);
  if (lane == 63) wsum[wid] = wx + c;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    const uint32_t v = wsum[w];
    if (w < wid) pre += v;
    tot += v;
  }
  loff[threadIdx.x] = pre + wx;
  if (threadIdx.x == 0) loff[kBlock] = tot;
  lz[threadIdx.x] = z;
  lpr[threadIdx.x] = pr;
  lpos[threadIdx.x] = pos;
  __syncthreads();
  // kExpU outputs per thread and step: their binary searches interleave and their sub-row loads are
  // all in flight before the first is used (one output per step waited for each load in turn).
  // Indices past the end are clamped to the last output (a fixed load count per step), and only
  // valid outputs are stored.
  for (uint32_t p0 = threadIdx.x; p0 < tot; p0 += kExpU * kBlock) {
    uint32_t lo[kExpU], q[kExpU], br[kExpU];
    bool ok[kExpU];
#pragma unroll
    for (int u = 0; u < kExpU; ++u) {
      const uint32_t p = p0 + u * kBlock;
      ok[u] = p < tot;
      lo[u] = 0;
    }
#pragma unroll
    for (int step = 0; step < 8; ++step) {  // largest t with loff[t] <= p (slots with c = 0 skipped)
#pragma unroll
      for (int u = 0; u < kExpU; ++u) {
        const uint32_t p = min(p0 + u * kBlock, tot - 1);
        const uint32_t md = lo[u] + (128u >> step);
        if (loff[md] <= p) lo[u] = md;
      }
    }
#pragma unroll
    for (int u = 0; u < kExpU; ++u) {
      const uint32_t p = min(p0 + u * kBlock, tot - 1);
      q[u] = p - loff[lo[u]];
      br[u] = sub[lz[lo[u]] + q[u]];
    }
#pragma unroll
    for (int u = 0; u < kExpU; ++u) {
      // one store per output slot of the step, straight-line (an invalid one goes to the sink):
      // a store under a branch drew its load into the branch, right before the store
      const uint32_t prow = lpr[lo[u]];
      const uint64_t o = lpos[lo[u]] + q[u];
      uint2* dst = ok[u] && o < out_cap ? out + o : sink;
      __builtin_nontemporal_store((uint64_t(br[u]) << 32) | prow, reinterpret_cast<uint64_t*>(dst));
      if (CK && ok[u]) {
        acc[4] += prow;
        acc[5] += br[u];
        const uint64_t ph = pair_hash(prow, br[u]);
        acc[7] += ph;
        acc[8] ^= ph;
      }
    }
  }
  // the output checksums only (the counts are the probe's): no partials without HJ3D_PROBE_CHECKSUM
  if (CK) block_store<kProbeFields, 1>(acc, partials + uint64_t(bid) * kProbeFields);
}

// hoff[q] = first flattened output of heavy slot q (exclusive scan of their counts, one workgroup;
// there are at most total outputs / kHeavyOut heavy slots).
__global__ __launch_bounds__(1024) void k_heavy_offsets(const uint32_t* __restrict__ heavy,
                                                        const uint32_t* __restrict__ nheavy,
                                                        const uint64_t* __restrict__ ooff, uint64_t* __restrict__ hoff) {
  __shared__ uint64_t wsum[1024 / kWave];
  __shared__ uint64_t carry_s;
  const uint32_t nh = *nheavy;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint32_t base = 0; base < nh; base += 1024) {
    const uint32_t q = base + threadIdx.x;
    uint64_t v = 0;
    if (q < nh) {
      const uint32_t i = heavy[q];
      v = ooff[i + 1] - ooff[i];
    }
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, kWave);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint64_t wpre = 0, tot = 0;
    for (int w = 0; w < 1024 / kWave; ++w) {
      const uint64_t t = wsum[w];
      if (w < wid) wpre += t;
      tot += t;
    }
    const uint64_t carry = carry_s;
    if (q < nh) hoff[q] = carry + wpre + x - v;
    __syncthreads();
    if (threadIdx.x == 0) carry_s = carry + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) hoff[nh] = carry_s;
}

// Heavy outputs flattened over all queued slots: wave w writes the kHeavySpan consecutive
// flattened outputs [w * kHeavySpan, ...), lane l every 64th of them, so stores and sub reads are
// coalesced and a lane binary-searches hoff only once (a heavy slot spans >= kHeavyOut outputs).
constexpr uint32_t kHeavySpan = 64 * 16;

template <bool SLOTS, bool CK>
__global__ __launch_bounds__(kBlock) void k_expand_heavy_flat(SlotSrc src, const uint64_t* __restrict__ ooff,
                                                              const uint32_t* __restrict__ sub,
                                                              const uint32_t* __restrict__ heavy,
                                                              const uint32_t* __restrict__ nheavy,
                                                              const uint64_t* __restrict__ hoff, uint2* __restrict__ out,
                                                              uint64_t out_cap, uint64_t* __restrict__ res) {
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t nh = *nheavy;
  const uint64_t total = hoff[nh];
  const int lane = threadIdx.x & 63;
  const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
  for (uint64_t w = (uint64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave; w * kHeavySpan < total; w += nwaves) {
    const uint64_t f0 = w * kHeavySpan + lane;
    if (f0 >= total) continue;
    uint32_t lo = 0, hi = nh;  // largest q with hoff[q] <= f0
    while (hi - lo > 1) {
      const uint32_t md = (lo + hi) >> 1;
      if (hoff[md] <= f0) lo = md; else hi = md;
    }
    uint32_t q = lo;
    uint64_t qb = hoff[q], qe = hoff[q + 1];
    uint32_t i = heavy[q], z, pr;
    src.get<SLOTS>(i, z, pr);
    uint64_t ob = ooff[i];
    for (uint64_t f = f0; f < total && f < (w + 1) * kHeavySpan; f += kWave) {
      while (f >= qe) {  // next heavy slot
        ++q;
        qb = qe;
        qe = hoff[q + 1];
        i = heavy[q];
        src.get<SLOTS>(i, z, pr);
        ob = ooff[i];
      }
      const uint64_t k = f - qb;
      const uint32_t br = sub[z + k];
      if (ob + k < out_cap)
        __builtin_nontemporal_store((uint64_t(br) << 32) | pr, reinterpret_cast<uint64_t*>(out + ob + k));
      if (CK) {
        acc[4] += pr;
        acc[5] += br;
        const uint64_t ph = pair_hash(pr, br);
        acc[7] += ph;
        acc[8] ^= ph;
      }
    }
  }
  if (CK) block_flush<kProbeFields, 1>(acc, res);
}

// ---- partitioned probe (radix_seg.hpp): the probe side is partitioned by bucket range and
// each partition's slice of the directory and main records is staged in LDS ----

// Probe of one tuple (hash h, row pr) against main records M[s .. s+n) of its bucket; mg0 =
// global index of M[0] (the slice start in LDS, 0 in HBM). Same counters as k_nested_probe.
template <int MODE, typename MT>
__device__ __forceinline__ void nested_bucket(uint32_t h, uint32_t pr, const MT* M, uint32_t s, uint32_t n,
                                              uint32_t mg0, uint64_t (&acc)[kProbeFields], uint64_t i,
                                              uint2* __restrict__ out, uint64_t out_cap, uint64_t* __restrict__ cnt,
                                              uint32_t* __restrict__ zo, uint32_t* __restrict__ po,
                                              const uint32_t* __restrict__ sub, Heavy* __restrict__ heavy,
                                              uint64_t* __restrict__ nheavy) {
  acc[0] += 1;
  uint32_t found = kInvalid;
  uint4 F = make_uint4(0, 0, 0, 0);
  for (uint32_t k = s; k < s + n; ++k) {
    const uint4 c = M[k];
    if (c.x == h) {
      found = k;
      F = c;
      break;
    }
  }
  if (found == kInvalid) {
    acc[3] += n;
  } else {
    uint32_t before = 0;  // mains of this bucket inserted before the matching one
    for (uint32_t k = s; k < s + n; ++k) before += M[k].y < F.y;
    acc[3] += 1 + before;
    acc[1] += 1;
  }
  if (MODE == kAggNU || MODE == kDenseNU) {
    if (found != kInvalid) {
      acc[2] += 1;
      acc[4] += pr;
      acc[5] += F.y;
      const uint64_t ph = pair_hash(pr, F.y);
      acc[7] += ph;
      acc[8] ^= ph;
    }
    if (MODE == kDenseNU && i < out_cap) out[i] = make_uint2(pr, found == kInvalid ? kInvalid : F.y);
  } else if (MODE == kAggUN) {
    if (found != kInvalid) {
      acc[2] += F.w;
      if (F.w <= kInline) {
        for (uint32_t q = 0; q < F.w; ++q) {
          const uint32_t br = sub[F.z + q];
          acc[4] += pr;
          acc[5] += br;
          const uint64_t ph = pair_hash(pr, br);
          acc[7] += ph;
          acc[8] ^= ph;
        }
      } else {
        const uint64_t slot = atomicAdd(reinterpret_cast<unsigned long long*>(nheavy), 1ull);
        heavy[slot] = Heavy{pr, mg0 + found};
      }
    }
  } else {  // kCountUN: the slot's output count, sub_off and probe row for the expansion
    acc[2] += found != kInvalid ? F.w : 0u;
    cnt[i] = found != kInvalid ? F.w : 0u;
    if (found != kInvalid) {
      zo[i] = F.z;
      po[i] = pr;
    }
  }
}

// The probe's small fills in one launch (they were three runtime fills / copies, and the count slots'
// fill wrote all |probe| + 1 words: 0.8 GB, 106 us at config D): the partials' atomic row, base0 =
// *src (n_probe before this call), and in the materialised unnest the count slots past the used
// ones (seg_tot region slots + *novf overflow slots; every used slot is written by the probe kernels).
__global__ __launch_bounds__(kBlock) void k_rn_prep(uint64_t* __restrict__ prow, uint64_t* __restrict__ base0,
                                                    const uint64_t* __restrict__ src, uint64_t* __restrict__ cnt,
                                                    const uint32_t* __restrict__ seg_tot,
                                                    const unsigned long long* __restrict__ novf, uint64_t n,
                                                    uint32_t* __restrict__ zero32) {
  if (blockIdx.x == 0) {
    if (threadIdx.x < kProbeFields) prow[threadIdx.x] = 0;
    if (threadIdx.x == 0) *base0 = *src;
    if (threadIdx.x == 64 && zero32) *zero32 = 0;  // the expansion's heavy-slot counter
  }
  if (!cnt) return;
  const uint64_t start = uint64_t(*seg_tot) + *novf;
  for (uint64_t i = start + uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock)
    cnt[i] = 0;
}

// PKD: the regions hold packed pairs {v, row} of pk_probe_slices (bucket in the slice v >> qbits, hash
// pk.hash_of(v, p): no modulo per pair), else {hash, row}.
template <int MODE, bool FITS, bool PKD>
__global__ __launch_bounds__(kJBlock) void k_rn_probe_seg(const uint2* __restrict__ region,
                                                          const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ seg, uint32_t G, uint32_t cap,
                                                          const uint32_t* __restrict__ off,
                                                          const uint4* __restrict__ mains,
                                                          const uint32_t* __restrict__ sub, FastMod fm, uint32_t lo,
                                                          uint32_t nbl, uint32_t W, uint32_t P, uint32_t splits,
                                                          bool flat, uint2* __restrict__ out, uint64_t out_cap,
                                                          uint64_t* __restrict__ cnt, uint32_t* __restrict__ zo,
                                                          uint32_t* __restrict__ po, Heavy* __restrict__ heavy,
                                                          uint64_t* __restrict__ nheavy, uint64_t* __restrict__ partials,
                                                          uint64_t* __restrict__ sink, bool xcd, PkGeom pk) {
  __shared__ uint32_t lds[kProbeLdsWords];
  // xcd: workgroup b runs on XCD b % 8; XCD x takes the x-th eighth of the (slice, share) pairs
  uint32_t bid = blockIdx.x;
  if (xcd) {
    const uint32_t per = gridDim.x / 8;
    if (bid < per * 8) bid = (bid % 8) * per + bid / 8;
  }
  const uint32_t p = bid / splits, sp = bid % splits;
  const uint32_t b0 = p * W;
  const uint32_t nbs = min(W, nbl - b0);
  const uint32_t m0 = off[b0], nm = off[b0 + nbs] - m0;
  const uint32_t dirw = (nbs + 4) & ~3u;  // main records 16-B aligned after the directory
  const bool fits = dirw + 4ull * nm <= kProbeLdsWords;
  if (fits != FITS) {  // the other kernel takes this partition; keep this block's partial row zero
    if (FITS && threadIdx.x < kProbeFields) partials[uint64_t(blockIdx.x) * kProbeFields + threadIdx.x] = 0;
    return;
  }
  uint32_t* ldir = lds;
  uint4* lmain = reinterpret_cast<uint4*>(lds + dirw);
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (MODE == kCountUN && FITS) {
    // materialised unnest: every item of a chunk writes its three slot words, in straight-line
    // code (absent items to the sink), so the chunk's store count is fixed and the wait for the
    // next chunk's pairs (loaded before these stores) leaves the stores in flight
    uint32_t* zsink = reinterpret_cast<uint32_t*>(sink + 1);
    seg_walk<true>(region, counts, seg, G, cap, P, p, splits, sp, flat,
                   [&] { stage_nested(off, mains, b0, nbs, m0, nm, ldir, lmain); },
                   [&](const uint64_t (&v)[kSegItems], const uint64_t (&sl)[kSegItems], uint32_t vm) {
#pragma unroll
                     for (int j = 0; j < kSegItems; ++j) {
                       const bool valid = (vm >> j) & 1u;
                       const uint32_t w0 = uint32_t(v[j]), row = uint32_t(v[j] >> 32);
                       const uint32_t hv = PKD ? pk.hash_of(w0, p) : w0;
                       const uint32_t bl = PKD ? w0 >> pk.qbits : fm.mod(hv) - lo - b0;
                       const uint32_t d = valid ? ldir[bl] : 0u;
                       const uint32_t s0 = d >> 16, n = d & 0xFFFFu;
                       uint32_t found = kInvalid;
                       uint4 F = make_uint4(0, 0, 0, 0);
                       for (uint32_t k = s0; k < s0 + n; ++k) {
                         const uint4 c = lmain[k];
                         if (c.x == hv) {
                           found = k;
                           F = c;
                           break;
                         }
                       }
                       uint32_t before = 0;  // mains of this bucket inserted before the matching one
                       if (found != kInvalid)
                         for (uint32_t k = s0; k < s0 + n; ++k) before += lmain[k].y < F.y;
                       if (valid) {
                         acc[0] += 1;
                         acc[1] += found != kInvalid;
                         acc[2] += found != kInvalid ? F.w : 0u;
                         acc[3] += found != kInvalid ? 1 + before : n;
                       }
                       const uint64_t i = sl[j];
                       uint64_t* cd = valid ? cnt + i : sink;
                       uint32_t* zd = valid ? zo + i : zsink;
                       uint32_t* pd = valid ? po + i : zsink + 1;
                       *cd = found != kInvalid ? F.w : 0u;
                       *zd = F.z;
                       *pd = row;
                     }
                   });
    block_store<kProbeFields, 1>(acc, partials + uint64_t(blockIdx.x) * kProbeFields);
    return;
  }
  seg_walk(region, counts, seg, G, cap, P, p, splits, sp, flat,
           [&] { if (FITS) stage_nested(off, mains, b0, nbs, m0, nm, ldir, lmain); },
           [&](uint32_t w0, uint32_t row, uint64_t i) {
             const uint32_t hv = PKD ? pk.hash_of(w0, p) : w0;
             const uint32_t bl = PKD ? w0 >> pk.qbits : fm.mod(hv) - lo - b0;
             if (FITS) {
               const uint32_t d = ldir[bl];
               nested_bucket<MODE>(hv, row, lmain, d >> 16, d & 0xFFFFu, m0, acc, i, out, out_cap, cnt, zo, po, sub,
                                   heavy, nheavy);
             } else {
               const uint32_t s = off[b0 + bl];
               nested_bucket<MODE>(hv, row, mains, s, off[b0 + bl + 1] - s, 0u, acc, i, out, out_cap, cnt, zo, po,
                                   sub, heavy, nheavy);
             }
           });
  if (FITS) block_store<kProbeFields, 1>(acc, partials + uint64_t(blockIdx.x) * kProbeFields);
  else block_flush<kProbeFields, 1>(acc, partials + uint64_t(gridDim.x) * kProbeFields);  // extra row (atomics)
}

// Overflow pairs (runs that did not fit their region), probed against the table in HBM; their
// slots follow the regions' (base = seg[P * G]).
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_rn_probe_ovf(const uint2* __restrict__ ovf,
                                                         const unsigned long long* __restrict__ novf,
                                                         const uint32_t* __restrict__ base_slot,
                                                         const uint32_t* __restrict__ off, const uint4* __restrict__ mains,
                                                         const uint32_t* __restrict__ sub, FastMod fm, uint32_t lo,
                                                         uint2* __restrict__ out, uint64_t out_cap,
                                                         uint64_t* __restrict__ cnt, uint32_t* __restrict__ zo,
                                                         uint32_t* __restrict__ po, Heavy* __restrict__ heavy,
                                                         uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res) {
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t n = *novf, b = *base_slot;
  for (uint64_t j = uint64_t(blockIdx.x) * kBlock + threadIdx.x; j < n; j += uint64_t(gridDim.x) * kBlock) {
    const uint2 e = ovf[j];
    const uint32_t bl = fm.mod(e.x) - lo;
    const uint32_t s = off[bl];
    nested_bucket<MODE>(e.x, e.y, mains, s, off[bl + 1] - s, 0u, acc, b + j, out, out_cap, cnt, zo, po, sub, heavy,
                        nheavy);
  }
  block_flush<kProbeFields, 1>(acc, res);
}

}  // namespace

namespace {

// Light expansion (one workgroup per 256 slots, partials per workgroup) then the heavy slots
// flattened over the chip (hoff in kScrD).
// ck: fold the output checksums (HJ3D_PROBE_CHECKSUM; the light kernel's per-workgroup partials
// are then reduced by the caller), otherwise the expansion only writes the pairs.
hipError_t expand(hj3d_ctx* ctx, const SlotSrc& src, bool slots, bool ck, uint64_t nslots, const uint64_t* ooff,
                  const uint32_t* sub, uint2* out, uint64_t out_cap, uint32_t* heavy, uint32_t* nheavy,
                  uint64_t* partials, uint64_t* res, hipStream_t s) {
  const uint32_t nblk = uint32_t((nslots + kBlock - 1) / kBlock);
  uint64_t* hoff = ctx->scratch[kScrD].as<uint64_t>();
  if (hipError_t e = ctx->ensure_ctl(); e != hipSuccess) return e;  // ctl words [64, 128): store sink
  auto launch = [&](auto slots_c, auto ck_c) {
    constexpr bool SL = decltype(slots_c)::value, CK = decltype(ck_c)::value;
    hipLaunchKernelGGL((k_expand_light<SL, CK>), dim3(nblk), dim3(kBlock), 0, s, src, nslots, ooff, sub, out, out_cap,
                       heavy, nheavy, partials, reinterpret_cast<uint2*>(ctx->ctl.as<uint64_t>() + 64));
    hipLaunchKernelGGL(k_heavy_offsets, dim3(1), dim3(1024), 0, s, heavy, nheavy, ooff, hoff);
    hipLaunchKernelGGL((k_expand_heavy_flat<SL, CK>), dim3(ctx->num_cus * 4), dim3(kBlock), 0, s, src, ooff, sub,
                       heavy, nheavy, hoff, out, out_cap, res);
  };
  using T = std::true_type;
  using F = std::false_type;
  if (slots) {
    if (ck) launch(T{}, T{});
    else launch(T{}, F{});
  } else {
    if (ck) launch(F{}, T{});
    else launch(F{}, F{});
  }
  return hipGetLastError();
}

}  // namespace

hipError_t nested_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s) {
  hipError_t e;
  const uint64_t n = r.n;
  const uint64_t nn = n ? n : 1;
  const uint32_t lo = uint32_t(t->desc.bucket_lo), nbl = t->nb_local;
  if ((e = t->off.ensure((uint64_t(nbl) + 1) * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = t->main.ensure(nn * sizeof(uint4))) != hipSuccess) return e;
  if ((e = t->sub.ensure(nn * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = t->counts.ensure(4 * sizeof(uint64_t))) != hipSuccess) return e;
  // scratch: hk | k1 | v1 | x(n+1) | mh | msub(n+1) | mfirst | mslot
  if ((e = ctx->scratch[kScrSortK].ensure(3 * nn * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrB].ensure((5 * nn + 2) * sizeof(uint32_t))) != hipSuccess) return e;
  uint32_t* hk = ctx->scratch[kScrSortK].as<uint32_t>();
  uint32_t* k1 = hk + nn;
  uint32_t* v1 = k1 + nn;
  uint32_t* x = ctx->scratch[kScrB].as<uint32_t>();
  uint32_t* mh = x + nn + 1;
  uint32_t* msub = mh + nn;
  uint32_t* mfirst = msub + nn + 1;
  uint32_t* mslot = mfirst + nn;
  uint32_t* rows = t->sub.as<uint32_t>();
  uint32_t* off = t->off.as<uint32_t>();
  uint64_t* counts = t->counts.as<uint64_t>();
  if ((e = hipMemsetAsync(counts, 0, 4 * sizeof(uint64_t), s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(off, 0, (uint64_t(nbl) + 1) * sizeof(uint32_t), s)) != hipSuccess) return e;
  const RelView v = view_of(r);
  const unsigned g = grid_for(ctx, nn, kBlock * 4);
  if (n) {
    hipLaunchKernelGGL(k_extract, dim3(g), dim3(kBlock), 0, s, v, t->fm, lo, nbl, hk, rows, counts);
    // sort by key, only over its significant bits (equal keys <=> equal hashes: murmur32 is a bijection)
    uint64_t maxkey = 0;
    if ((e = hipMemcpyAsync(&maxkey, counts + 3, sizeof(maxkey), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    const int bits = maxkey ? 32 - __builtin_clz(uint32_t(maxkey)) : 0;
    bool alt = false;
    if ((e = radix_sort_pairs(ctx, hk, rows, k1, v1, n, bits, s, &alt)) != hipSuccess) return e;
    if (alt) {  // odd number of passes: the sorted keys are in k1, the sorted rows in v1
      hk = k1;
      if ((e = hipMemcpyAsync(rows, v1, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    }
    const bool rows_sorted = r.row_off == HJ3D_ROW_IMPLICIT;  // stable sort keeps input (= row) order
    hipLaunchKernelGGL(k_heads, dim3(g), dim3(kBlock), 0, s, hk, n, x);
    if ((e = exclusive_scan_u32(ctx, x, x, n, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_runs, dim3(g), dim3(kBlock), 0, s, hk, n, x, rows, rows_sorted, mh, msub, mfirst);
    if (!rows_sorted) hipLaunchKernelGGL(k_run_min, dim3(g), dim3(kBlock), 0, s, hk, rows, n, x, mfirst);
    hipLaunchKernelGGL(k_main_count, dim3(g), dim3(kBlock), 0, s, mh, x, n, t->fm, lo, nbl, off, mslot);
  }
  if ((e = exclusive_scan_u32(ctx, off, off, nbl, s)) != hipSuccess) return e;
  if (n) {
    hipLaunchKernelGGL(k_main_scatter, dim3(g), dim3(kBlock), 0, s, mh, mfirst, msub, mslot, x, n, t->fm, lo, off,
                       t->main.as<uint4>(), counts);
  }
  t->n_build = n;
  return hipGetLastError();
}

hipError_t nested_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                        uint64_t out_cap, uint64_t* res, hipStream_t s) {
  if (r.n == 0) return hipSuccess;
  const RelView v = view_of(r);
  const bool unnest = flags & HJ3D_PROBE_UNNEST;
  const bool emit = (flags & HJ3D_PROBE_EMIT) && out;
  const uint32_t lo = uint32_t(t->desc.bucket_lo), nbl = t->nb_local;
  const uint32_t* off = t->off.as<const uint32_t>();
  const uint4* mains = t->main.as<const uint4>();
  const uint32_t* sub = t->sub.as<const uint32_t>();
  uint2* o = static_cast<uint2*>(out);
  const unsigned g = grid_for(ctx, r.n, kBlock * kItems);
  hipError_t e;
  if (!unnest) {
    if (emit)
      hipLaunchKernelGGL(k_nested_probe<kDenseNU>, dim3(g), dim3(kBlock), 0, s, v, t->fm, lo, nbl, off, mains, sub, o,
                         out_cap, nullptr, nullptr, nullptr, nullptr, res);
    else
      hipLaunchKernelGGL(k_nested_probe<kAggNU>, dim3(g), dim3(kBlock), 0, s, v, t->fm, lo, nbl, off, mains, sub,
                         nullptr, 0, nullptr, nullptr, nullptr, nullptr, res);
    return hipGetLastError();
  }
  if (!emit) {
    if ((e = ctx->scratch[kScrC].ensure(r.n * sizeof(Heavy) + 16)) != hipSuccess) return e;
    uint64_t* nheavy = ctx->scratch[kScrC].as<uint64_t>();
    Heavy* heavy = reinterpret_cast<Heavy*>(nheavy + 2);
    if ((e = hipMemsetAsync(nheavy, 0, sizeof(uint64_t), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_nested_probe<kAggUN>, dim3(g), dim3(kBlock), 0, s, v, t->fm, lo, nbl, off, mains, sub,
                       nullptr, 0, nullptr, nullptr, heavy, nheavy, res);
    hipLaunchKernelGGL(k_expand_heavy, dim3(ctx->num_cus * 4), dim3(kBlock), 0, s, heavy, nheavy, mains, sub, res);
    return hipGetLastError();
  }
  // materialised unnest: count -> scan -> expansion (light: per 256 probes; heavy: all workgroups)
  const uint32_t nblk = uint32_t((r.n + kBlock - 1) / kBlock);
  if ((e = ctx->scratch[kScrA].ensure((r.n + 1) * sizeof(uint64_t))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrC].ensure(2 * r.n * sizeof(uint32_t) + 64)) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrD].ensure((r.n + 2) * sizeof(uint64_t))) != hipSuccess) return e;  // hoff
  if ((e = ctx->scratch[kScrPartial].ensure(uint64_t(nblk) * kProbeFields * sizeof(uint64_t))) != hipSuccess) return e;
  uint64_t* cnt = ctx->scratch[kScrA].as<uint64_t>();
  uint32_t* nheavy = ctx->scratch[kScrC].as<uint32_t>();
  uint32_t* mid = nheavy + 16;
  uint32_t* heavy = mid + r.n;
  uint64_t* partials = ctx->scratch[kScrPartial].as<uint64_t>();
  if ((e = hipMemsetAsync(nheavy, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_nested_probe<kCountUN>, dim3(g), dim3(kBlock), 0, s, v, t->fm, lo, nbl, off, mains, sub,
                     nullptr, 0, cnt, mid, nullptr, nullptr, res);
  if ((e = exclusive_scan_u64(ctx, cnt, cnt, r.n, s)) != hipSuccess) return e;
  SlotSrc src{v, mid, mains, nullptr, nullptr};
  const bool ck = flags & HJ3D_PROBE_CHECKSUM;
  if ((e = expand(ctx, src, false, ck, r.n, cnt, sub, o, out_cap, heavy, nheavy, partials, res, s)) != hipSuccess)
    return e;
  return ck ? reduce_partials(partials, nblk, kProbeFields, 1, res, s) : hipSuccess;
}

bool radix_nested_applicable(const hj3d_ctx* ctx, const hj3d_table* t, uint64_t n_probe) {
  return t->desc.kind == HJ3D_NESTED && !ctx->force_direct && n_probe >= ctx->radix_min && t->nb_local >= 64 &&
         n_probe < (1ull << 32) && t->n_mains > 0;
}

hipError_t radix_nested_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                              uint64_t out_cap, uint64_t* res, hipStream_t s, const SelArgs* sel, const ZeroList* also) {
  hipError_t e;
  const uint32_t lo = uint32_t(t->desc.bucket_lo), nbl = t->nb_local;
  // slice width: 80% of the LDS budget at the mean number of main records per bucket (a
  // directory word + a 4-word main record per bucket at fill 1)
  const double fill = double(t->n_mains) / double(nbl);
  ProbeParts pp;
  unsigned long long* npass = nullptr;  // fused selection: tuples passing it (n_probe)
  uint32_t w_fit = uint32_t(0.8 * kProbeLdsWords / (1.0 + 4.0 * fill));
  if (ctx->pk_slice_max && w_fit > ctx->pk_slice_max) w_fit = ctx->pk_slice_max;  // HJ3D_OPT_PK_SLICE (tests)
  // more LDS slices than the one-level partitioner's 2048 (config D's 1e8-bucket table on one GPU,
  // 2.5e7 / 5e7 buckets per rank at 4 / 2 owners): the packed partitioner's two levels give every
  // slice its LDS width (pk_probe_slices); before, such tables were probed in ~1 MB slices through L2
  PkGeom pk{};
  bool pkd = false;
  // once the packed partitioner has run, its control words (overflow count, n_probe) go back to zero
  // on every exit, early returns included: the probes that share them rely on that
  struct CtlReset {
    hj3d_ctx* c;
    hipStream_t st;
    bool armed = false;
    ~CtlReset() {
      if (armed) (void)pk_ctl_reset(c, st);
    }
  } ctl_reset{ctx, s};
  {
    const uint64_t P0 = (uint64_t(nbl) + w_fit - 1) / w_fit;
    if (!sel && w_fit >= 64 && P0 > 2048 && P0 <= 65536) {
      const uint64_t G = uint64_t(ctx->num_cus);
      const uint64_t P1 = (P0 + G - 1) / G * G;  // whole waves of probe workgroups
      const uint32_t W1 = uint32_t((uint64_t(nbl) + P1 - 1) / P1);
      e = pk_probe_slices(ctx, t, r, W1 >= 64 ? W1 : w_fit, &pp, &pk, s);
      if (e == hipSuccess) pkd = ctl_reset.armed = true;
      else if (e != hipErrorNotSupported) return e;
      if (pkd && also && (e = zero_words(*also, s)) != hipSuccess) return e;
    }
  }
  if (!pkd && (e = radix_partition_probe(ctx, t, r, w_fit, &pp, s, sel, sel ? &npass : nullptr, true, also)) != hipSuccess)
    return e;
  // slices wider than LDS (more than the partitioner's 2048 slices at the fitting width: config D's
  // 1e8-bucket table) are probed through the cache. Then kHbmSplits workgroups share each slice and
  // the blocks are ordered so that an XCD's workgroups take consecutive (slice, share) pairs: the
  // ~32 workgroups of an XCD work on two slices at a time, whose directory and main records
  // (~1 MB each) stay in its 4 MB L2 instead of 32 different slices thrashing it.
  const bool wide = !pkd && pp.W > w_fit && pp.splits < kHbmSplits && pp.G >= kHbmSplits;
  if (wide) pp.splits = kHbmSplits;
  const uint32_t nblocks = pp.P * pp.splits;
  if ((e = ctx->scratch[kScrPartial].ensure(uint64_t(nblocks + 2) * kProbeFields * sizeof(uint64_t))) != hipSuccess)
    return e;
  uint64_t* partials = ctx->scratch[kScrPartial].as<uint64_t>();
  uint64_t* base0 = partials + uint64_t(nblocks + 1) * kProbeFields;
  const uint64_t* base_src = sel ? reinterpret_cast<const uint64_t*>(npass) : res;
  const bool unnest = flags & HJ3D_PROBE_UNNEST;
  const bool emit = (flags & HJ3D_PROBE_EMIT) && out;
  const uint32_t* off = t->off.as<const uint32_t>();
  const uint4* mains = t->main.as<const uint4>();
  const uint32_t* sub = t->sub.as<const uint32_t>();
  uint2* o = static_cast<uint2*>(out);
  uint64_t* cnt = nullptr;
  uint32_t *zo = nullptr, *po = nullptr;
  Heavy* hq = nullptr;
  uint64_t* nhq = nullptr;
  const int mode = !unnest ? (emit ? kDenseNU : kAggNU) : (emit ? kCountUN : kAggUN);
  if (mode == kCountUN) {
    if ((e = ctx->scratch[kScrA].ensure((r.n + 1) * sizeof(uint64_t))) != hipSuccess) return e;
    if ((e = ctx->scratch[kScrC].ensure(3 * r.n * sizeof(uint32_t) + 64)) != hipSuccess) return e;
    cnt = ctx->scratch[kScrA].as<uint64_t>();
    zo = ctx->scratch[kScrC].as<uint32_t>() + 16;
    po = zo + r.n;
  } else if (mode == kAggUN) {
    if ((e = ctx->scratch[kScrC].ensure(r.n * sizeof(Heavy) + 16)) != hipSuccess) return e;
    nhq = ctx->scratch[kScrC].as<uint64_t>();
    hq = reinterpret_cast<Heavy*>(nhq + 2);
    if ((e = hipMemsetAsync(nhq, 0, sizeof(uint64_t), s)) != hipSuccess) return e;
  }
  if ((e = ctx->ensure_ctl()) != hipSuccess) return e;
  uint64_t* sink = ctx->ctl.as<uint64_t>() + 64;  // ctl words [64, 128): store sink
  // the materialised expansion's heavy-slot counter (scratch kScrSortK, word 0) is zeroed by the prep
  // launch (no runtime fill behind the probe)
  uint32_t* nheavy = nullptr;
  if (mode == kCountUN) {
    if ((e = ctx->scratch[kScrSortK].ensure((r.n + 64) * sizeof(uint32_t))) != hipSuccess) return e;
    nheavy = ctx->scratch[kScrSortK].as<uint32_t>();
  }
  hipLaunchKernelGGL(k_rn_prep, dim3(cnt ? ctx->num_cus * 4 : 1), dim3(kBlock), 0, s,
                     partials + uint64_t(nblocks) * kProbeFields, base0, base_src, cnt, pp.seg + uint64_t(pp.G) * pp.P,
                     pp.novf, r.n, nheavy);
  {
    PhaseTimer tk(ctx, HJ3D_T_PROBE_KERNEL);
    auto launch = [&](auto mode_c) {
      constexpr int M = decltype(mode_c)::value;
      auto seg_kernels = [&](auto pkd_c) {
        constexpr bool PKD = decltype(pkd_c)::value;
        hipLaunchKernelGGL((k_rn_probe_seg<M, true, PKD>), dim3(nblocks), dim3(kJBlock), 0, s, pp.region, pp.counts,
                           pp.seg, pp.G, pp.cap, off, mains, sub, t->fm, lo, nbl, pp.W, pp.P, pp.splits, pp.flat, o,
                           out_cap, cnt, zo, po, hq, nhq, partials, sink, wide, pk);
        hipLaunchKernelGGL((k_rn_probe_seg<M, false, PKD>), dim3(nblocks), dim3(kJBlock), 0, s, pp.region, pp.counts,
                           pp.seg, pp.G, pp.cap, off, mains, sub, t->fm, lo, nbl, pp.W, pp.P, pp.splits, pp.flat, o,
                           out_cap, cnt, zo, po, hq, nhq, partials, sink, wide, pk);
      };
      if (pkd) seg_kernels(std::true_type{});
      else seg_kernels(std::false_type{});
      hipLaunchKernelGGL((k_rn_probe_ovf<M>), dim3(ctx->num_cus), dim3(kBlock), 0, s, pp.ovf, pp.novf,
                         pp.seg + uint64_t(pp.G) * pp.P, off, mains, sub, t->fm, lo, o, out_cap, cnt, zo, po, hq, nhq,
                         res);
    };
    switch (mode) {
      case kAggNU: launch(std::integral_constant<int, kAggNU>{}); break;
      case kDenseNU: launch(std::integral_constant<int, kDenseNU>{}); break;
      case kAggUN: launch(std::integral_constant<int, kAggUN>{}); break;
      default: launch(std::integral_constant<int, kCountUN>{}); break;
    }
    if (mode == kAggUN)
      hipLaunchKernelGGL(k_expand_heavy, dim3(ctx->num_cus * 4), dim3(kBlock), 0, s, hq, nhq, mains, sub, res);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // the packed partitioner's control words (overflow count, n_probe) back to zero, the invariant of
  // the probes that share them
  if (pkd) {
    ctl_reset.armed = false;
    if ((e = pk_ctl_reset(ctx, s)) != hipSuccess) return e;
  }
  // n_probe counts every scanned tuple, also those of unowned buckets (dropped by the partition)
  if ((e = reduce_partials(partials, nblocks + 1, kProbeFields, 1, res, s, sel ? 0ull : r.n, base0)) != hipSuccess)
    return e;
  if (mode != kCountUN) return hipSuccess;
  // expansion over the slots: regions' then overflow pairs' (unused slots have count 0)
  if ((e = exclusive_scan_u64(ctx, cnt, cnt, r.n, s)) != hipSuccess) return e;
  const uint32_t nblk = uint32_t((r.n + kBlock - 1) / kBlock);
  // heavy slots: at most one per slot (many probe tuples may match one hot key); nheavy zeroed above
  if ((e = ctx->scratch[kScrD].ensure((r.n + 2) * sizeof(uint64_t))) != hipSuccess) return e;  // hoff
  if ((e = ctx->scratch[kScrPartial].ensure(uint64_t(nblk) * kProbeFields * sizeof(uint64_t))) != hipSuccess) return e;
  uint32_t* heavy = nheavy + 64;
  partials = ctx->scratch[kScrPartial].as<uint64_t>();
  SlotSrc src{view_of(r), nullptr, mains, zo, po};
  const bool ck = flags & HJ3D_PROBE_CHECKSUM;
  if ((e = expand(ctx, src, true, ck, r.n, cnt, sub, o, out_cap, heavy, nheavy, partials, res, s)) != hipSuccess)
    return e;
  return ck ? reduce_partials(partials, nblk, kProbeFields, 1, res, s) : hipSuccess;
}

}  // namespace hj3d

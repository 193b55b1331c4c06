// chain.hip — chaining hash table (HtChaining1, ht_chaining.hh) on MI355X.
//
// Layout (CSR-bucketized instead of the reference's 24-B pointer nodes):
//   off[b]    u32, b in [0, nb_local]: entries of bucket b are ent[off[b] .. off[b+1])
//   ent[j]    {u32 hash, u32 row}: 8 B per stored tuple (vs 24 B per reference node)
// The reference visits a bucket as [first insert, newest, ..., second insert]
// (ht_chaining.hh:185-194: the directory slot keeps the first insert, later inserts are
// head-inserted behind it). We never materialise that order: the probe reads the whole
// (tiny) bucket and derives the 1-based position of the reference's first match from row
// ids, which reproduces AlgHashJoinProbe's comparison count (algebra.hh:640-658) exactly.
//
// Build = count (atomic slot per tuple) -> exclusive scan -> scatter; 3 streaming passes.
// Probe = one pass: tuple key (streamed, non-temporal) -> bucket range -> bucket entries.
// At |R| = 1e7 the table is 40 MB + 80 MB and stays in the 256 MB Infinity Cache while
// S streams past it (roofline section).
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

constexpr int kBuildItems = 4;
constexpr int kProbeItems = 4;

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Atomic slot allocation with wave-level aggregation of the most common bucket(s): lanes that
// share the first pending lane's bucket take consecutive slots from ONE atomic (skewed builds
// hammer a few hot counters; uniform builds pay two ballots). Must be called wave-converged.
__device__ __forceinline__ uint32_t agg_slot(uint32_t* cnt, uint32_t b, bool valid) {
  uint32_t res = kInvalid;
  bool pending = valid;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const uint64_t pm = __ballot(pending);
    if (pm == 0) return res;
    const int leader = __ffsll((unsigned long long)pm) - 1;
    const uint32_t lb = __shfl(b, leader, kWave);
    const bool same = pending && b == lb;
    const uint64_t sm = __ballot(same);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&cnt[lb], uint32_t(__popcll(sm)));
    base = __shfl(base, leader, kWave);
    if (same) {
      res = base + uint32_t(__popcll(sm & lanemask_lt()));
      pending = false;
    }
  }
  if (pending) res = atomicAdd(&cnt[b], 1u);
  return res;
}

__global__ __launch_bounds__(kBlock) void k_chain_count(RelView r, FastMod fm, uint32_t lo, uint32_t nbl,
                                                        uint32_t* __restrict__ cnt, uint32_t* __restrict__ slot) {
  const uint64_t stride = uint64_t(gridDim.x) * kBlock * kBuildItems;
  for (uint64_t base = uint64_t(blockIdx.x) * kBlock * kBuildItems; base < r.n; base += stride) {
    uint32_t b[kBuildItems];
    bool v[kBuildItems];
#pragma unroll
    for (int j = 0; j < kBuildItems; ++j) {
      const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
      v[j] = i < r.n;
      const uint32_t key = v[j] ? r.key(i) : 0u;
      b[j] = fm.mod(murmur32(key)) - lo;  // unowned buckets wrap to >= nbl
      v[j] = v[j] && b[j] < nbl;
    }
#pragma unroll
    for (int j = 0; j < kBuildItems; ++j) {
      const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
      const uint32_t sl = agg_slot(cnt, b[j], v[j]);
      if (i < r.n) slot[i] = sl;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_chain_scatter(RelView r, FastMod fm, uint32_t lo,
                                                          const uint32_t* __restrict__ off,
                                                          const uint32_t* __restrict__ slot,
                                                          uint2* __restrict__ ent) {
  const uint64_t stride = uint64_t(gridDim.x) * kBlock * kBuildItems;
  for (uint64_t base = uint64_t(blockIdx.x) * kBlock * kBuildItems; base < r.n; base += stride) {
#pragma unroll
    for (int j = 0; j < kBuildItems; ++j) {
      const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
      if (i >= r.n) continue;
      const uint32_t sl = slot[i];
      if (sl == kInvalid) continue;
      const uint32_t h = murmur32(r.key(i));
      const uint32_t b = fm.mod(h) - lo;
      ent[off[b] + sl] = make_uint2(h, r.row(i));
    }
  }
}

enum ProbeMode { kAgg = 0, kDense = 1, kCount = 2, kWrite = 3 };

constexpr int kRegEnt = 4;  // bucket entries held in registers per probe item (covers ~98% of
                            // probes at #buckets = |R|; longer buckets take the loop below)

// One probe strand over a chaining table.
//   kAgg   : counters + output checksums only (what the reference's AlgTop observes)
//   kDense : kAgg + out[i] = {probe row, build row | 0xFFFFFFFF} per probe tuple (UNIQUE only)
//   kCount : kAgg + cnt[i] = #output pairs of probe tuple i (u64)
//   kWrite : out[ooff[i] + k] = k-th output pair of probe tuple i (after a scan of kCount)
// Memory-level parallelism: every item's key, bucket range and first kRegEnt entries are issued
// as independent loads (three dependent rounds per kProbeItems tuples), then evaluated from
// registers.
template <bool UNIQUE, int MODE>
__global__ __launch_bounds__(kBlock) void k_chain_probe(RelView r, FastMod fm, uint32_t lo, uint32_t nbl,
                                                        const uint32_t* __restrict__ off,
                                                        const uint2* __restrict__ ent, uint2* __restrict__ out,
                                                        uint64_t out_cap, uint64_t* __restrict__ cnt,
                                                        uint64_t* __restrict__ res) {
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t stride = uint64_t(gridDim.x) * kBlock * kProbeItems;
  for (uint64_t base = uint64_t(blockIdx.x) * kBlock * kProbeItems; base < r.n; base += stride) {
    uint32_t h[kProbeItems], b[kProbeItems], pr[kProbeItems], s[kProbeItems], n[kProbeItems];
    uint2 E[kProbeItems][kRegEnt];
    // round 1: stream the probe keys (non-temporal: S is read once)
#pragma unroll
    for (int j = 0; j < kProbeItems; ++j) {
      const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
      const bool v = i < r.n;
      h[j] = murmur32(v ? r.key(i) : 0u);
      pr[j] = v ? r.row(i) : 0u;
      b[j] = v ? fm.mod(h[j]) - lo : kInvalid;
    }
    // round 2: bucket ranges (random; the directory is Infinity-Cache resident)
#pragma unroll
    for (int j = 0; j < kProbeItems; ++j) {
      s[j] = 0;
      n[j] = 0;
      if (b[j] < nbl) {
        s[j] = off[b[j]];
        n[j] = off[b[j] + 1] - s[j];
      }
    }
    // round 3: the first kRegEnt entries of every bucket, all in flight together
#pragma unroll
    for (int k = 0; k < kRegEnt; ++k) {
#pragma unroll
      for (int j = 0; j < kProbeItems; ++j) {
        E[j][k] = make_uint2(~h[j], kInvalid);  // never matches
        if (uint32_t(k) < n[j]) E[j][k] = ent[s[j] + k];
      }
    }
#pragma unroll
    for (int j = 0; j < kProbeItems; ++j) {
      const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
      if (i >= r.n) continue;
      if (MODE != kWrite) acc[0] += 1;  // n_probe
      const uint32_t nj = n[j];
      uint32_t nout = 0;
      if (UNIQUE) {
        // the reference walks [first insert, newest, ..., second]: the first match it meets is
        // the minimum-row entry if that matches, else the largest matching row
        uint32_t minrow = kInvalid, lo_m = kInvalid, hi_m = 0, nm = 0;
#pragma unroll
        for (int k = 0; k < kRegEnt; ++k) {
          if (uint32_t(k) < nj) {
            minrow = min(minrow, E[j][k].y);
            if (E[j][k].x == h[j]) {
              ++nm;
              lo_m = min(lo_m, E[j][k].y);
              hi_m = max(hi_m, E[j][k].y);
            }
          }
        }
        for (uint32_t k = kRegEnt; k < nj; ++k) {  // long buckets
          const uint2 e2 = ent[s[j] + k];
          minrow = min(minrow, e2.y);
          if (e2.x == h[j]) {
            ++nm;
            lo_m = min(lo_m, e2.y);
            hi_m = max(hi_m, e2.y);
          }
        }
        uint32_t match = kInvalid;
        if (nj != 0) {
          if (nm == 0) {
            acc[3] += nj;  // no match: the whole chain is compared
          } else if (lo_m == minrow) {
            acc[3] += 1;  // the directory entry (first insert) matches
            match = lo_m;
          } else {
            uint32_t gt = 0;
#pragma unroll
            for (int k = 0; k < kRegEnt; ++k) gt += (uint32_t(k) < nj) && E[j][k].y > hi_m;
            for (uint32_t k = kRegEnt; k < nj; ++k) gt += ent[s[j] + k].y > hi_m;
            acc[3] += 2 + gt;
            match = hi_m;
          }
        }
        if (match != kInvalid) {
          nout = 1;
          if (MODE != kWrite) {
            acc[1] += 1;
            acc[2] += 1;
            acc[4] += pr[j];
            acc[5] += match;
            const uint64_t ph = pair_hash(pr[j], match);
            acc[7] += ph;
            acc[8] ^= ph;
          }
          if (MODE == kWrite) {
            const uint64_t o = cnt[i];
            if (o < out_cap) out[o] = make_uint2(pr[j], match);
          }
        }
        if (MODE == kDense && i < out_cap)
          __builtin_nontemporal_store((uint64_t(match) << 32) | pr[j], reinterpret_cast<uint64_t*>(out + i));
      } else {
        if (MODE != kWrite) acc[3] += nj;
        uint64_t o = (MODE == kWrite) ? cnt[i] : 0;
        for (uint32_t k = 0; k < nj; ++k) {
          uint2 e2;
          if (k < kRegEnt) {
            e2 = E[j][0];
#pragma unroll
            for (int q = 1; q < kRegEnt; ++q) e2 = (k == uint32_t(q)) ? E[j][q] : e2;
          } else {
            e2 = ent[s[j] + k];
          }
          if (e2.x != h[j]) continue;
          ++nout;
          if (MODE == kWrite) {
            if (o < out_cap) out[o] = make_uint2(pr[j], e2.y);
            ++o;
          } else {
            acc[4] += pr[j];
            acc[5] += e2.y;
            const uint64_t ph = pair_hash(pr[j], e2.y);
            acc[7] += ph;
            acc[8] ^= ph;
          }
        }
        if (MODE != kWrite) {
          acc[1] += nout != 0;
          acc[2] += nout;
        }
      }
      if (MODE == kCount) cnt[i] = nout;
    }
  }
  if (MODE != kWrite) block_flush<kProbeFields, 1>(acc, res);
}

template <bool UNIQUE, int MODE>
void launch_probe(hj3d_ctx* ctx, const hj3d_table* t, const RelView& v, uint2* out, uint64_t cap, uint64_t* cnt,
                  uint64_t* res, hipStream_t s) {
  const unsigned grid = grid_for(ctx, v.n, kBlock * kProbeItems);
  hipLaunchKernelGGL((k_chain_probe<UNIQUE, MODE>), dim3(grid), dim3(kBlock), 0, s, v, t->fm,
                     uint32_t(t->desc.bucket_lo), t->nb_local, t->off.as<const uint32_t>(),
                     t->ent.as<const uint2>(), out, cap, cnt, res);
}

}  // namespace

hipError_t chain_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s) {
  hipError_t e;
  if ((e = t->off.ensure((uint64_t(t->nb_local) + 1) * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = t->ent.ensure((r.n ? r.n : 1) * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrSlot].ensure((r.n ? r.n : 1) * sizeof(uint32_t))) != hipSuccess) return e;
  uint32_t* off = t->off.as<uint32_t>();
  uint32_t* slot = ctx->scratch[kScrSlot].as<uint32_t>();
  if ((e = hipMemsetAsync(off, 0, (uint64_t(t->nb_local) + 1) * sizeof(uint32_t), s)) != hipSuccess) return e;
  const RelView v = view_of(r);
  const uint32_t lo = uint32_t(t->desc.bucket_lo);
  if (r.n) {
    const unsigned grid = grid_for(ctx, r.n, kBlock * kBuildItems);
    hipLaunchKernelGGL(k_chain_count, dim3(grid), dim3(kBlock), 0, s, v, t->fm, lo, t->nb_local, off, slot);
  }
  if ((e = exclusive_scan_u32(ctx, off, off, t->nb_local, s)) != hipSuccess) return e;
  if (r.n) {
    const unsigned grid = grid_for(ctx, r.n, kBlock * kBuildItems);
    hipLaunchKernelGGL(k_chain_scatter, dim3(grid), dim3(kBlock), 0, s, v, t->fm, lo, off, slot,
                       t->ent.as<uint2>());
  }
  t->n_build = r.n;
  return hipGetLastError();
}

hipError_t chain_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                       uint64_t out_cap, uint64_t* res, hipStream_t s) {
  const RelView v = view_of(r);
  const bool unique = flags & HJ3D_PROBE_UNIQUE;
  const bool emit = (flags & HJ3D_PROBE_EMIT) && out;
  uint2* o = static_cast<uint2*>(out);
  if (r.n == 0) return hipSuccess;
  if (!emit) {
    if (unique) launch_probe<true, kAgg>(ctx, t, v, nullptr, 0, nullptr, res, s);
    else launch_probe<false, kAgg>(ctx, t, v, nullptr, 0, nullptr, res, s);
    return hipGetLastError();
  }
  if (unique) {
    launch_probe<true, kDense>(ctx, t, v, o, out_cap, nullptr, res, s);
    return hipGetLastError();
  }
  // variable-length output: count -> scan -> write (deterministic positions, probe order)
  hipError_t e = ctx->scratch[kScrA].ensure((r.n + 1) * sizeof(uint64_t));
  if (e != hipSuccess) return e;
  uint64_t* cnt = ctx->scratch[kScrA].as<uint64_t>();
  launch_probe<false, kCount>(ctx, t, v, nullptr, 0, cnt, res, s);
  if ((e = exclusive_scan_u64(ctx, cnt, cnt, r.n, s)) != hipSuccess) return e;
  launch_probe<false, kWrite>(ctx, t, v, o, out_cap, cnt, res, s);
  return hipGetLastError();
}

}  // namespace hj3d

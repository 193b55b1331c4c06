// nested_radix.hip — build of the nested ("3D") table from the radix-partitioned bucket CSR.
//
// The nested table needs, per bucket, one main record per distinct key {hash, first row,
// sub_off, sub_len} and the rows of every key contiguous in `sub` (ht_nested.hh:287-311: a main
// node per distinct key, duplicates in its sub-chain). The order of the mains inside a bucket
// and of the rows inside a key do not matter: the probe derives the reference's comparison
// count from first-row ranks (nested.hip), and unnest counts/checksums are order-free. So
// instead of sorting all tuples by hash (4 LSD passes over 16 B/tuple) this path:
//   1. radix-partitions the tuples into the bucket CSR of (hash, row) entries (radix.hip,
//      the chaining build: two streaming passes + one LDS pass per bucket slice);
//   2. groups every bucket by key in place: buckets of <= 32 entries by one thread (insertion
//      sort on (hash, row)); longer buckets (Zipf hot keys) by one workgroup that splits off one
//      key per pass with a block-wide partition (cost = #distinct keys in the bucket x its size;
//      a bucket needing more than kMaxPasses passes flags the table for the sort-based build);
//   3. writes the main records (per bucket: #keys -> scan -> records) and the sub rows.
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

constexpr uint32_t kSmall = 32;
constexpr uint32_t kMaxPasses = 64;
constexpr int kGBlock = 256;

__global__ __launch_bounds__(kBlock) void k_group_small(const uint32_t* __restrict__ eoff, uint32_t nbl,
                                                        uint2* __restrict__ ent, uint32_t* __restrict__ dcount,
                                                        uint32_t* __restrict__ large, uint32_t* __restrict__ nlarge) {
  for (uint32_t b = blockIdx.x * kBlock + threadIdx.x; b < nbl; b += gridDim.x * kBlock) {
    const uint32_t s = eoff[b], n = eoff[b + 1] - s;
    if (n > kSmall) {
      large[atomicAdd(nlarge, 1u)] = b;
      dcount[b] = 0;
      continue;
    }
    uint32_t d = 0;
    if (n) {
      for (uint32_t k = 1; k < n; ++k) {  // insertion sort by (hash, row)
        const uint2 x = ent[s + k];
        const uint64_t kx = (uint64_t(x.x) << 32) | x.y;
        uint32_t j = k;
        while (j > 0) {
          const uint2 y = ent[s + j - 1];
          if (((uint64_t(y.x) << 32) | y.y) <= kx) break;
          ent[s + j] = y;
          --j;
        }
        ent[s + j] = x;
      }
      uint32_t prev = ent[s].x;
      d = 1;
      for (uint32_t k = 1; k < n; ++k) {
        const uint32_t h = ent[s + k].x;
        d += h != prev;
        prev = h;
      }
    }
    dcount[b] = d;
  }
}

__device__ __forceinline__ uint32_t block_excl_scan_256(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t wt;
  const uint32_t x = wave_excl_scan(v, &wt) + v;  // inclusive within the wave
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kGBlock / kWave; ++w) {
    const uint32_t s = wsum[w];
    if (w < wid) pre += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// One workgroup per long bucket: split off the key of the first remaining entry per pass.
// Pass d of long bucket q records its run start and min row in slot q * kMaxPasses + d.
__global__ __launch_bounds__(kGBlock) void k_group_large(const uint32_t* __restrict__ eoff, uint2* __restrict__ ent,
                                                         uint2* __restrict__ tmp, const uint32_t* __restrict__ large,
                                                         const uint32_t* __restrict__ nlarge,
                                                         uint32_t* __restrict__ dcount, uint2* __restrict__ runs,
                                                         uint32_t* __restrict__ flag) {
  __shared__ uint32_t wsum[kGBlock / kWave];
  __shared__ uint32_t wmin[kGBlock / kWave];
  const uint32_t nl = *nlarge;
  for (uint32_t q = blockIdx.x; q < nl; q += gridDim.x) {
    const uint32_t b = large[q];
    const uint32_t s = eoff[b], e = eoff[b + 1];
    uint32_t cur = s, d = 0;
    while (cur < e) {
      if (d == kMaxPasses) {  // too many distinct keys in one bucket: sort-based build instead
        if (threadIdx.x == 0) *flag = 1u;
        break;
      }
      const uint32_t K = ent[cur].x;
      uint32_t m = 0, nm = 0, mn = kInvalid;
      for (uint32_t c0 = cur; c0 < e; c0 += kGBlock) {
        const uint32_t i = c0 + threadIdx.x;
        const bool valid = i < e;
        const uint2 v = valid ? ent[i] : make_uint2(0, 0);
        const bool f = valid && v.x == K;
        uint32_t tm, tn;
        const uint32_t pm = block_excl_scan_256(f ? 1u : 0u, wsum, &tm);
        const uint32_t pn = block_excl_scan_256((valid && !f) ? 1u : 0u, wsum, &tn);
        if (f) {
          tmp[cur + m + pm] = v;
          mn = min(mn, v.y);
        } else if (valid) {
          tmp[e - 1 - (nm + pn)] = v;
        }
        m += tm;
        nm += tn;
      }
      __syncthreads();
      for (uint32_t i = cur + threadIdx.x; i < e; i += kGBlock) ent[i] = tmp[i];
      // block min of the key's rows
      mn = min(mn, __shfl_xor(mn, 32, kWave));
      mn = min(mn, __shfl_xor(mn, 16, kWave));
      mn = min(mn, __shfl_xor(mn, 8, kWave));
      mn = min(mn, __shfl_xor(mn, 4, kWave));
      mn = min(mn, __shfl_xor(mn, 2, kWave));
      mn = min(mn, __shfl_xor(mn, 1, kWave));
      if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = mn;
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t bm = wmin[0];
        for (int w = 1; w < kGBlock / kWave; ++w) bm = min(bm, wmin[w]);
        runs[uint64_t(q) * kMaxPasses + d] = make_uint2(cur, bm);
      }
      __syncthreads();
      cur += m;
      ++d;
    }
    if (threadIdx.x == 0) dcount[b] = d;
  }
}

__global__ __launch_bounds__(kBlock) void k_mains_small(const uint32_t* __restrict__ eoff, uint32_t nbl,
                                                        const uint2* __restrict__ ent, const uint32_t* __restrict__ moff,
                                                        uint4* __restrict__ mains, uint64_t* __restrict__ counts) {
  uint32_t mx = 0;
  for (uint32_t b = blockIdx.x * kBlock + threadIdx.x; b < nbl; b += gridDim.x * kBlock) {
    const uint32_t s = eoff[b], n = eoff[b + 1] - s;
    if (n == 0 || n > kSmall) continue;
    uint32_t j = moff[b], rs = s;
    for (uint32_t k = 1; k <= n; ++k) {
      if (k == n || ent[s + k].x != ent[rs].x) {
        const uint2 f = ent[rs];  // sorted by (hash, row): the run's first entry has its min row
        mains[j++] = make_uint4(f.x, f.y, rs, s + k - rs);
        mx = max(mx, s + k - rs);
        rs = s + k;
      }
    }
  }
  const uint64_t wm = wave_max(uint64_t(mx));
  if ((threadIdx.x & 63) == 0 && wm) atomicMax(reinterpret_cast<unsigned long long*>(counts + 2), wm);
}

// One thread per (long bucket, pass) slot: the pass-d key of bucket large[q] becomes main d.
__global__ __launch_bounds__(kBlock) void k_mains_large(const uint2* __restrict__ runs, const uint32_t* __restrict__ large,
                                                        uint32_t nlarge, const uint32_t* __restrict__ eoff,
                                                        const uint32_t* __restrict__ dcnt, const uint32_t* __restrict__ moff,
                                                        const uint2* __restrict__ ent, uint4* __restrict__ mains,
                                                        uint64_t* __restrict__ counts) {
  uint32_t mx = 0;
  const uint64_t slots = uint64_t(nlarge) * kMaxPasses;
  for (uint64_t idx = uint64_t(blockIdx.x) * kBlock + threadIdx.x; idx < slots; idx += uint64_t(gridDim.x) * kBlock) {
    const uint32_t q = uint32_t(idx / kMaxPasses), d = uint32_t(idx % kMaxPasses);
    const uint32_t b = large[q];
    const uint32_t nd = moff[b + 1] - moff[b];
    if (d >= nd) continue;
    const uint2 r = runs[idx];
    const uint32_t end = d + 1 < nd ? runs[idx + 1].x : eoff[b + 1];
    mains[moff[b] + d] = make_uint4(ent[r.x].x, r.y, r.x, end - r.x);
    mx = max(mx, end - r.x);
  }
  const uint64_t wm = wave_max(uint64_t(mx));
  if ((threadIdx.x & 63) == 0 && wm) atomicMax(reinterpret_cast<unsigned long long*>(counts + 2), wm);
}

__global__ __launch_bounds__(kBlock) void k_sub_rows(const uint2* __restrict__ ent, uint64_t n, uint32_t* __restrict__ sub) {
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kBlock)
    sub[i] = ent[i].y;
}

__global__ void k_nested_counts(const uint32_t* __restrict__ eoff, const uint32_t* __restrict__ moff, uint32_t nbl,
                                uint64_t* __restrict__ counts) {
  counts[0] = eoff[nbl] - eoff[0];
  counts[1] = moff[nbl];
}

}  // namespace

bool nested_radix_applicable(const hj3d_ctx* ctx, const hj3d_table* t, uint64_t n) {
  return ctx->nested_radix && !ctx->force_direct && n >= (ctx->radix_min >> 4) && n > 0 && t->nb_local >= 64 && n < (1ull << 31);
}

// Returns hipErrorNotSupported (table untouched apart from scratch) when a bucket holds more
// than kMaxPasses distinct keys; the caller then uses the sort-based build.
hipError_t nested_build_radix(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s) {
  hipError_t e;
  const uint64_t n = r.n;
  const uint32_t nbl = t->nb_local;
  if ((e = radix_build(ctx, t, r, s)) != hipSuccess) return e;  // t->off / t->ent: the bucket CSR
  if ((e = t->main.ensure(n * sizeof(uint4))) != hipSuccess) return e;
  if ((e = t->sub.ensure(n * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = t->counts.ensure(4 * sizeof(uint64_t))) != hipSuccess) return e;
  // scratch: tmp (n uint2) | dcount -> moff (nbl+1) | large (nbl) | run slots | 3 counters
  if ((e = ctx->scratch[kScrSortK].ensure(n * sizeof(uint2))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrB].ensure((2 * uint64_t(nbl) + 2) * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = ctx->scratch[kScrD].ensure(64)) != hipSuccess) return e;
  uint2* tmp = ctx->scratch[kScrSortK].as<uint2>();
  uint32_t* dcount = ctx->scratch[kScrB].as<uint32_t>();
  uint32_t* large = dcount + nbl + 1;
  uint32_t* ctr = ctx->scratch[kScrD].as<uint32_t>();  // [0] #long buckets, [1] too-many-keys flag
  uint32_t* eoff = t->off.as<uint32_t>();
  uint2* ent = t->ent.as<uint2>();
  uint64_t* counts = t->counts.as<uint64_t>();
  if ((e = hipMemsetAsync(ctr, 0, 64, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(counts, 0, 4 * sizeof(uint64_t), s)) != hipSuccess) return e;
  const unsigned gb = grid_for(ctx, nbl, kBlock);
  hipLaunchKernelGGL(k_group_small, dim3(gb), dim3(kBlock), 0, s, eoff, nbl, ent, dcount, large, ctr);
  uint32_t hc[2] = {0, 0};
  if ((e = hipMemcpyAsync(hc, ctr, sizeof(hc), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  const uint32_t nlarge = hc[0];
  if ((e = ctx->scratch[kScrC].ensure((uint64_t(nlarge) * kMaxPasses + 1) * sizeof(uint2))) != hipSuccess) return e;
  uint2* runs = ctx->scratch[kScrC].as<uint2>();
  if (nlarge) {
    hipLaunchKernelGGL(k_group_large, dim3(ctx->num_cus * 8), dim3(kGBlock), 0, s, eoff, ent, tmp, large, ctr,
                       dcount, runs, ctr + 1);
    if ((e = hipMemcpyAsync(hc, ctr, sizeof(hc), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if (hc[1]) return hipErrorNotSupported;
  }
  uint32_t* moff = dcount;  // exclusive scan in place: moff[b] = first main of bucket b, moff[nbl] = #mains
  if ((e = exclusive_scan_u32(ctx, dcount, moff, nbl, s)) != hipSuccess) return e;
  uint4* mains = t->main.as<uint4>();
  hipLaunchKernelGGL(k_mains_small, dim3(gb), dim3(kBlock), 0, s, eoff, nbl, ent, moff, mains, counts);
  if (nlarge)
    hipLaunchKernelGGL(k_mains_large, dim3(grid_for(ctx, uint64_t(nlarge) * kMaxPasses, kBlock)), dim3(kBlock), 0, s,
                       runs, large, nlarge, eoff, dcount, moff, ent, mains, counts);
  hipLaunchKernelGGL(k_sub_rows, dim3(grid_for(ctx, n, kBlock * 4)), dim3(kBlock), 0, s, ent, n, t->sub.as<uint32_t>());
  hipLaunchKernelGGL(k_nested_counts, dim3(1), dim3(1), 0, s, eoff, moff, nbl, counts);
  // the table's directory becomes the main-record offsets
  if ((e = hipMemcpyAsync(eoff, moff, (uint64_t(nbl) + 1) * sizeof(uint32_t), hipMemcpyDeviceToDevice, s)) !=
      hipSuccess)
    return e;
  t->n_build = n;
  return hipGetLastError();
}

}  // namespace hj3d

// micro_radix.hip — diagnostic microbenchmark of the radix-join probe kernels (not product).
//
// Compiles radix.hip + scan.hip into this translation unit (under a renamed namespace) so the
// real kernels can be launched with other template parameters and next to streaming floors on
// the same data. Config B shapes: |R| = 1e7 keys, |S| = 1e8 AoS {k,a,b}, S.a uniform in [0,|R|).
//   part1<B,R,MAXP>  single-pass partitioner variants (workgroup size, tile, occupancy)
//   probe_seg        the segmented probe on each variant's regions
//   stream floors    read the tuple + write a pair in place; read pairs + write pairs
#define hj3d hj3d_micro
#include "../csrc/radix.hip"
#include "../csrc/scan.hip"
#undef hj3d

#include <cstdio>
#include <cstdlib>

using namespace hj3d_micro;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

namespace {

__global__ void k_fill(uint32_t* t, uint64_t n, uint32_t stride_w, uint32_t nr, bool fk) {
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    if (fk) {
      t[i * stride_w] = uint32_t(i);
      t[i * stride_w + 1] = uint32_t(mix64(i * 0x9E3779B97F4A7C15ull + 7) % nr);
      t[i * stride_w + 2] = 0;
    } else {
      t[i * stride_w] = uint32_t(i);
    }
  }
}

__global__ __launch_bounds__(1024) void k_stream_pairs(RelView r, uint2* __restrict__ out) {
  const uint64_t stride = uint64_t(gridDim.x) * 1024 * 16;
  for (uint64_t base = uint64_t(blockIdx.x) * 1024 * 16; base < r.n; base += stride) {
    uint32_t h[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t i = base + uint64_t(j) * 1024 + threadIdx.x;
      h[j] = i < r.n ? r.key(i) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t i = base + uint64_t(j) * 1024 + threadIdx.x;
      if (i < r.n) out[i] = make_uint2(murmur32(h[j]), uint32_t(i));
    }
  }
}

__global__ __launch_bounds__(256) void k_copy_pairs(const uint2* __restrict__ in, uint64_t n, uint2* __restrict__ out) {
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(in + i)) ^ 1ull,
                                reinterpret_cast<uint64_t*>(out + i));
}


// Diagnostic copy of k_rp_part1 with phases switched off (timing only; results are garbage).
// KNOB bit 0: skip rank atomics (rank = round), bit 1: skip staging, bit 2: skip global stores,
// bit 3: skip the write-out loop entirely, bit 4: skip key loads (keys = index hash)
template <int KNOB>
__global__ __launch_bounds__(1024) void k_part1_knob(RelView r, FastMod fm, uint32_t lo, uint32_t nbl, FastDiv fw,
                                                     uint32_t P, uint32_t ntiles, uint32_t cap,
                                                     uint2* __restrict__ region, uint32_t* __restrict__ counts) {
  constexpr int BLOCK = 1024, ROUNDS = 16, TILE = BLOCK * ROUNDS, TBITS = 14;
  __shared__ uint2 stage[TILE];
  __shared__ uint32_t loc[2049];
  __shared__ uint32_t cur[2048];
  __shared__ uint32_t wsum[BLOCK / kWave];
  const uint64_t gbase = uint64_t(blockIdx.x) * P;
  for (uint32_t p = threadIdx.x; p < P; p += BLOCK) cur[p] = 0;
  uint32_t h[ROUNDS];
#pragma unroll
  for (int j = 0; j < ROUNDS; ++j) {
    const uint64_t i = uint64_t(blockIdx.x) * TILE + uint64_t(j) * BLOCK + threadIdx.x;
    h[j] = (KNOB & 16) ? uint32_t(i * 2654435761u) : (i < r.n ? r.key(i) : 0u);
  }
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
        rk[j] = (part << TBITS) | ((KNOB & 1) ? uint32_t(j) : atomicAdd(&loc[part], 1u));
      } else {
        rk[j] = kInvalid;
      }
    }
    __syncthreads();
    const uint32_t m = lds_excl_scan<BLOCK>(loc, P, wsum);
    if (threadIdx.x == 0) loc[P] = m;
    if (!(KNOB & 2)) {
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j) {
        if (rk[j] == kInvalid) continue;
        const uint64_t i = base + uint64_t(j) * BLOCK + threadIdx.x;
        stage[(loc[rk[j] >> TBITS] + (rk[j] & (TILE - 1))) & (TILE - 1)] = make_uint2(h[j], r.row(i));
      }
    }
    __syncthreads();
    const uint64_t nbase = uint64_t(tile + gridDim.x) * TILE;
#pragma unroll
    for (int j = 0; j < ROUNDS; ++j) {
      const uint64_t i = nbase + uint64_t(j) * BLOCK + threadIdx.x;
      h[j] = (KNOB & 16) ? uint32_t(i * 2654435761u) : (i < r.n ? r.key(i) : 0u);
    }
    if (!(KNOB & 8)) {
      for (uint32_t k = threadIdx.x; k < TILE; k += BLOCK) {
        const uint2 e = stage[k];
        const uint32_t p = fw.div(fm.mod(e.x) - lo) % P;
        const uint32_t o = (cur[p] + (k - loc[p])) % cap;
        if (!(KNOB & 4)) region[(gbase + p) * cap + o] = e;
        else if (e.x == 0x12345678u && o == 7u) region[0] = e;
      }
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < P; p += BLOCK) cur[p] += loc[p + 1] - loc[p];
    __syncthreads();
  }
  for (uint32_t p = threadIdx.x; p < P; p += BLOCK) counts[gbase + p] = min(cur[p], cap);
}

template <int KNOB>
__global__ __launch_bounds__(kJBlock) void k_probe_knob(const uint2* __restrict__ region,
                                                          const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ seg, uint32_t G, uint32_t cap,
                                                          const uint32_t* __restrict__ off, const uint2* __restrict__ ent,
                                                          FastMod fm, uint32_t lo, uint32_t nbl, uint32_t W, uint32_t P,
                                                          uint32_t splits, uint2* __restrict__ out, uint64_t out_cap,
                                                          uint64_t* __restrict__ cnt, uint64_t* __restrict__ partials) {
  __shared__ uint32_t lds[kProbeLdsWords];
  const uint32_t p = blockIdx.x / splits, sp = blockIdx.x % splits;
  const uint32_t b0 = p * W;
  const uint32_t nbs = min(W, nbl - b0);
  const uint32_t e0 = off[b0], e1 = off[b0 + nbs];
  const uint32_t ne = e1 - e0;
  const bool fits = (nbs + 1) + 2ull * ne + 1 <= kProbeLdsWords;
  uint32_t* loff = lds;
  uint2* lent = reinterpret_cast<uint2*>(lds + ((nbs + 2) & ~1u));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kWaves = kJBlock / kWave;
  const uint32_t g_lo = uint32_t(uint64_t(G) * sp / splits), g_hi = uint32_t(uint64_t(G) * (sp + 1) / splits);
  constexpr uint32_t kChunk = 64 * kSegItems;
  // The regions of wave wid are g = g_lo + wid + kWaves * r; lane r holds region r's pair count and
  // output base, so the walk below never waits on a global load for its bookkeeping.
  const uint32_t nr = g_hi > g_lo + wid ? (g_hi - g_lo - wid + kWaves - 1) / kWaves : 0u;  // <= 64 (G <= 1024)
  uint32_t my_len = 0, my_seg = 0;
  if (uint32_t(lane) < nr) {
    const uint32_t gg = g_lo + wid + kWaves * lane;
    my_len = counts[uint64_t(gg) * P + p];
    my_seg = seg[uint64_t(p) * G + gg];
  }
  // wave-uniform cursor: region index r, offset q
  uint32_t r = 0, q = 0;
  uint32_t len = __shfl(my_len, 0, kWave);
  while (r < nr && len == 0) {
    ++r;
    len = __shfl(my_len, int(r & 63), kWave);
  }
  auto load = [&](uint64_t (&v)[kSegItems], uint32_t rr, uint32_t qq, uint32_t ll) {
    const uint2* src = region + (uint64_t(g_lo + wid + kWaves * rr) * P + p) * cap;
#pragma unroll
    for (int j = 0; j < kSegItems; ++j) {
      const uint32_t k = qq + j * 64 + lane;
      v[j] = (rr < nr && k < ll) ? __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(src + k)) : 0ull;
    }
  };
  uint64_t cur[kSegItems];
  load(cur, r, q, len);
  if (fits && !(KNOB & 1)) stage_slice(off, ent, b0, nbs, e0, ne, loff, lent);
  __syncthreads();
  uint64_t acc[kProbeFields] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  while (r < nr) {
    uint32_t nr_ = r, nq = q + kChunk, nl = len;
    while (nr_ < nr && nq >= nl) {
      ++nr_;
      nq = 0;
      nl = __shfl(my_len, int(nr_ & 63), kWave);
    }
    uint64_t nxt[kSegItems];
    load(nxt, nr_, nq, nl);
    const uint64_t obase = uint64_t(__shfl(my_seg, int(r & 63), kWave)) + q;
#pragma unroll
    for (int j = 0; j < kSegItems; ++j) {
      const uint32_t k = q + j * 64 + lane;
      if (k >= len) continue;
      const uint32_t hv = uint32_t(cur[j]), row = uint32_t(cur[j] >> 32);
      const uint32_t bl = fm.mod(hv) - lo - b0;
      const uint64_t i = obase + j * 64 + lane;
      if (KNOB & 2) {
        acc[0] += bl;
        if (!(KNOB & 4)) __builtin_nontemporal_store(cur[j] ^ bl, reinterpret_cast<uint64_t*>(out + i));
      } else if (KNOB & 4) {
        const uint32_t d = loff[bl];
        probe_bucket<true, kAgg, false>(hv, row, lent, d >> 16, d & 0xFFFFu, acc, i, out, out_cap, cnt);
      } else if (KNOB & 8) {  // directory lookup only
        const uint32_t s = loff[bl], e = loff[bl + 1];
        acc[0] += s ^ e;
        __builtin_nontemporal_store(cur[j] ^ (uint64_t(s) << 32 | e), reinterpret_cast<uint64_t*>(out + i));
      } else {
        const uint32_t d = loff[bl];
        probe_bucket<true, kDense, false>(hv, row, lent, d >> 16, d & 0xFFFFu, acc, i, out, out_cap, cnt);
      }
    }
    r = nr_;
    q = nq;
    len = nl;
#pragma unroll
    for (int j = 0; j < kSegItems; ++j) cur[j] = nxt[j];
  }
  block_store<kProbeFields, 1>(acc, partials + uint64_t(blockIdx.x) * kProbeFields);
}


}  // namespace

int main(int argc, char** argv) {
  const uint32_t nR = argc > 1 ? atoi(argv[1]) : 10000000;
  const uint64_t nS = argc > 2 ? atoll(argv[2]) : 100000000ull;
  const int reps = 5;
  hj3d_ctx ctx;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  ctx.num_cus = prop.multiProcessorCount;
  ctx.stream = nullptr;
  uint32_t *R, *S;
  CK(hipMalloc(&R, uint64_t(nR) * 4));
  CK(hipMalloc(&S, nS * 12));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, R, nR, 1, nR, false);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, S, nS, 3, nR, true);
  hj3d_rel rr{R, nR, 4, 0, HJ3D_ROW_IMPLICIT, 0, 0};
  hj3d_rel rs{S, nS, 12, 4, HJ3D_ROW_IMPLICIT, 0, 0};
  hj3d_table t;
  t.desc.kind = HJ3D_CHAIN;
  t.desc.num_buckets = nR;
  t.desc.bucket_lo = 0;
  t.desc.bucket_hi = nR;
  t.nb_local = nR;
  t.fm = FastMod::make(nR);
  CK(t.counts.ensure(32));
  CK(radix_build(&ctx, &t, rr, 0));
  CK(sort_small_buckets(&ctx, &t, 0));
  uint2 *out, *pairs;
  CK(hipMalloc(&out, nS * 8));
  CK(hipMalloc(&pairs, nS * 8));
  uint64_t* res;
  CK(hipMalloc(&res, 16 * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, auto fn, double bytes) {
    fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) fn();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-40s %8.3f ms  %7.0f GB/s (alg)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    return ms;
  };
  timeit("radix_probe dense (product, all)",
         [&] { CK(radix_probe(&ctx, &t, rs, HJ3D_PROBE_UNIQUE | HJ3D_PROBE_EMIT, out, nS, res, 0)); }, nS * 28.0);
  // chunked: the same probe over S in C consecutive pieces (regions reused: do they stay in the
  // 256 MB Infinity Cache between the partition and the probe of one piece?)
  for (int C : {2, 4, 8, 16}) {
    char nm[64];
    snprintf(nm, sizeof nm, "radix_probe dense, %d chunks", C);
    timeit(nm, [&] {
      const uint64_t step = (nS + C - 1) / C;
      for (uint64_t o = 0; o < nS; o += step) {
        hj3d_rel c = rs;
        c.base = reinterpret_cast<const char*>(S) + o * 12;
        c.n = o + step < nS ? step : nS - o;
        c.row_base = o;
        CK(radix_probe(&ctx, &t, c, HJ3D_PROBE_UNIQUE | HJ3D_PROBE_EMIT, out + o, c.n, res, 0));
      }
    }, nS * 28.0);
  }
  const RelView v = view_of(rs);
  timeit("floor: read tuple, write pair", [&] { hipLaunchKernelGGL(k_stream_pairs, dim3(1024), dim3(1024), 0, 0, v, pairs); },
         nS * 20.0);
  timeit("floor: read pair, write pair", [&] { hipLaunchKernelGGL(k_copy_pairs, dim3(4096), dim3(256), 0, 0, pairs, nS, out); },
         nS * 16.0);

  const double fill = 1.0;
  const uint32_t W = uint32_t(0.8 * kProbeLdsWords / (1.0 + 2.0 * fill));
  const Plan pl0 = plan_for(nR, W, nS);
  const uint32_t P = pl0.P;
  uint32_t* counts;
  uint32_t* seg;
  uint2* ovf;
  unsigned long long* novf;
  uint2* region;
  const uint64_t region_bytes = 3ull << 30;
  CK(hipMalloc(&region, region_bytes));
  CK(hipMalloc(&counts, 4096ull * P * 4));
  CK(hipMalloc(&seg, (4096ull * P + 1) * 4));
  CK(hipMalloc(&ovf, nS * 8));
  CK(hipMalloc(&novf, 8));
  uint64_t* partials;
  CK(hipMalloc(&partials, 1ull << 24));

  auto variant = [&](const char* name, auto kern, int block, int tile, int per_cu) {
    const uint32_t ntiles = uint32_t((nS + tile - 1) / tile);
    uint32_t G = uint32_t(ctx.num_cus) * per_cu;
    if (G > ntiles) G = ntiles;
    const uint64_t per_g = uint64_t((ntiles + G - 1) / G) * tile;
    const double ex = double(per_g) / P;
    uint64_t cap = uint64_t(ex + 8.0 * std::sqrt(ex) + 32.0);
    cap = (cap + 15) & ~uint64_t(15);
    if (uint64_t(G) * P * cap * 8 > region_bytes) {
      printf("%s: region too large\n", name);
      return;
    }
    char nm[128];
    snprintf(nm, sizeof nm, "part1 %s (G=%u cap=%llu)", name, G, (unsigned long long)cap);
    timeit(nm, [&] {
      CK(hipMemsetAsync(novf, 0, 8, 0));
      hipLaunchKernelGGL(kern, dim3(G), dim3(block), 0, 0, v, t.fm, 0u, nR, pl0.fw, P, ntiles, uint32_t(cap), region,
                         counts, ovf, novf);
    }, nS * 20.0);
    unsigned long long h_novf = 0;
    CK(hipMemcpy(&h_novf, novf, 8, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(k_transpose_counts, dim3(1024), dim3(256), 0, 0, counts, G, P, seg);
    CK(exclusive_scan_u32(&ctx, seg, seg, uint64_t(G) * P, 0));
    uint32_t splits = 1;
    if (P < uint32_t(ctx.num_cus) * 2) splits = (uint32_t(ctx.num_cus) * 2 + P - 1) / P;
    snprintf(nm, sizeof nm, "  probe_seg on it (ovf=%llu)", h_novf);
    timeit(nm, [&] {
      hipLaunchKernelGGL((k_rp_probe_seg<true, kDense, false, true>), dim3(P * splits), dim3(kJBlock), 0, 0, region, counts,
                         seg, G, uint32_t(cap), t.off.as<const uint32_t>(), t.ent.as<const uint2>(), t.fm, 0u, nR,
                         pl0.W, P, splits, false, out, nS, nullptr, partials);
    }, nS * 16.0 + nR * 12.0);
  };
  variant("1024x16 (1/CU)", k_rp_part1<1024, 16, 2048, true>, 1024, 16384, 1);
  variant("regcarry 1024x8 (1/CU)", k_rp_part1r<1024, 8, true>, 1024, 8192, 1);
  {
    const uint32_t ntiles = uint32_t((nS + 16383) / 16384), G = 256;
    const uint32_t cap = 576;
    auto knob = [&](const char* nm, auto kern) {
      timeit(nm, [&] { hipLaunchKernelGGL(kern, dim3(G), dim3(1024), 0, 0, v, t.fm, 0u, nR, pl0.fw, P, ntiles, cap,
                                          region, counts); }, nS * 20.0);
    };
    knob("knob full copy", k_part1_knob<0>);
    CK(hipMemsetAsync(novf, 0, 8, 0));
    hipLaunchKernelGGL((k_rp_part1<1024, 16, 2048, true>), dim3(G), dim3(1024), 0, 0, v, t.fm, 0u, nR, pl0.fw, P, ntiles, cap,
                       region, counts, ovf, novf);
    hipLaunchKernelGGL(k_transpose_counts, dim3(1024), dim3(256), 0, 0, counts, G, P, seg);
    CK(exclusive_scan_u32(&ctx, seg, seg, uint64_t(G) * P, 0));
    auto pk = [&](const char* nm, auto kern) {
      timeit(nm, [&] { hipLaunchKernelGGL(kern, dim3(P), dim3(1024), 0, 0, region, counts, seg, G, cap,
                                          t.off.as<const uint32_t>(), t.ent.as<const uint2>(), t.fm, 0u, nR, pl0.W, P,
                                          1u, out, nS, nullptr, partials); }, nS * 16.0 + nR * 12.0);
    };
    pk("probe knob full (dense)", k_probe_knob<0>);
    pk("probe knob no slice stage", k_probe_knob<1>);
    pk("probe knob no probe (copy)", k_probe_knob<2>);
    pk("probe knob no probe no store", k_probe_knob<2 | 4>);
    pk("probe knob probe agg (no store)", k_probe_knob<4>);
    pk("probe knob dir lookup only", k_probe_knob<8>);
    knob("knob no rank atomics", k_part1_knob<1>);
    knob("knob no staging", k_part1_knob<2>);
    knob("knob no global stores", k_part1_knob<4>);
    knob("knob no write-out loop", k_part1_knob<8>);
    knob("knob no key loads", k_part1_knob<16>);
    knob("knob only loads+hash+rank+scan", k_part1_knob<2 | 8>);
    knob("knob only loads+hash+scan", k_part1_knob<1 | 2 | 8>);
  }
  CK(hipDeviceSynchronize());
  printf("ok\n");
  return 0;
}

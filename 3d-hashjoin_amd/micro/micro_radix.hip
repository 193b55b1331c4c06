// micro_radix.hip — diagnostic microbenchmark of the radix-join kernels (not product).
//
// Compiles radix.hip + scan.hip into this translation unit (under a renamed namespace) so the
// real kernels can be launched next to stripped variants on the same data:
//   probe:   real k_rp_probe (dense EMIT / aggregate) vs copy-only (pairs -> out at the same
//            geometry) vs copy + slice staging
//   scatter: real k_rp_scatter vs a streaming floor (read tuple, write pair in place)
// Config B shapes: |R| = 1e7 keys, |S| = 1e8 AoS {k,a,b} with S.a uniform in [0, |R|).
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

// copy-only: same grid/partition geometry as k_rp_probe, pairs -> out, optional slice stage
template <bool STAGE>
__global__ __launch_bounds__(1024) void k_copy(const uint2* __restrict__ pairs, const uint32_t* __restrict__ ps,
                                               const uint32_t* __restrict__ off, const uint2* __restrict__ ent,
                                               uint32_t nbl, uint32_t W, uint2* __restrict__ out) {
  __shared__ uint32_t lds[36864];
  const uint32_t p = blockIdx.x;
  const uint32_t b0 = p * W;
  const uint32_t nbs = min(W, nbl - b0);
  if (STAGE) {
    const uint32_t e0 = off[b0], ne = off[b0 + nbs] - e0;
    for (uint32_t k = threadIdx.x; k <= nbs; k += 1024) lds[k] = off[b0 + k] - e0;
    uint2* lent = reinterpret_cast<uint2*>(lds + ((nbs + 2) & ~1u));
    for (uint32_t k = threadIdx.x; k < ne; k += 1024) lent[k] = ent[e0 + k];
    __syncthreads();
  }
  const uint32_t s0 = ps[p], s1 = ps[p + 1];
  uint32_t x = 0;
  for (uint32_t base = s0; base < s1; base += 1024 * 12) {
    uint64_t v[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const uint32_t i = base + j * 1024 + threadIdx.x;
      v[j] = i < s1 ? __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(pairs + i)) : 0ull;
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const uint32_t i = base + j * 1024 + threadIdx.x;
      if (STAGE) x += lds[uint32_t(v[j]) % (nbs + 1)];
      if (i < s1) __builtin_nontemporal_store(v[j] ^ x, reinterpret_cast<uint64_t*>(out + i));
    }
  }
}

// streaming floor of the scatter: read the AoS key, hash, write (hash,row) in place
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
  uint2* out;
  CK(hipMalloc(&out, nS * 8));
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
    printf("%-28s %8.3f ms  %7.0f GB/s (alg)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  // the real probe (partition + probe); afterwards the scratch holds the partitioned pairs
  ctx.timing = false;
  timeit("radix_probe dense (all)", [&] { CK(radix_probe(&ctx, &t, rs, HJ3D_PROBE_UNIQUE | HJ3D_PROBE_EMIT, out, nS, res, 0)); }, nS * 28.0);
  // reconstruct the probe plan
  const double fill = double(nR) / nR;
  uint32_t W = uint32_t(0.8 * kProbeLdsWords / (1.0 + 2.0 * fill));
  const Plan pl = plan_for(nR, W, nS);
  const uint2* pairs = ctx.scratch[kScrPairs].as<uint2>();
  const uint32_t* ps = ctx.scratch[kScrPStart].as<uint32_t>();
  uint64_t* partials = ctx.scratch[kScrPartial].as<uint64_t>();
  uint32_t splits = 1;
  if (pl.P < uint32_t(ctx.num_cus) * 2) splits = (uint32_t(ctx.num_cus) * 2 + pl.P - 1) / pl.P;
  printf("P=%u W=%u splits=%u ntiles=%u\n", pl.P, pl.W, splits, pl.ntiles);
  const double pb = nS * 16.0 + nR * 12.0;
  timeit("k_rp_probe dense", [&] { launch_probe<true, kDense>(&t, pl, splits, pairs, ps, out, nS, nullptr, partials, false, 0); }, pb);
  timeit("k_rp_probe agg", [&] { launch_probe<true, kAgg>(&t, pl, splits, pairs, ps, nullptr, 0, nullptr, partials, false, 0); }, nS * 8.0 + nR * 12.0);
  timeit("copy (no stage)", [&] { hipLaunchKernelGGL(k_copy<false>, dim3(pl.P), dim3(1024), 0, 0, pairs, ps, t.off.as<const uint32_t>(), t.ent.as<const uint2>(), nR, pl.W, out); }, pb);
  timeit("copy + stage + 1 lds", [&] { hipLaunchKernelGGL(k_copy<true>, dim3(pl.P), dim3(1024), 0, 0, pairs, ps, t.off.as<const uint32_t>(), t.ent.as<const uint2>(), nR, pl.W, out); }, pb);
  // scatter side
  uint2* pout = ctx.scratch[kScrPairs].as<uint2>();
  timeit("partition_pairs (hist+scan+scatter)", [&] { CK(partition_pairs(&ctx, &t, rs, pl, pout, ctx.scratch[kScrPStart].as<uint32_t>(), 0)); }, nS * 32.0);
  const RelView v = view_of(rs);
  const uint32_t* hist = ctx.scratch[kScrPHist].as<uint32_t>();
  const uint32_t g = pl.ntiles < uint32_t(ctx.num_cus) ? pl.ntiles : uint32_t(ctx.num_cus);
  timeit("k_rp_scatter", [&] { hipLaunchKernelGGL(k_rp_scatter, dim3(g), dim3(kPBlock), 0, 0, v, t.fm, 0u, nR, pl.fw, pl.P, pl.ntiles, hist, pout); }, nS * 20.0);
  timeit("k_rp_hist", [&] { hipLaunchKernelGGL(k_rp_hist, dim3(pl.ntiles), dim3(kPBlock), 0, 0, v, t.fm, 0u, nR, pl.fw, pl.P, pl.ntiles, const_cast<uint32_t*>(hist)); }, nS * 12.0);
  for (unsigned gg : {256u, 512u, 1024u, 2048u})
    timeit(gg == 256 ? "stream pairs g=256" : gg == 512 ? "stream pairs g=512" : gg == 1024 ? "stream pairs g=1024" : "stream pairs g=2048",
           [&] { hipLaunchKernelGGL(k_stream_pairs, dim3(gg), dim3(1024), 0, 0, v, out); }, nS * 20.0);
  // restore the partitioned pairs for any later use and check nothing faulted
  CK(hipDeviceSynchronize());
  printf("ok\n");
  return 0;
}

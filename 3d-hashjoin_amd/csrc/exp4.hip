// exp4.hip — the experiment-4 probe strand: R probes the table on S, then (keyed by the same
// R.k) the table on T; results are triples (r, s, t).
//
//   Ndu (nested tables, main_experiment4.cc:831-941): AlgNestJoinProbe(S) -> AlgNestJoinProbe(T)
//       -> AlgUnnestHt(T) -> AlgUnnestHt(S) -> AlgTop. The S matches stay nested until T also
//       matched ("deferred unnesting"), so R tuples that fail the second join never expand S.
//   Chj (chaining tables, main_experiment4.cc:943-1043): AlgHashJoinProbe(S) emits every (r,s)
//       pair, and each pair probes T (full chain walk, no early exit).
// Counters are the reference's CSV columns; with the GPU layouts they are closed forms per r:
//   Ndu: cmps as nested probes; unnest_1 += |T(k)|; unnest_2 = top += |S(k)|*|T(k)|
//   Chj: c_probe_rs += mS; cmp_rs += nS; cmp_rt += mS*nT (only if T's bucket is non-empty);
//        c_probe_rt = top += mS*mT
// Triples are enumerated only for the checksums; products above kInline2 are handed to whole
// workgroups (heavy queue), as in nested.hip.
#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

constexpr int kItems = 2;
constexpr uint64_t kInline2 = 64;
constexpr int kF = 12;  // c_probe_rs, cmp_rs, c_probe_rt, cmp_rt, unnest_1, unnest_2, top, sum_a, sum_b, sum_c, sum_h, xor_h

struct Heavy2 {
  uint32_t r;   // probe row
  uint32_t ms;  // S side: nested main index, or chaining bucket entry range start
  uint32_t mt;  // T side
  uint32_t pad;
};

__device__ __forceinline__ void add_triple(uint64_t (&a)[kF], uint32_t r, uint32_t s, uint32_t t) {
  a[7] += r;
  a[8] += s;
  a[9] += t;
  const uint64_t h = triple_hash(r, s, t);
  a[10] += h;
  a[11] ^= h;
}

struct NTab {  // nested table view
  const uint32_t* off;
  const uint4* mains;
  const uint32_t* sub;
  FastMod fm;
  uint32_t lo, nbl;
  // returns main index or kInvalid; adds the reference's comparison count to *cmps
  __device__ __forceinline__ uint32_t find(uint32_t h, uint64_t* cmps, uint4* M) const {
    const uint32_t b = fm.mod(h) - lo;
    if (b >= nbl) return kInvalid;
    const uint32_t s = off[b], e = off[b + 1];
    uint32_t found = kInvalid;
    for (uint32_t k = s; k < e; ++k) {
      const uint4 c = mains[k];
      if (c.x == h) { found = k; *M = c; break; }
    }
    if (found == kInvalid) { *cmps += e - s; return kInvalid; }
    uint32_t before = 0;
    for (uint32_t k = s; k < e; ++k) before += mains[k].y < M->y;
    *cmps += 1 + before;
    return found;
  }
};

struct CTab {  // chaining table view
  const uint32_t* off;
  const uint2* ent;
  FastMod fm;
  uint32_t lo, nbl;
  __device__ __forceinline__ void range(uint32_t h, uint32_t* s, uint32_t* e) const {
    const uint32_t b = fm.mod(h) - lo;
    *s = 0;
    *e = 0;
    if (b < nbl) { *s = off[b]; *e = off[b + 1]; }
  }
};

__global__ __launch_bounds__(kBlock) void k_ndu(RelView r, NTab S, NTab T, Heavy2* __restrict__ heavy,
                                                uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res) {
  uint64_t a[kF] = {0};
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < r.n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t h = murmur32(r.key(i));
    const uint32_t pr = r.row(i);
    uint4 MS, MT;
    const uint32_t ms = S.find(h, &a[1], &MS);
    if (ms == kInvalid) continue;
    a[0] += 1;
    const uint32_t mt = T.find(h, &a[3], &MT);
    if (mt == kInvalid) continue;
    a[2] += 1;
    a[4] += MT.w;
    const uint64_t prod = uint64_t(MS.w) * MT.w;
    a[5] += prod;
    a[6] += prod;
    if (prod <= kInline2) {
      for (uint32_t q = 0; q < MT.w; ++q) {
        const uint32_t tr = T.sub[MT.z + q];
        for (uint32_t p = 0; p < MS.w; ++p) add_triple(a, pr, S.sub[MS.z + p], tr);
      }
    } else {
      const uint64_t slot = atomicAdd(reinterpret_cast<unsigned long long*>(nheavy), 1ull);
      heavy[slot] = Heavy2{pr, ms, mt, 0};
    }
  }
  block_flush<kF, 1>(a, res);
}

__global__ __launch_bounds__(kBlock) void k_ndu_heavy(NTab S, NTab T, const Heavy2* __restrict__ heavy,
                                                      const uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res) {
  uint64_t a[kF] = {0};
  const uint64_t nh = *nheavy;
  for (uint64_t q = blockIdx.x; q < nh; q += gridDim.x) {
    const Heavy2 hv = heavy[q];
    const uint4 MS = S.mains[hv.ms], MT = T.mains[hv.mt];
    const uint64_t prod = uint64_t(MS.w) * MT.w;
    for (uint64_t k = threadIdx.x; k < prod; k += kBlock) {
      const uint32_t tq = uint32_t(k / MS.w), sq = uint32_t(k % MS.w);
      add_triple(a, hv.r, S.sub[MS.z + sq], T.sub[MT.z + tq]);
    }
  }
  block_flush<kF, 1>(a, res);
}

__global__ __launch_bounds__(kBlock) void k_chj(RelView r, CTab S, CTab T, Heavy2* __restrict__ heavy,
                                                uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res) {
  uint64_t a[kF] = {0};
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < r.n; i += uint64_t(gridDim.x) * kBlock) {
    const uint32_t h = murmur32(r.key(i));
    const uint32_t pr = r.row(i);
    uint32_t s0, s1, t0, t1;
    S.range(h, &s0, &s1);
    if (s0 == s1) continue;  // empty S bucket: no comparisons (algebra.hh:640-643)
    a[1] += s1 - s0;
    uint32_t mS = 0;
    for (uint32_t k = s0; k < s1; ++k) mS += S.ent[k].x == h;
    if (mS == 0) continue;
    a[0] += mS;
    T.range(h, &t0, &t1);
    if (t0 == t1) continue;
    a[3] += uint64_t(mS) * (t1 - t0);
    uint32_t mT = 0;
    for (uint32_t k = t0; k < t1; ++k) mT += T.ent[k].x == h;
    const uint64_t prod = uint64_t(mS) * mT;
    a[2] += prod;
    a[6] += prod;
    if (prod == 0) continue;
    if (prod <= kInline2) {
      for (uint32_t ks = s0; ks < s1; ++ks) {
        const uint2 es = S.ent[ks];
        if (es.x != h) continue;
        for (uint32_t kt = t0; kt < t1; ++kt) {
          const uint2 et = T.ent[kt];
          if (et.x == h) add_triple(a, pr, es.y, et.y);
        }
      }
    } else {
      const uint64_t slot = atomicAdd(reinterpret_cast<unsigned long long*>(nheavy), 1ull);
      heavy[slot] = Heavy2{pr, h, 0, 0};
    }
  }
  block_flush<kF, 1>(a, res);
}

// Heavy chaining products: the block walks the S bucket; its threads stride over the T bucket.
__global__ __launch_bounds__(kBlock) void k_chj_heavy(CTab S, CTab T, const Heavy2* __restrict__ heavy,
                                                      const uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res) {
  uint64_t a[kF] = {0};
  const uint64_t nh = *nheavy;
  for (uint64_t q = blockIdx.x; q < nh; q += gridDim.x) {
    const Heavy2 hv = heavy[q];
    const uint32_t h = hv.ms;
    uint32_t s0, s1, t0, t1;
    S.range(h, &s0, &s1);
    T.range(h, &t0, &t1);
    for (uint32_t ks = s0; ks < s1; ++ks) {
      const uint2 es = S.ent[ks];
      if (es.x != h) continue;
      for (uint32_t kt = t0 + threadIdx.x; kt < t1; kt += kBlock) {
        const uint2 et = T.ent[kt];
        if (et.x == h) add_triple(a, hv.r, es.y, et.y);
      }
    }
  }
  block_flush<kF, 1>(a, res);
}

}  // namespace

hipError_t probe2(hj3d_ctx* ctx, const hj3d_table* ts, const hj3d_table* tt, const hj3d_rel& r, uint32_t flags,
                  void* out, uint64_t out_cap, uint64_t* res, hipStream_t s) {
  (void)out;
  (void)out_cap;
  if (flags & HJ3D_PROBE_EMIT) return hipErrorNotSupported;
  if (r.n == 0) return hipSuccess;
  hipError_t e = ctx->scratch[kScrC].ensure(r.n * sizeof(Heavy2) + 16);
  if (e != hipSuccess) return e;
  uint64_t* nheavy = ctx->scratch[kScrC].as<uint64_t>();
  Heavy2* heavy = reinterpret_cast<Heavy2*>(nheavy + 2);
  if ((e = hipMemsetAsync(nheavy, 0, sizeof(uint64_t), s)) != hipSuccess) return e;
  const RelView v = view_of(r);
  const unsigned g = grid_for(ctx, r.n, kBlock * kItems);
  if (ts->desc.kind == HJ3D_NESTED) {
    NTab S{ts->off.as<const uint32_t>(), ts->main.as<const uint4>(), ts->sub.as<const uint32_t>(), ts->fm,
           uint32_t(ts->desc.bucket_lo), ts->nb_local};
    NTab T{tt->off.as<const uint32_t>(), tt->main.as<const uint4>(), tt->sub.as<const uint32_t>(), tt->fm,
           uint32_t(tt->desc.bucket_lo), tt->nb_local};
    hipLaunchKernelGGL(k_ndu, dim3(g), dim3(kBlock), 0, s, v, S, T, heavy, nheavy, res);
    hipLaunchKernelGGL(k_ndu_heavy, dim3(ctx->num_cus * 4), dim3(kBlock), 0, s, S, T, heavy, nheavy, res);
  } else {
    CTab S{ts->off.as<const uint32_t>(), ts->ent.as<const uint2>(), ts->fm, uint32_t(ts->desc.bucket_lo),
           ts->nb_local};
    CTab T{tt->off.as<const uint32_t>(), tt->ent.as<const uint2>(), tt->fm, uint32_t(tt->desc.bucket_lo),
           tt->nb_local};
    hipLaunchKernelGGL(k_chj, dim3(g), dim3(kBlock), 0, s, v, S, T, heavy, nheavy, res);
    hipLaunchKernelGGL(k_chj_heavy, dim3(ctx->num_cus * 4), dim3(kBlock), 0, s, S, T, heavy, nheavy, res);
  }
  return hipGetLastError();
}

}  // namespace hj3d

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
#include "radix_seg.hpp"

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

// One output triple: its row sums always (the unnest reads every sub row, as AlgUnnestHt::step,
// algebra.hh:510-541, produces every tuple), its hash only with HJ3D_PROBE_CHECKSUM (ck; the
// verification checksums, which the reference does not compute; two mix64 per triple).
__device__ __forceinline__ void add_triple(uint64_t (&a)[kF], uint32_t r, uint32_t s, uint32_t t, bool ck) {
  a[7] += r;
  a[8] += s;
  a[9] += t;
  if (ck) {
    const uint64_t h = triple_hash(r, s, t);
    a[10] += h;
    a[11] ^= h;
  }
}

struct NTab {  // nested table view
  const uint32_t* off;
  const uint4* mains;
  const uint32_t* sub;
  FastMod fm;
  uint32_t lo, nbl;
  // returns main index or kInvalid; adds the reference's comparison count to *cmps
  __device__ __forceinline__ uint32_t find(uint32_t h, uint64_t* cmps, uint4* M) const;
};

// Main record of hash h among M[s .. s+n) (one bucket), or kInvalid; adds the reference's
// comparison count (findMainNodeByOther, ht_nested.hh:354-382) to *cmps. M: HBM or LDS.
template <typename MT>
__device__ __forceinline__ uint32_t nfind(uint32_t h, const MT* M, uint32_t s, uint32_t n, uint64_t* cmps, uint4* F) {
  uint32_t found = kInvalid;
  for (uint32_t k = s; k < s + n; ++k) {
    const uint4 c = M[k];
    if (c.x == h) { found = k; *F = c; break; }
  }
  if (found == kInvalid) { *cmps += n; return kInvalid; }
  uint32_t before = 0;
  for (uint32_t k = s; k < s + n; ++k) before += M[k].y < F->y;
  *cmps += 1 + before;
  return found;
}

__device__ __forceinline__ uint32_t NTab::find(uint32_t h, uint64_t* cmps, uint4* M) const {
  const uint32_t b = fm.mod(h) - lo;
  if (b >= nbl) return kInvalid;
  const uint32_t s = off[b];
  return nfind(h, mains, s, off[b + 1] - s, cmps, M);
}

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

// Triples of one light match (|S(k)| x |T(k)| <= kInline2): the sub rows are loaded in blocks
// of 8 into registers before they are combined, so a match costs one or two memory latencies
// instead of one per sub row.
__device__ __forceinline__ void light_triples(uint64_t (&a)[kF], uint32_t pr, const NTab& S, const NTab& T, uint32_t zs,
                                              uint32_t ws, uint32_t zt, uint32_t wt, bool ck) {
  constexpr uint32_t kB = 8;
  for (uint32_t qb = 0; qb < wt; qb += kB) {
    uint32_t tv[kB];
#pragma unroll
    for (uint32_t u = 0; u < kB; ++u) tv[u] = qb + u < wt ? T.sub[zt + qb + u] : 0u;
    for (uint32_t pb = 0; pb < ws; pb += kB) {
      uint32_t sv[kB];
#pragma unroll
      for (uint32_t u = 0; u < kB; ++u) sv[u] = pb + u < ws ? S.sub[zs + pb + u] : 0u;
#pragma unroll
      for (uint32_t qu = 0; qu < kB; ++qu) {
        if (qb + qu >= wt) break;
#pragma unroll
        for (uint32_t pu = 0; pu < kB; ++pu)
          if (pb + pu < ws) add_triple(a, pr, sv[pu], tv[qu], ck);
      }
    }
  }
}

// Ndu for one probe tuple after its two lookups (ms / mt: global main indices or kInvalid).
__device__ __forceinline__ void ndu_tail(uint64_t (&a)[kF], uint32_t pr, const NTab& S, const NTab& T, uint32_t ms,
                                         const uint4& MS, uint32_t mt, const uint4& MT, Heavy2* __restrict__ heavy,
                                         uint64_t* __restrict__ nheavy, bool ck) {
  a[2] += 1;
  a[4] += MT.w;
  const uint64_t prod = uint64_t(MS.w) * MT.w;
  a[5] += prod;
  a[6] += prod;
  if (prod <= kInline2) {
    light_triples(a, pr, S, T, MS.z, MS.w, MT.z, MT.w, ck);
  } else {
    const uint64_t slot = atomicAdd(reinterpret_cast<unsigned long long*>(nheavy), 1ull);
    heavy[slot] = Heavy2{pr, ms, mt, 0};
  }
}

// AlgNestJoinProbe(S) -> AlgNestJoinProbe(T) -> unnest both, for one probe tuple (HBM tables).
__device__ __forceinline__ void ndu_probe(uint64_t (&a)[kF], uint32_t h, uint32_t pr, const NTab& S, const NTab& T,
                                          Heavy2* __restrict__ heavy, uint64_t* __restrict__ nheavy, bool ck) {
  uint4 MS, MT;
  const uint32_t ms = S.find(h, &a[1], &MS);
  if (ms == kInvalid) return;
  a[0] += 1;
  const uint32_t mt = T.find(h, &a[3], &MT);
  if (mt == kInvalid) return;
  ndu_tail(a, pr, S, T, ms, MS, mt, MT, heavy, nheavy, ck);
}

__global__ __launch_bounds__(kBlock) void k_ndu(RelView r, NTab S, NTab T, Heavy2* __restrict__ heavy,
                                                uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res, bool ck) {
  uint64_t a[kF] = {0};
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < r.n; i += uint64_t(gridDim.x) * kBlock)
    ndu_probe(a, murmur32(r.key(i)), r.row(i), S, T, heavy, nheavy, ck);
  block_flush<kF, 1>(a, res);
}

// Partitioned Ndu (S and T tables with the same bucket function): the probe side is
// partitioned by bucket range (radix_partition_probe) and each partition's slices of BOTH
// tables (directories + main records) are staged in LDS; the lookups of both joins then run
// against LDS. FITS as in k_rp_probe_seg (false: the slices are read through L2).
template <bool FITS>
__global__ __launch_bounds__(kJBlock) void k_ndu_seg(const uint2* __restrict__ region, const uint32_t* __restrict__ counts,
                                                     const uint32_t* __restrict__ seg, uint32_t G, uint32_t cap, NTab S,
                                                     NTab T, uint32_t W, uint32_t P, uint32_t splits, bool flat,
                                                     Heavy2* __restrict__ heavy, uint64_t* __restrict__ nheavy,
                                                     uint64_t* __restrict__ res, bool ck) {
  __shared__ uint32_t lds[kProbeLdsWords];
  const uint32_t p = blockIdx.x / splits, sp = blockIdx.x % splits;
  const uint32_t b0 = p * W;
  const uint32_t nbs = min(W, S.nbl - b0);
  const uint32_t s0 = S.off[b0], ns = S.off[b0 + nbs] - s0;
  const uint32_t t0 = T.off[b0], nt = T.off[b0 + nbs] - t0;
  const uint32_t dirw = (2 * nbs + 4) & ~3u;  // both directories, then 16-B aligned main records
  const bool fits = dirw + 4ull * (ns + nt) <= kProbeLdsWords;
  if (fits != FITS) return;
  uint32_t* ldS = lds;
  uint32_t* ldT = lds + nbs;
  uint4* lmS = reinterpret_cast<uint4*>(lds + dirw);
  uint4* lmT = lmS + ns;
  uint64_t a[kF] = {0};
  seg_walk(region, counts, seg, G, cap, P, p, splits, sp, flat,
           [&] {
             if (FITS) {
               stage_nested(S.off, S.mains, b0, nbs, s0, ns, ldS, lmS);
               stage_nested(T.off, T.mains, b0, nbs, t0, nt, ldT, lmT);
             }
           },
           [&](uint32_t h, uint32_t pr, uint64_t) {
             if (!FITS) {
               ndu_probe(a, h, pr, S, T, heavy, nheavy, ck);
               return;
             }
             const uint32_t bl = S.fm.mod(h) - S.lo - b0;
             uint4 MS, MT;
             const uint32_t ds = ldS[bl];
             const uint32_t ms = nfind(h, lmS, ds >> 16, ds & 0xFFFFu, &a[1], &MS);
             if (ms == kInvalid) return;
             a[0] += 1;
             const uint32_t dt = ldT[bl];
             const uint32_t mt = nfind(h, lmT, dt >> 16, dt & 0xFFFFu, &a[3], &MT);
             if (mt == kInvalid) return;
             ndu_tail(a, pr, S, T, s0 + ms, MS, t0 + mt, MT, heavy, nheavy, ck);
           });
  block_flush<kF, 1>(a, res);
}

// Overflow pairs of the partition (runs that did not fit their region), against the HBM tables.
__global__ __launch_bounds__(kBlock) void k_ndu_ovf(const uint2* __restrict__ ovf, const unsigned long long* __restrict__ novf,
                                                    NTab S, NTab T, Heavy2* __restrict__ heavy,
                                                    uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res, bool ck) {
  uint64_t a[kF] = {0};
  const uint64_t n = *novf;
  for (uint64_t j = uint64_t(blockIdx.x) * kBlock + threadIdx.x; j < n; j += uint64_t(gridDim.x) * kBlock)
    ndu_probe(a, ovf[j].x, ovf[j].y, S, T, heavy, nheavy, ck);
  block_flush<kF, 1>(a, res);
}

__global__ __launch_bounds__(kBlock) void k_ndu_heavy(NTab S, NTab T, const Heavy2* __restrict__ heavy,
                                                      const uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res,
                                                      bool ck) {
  uint64_t a[kF] = {0};
  const uint64_t nh = *nheavy;
  for (uint64_t q = blockIdx.x; q < nh; q += gridDim.x) {
    const Heavy2 hv = heavy[q];
    const uint4 MS = S.mains[hv.ms], MT = T.mains[hv.mt];
    const uint64_t prod = uint64_t(MS.w) * MT.w;
    for (uint64_t k = threadIdx.x; k < prod; k += kBlock) {
      const uint32_t tq = uint32_t(k / MS.w), sq = uint32_t(k % MS.w);
      add_triple(a, hv.r, S.sub[MS.z + sq], T.sub[MT.z + tq], ck);
    }
  }
  block_flush<kF, 1>(a, res);
}

__global__ __launch_bounds__(kBlock) void k_chj(RelView r, CTab S, CTab T, Heavy2* __restrict__ heavy,
                                                uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res, bool ck) {
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
          if (et.x == h) add_triple(a, pr, es.y, et.y, ck);
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
                                                      const uint64_t* __restrict__ nheavy, uint64_t* __restrict__ res,
                                                      bool ck) {
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
        if (et.x == h) add_triple(a, hv.r, es.y, et.y, ck);
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
  const bool ck = flags & HJ3D_PROBE_CHECKSUM;  // triple hashes (sum_h, xor_h); row sums always
  // the result slot and the heavy-item counter start at zero: one launch clears both (with the
  // partitioner's own counters on the partitioned path)
  ZeroList z;
  z.add(res, kResFields);
  if (r.n == 0) return zero_words(z, s);
  hipError_t e = ctx->scratch[kScrC].ensure(r.n * sizeof(Heavy2) + 16);
  if (e != hipSuccess) return e;
  uint64_t* nheavy = ctx->scratch[kScrC].as<uint64_t>();
  Heavy2* heavy = reinterpret_cast<Heavy2*>(nheavy + 2);
  z.add(nheavy, 1);
  const RelView v = view_of(r);
  const unsigned g = grid_for(ctx, r.n, kBlock * kItems);
  if (ts->desc.kind == HJ3D_NESTED) {
    NTab S{ts->off.as<const uint32_t>(), ts->main.as<const uint4>(), ts->sub.as<const uint32_t>(), ts->fm,
           uint32_t(ts->desc.bucket_lo), ts->nb_local};
    NTab T{tt->off.as<const uint32_t>(), tt->main.as<const uint4>(), tt->sub.as<const uint32_t>(), tt->fm,
           uint32_t(tt->desc.bucket_lo), tt->nb_local};
    // partitioned when both tables share the bucket function (and their main counts are known)
    const bool same = ts->desc.num_buckets == tt->desc.num_buckets && ts->desc.bucket_lo == tt->desc.bucket_lo &&
                      ts->nb_local == tt->nb_local;
    e = hipErrorNotSupported;
    if (same && radix_nested_applicable(ctx, ts, r.n) && radix_nested_applicable(ctx, tt, r.n)) {
      const double fill = double(ts->n_mains + tt->n_mains) / double(ts->nb_local);
      ProbeParts pp;
      // no output: the regions' output slots are not needed
      e = radix_partition_probe(ctx, ts, r, uint32_t(0.8 * kProbeLdsWords / (2.0 + 4.0 * fill)), &pp, s, nullptr,
                                nullptr, false, &z);
      if (e == hipSuccess) {
        const uint32_t nblocks = pp.P * pp.splits;
        hipLaunchKernelGGL(k_ndu_seg<true>, dim3(nblocks), dim3(kJBlock), 0, s, pp.region, pp.counts, pp.seg, pp.G,
                           pp.cap, S, T, pp.W, pp.P, pp.splits, pp.flat, heavy, nheavy, res, ck);
        hipLaunchKernelGGL(k_ndu_seg<false>, dim3(nblocks), dim3(kJBlock), 0, s, pp.region, pp.counts, pp.seg, pp.G,
                           pp.cap, S, T, pp.W, pp.P, pp.splits, pp.flat, heavy, nheavy, res, ck);
        hipLaunchKernelGGL(k_ndu_ovf, dim3(ctx->num_cus), dim3(kBlock), 0, s, pp.ovf, pp.novf, S, T, heavy, nheavy,
                           res, ck);
      }
    }
    if (e == hipErrorNotSupported) {
      if ((e = zero_words(z, s)) != hipSuccess) return e;
      hipLaunchKernelGGL(k_ndu, dim3(g), dim3(kBlock), 0, s, v, S, T, heavy, nheavy, res, ck);
    } else if (e != hipSuccess) {
      return e;
    }
    hipLaunchKernelGGL(k_ndu_heavy, dim3(ctx->num_cus * 4), dim3(kBlock), 0, s, S, T, heavy, nheavy, res, ck);
  } else {
    if ((e = zero_words(z, s)) != hipSuccess) return e;
    CTab S{ts->off.as<const uint32_t>(), ts->ent.as<const uint2>(), ts->fm, uint32_t(ts->desc.bucket_lo),
           ts->nb_local};
    CTab T{tt->off.as<const uint32_t>(), tt->ent.as<const uint2>(), tt->fm, uint32_t(tt->desc.bucket_lo),
           tt->nb_local};
    hipLaunchKernelGGL(k_chj, dim3(g), dim3(kBlock), 0, s, v, S, T, heavy, nheavy, res, ck);
    hipLaunchKernelGGL(k_chj_heavy, dim3(ctx->num_cus * 4), dim3(kBlock), 0, s, S, T, heavy, nheavy, res, ck);
  }
  return hipGetLastError();
}

}  // namespace hj3d

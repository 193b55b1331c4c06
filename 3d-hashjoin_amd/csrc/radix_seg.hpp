// radix_seg.hpp — device side of the partitioned probe shared by the chaining probe (radix.hip)
// and the nested probe (nested.hip): the walk of one partition's regions.
//
// k_rp_part1 (radix.hip) leaves, for every partitioning workgroup g and partition p, a region of
// counts[g * P + p] (hash, row) pairs at region[(g * P + p) * cap]; seg[p * G + g] is the dense
// output slot of the region's first pair (exclusive scan, partition-major). A probe workgroup
// owns partition p (or one of `splits` shares of its regions) and stages the partition's table
// slice in LDS before probing.
#pragma once

#include "hj3d_internal.hpp"

namespace hj3d {

// Index of region (partitioning workgroup g, partition p) among the G * P regions: g-major, so a
// partitioning workgroup's regions are contiguous (a partition-major layout measured the same).
__host__ __device__ __forceinline__ uint64_t region_idx(uint32_t g, uint32_t p, uint32_t G, uint32_t P) {
  return uint64_t(g) * P + p;
}

constexpr int kJBlock = 1024;               // build / probe workgroups (16 waves, 1 per CU)
constexpr uint32_t kProbeLdsWords = 36864;  // 144 KB LDS table slice per probe workgroup
// the packed probe (chain_pk.hip): everything of the 160 KB LDS but its ~5.3 KB of walk state
constexpr uint32_t kPkLdsWords = 39552;
constexpr int kSegItems = 8;                // pairs per lane and step of the region walk (4, 12, 16: slower)

// Walks the regions of partition p assigned to share sp (of `splits`): wave w takes regions
// g = g_lo + w, g_lo + w + 16, ... (at most 64; lane r holds region r's pair count and output
// base) in chunks of 64 * kSegItems pairs, the next chunk in flight while the current one is
// probed. `stage()` runs once after the first chunk's loads are issued (table slice -> LDS) and
// is followed by a barrier; `probe(hash, row, slot)` is called for every pair.
// Long regions (a large probe side) are walked one region at a time. Short ones (`flat`: a small
// probe side leaves a few dozen pairs per region) are walked as ONE flattened stream so that
// every lane stays busy; the region of each 64-item block is then found with wave-uniform steps
// only (readlane of the lane holding region r): the block's first region advances
// monotonically and the region starts inside a block are few.
// CHUNK: `probe(v, slot, valid)` is called once per chunk with all kSegItems items of the lane
// (pair v[j], output slot slot[j], item j present iff bit j of valid), so that the probe can
// batch its LDS lookups across items.
template <bool CHUNK = false, class Stage, class Probe>
__device__ __forceinline__ void seg_walk(const uint2* __restrict__ region, const uint32_t* __restrict__ counts,
                                         const uint32_t* __restrict__ seg, uint32_t G, uint32_t cap, uint32_t P,
                                         uint32_t p, uint32_t splits, uint32_t sp, bool flat, Stage&& stage,
                                         Probe&& probe) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kWaves = kJBlock / kWave;
  const uint32_t g_lo = uint32_t(uint64_t(G) * sp / splits), g_hi = uint32_t(uint64_t(G) * (sp + 1) / splits);
  constexpr uint32_t kChunk = 64 * kSegItems;
  const uint32_t nr = g_hi > g_lo + wid ? (g_hi - g_lo - wid + kWaves - 1) / kWaves : 0u;  // <= 64 (G <= 1024)
  uint32_t my_len = 0, my_seg = 0;
  if (uint32_t(lane) < nr) {
    const uint32_t gg = g_lo + wid + kWaves * lane;
    my_len = counts[uint64_t(gg) * P + p];
    my_seg = seg[uint64_t(p) * G + gg];
  }
  if (flat) {
    uint32_t total;
    const uint32_t my_pre = wave_excl_scan(my_len, &total);  // stream offset of region `lane`
    auto pre_at = [&](uint32_t r) { return uint32_t(__builtin_amdgcn_readlane(int(my_pre), int(r))); };
    auto seg_at = [&](uint32_t r) { return uint32_t(__builtin_amdgcn_readlane(int(my_seg), int(r))); };
    uint32_t rb = 0;  // wave-uniform: last region starting at or before the current block
    auto load = [&](uint64_t (&v)[kSegItems], uint32_t (&slot)[kSegItems], uint32_t f0) {
  #pragma unroll
      for (int j = 0; j < kSegItems; ++j) {
        const uint32_t b = f0 + j * 64, f = b + lane;
        while (rb + 1 < nr && pre_at(rb + 1) <= b) ++rb;
        uint32_t r = rb, pr = pre_at(rb), sg = seg_at(rb);
        for (uint32_t t = rb + 1; t < nr; ++t) {  // region starts inside the block
          const uint32_t pt = pre_at(t);
          if (pt > b + 63) break;
          if (pt <= f) {
            r = t;
            pr = pt;
            sg = seg_at(t);
          }
        }
        const uint2* src = region + region_idx(g_lo + wid + kWaves * r, p, G, P) * cap;
        // unconditional (an absent item reads the region base): a fixed load count per chunk, so
        // waiting for it needs no vmcnt(0)
        const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(f < total ? src + (f - pr) : region));
        v[j] = f < total ? x : 0ull;
        slot[j] = sg + (f - pr);
      }
    };
    uint64_t cur[kSegItems];
    uint32_t cslot[kSegItems];
    load(cur, cslot, 0);
    stage();
    __syncthreads();
    for (uint32_t f0 = 0; f0 < total; f0 += kChunk) {
      uint64_t nxt[kSegItems];
      uint32_t nslot[kSegItems];
      if (f0 + kChunk < total) load(nxt, nslot, f0 + kChunk);
      if constexpr (CHUNK) {
        uint64_t sl[kSegItems];
        uint32_t vm = 0;
  #pragma unroll
        for (int j = 0; j < kSegItems; ++j) {
          sl[j] = cslot[j];
          vm |= uint32_t(f0 + j * 64 + lane < total) << j;
        }
        probe(cur, sl, vm);
      } else {
  #pragma unroll
        for (int j = 0; j < kSegItems; ++j)
          if (f0 + j * 64 + lane < total) probe(uint32_t(cur[j]), uint32_t(cur[j] >> 32), uint64_t(cslot[j]));
      }
  #pragma unroll
      for (int j = 0; j < kSegItems; ++j) {
        cur[j] = nxt[j];
        cslot[j] = nslot[j];
      }
    }
    return;
  }
  // wave-uniform cursor: region index r, offset q
  uint32_t r = 0, q = 0;
  uint32_t len = __shfl(my_len, 0, kWave);
  while (r < nr && len == 0) {
    ++r;
    len = __shfl(my_len, int(r & 63), kWave);
  }
  auto load = [&](uint64_t (&v)[kSegItems], uint32_t rr, uint32_t qq, uint32_t ll) {
    const uint2* src = region + region_idx(g_lo + wid + kWaves * rr, p, G, P) * cap;
#pragma unroll
    for (int j = 0; j < kSegItems; ++j) {
      const uint32_t k = qq + j * 64 + lane;
      const bool ok = rr < nr && k < ll;
      const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(ok ? src + k : region));
      v[j] = ok ? x : 0ull;
    }
  };
  uint64_t cur[kSegItems];
  load(cur, r, q, len);
  stage();
  __syncthreads();
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
    if constexpr (CHUNK) {
      uint64_t sl[kSegItems];
      uint32_t vm = 0;
#pragma unroll
      for (int j = 0; j < kSegItems; ++j) {
        sl[j] = obase + j * 64 + lane;
        vm |= uint32_t(q + j * 64 + lane < len) << j;
      }
      probe(cur, sl, vm);
    } else {
#pragma unroll
      for (int j = 0; j < kSegItems; ++j) {
        const uint32_t k = q + j * 64 + lane;
        if (k < len) probe(uint32_t(cur[j]), uint32_t(cur[j] >> 32), obase + j * 64 + lane);
      }
    }
    r = nr_;
    q = nq;
    len = nl;
#pragma unroll
    for (int j = 0; j < kSegItems; ++j) cur[j] = nxt[j];
  }
}

// Directory words (start << 16 | count, relative to the slice) then the main records of buckets
// [b0, b0 + nbs); all loads of a batch of kStage rounds are issued before the first LDS write.
__device__ __forceinline__ void stage_nested(const uint32_t* __restrict__ off, const uint4* __restrict__ mains,
                                             uint32_t b0, uint32_t nbs, uint32_t m0, uint32_t nm, uint32_t* ldir,
                                             uint4* lmain) {
  constexpr int kStage = 8;
  const uint32_t nmax = max(nbs, nm);
  for (uint32_t k0 = threadIdx.x; k0 < nmax; k0 += kJBlock * kStage) {
    uint32_t v[kStage], w[kStage];
    uint4 x[kStage];
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const uint32_t k = k0 + u * kJBlock;
      v[u] = k < nbs ? off[b0 + k] : 0u;
      w[u] = k < nbs ? off[b0 + k + 1] : 0u;
      x[u] = k < nm ? mains[m0 + k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const uint32_t k = k0 + u * kJBlock;
      if (k < nbs) ldir[k] = ((v[u] - m0) << 16) | (w[u] - v[u]);
      if (k < nm) lmain[k] = x[u];
    }
  }
}

}  // namespace hj3d

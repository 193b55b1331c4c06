// hj3d_device.hpp — device-side building blocks shared by the hj3d kernels (gfx950 / CDNA4).
//
// Everything on the join path is integer work: u32 keys, murmur3 fmix32 hashes, a u32
// modulo by a runtime (non power of two) bucket count, u32 row ids and u64 counters.
// No MFMA anywhere; the kernels are HBM / Infinity-Cache bound.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hj3d {

constexpr int kWave = 64;  // CDNA wavefront

// murmur3 fmix32 — ht::murmur_hash<uint32_t> (util/hasht.hh:52-61). A bijection on u32,
// so equal hashes imply equal u32 keys (the reference's joinpred after the hash compare is
// therefore implied).
__host__ __device__ __forceinline__ uint32_t murmur32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// splitmix64 finalizer and the pair/triple hashes used for order-independent output checksums
// (same definitions as oracle/hj3d_oracle.c and include/hj3d.h).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t pair_hash(uint32_t a, uint32_t b) {
  return mix64((uint64_t(a) << 32) | uint64_t(b));
}
__host__ __device__ __forceinline__ uint64_t triple_hash(uint32_t a, uint32_t b, uint32_t c) {
  return mix64(pair_hash(a, b) ^ uint64_t(c));
}

// Exact a % d for u32 a and 1 <= d < 2^32 without a division (Lemire, Kaser, Kurz 2019:
// M = ceil(2^64 / d); a % d = ((M * a mod 2^64) * d) >> 64). The reference computes
// `hash % numBuckets` with a 64-bit division per tuple (ht_chaining.hh:139-140).
struct FastMod {
  uint64_t m;
  uint32_t d;
  static FastMod make(uint32_t d) {
    FastMod f;
    f.d = d;
    f.m = (d <= 1) ? 0 : (~uint64_t(0) / d + 1);
    return f;
  }
  __device__ __forceinline__ uint32_t mod(uint32_t a) const {
    const uint64_t low = m * uint64_t(a);
    return uint32_t(__umul64hi(low, uint64_t(d)));
  }
};

// Exact n / d for u32 n and 2 <= d < 2^32 with one 32-bit high multiply (the branch-free form of
// division by an invariant integer, Granlund & Montgomery 1994): q = mulhi(magic, n),
// n / d = (((n - q) >> 1) + q) >> shift. Powers of two take magic = 0.
struct FastDiv32 {
  uint32_t magic = 0, shift = 0;
  static FastDiv32 make(uint32_t d) {
    FastDiv32 f;
    const uint32_t L = 31u - uint32_t(__builtin_clz(d));
    if ((d & (d - 1)) == 0) {
      f.shift = L - 1;
      return f;
    }
    const uint64_t num = uint64_t(1) << (32 + L);
    uint32_t m = uint32_t(num / d);
    const uint32_t rem = uint32_t(num % d);
    m += m;
    const uint32_t twice = rem + rem;
    if (twice >= d || twice < rem) m += 1;
    f.magic = m + 1;
    f.shift = L;
    return f;
  }
  __host__ __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint32_t q = uint32_t((uint64_t(magic) * n) >> 32);
    return (((n - q) >> 1) + q) >> shift;
  }
};

// Device view of an hj3d_rel (AoS tuples in HBM).
struct RelView {
  const char* base;
  uint64_t n;
  uint32_t stride;
  uint32_t key_off;
  uint32_t row_off;  // 0xFFFFFFFF = implicit
  uint32_t pad;
  uint64_t row_base;

  __device__ __forceinline__ uint32_t key(uint64_t i) const {
    return *reinterpret_cast<const uint32_t*>(base + i * stride + key_off);
  }
  __device__ __forceinline__ uint32_t row(uint64_t i) const {
    if (row_off == 0xFFFFFFFFu) return uint32_t(row_base + i);
    return __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(base + i * stride + row_off));
  }
};

// Counters of one probe strand, accumulated per thread, reduced per block, then one device
// atomic per field per block (Guideline 12: per-block partial reduction first).
struct ProbeAcc {
  uint64_t n_probe, n_matched, n_out, n_cmps, sum_a, sum_b, sum_c, sum_h, xor_h;
};
constexpr int kResFields = 16;   // u64 words of the context's result slot (hj3d_probe_result + marks)
constexpr int kProbeFields = 9;  // xor_h is the last field (reduced with xor)

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ uint64_t wave_xor(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const uint64_t w = __shfl_xor(v, o, kWave); v = w < v ? w : v; }
  return v;
}
__device__ __forceinline__ uint64_t wave_max(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const uint64_t w = __shfl_xor(v, o, kWave); v = w > v ? w : v; }
  return v;
}

// Block-reduce `nf` u64 fields (last `nxor` of them with xor, the rest with +) and add
// them to dst with one atomic per field. Block size must be a multiple of 64, <= 1024.
template <int NF, int NXOR>
__device__ __forceinline__ void block_flush(const uint64_t (&v)[NF], uint64_t* dst) {
  __shared__ uint64_t red[16][NF];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint64_t w[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) w[f] = (f >= NF - NXOR) ? wave_xor(v[f]) : wave_sum(v[f]);
  if (lane == 0) {
#pragma unroll
    for (int f = 0; f < NF; ++f) red[wid][f] = w[f];
  }
  __syncthreads();
  if (threadIdx.x < NF) {
    const int f = threadIdx.x;
    uint64_t acc = 0;
    for (int k = 0; k < nw; ++k) acc = (f >= NF - NXOR) ? (acc ^ red[k][f]) : (acc + red[k][f]);
    if (acc != 0) {
      if (f >= NF - NXOR) atomicXor(reinterpret_cast<unsigned long long*>(dst + f), acc);
      else atomicAdd(reinterpret_cast<unsigned long long*>(dst + f), acc);
    }
  }
}

// Block-reduce NF u64 fields (last NXOR with xor) and store the block's totals to
// dst_row[0..NF) without atomics (per-block partials, summed by reduce_partials: deterministic
// and free of same-address atomic serialisation, ~12 ns per same-line atomic on MI355X).
template <int NF, int NXOR>
__device__ __forceinline__ void block_store(const uint64_t (&v)[NF], uint64_t* dst_row) {
  __shared__ uint64_t red[16][NF];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint64_t w[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) w[f] = (f >= NF - NXOR) ? wave_xor(v[f]) : wave_sum(v[f]);
  if (lane == 0) {
#pragma unroll
    for (int f = 0; f < NF; ++f) red[wid][f] = w[f];
  }
  __syncthreads();
  if (threadIdx.x < NF) {
    const int f = threadIdx.x;
    uint64_t acc = 0;
    for (int k = 0; k < nw; ++k) acc = (f >= NF - NXOR) ? (acc ^ red[k][f]) : (acc + red[k][f]);
    dst_row[f] = acc;
  }
}

// Exclusive prefix sum over a wave (64 lanes) of u32 values; returns the wave total in *total.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
  const int lane = threadIdx.x & 63;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  *total = __shfl(x, 63, kWave);
  return x - v;
}

}  // namespace hj3d

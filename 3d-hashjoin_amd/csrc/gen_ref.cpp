// gen_ref.cpp — the reference's own input generators, bit-exact, on the host.
//
// The reference draws every input column from ONE sequential std::mt19937 stream (default seed
// 5489): Experiment1::init (main_experiment1.cc:415-457) shuffles R.k = iota(|R|) with
// std::shuffle, draws S.a with GenRandIntVec::generate_uni (util/GenRandIntVec.cc:72-98:
// uniform_int_distribution<int>(0, fkMax-1)) or generate_zipf (:167-200: zipf_distribution,
// util/zipf_distribution.hh:48-58, value - 1), then vec_permute's S.a (:335-340);
// Experiment4::init (main_experiment4.cc:517-575) shuffles the FK blocks with std::shuffle. The
// distributions are libstdc++ 11's (bits/uniform_int_dist.h:241-330 Lemire downscaling,
// bits/stl_algo.h:3706-3792 shuffle, bits/random.tcc generate_canonical<double,53>) and the
// Zipf sampler calls glibc libm. This file re-implements that stream for the engine's own full-size
// runs (config B / C / E relations equal to the reference's, so counters can be compared with the
// reference's at the headline sizes) and is built for speed rather than as a transcription:
//   * the Mersenne twister refills its 624-word state block at a time, without modulo indexing;
//   * Fisher-Yates swap positions do not depend on the array, so they are drawn a block ahead and
//     the swapped cache lines prefetched (the swaps are a random walk over up to 400 MB);
//   * each Zipf attempt consumes exactly two words (generate_canonical), so attempt m always reads
//     stream words (2m, 2m+1) of the Zipf phase: all attempts of a block are evaluated in parallel
//     threads and the accepted ones kept in order, then the twister is re-advanced to exactly the
//     words the sequential sampler would have consumed.
// Compiled with g++ -O2 -ffp-contract=off (no FMA contraction: the Zipf arithmetic must round as the
// reference binary's does). Host-only, synchronous; no GPU is touched.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "hj3d.h"

namespace {

class Twister {  // std::mt19937 (MT19937, 32-bit), default seed 5489
 public:
  explicit Twister(uint32_t seed = 5489u) {
    s_[0] = seed;
    for (uint32_t i = 1; i < kN; ++i) s_[i] = 1812433253u * (s_[i - 1] ^ (s_[i - 1] >> 30)) + i;
    pos_ = kN;
  }
  uint32_t operator()() {
    if (pos_ == kN) refill();
    uint32_t y = s_[pos_++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    return y ^ (y >> 18);
  }
  void discard(uint64_t n) {
    while (n) {
      if (pos_ == kN) refill();
      const uint64_t k = std::min<uint64_t>(n, kN - pos_);
      pos_ += uint32_t(k);
      n -= k;
    }
  }
  void fill(uint32_t* out, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) out[i] = (*this)();
  }

 private:
  static constexpr uint32_t kN = 624, kM = 397;
  static uint32_t twist(uint32_t hi, uint32_t lo, uint32_t far) {
    const uint32_t y = (hi & 0x80000000u) | (lo & 0x7fffffffu);
    return far ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  void refill() {
    uint32_t k = 0;
    for (; k < kN - kM; ++k) s_[k] = twist(s_[k], s_[k + 1], s_[k + kM]);
    for (; k < kN - 1; ++k) s_[k] = twist(s_[k], s_[k + 1], s_[k + kM - kN]);
    s_[kN - 1] = twist(s_[kN - 1], s_[0], s_[kM - 1]);
    pos_ = 0;
  }
  uint32_t s_[kN];
  uint32_t pos_;
};

// uniform_int_distribution<u32/size_t>(0, range-1) over a 32-bit engine (Lemire, libstdc++ 11).
// range == 2^32 (urange == engine range) takes the raw word.
inline uint32_t draw_below(Twister& g, uint64_t range) {
  if (range > 0xffffffffull) return g();
  const uint32_t r = uint32_t(range);
  uint64_t prod = uint64_t(g()) * r;
  if (uint32_t(prod) < r) {
    const uint32_t thresh = (0u - r) % r;
    while (uint32_t(prod) < thresh) prod = uint64_t(g()) * r;
  }
  return uint32_t(prod >> 32);
}

constexpr int kAhead = 512;  // swap positions drawn per block
constexpr int kPf = 24;      // prefetch distance (swaps)

inline void swap_at(uint32_t* v, uint64_t i, uint64_t j) {
  const uint32_t t = v[i];
  v[i] = v[j];
  v[j] = t;
}

// std::shuffle of v[0, n) (bits/stl_algo.h:3729-3792).
void shuffle(uint32_t* v, uint64_t n, Twister& g) {
  if (n < 2) {
    return;
  }
  if (0xffffffffull / n >= n) {  // small range: two positions per draw (__gen_two_uniform_ints)
    uint64_t i = 1;
    if (n % 2 == 0) swap_at(v, i++, draw_below(g, 2));
    while (i != n) {
      const uint64_t b0 = i + 1, b1 = i + 2;
      const uint64_t x = draw_below(g, b0 * b1);
      swap_at(v, i++, x / b1);
      swap_at(v, i++, x % b1);
    }
    return;
  }
  uint32_t js[kAhead];
  for (uint64_t i0 = 1; i0 < n; i0 += kAhead) {
    const int m = int(std::min<uint64_t>(kAhead, n - i0));
    for (int k = 0; k < m; ++k) js[k] = draw_below(g, i0 + k + 1);
    for (int k = 0; k < std::min(m, kPf); ++k) __builtin_prefetch(v + js[k], 1);
    for (int k = 0; k < m; ++k) {
      if (k + kPf < m) __builtin_prefetch(v + js[k + kPf], 1);
      swap_at(v, i0 + k, js[k]);
    }
  }
}

// GenRandIntVec::vec_permute (util/GenRandIntVec.cc:335-340): i = n-1 .. 1, swap(v[i], v[g() % i]).
void vec_permute(uint32_t* v, uint64_t n, Twister& g) {
  if (n < 2) return;
  uint64_t js[kAhead];
  for (uint64_t i0 = n - 1; i0 > 0;) {
    const int m = int(std::min<uint64_t>(kAhead, i0));
    for (int k = 0; k < m; ++k) {
      const uint64_t i = i0 - k;
      const uint32_t w = g();
      js[k] = i <= 0xffffffffull ? uint32_t(w % uint32_t(i)) : w % i;
    }
    for (int k = 0; k < std::min(m, kPf); ++k) __builtin_prefetch(v + js[k], 1);
    for (int k = 0; k < m; ++k) {
      if (k + kPf < m) __builtin_prefetch(v + js[k + kPf], 1);
      swap_at(v, i0 - k, js[k]);
    }
    i0 -= m;
  }
}

// zipf_distribution<uint, double>(n, q) (util/zipf_distribution.hh:22-147): rejection-inversion
// (Hoermann & Derflinger) with the hat integral H and its inverse.
struct Zipf {
  double q, H_x1, H_n;
  uint32_t n;
  static double expm1_over(double x) {
    return std::fabs(x) > 1e-8 ? std::expm1(x) / x : 1.0 + x / 2.0 * (1.0 + x / 3.0 * (1.0 + x / 4.0));
  }
  static double log1p_over(double x) {
    return std::fabs(x) > 1e-8 ? std::log1p(x) / x : 1.0 - x * ((1 / 2.0) - x * ((1 / 3.0) - x * (1 / 4.0)));
  }
  double H(double x) const {
    const double lx = std::log(x);
    return expm1_over((1.0 - q) * lx) * lx;
  }
  double H_inv(double x) const { return std::exp(log1p_over(std::max(-1.0, x * (1.0 - q))) * x); }
  double h(double x) const { return std::exp(-q * std::log(x)); }
  Zipf(uint32_t n_, double q_) : q(q_), n(n_) {
    H_x1 = H(1.5) - 1.0;
    H_n = H(double(n_) + 0.5);
  }
  // one attempt from the two words (lo, hi) of generate_canonical<double,53>; 0 = rejected
  uint32_t attempt(uint32_t lo, uint32_t hi) const {
    double r = (double(lo) + double(hi) * 4294967296.0) / 18446744073709551616.0;
    if (r >= 1.0) r = std::nextafter(1.0, 0.0);
    const double u = r * (H_n - H_x1) + H_x1;  // uniform_real_distribution(H_x1, H_n)
    const double x = H_inv(u);
    const double rx = std::round(x);
    uint32_t k = uint32_t(rx);
    k = std::max<uint32_t>(1u, std::min<uint32_t>(n, k));
    return u >= H(double(k) + 0.5) - h(double(k)) ? k : 0u;
  }
};

int worker_count(int threads) {
  if (threads > 0) return std::min(threads, 64);
  const unsigned hw = std::thread::hardware_concurrency();
  return int(std::max(1u, std::min(hw ? hw : 1u, 16u)));
}

template <class F>
void parallel_for(uint64_t n, int workers, F&& f) {
  if (workers <= 1 || n < 4096) {
    f(uint64_t(0), n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(workers);
  for (int w = 0; w < workers; ++w) {
    const uint64_t a = n * w / workers, b = n * (w + 1) / workers;
    th.emplace_back([&f, a, b] { f(a, b); });
  }
  for (auto& t : th) t.join();
}

// n Zipf values ((draw - 1) % fk_max, GenRandIntVec::genval_zipf) from g, leaving g exactly where
// the sequential sampler would.
void zipf_values(uint32_t* out, uint64_t n, uint32_t fk_max, double theta, Twister& g, int workers) {
  const Zipf z(fk_max, theta);
  constexpr uint64_t kBlock = uint64_t(1) << 22;  // attempts per block
  std::vector<uint32_t> words(2 * kBlock), res(kBlock);
  uint64_t done = 0;
  while (done < n) {
    const uint64_t want = n - done;
    // a few percent of the attempts are rejected: draw a little more than needed
    const uint64_t m = std::min<uint64_t>(kBlock, want + want / 16 + 64);
    Twister mark = g;
    g.fill(words.data(), 2 * m);
    parallel_for(m, workers, [&](uint64_t a, uint64_t b) {
      for (uint64_t i = a; i < b; ++i) res[i] = z.attempt(words[2 * i], words[2 * i + 1]);
    });
    uint64_t used = 0;
    for (; used < m && done < n; ++used)
      if (res[used]) out[done++] = (res[used] - 1u) % fk_max;
    if (used < m) {  // rewind to just after the last consumed attempt
      g = mark;
      g.discard(2 * used);
    }
  }
}

}  // namespace

extern "C" {

hj3d_status hj3d_gen_exp1_ref(uint64_t nR, uint64_t nS, int skew, double theta, uint32_t t, uint32_t* Rk,
                              uint32_t* Sa, int threads) {
  if ((nR && !Rk) || (nS && !Sa) || nR == 0 || nR > 0xffffffffull || nS > 0xffffffffull || t >= 32)
    return HJ3D_EINVAL;
  const uint32_t fk_max = uint32_t(nR >> t);  // Experiment1::getFkMax (main_experiment1.cc:190)
  if (fk_max == 0 || (skew && !(theta >= 0.0))) return HJ3D_EINVAL;
  Twister g;
  for (uint64_t i = 0; i < nR; ++i) Rk[i] = uint32_t(i);
  shuffle(Rk, nR, g);
  if (!skew) {
    for (uint64_t i = 0; i < nS; ++i) Sa[i] = draw_below(g, fk_max);
  } else {
    zipf_values(Sa, nS, fk_max, theta, g, worker_count(threads));
  }
  vec_permute(Sa, nS, g);
  return HJ3D_OK;
}

hj3d_status hj3d_gen_exp4_ref(uint32_t log2R, uint32_t alpha, uint32_t mult_a, uint32_t beta, uint32_t mult_b,
                              uint32_t* Sa, uint32_t* Ta, uint64_t* card) {
  if (log2R >= 32 || alpha >= 32 || beta >= 32) return HJ3D_EINVAL;
  const uint64_t nR = uint64_t(1) << log2R;
  const uint64_t n_common = nR >> alpha, n_excl = nR >> beta;  // numFkCommon / numFkExclusive
  const uint64_t c_common = n_common * mult_a, c_excl = n_excl * mult_b, total = c_common + c_excl;
  if (card) *card = total;
  if (!Sa || !Ta) return card ? HJ3D_OK : HJ3D_EINVAL;
  if (nR < n_common + 2 * n_excl) return HJ3D_EINVAL;  // Experiment4::init's assertion
  // blocks of repeated values: common [0, nc) x A, S-exclusive [nc, nc+ne) x B, T-exclusive after
  std::vector<uint32_t> common(c_common), ex_s(c_excl), ex_t(c_excl);
  for (uint64_t i = 0; i < c_common; ++i) common[i] = uint32_t(i / mult_a);
  for (uint64_t i = 0; i < c_excl; ++i) {
    ex_s[i] = uint32_t(n_common + i / mult_b);
    ex_t[i] = uint32_t(n_common + n_excl + i / mult_b);
  }
  Twister g;
  shuffle(ex_s.data(), c_excl, g);
  shuffle(ex_t.data(), c_excl, g);
  shuffle(common.data(), c_common, g);
  std::memcpy(Sa, common.data(), c_common * 4);
  std::memcpy(Sa + c_common, ex_s.data(), c_excl * 4);
  shuffle(common.data(), c_common, g);  // T gets the common block reshuffled
  std::memcpy(Ta, common.data(), c_common * 4);
  std::memcpy(Ta + c_common, ex_t.data(), c_excl * 4);
  return HJ3D_OK;
}

}  // extern "C"

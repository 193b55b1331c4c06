// ref_golden.cc — golden-fixture generator that drives the REAL reference code.
//
// TEST INFRASTRUCTURE ONLY (oracle/). This file is never part of the product path.
// It is compiled by oracle/Makefile against the read-only reference sources under
// $(REF) (/root/reference) and its binary lands in oracle/_ref/ (git-ignored).
// It #includes the reference's own hash tables / operators / generators; nothing
// from the reference is copied here. The functor structs below are this repo's own
// restatement of the experiment plumbing (hash on a field, equality on a field,
// concat into pointer pairs) so that the reference operators can be instantiated
// with an AlgTop whose print hook folds every output tuple into order-independent
// checksums.
//
// Reference entities exercised (file:line in /root/reference):
//   input generation   main_experiment1.cc:415-457, util/GenRandIntVec.cc:72-98,167-200,335-340
//                      main_experiment4.cc:517-575
//   chaining HT        ht_chaining.hh:181-196 (insert), 236-248 (probe dir), 260-292 (stats)
//   nested HT          ht_nested.hh:287-311 (insert), 354-382 (probe), 450-482 (stats)
//   operators          algebra.hh:247-275 (scan), 362-473 (nest build/probe), 489-552 (unnest),
//                      555-672 (chaining build/probe), 204-243 (top)
//
// Usage:
//   ref_golden exp1 <nR> <nS> <skew 0|1> <theta> <t> <b> [dump]
//   ref_golden exp4 <log2R> <alpha> <multA> <beta> <multB> [dump]
//   ref_golden time_csr <nR> <nS> <min_reps> [prefix]  (CPU baseline timing of the reference Csr plan,
//                                      repeat_mintime; probe side = the first `prefix` S tuples)
//   ref_golden time_nrs <nR> <nS> <theta> <reps>  (the same for the Nrs plan, Zipf FKs: config C)
//   ref_golden time_ndu <log2R> <a> <A> <b> <B> <reps>  (the experiment-4 Ndu plan: config E)
// Prints one JSON object on stdout. With "dump", the generated key columns are
// also emitted (small sizes only; used for generator known-answer fixtures).

#include "util/standard_includes.hh"

#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <unordered_set>

#include "util/GenRandIntVec.hh"
#include "util/hasht.hh"
#include "util/measure_helpers.hh"
#include "algebra.hh"
#include "ht_chaining.hh"
#include "ht_nested.hh"

namespace {

// ---- checksums shared with include/hj3d.h (HJ3D_MIX64 / pair / triple hashes) ----
inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
inline uint64_t pairHash(uint64_t a, uint64_t b) { return mix64((a << 32) | (b & 0xffffffffULL)); }
inline uint64_t tripleHash(uint64_t a, uint64_t b, uint64_t c) { return mix64(pairHash(a, b) ^ c); }
inline uint64_t colsum(const std::vector<uint32_t>& v) {
  uint64_t s = 0;
  for (size_t i = 0; i < v.size(); ++i) s += pairHash(i, v[i]);
  return s;
}

struct Agg {  // order-independent aggregate over emitted tuples
  uint64_t n = 0, sumA = 0, sumB = 0, sumC = 0, sumH = 0, xorH = 0;
  void add2(uint64_t a, uint64_t b) {
    ++n; sumA += a; sumB += b; const uint64_t h = pairHash(a, b); sumH += h; xorH ^= h;
  }
  void add3(uint64_t a, uint64_t b, uint64_t c) {
    ++n; sumA += a; sumB += b; sumC += c; const uint64_t h = tripleHash(a, b, c); sumH += h; xorH ^= h;
  }
};

std::ostream gNull(nullptr);

void printStats(const HtStatistics& s) {
  std::printf("\"stats\":{\"nb\":%zu,\"empty\":%zu,\"entries\":%zu,\"distinct\":%zu,"
              "\"cc0_min\":%zu,\"cc0_max\":%zu,\"cc0_sum\":%zu,\"cc0_cnt\":%zu,"
              "\"cc1_min\":%zu,\"cc1_max\":%zu,\"cc1_sum\":%zu,\"cc1_cnt\":%zu,"
              "\"frac_empty\":%.17g,\"cc0_avg\":%.17g,\"cc1_avg\":%.17g}",
              s._numBuckets, s._numEmptyBuckets, s._numEntries, s._numDistinctKeys,
              s._collisionChainLen.min(), s._collisionChainLen.max(), s._collisionChainLen.sum(),
              s._collisionChainLen.count(),
              s._collisionChainLenNonempty.min(), s._collisionChainLenNonempty.max(),
              s._collisionChainLenNonempty.sum(), s._collisionChainLenNonempty.count(),
              s.fracEmptyBuckets(), s._collisionChainLen.avg(), s._collisionChainLenNonempty.avg());
}

void printAgg(const char* name, const Agg& a) {
  std::printf("\"%s\":{\"n\":%" PRIu64 ",\"sum_a\":%" PRIu64 ",\"sum_b\":%" PRIu64
              ",\"sum_c\":%" PRIu64 ",\"sum_h\":%" PRIu64 ",\"xor_h\":%" PRIu64 "}",
              name, a.n, a.sumA, a.sumB, a.sumC, a.sumH, a.xorH);
}

void printHead(const char* name, const std::vector<uint32_t>& v, size_t k = 16) {
  std::printf("\"%s\":[", name);
  for (size_t i = 0; i < std::min(k, v.size()); ++i) std::printf("%s%u", i ? "," : "", v[i]);
  std::printf("]");
}

void printAll(const char* name, const std::vector<uint32_t>& v) { printHead(name, v, v.size()); }

// =============================== experiment 1 ===================================
namespace e1 {
struct Tup { uint32_t k, a, b; };
using hv_t = uint32_t;
inline hv_t H(uint32_t x) { return ht::murmur_hash<uint32_t>(x); }

struct GS {};
struct HashK { using input_t = Tup; using output_t = hv_t;
  static output_t eval(const input_t* t) { return H(t->k); } };
struct HashA { using input_t = Tup; using output_t = hv_t;
  static output_t eval(const input_t* t) { return H(t->a); } };
struct EqK { using left_t = Tup; using right_t = Tup;
  static bool eval(const left_t* l, const right_t* r) { return l->k == r->k; } };
struct EqA { using left_t = Tup; using right_t = Tup;
  static bool eval(const left_t* l, const right_t* r) { return l->a == r->a; } };
struct PredKA { using left_t = Tup; using right_t = Tup;   // probe R.k vs build S.a
  static bool eval(const left_t* l, const right_t* r) { return l->k == r->a; } };
struct PredAK { using left_t = Tup; using right_t = Tup;   // probe S.a vs build R.k
  static bool eval(const left_t* l, const right_t* r) { return l->a == r->k; } };

struct Pair { const Tup* _left; const Tup* _right; };
struct CatPair { using left_t = Tup; using right_t = Tup; using output_t = Pair;
  static output_t eval(left_t* l, const right_t* r) { return {l, r}; } };

template <typename Tmain> struct Nested { Tup* _left; const Tmain* _right; };
template <typename Tht> struct CatNested {
  using left_t = Tup; using right_t = typename Tht::MainNode; using output_t = Nested<right_t>;
  static output_t eval(left_t* l, const right_t* r) { return {l, r}; } };
template <typename Tht> struct Unnest {
  using input_t = Nested<typename Tht::MainNode>; using output_t = Pair;
  using MainNode = typename Tht::MainNode; using data_t = typename Tht::data_t;
  static const MainNode* getMainNode(input_t* n) { return n->_right; }
  static void eval_left(output_t* o, input_t* n) { o->_left = n->_left; }
  static void eval_right(output_t* o, input_t*, const data_t* d) { o->_right = d; }
};

// The reference operators stream their inputs in (compiled-out) trace statements.
inline std::ostream& operator<<(std::ostream& os, const Tup& t) { return os << t.k << "|" << t.a; }
inline std::ostream& operator<<(std::ostream& os, const Pair& p) { return os << p._left << p._right; }
template <typename M> std::ostream& operator<<(std::ostream& os, const Nested<M>& n) { return os << n._left; }

// chaining plan: build on `build`, probe with `probe`
template <typename HB, typename EB, typename HP, typename PP, bool Unique>
void planChaining(const char* name, RelationRS<Tup>& build, RelationRS<Tup>& probe, size_t nb) {
  using build_t = AlgHashJoinBuild<HB, EB, GS>;
  using top_t = AlgTop<Pair, GS>;
  using probe_t = AlgHashJoinProbe<top_t, build_t, HP, PP, CatPair, Unique>;
  GS gs;
  Agg agg;
  const Tup* bb = build._tuples.data();
  const Tup* pb = probe._tuples.data();
  build_t opBuild(nb, 10);
  AlgScan<build_t> scanB(&opBuild, &build);
  top_t top(gNull, true, [&](const Pair* p, std::ostream&) {
    agg.add2(static_cast<uint64_t>(p->_left - pb), static_cast<uint64_t>(p->_right - bb));
  });
  probe_t opProbe(&top, &opBuild);
  AlgScan<probe_t> scanP(&opProbe, &probe);
  scanB.run(&gs);
  scanP.run(&gs);
  std::printf("\"%s\":{\"nb\":%zu,\"c_build\":%" PRIu64 ",\"c_probe\":%" PRIu64
              ",\"c_cmp\":%" PRIu64 ",\"c_top\":%" PRIu64 ",",
              name, opBuild.hashtable().numBuckets(), opBuild.count(), opProbe.count(),
              opProbe.numCmps(), top.count());
  printStats(opBuild.hashtable().makeStatistics());
  std::printf(",");
  printAgg("out", agg);
  std::printf("}");
}

// nested plan: build on `build`, probe with `probe`, optional unnest
template <typename HB, typename EB, typename HP, typename PP>
void planNested(const char* name, RelationRS<Tup>& build, RelationRS<Tup>& probe, size_t nb, bool unnest) {
  using build_t = AlgNestJoinBuild<HB, EB, GS>;
  using ht_t = typename build_t::hashtable_t;
  using nested_t = Nested<typename ht_t::MainNode>;
  GS gs;
  Agg agg;
  const Tup* bb = build._tuples.data();
  const Tup* pb = probe._tuples.data();
  build_t opBuild(nb, 10, 10);
  AlgScan<build_t> scanB(&opBuild, &build);
  uint64_t cProbe = 0, cCmp = 0, cUnnest = 0, cTop = 0;
  if (unnest) {
    using top_t = AlgTop<Pair, GS>;
    using unnest_t = AlgUnnestHt<top_t, Unnest<ht_t>, ht_t>;
    using probe_t = AlgNestJoinProbe<unnest_t, build_t, HP, PP, CatNested<ht_t>>;
    top_t top(gNull, true, [&](const Pair* p, std::ostream&) {
      agg.add2(static_cast<uint64_t>(p->_left - pb), static_cast<uint64_t>(p->_right - bb));
    });
    unnest_t opUnnest(&top);
    probe_t opProbe(&opUnnest, &opBuild);
    AlgScan<probe_t> scanP(&opProbe, &probe);
    scanB.run(&gs);
    scanP.run(&gs);
    cProbe = opProbe.count(); cCmp = opProbe.numCmps(); cUnnest = opUnnest.count(); cTop = top.count();
  } else {
    using top_t = AlgTop<nested_t, GS>;
    using probe_t = AlgNestJoinProbe<top_t, build_t, HP, PP, CatNested<ht_t>>;
    top_t top(gNull, true, [&](const nested_t* p, std::ostream&) {
      agg.add2(static_cast<uint64_t>(p->_left - pb), static_cast<uint64_t>(p->_right->data() - bb));
    });
    probe_t opProbe(&top, &opBuild);
    AlgScan<probe_t> scanP(&opProbe, &probe);
    scanB.run(&gs);
    scanP.run(&gs);
    cProbe = opProbe.count(); cCmp = opProbe.numCmps(); cTop = top.count();
  }
  std::printf("\"%s\":{\"nb\":%zu,\"c_build\":%" PRIu64 ",\"c_probe\":%" PRIu64 ",\"c_cmp\":%" PRIu64
              ",\"c_unnest\":%" PRIu64 ",\"c_top\":%" PRIu64 ",",
              name, opBuild.hashtable().numBuckets(), opBuild.count(), cProbe, cCmp,
              unnest ? cUnnest : 0, cTop);
  printStats(opBuild.hashtable().makeStatistics());
  std::printf(",");
  printAgg("out", agg);
  std::printf("}");
}

int run(size_t nR, size_t nS, bool skew, double theta, uint32_t t, uint32_t b, bool dump, const std::string& only) {
  // Same generation sequence as main_experiment1.cc:415-457 (exact cardinalities instead of 2^x).
  std::mt19937 rng;
  std::vector<uint32_t> keysR(nR);
  for (size_t i = 0; i < nR; ++i) keysR[i] = static_cast<uint32_t>(i);
  std::shuffle(keysR.begin(), keysR.end(), rng);
  const uint32_t fkMax = static_cast<uint32_t>(nR >> t);
  std::vector<uint32_t> fk;
  GenRandIntVec griv;
  GenRandIntVec::param_t p = skew
      ? GenRandIntVec::param_t(GenRandIntVec::dist_t::kZipf, fkMax, 0, theta, 0, -1)
      : GenRandIntVec::param_t(GenRandIntVec::dist_t::kUni, fkMax, 0, 0.0, 0, -1);
  griv.generate(fk, static_cast<uint>(nS), p, rng);
  const size_t numDv = std::unordered_set<uint32_t>(fk.cbegin(), fk.cend()).size();

  RelationRS<Tup> R, S;
  R._tuples.resize(nR);
  for (size_t i = 0; i < nR; ++i) R._tuples[i] = Tup{keysR[i], 0, 0};
  S._tuples.resize(nS);
  for (size_t i = 0; i < nS; ++i) S._tuples[i] = Tup{static_cast<uint32_t>(i), fk[i], 0};

  const size_t nbR = std::max<size_t>(nR / b, 1);
  const size_t nbS = std::max<size_t>(numDv / b, 1);

  std::printf("{\"exp\":1,\"nR\":%zu,\"nS\":%zu,\"skew\":%d,\"theta\":%.17g,\"t\":%u,\"b\":%u,"
              "\"fkMax\":%u,\"numDvSa\":%zu,\"colsum_Rk\":%" PRIu64 ",\"colsum_Sa\":%" PRIu64 ",",
              nR, nS, skew ? 1 : 0, theta, t, b, fkMax, numDv, colsum(keysR), colsum(fk));
  printHead("head_Rk", keysR);
  std::printf(",");
  printHead("head_Sa", fk);
  std::printf(",");
  if (dump) {
    printAll("Rk", keysR);
    std::printf(",");
    printAll("Sa", fk);
    std::printf(",");
  }
  // `only` (comma-separated plan names, empty = all) restricts the plans, for the largest inputs
  const auto want = [&](const char* plan) { return only.empty() || ("," + only + ",").find(std::string(",") + plan + ",") != std::string::npos; };
  bool first = true;
  const auto sep = [&]() { if (!first) std::printf(","); first = false; };
  std::printf("\"plans\":{");
  if (want("Csr")) { sep(); planChaining<HashK, EqK, HashA, PredAK, true>("Csr", R, S, nbR); }
  if (want("CsrUU")) { sep(); planChaining<HashK, EqK, HashA, PredAK, false>("CsrUU", R, S, nbR); }
  if (want("Crs")) { sep(); planChaining<HashA, EqA, HashK, PredKA, false>("Crs", S, R, nbS); }
  if (want("Nsr")) { sep(); planNested<HashK, EqK, HashA, PredAK>("Nsr", R, S, nbR, true); }
  if (want("Nrs")) { sep(); planNested<HashA, EqA, HashK, PredKA>("Nrs", S, R, nbS, true); }
  if (want("NrsNU")) { sep(); planNested<HashA, EqA, HashK, PredKA>("NrsNU", S, R, nbS, false); }
  std::printf("}}\n");
  return 0;
}

// CPU baseline (bench.py cpu_baseline, kind "reference"): the reference's own Csr plan
// (main_experiment1.cc:636-699: AlgScan(R) -> AlgHashJoinBuild, AlgScan(S) -> AlgHashJoinProbe
// unique -> counting AlgTop, clear_ht between repetitions) timed on a uniform key/FK input of
// |R| = nR, |S| = nS generated as in main_experiment1.cc:415-457. Build and probe are timed
// separately with steady_clock, averaged over `reps` repetitions.
int timeCsr(size_t nR, size_t nS, int reps, size_t prefix) {
  std::mt19937 rng;
  std::vector<uint32_t> keysR(nR);
  for (size_t i = 0; i < nR; ++i) keysR[i] = static_cast<uint32_t>(i);
  std::shuffle(keysR.begin(), keysR.end(), rng);
  std::vector<uint32_t> fk;
  GenRandIntVec griv;
  GenRandIntVec::param_t p(GenRandIntVec::dist_t::kUni, static_cast<uint32_t>(nR), 0, 0.0, 0, -1);
  griv.generate(fk, static_cast<uint>(nS), p, rng);
  // the probe side: the first `prefix` tuples of the generated |S| = nS relation (all of it when
  // prefix is 0), so a bounded sample is a prefix of exactly the relation the GPU line joins
  const size_t nP = prefix && prefix < nS ? prefix : nS;
  RelationRS<Tup> R, S;
  R._tuples.resize(nR);
  for (size_t i = 0; i < nR; ++i) R._tuples[i] = Tup{keysR[i], 0, 0};
  S._tuples.resize(nP);
  for (size_t i = 0; i < nP; ++i) S._tuples[i] = Tup{static_cast<uint32_t>(i), fk[i], 0};
  fk.clear();
  fk.shrink_to_fit();

  using build_t = AlgHashJoinBuild<HashK, EqK, GS>;
  using top_t = AlgTop<Pair, GS>;
  using probe_t = AlgHashJoinProbe<top_t, build_t, HashA, PredAK, CatPair, true>;
  GS gs;
  build_t opBuild(std::max<size_t>(nR, 1), 10);
  AlgScan<build_t> scanB(&opBuild, &R);
  top_t top(gNull, false);
  probe_t opProbe(&top, &opBuild);
  AlgScan<probe_t> scanP(&opProbe, &S);
  using clk = std::chrono::steady_clock;
  std::chrono::nanoseconds tb{0}, tp{0};
  // main_experiment1.cc:663-699: repeat_mintime (util/measure_helpers.hh:15-41) with >= 300 ms and
  // `reps` minimum repetitions, clear_ht between repetitions (not after the last)
  const auto [tot, n] = df::infra::repeat_mintime(
      std::chrono::milliseconds(300),
      [&]() {
        const auto t0 = clk::now();
        scanB.run(&gs);
        const auto t1 = clk::now();
        scanP.run(&gs);
        const auto t2 = clk::now();
        tb += t1 - t0;
        tp += t2 - t1;
      },
      [&]() { opBuild.clear_ht(); }, false, size_t(reps > 0 ? reps : 1));
  (void)tot;
  const double nr = double(n);
  std::printf("{\"plan\":\"Csr\",\"nR\":%zu,\"nS\":%zu,\"probe_prefix\":%zu,\"reps\":%zu,\"build_ns\":%.1f,"
              "\"probe_ns\":%.1f,\"c_probe\":%" PRIu64 ",\"c_cmp\":%" PRIu64 ",\"c_top\":%" PRIu64 "}\n",
              nR, nS, nP, n, double(tb.count()) / nr, double(tp.count()) / nr, opProbe.count(),
              opProbe.numCmps(), top.count());  // counters of the last repetition (AlgScan::run resets them)
  return 0;
}

// CPU baseline of config C (bench.py --workload C, kind "reference"): the reference's Nrs plan
// (main_experiment1.cc:1001-1185: AlgScan(S) -> AlgNestJoinBuild on S.a with NB = #dv(S.a),
// AlgScan(R) -> AlgNestJoinProbe -> AlgUnnestHt -> counting AlgTop) on |R| = nR unique keys and
// |S| = nS FKs ~ Zipf(theta) over [0, nR), generated as in main_experiment1.cc:415-457.
int timeNrs(size_t nR, size_t nS, double theta, int reps) {
  std::mt19937 rng;
  std::vector<uint32_t> keysR(nR);
  for (size_t i = 0; i < nR; ++i) keysR[i] = static_cast<uint32_t>(i);
  std::shuffle(keysR.begin(), keysR.end(), rng);
  std::vector<uint32_t> fk;
  GenRandIntVec griv;
  GenRandIntVec::param_t p(GenRandIntVec::dist_t::kZipf, static_cast<uint32_t>(nR), 0, theta, 0, -1);
  griv.generate(fk, static_cast<uint>(nS), p, rng);
  RelationRS<Tup> R, S;
  R._tuples.resize(nR);
  for (size_t i = 0; i < nR; ++i) R._tuples[i] = Tup{keysR[i], 0, 0};
  S._tuples.resize(nS);
  for (size_t i = 0; i < nS; ++i) S._tuples[i] = Tup{static_cast<uint32_t>(i), fk[i], 0};
  const size_t nb = std::max<size_t>(std::unordered_set<uint32_t>(fk.begin(), fk.end()).size(), 1);
  using build_t = AlgNestJoinBuild<HashA, EqA, GS>;
  using ht_t = build_t::hashtable_t;
  using top_t = AlgTop<Pair, GS>;
  using unnest_t = AlgUnnestHt<top_t, Unnest<ht_t>, ht_t>;
  using probe_t = AlgNestJoinProbe<unnest_t, build_t, HashK, PredKA, CatNested<ht_t>>;
  GS gs;
  build_t opBuild(nb, 10, 10);
  AlgScan<build_t> scanB(&opBuild, &S);
  top_t top(gNull, false);
  unnest_t opUnnest(&top);
  probe_t opProbe(&opUnnest, &opBuild);
  AlgScan<probe_t> scanP(&opProbe, &R);
  using clk = std::chrono::steady_clock;
  std::chrono::nanoseconds tb{0}, tp{0};
  // repeat_mintime (util/measure_helpers.hh:15-41): >= 300 ms, >= `reps` repetitions, clear_ht between
  const size_t n = df::infra::repeat_mintime(
      std::chrono::milliseconds(300),
      [&]() {
        const auto t0 = clk::now();
        scanB.run(&gs);
        const auto t1 = clk::now();
        scanP.run(&gs);
        const auto t2 = clk::now();
        tb += t1 - t0;
        tp += t2 - t1;
      },
      [&]() { opBuild.clear_ht(); }, false, size_t(reps > 0 ? reps : 1)).second;
  std::printf("{\"plan\":\"Nrs\",\"nR\":%zu,\"nS\":%zu,\"theta\":%g,\"nb\":%zu,\"reps\":%zu,\"build_ns\":%.1f,"
              "\"probe_ns\":%.1f,\"c_probe\":%" PRIu64 ",\"c_cmp\":%" PRIu64 ",\"c_unnest\":%" PRIu64
              ",\"c_top\":%" PRIu64 "}\n",
              nR, nS, theta, nb, n, double(tb.count()) / n, double(tp.count()) / n, opProbe.count(),
              opProbe.numCmps(), opUnnest.count(), top.count());
  return 0;
}
}  // namespace e1

// =============================== experiment 4 ===================================
namespace e4 {
struct Tup { uint32_t k, a; };
using hv_t = uint32_t;
inline hv_t H(uint32_t x) { return ht::murmur_hash<uint32_t>(x); }
struct GS {};
struct HashFk { using input_t = Tup; using output_t = hv_t;
  static output_t eval(const input_t* t) { return H(t->a); } };
struct EqFk { using left_t = Tup; using right_t = Tup;
  static bool eval(const left_t* l, const right_t* r) { return l->a == r->a; } };
struct HashR { using input_t = Tup; using output_t = hv_t;
  static output_t eval(const input_t* t) { return H(t->k); } };
struct PredR { using left_t = Tup; using right_t = Tup;
  static bool eval(const left_t* l, const right_t* r) { return l->k == r->a; } };

using nbuild_t = AlgNestJoinBuild<HashFk, EqFk, GS>;
using nht_t = nbuild_t::hashtable_t;
using Main = nht_t::MainNode;

struct Triple { const Tup* _r; const Tup* _s; const Tup* _t; };
struct NRS { Tup* _r; const Main* _s; };
struct NRST { Tup* _r; const Main* _s; const Main* _t; };
struct RnSxT { Tup* _r; const Main* _s; const Tup* _t; };

struct CatNRS { using left_t = Tup; using right_t = const Main; using output_t = NRS;
  static output_t eval(left_t* l, const right_t* r) { return {l, r}; } };
struct HashNRS { using input_t = NRS; using output_t = hv_t;
  static output_t eval(const input_t* n) { return H(n->_r->k); } };
struct PredNRS { using left_t = NRS; using right_t = Tup;
  static bool eval(const left_t* l, const right_t* r) { return l->_r->k == r->a; } };
struct CatNRST { using left_t = NRS; using right_t = const Main; using output_t = NRST;
  static output_t eval(left_t* l, const right_t* r) { return {l->_r, l->_s, r}; } };
struct UnT { using input_t = NRST; using output_t = RnSxT; using MainNode = Main; using data_t = nht_t::data_t;
  static const MainNode* getMainNode(input_t* n) { return n->_t; }
  static void eval_left(output_t* o, input_t* n) { o->_r = n->_r; o->_s = n->_s; }
  static void eval_right(output_t* o, input_t*, const data_t* d) { o->_t = d; } };
struct UnS { using input_t = RnSxT; using output_t = Triple; using MainNode = Main; using data_t = nht_t::data_t;
  static const MainNode* getMainNode(input_t* n) { return n->_s; }
  static void eval_left(output_t* o, input_t* n) { o->_r = n->_r; o->_t = n->_t; }
  static void eval_right(output_t* o, input_t*, const data_t* d) { o->_s = d; } };

struct PairRS { const Tup* _r; const Tup* _s; };
inline std::ostream& operator<<(std::ostream& os, const Tup& t) { return os << t.k << "|" << t.a; }
inline std::ostream& operator<<(std::ostream& os, const PairRS& p) { return os << p._r; }
inline std::ostream& operator<<(std::ostream& os, const NRS& p) { return os << p._r; }
inline std::ostream& operator<<(std::ostream& os, const NRST& p) { return os << p._r; }
inline std::ostream& operator<<(std::ostream& os, const RnSxT& p) { return os << p._r; }
inline std::ostream& operator<<(std::ostream& os, const Triple& p) { return os << p._r; }
struct CatRS { using left_t = Tup; using right_t = Tup; using output_t = PairRS;
  static output_t eval(left_t* l, const right_t* r) { return {l, r}; } };
struct HashRS { using input_t = PairRS; using output_t = hv_t;
  static output_t eval(const input_t* p) { return H(p->_r->k); } };
struct PredRS_T { using left_t = PairRS; using right_t = Tup;
  static bool eval(const left_t* l, const right_t* r) { return l->_r->k == r->a; } };
struct CatRS_T { using left_t = PairRS; using right_t = Tup; using output_t = Triple;
  static output_t eval(left_t* l, const right_t* r) { return {l->_r, l->_s, r}; } };

int run(uint32_t log2R, uint32_t alpha, uint32_t mA, uint32_t beta, uint32_t mB, bool dump) {
  // Same generation sequence as main_experiment4.cc:517-575.
  const size_t cardR = size_t(1) << log2R;
  const size_t numFkCommon = cardR / (size_t(1) << alpha);
  const size_t numFkExcl = cardR / (size_t(1) << beta);
  const size_t cardFkCommon = numFkCommon * mA, cardFkExcl = numFkExcl * mB;
  const size_t cardFk = cardFkCommon + cardFkExcl;
  std::mt19937 rng;
  std::vector<uint32_t> keys(std::max(cardR, cardFk));
  std::iota(keys.begin(), keys.end(), 0u);
  std::vector<uint32_t> fkC(cardFkCommon), fkS(cardFkExcl), fkT(cardFkExcl);
  uint32_t v = 0;
  size_t idx = 0;
  for (; v < numFkCommon; ++v) for (uint32_t i = 0; i < mA; ++i) fkC[idx++] = v;
  idx = 0;
  for (; v < numFkCommon + numFkExcl; ++v) for (uint32_t i = 0; i < mB; ++i) fkS[idx++] = v;
  idx = 0;
  for (; v < numFkCommon + 2 * numFkExcl; ++v) for (uint32_t i = 0; i < mB; ++i) fkT[idx++] = v;
  RelationRS<Tup> R, S, T;
  R._tuples.resize(cardR);
  for (size_t i = 0; i < cardR; ++i) R._tuples[i] = Tup{keys[i], 0};
  std::shuffle(fkS.begin(), fkS.end(), rng);
  std::shuffle(fkT.begin(), fkT.end(), rng);
  std::shuffle(fkC.begin(), fkC.end(), rng);
  std::vector<uint32_t> colS(cardFk), colT(cardFk);
  S._tuples.resize(cardFk);
  for (size_t i = 0; i < cardFk; ++i) {
    colS[i] = i < cardFkCommon ? fkC[i] : fkS[i - cardFkCommon];
    S._tuples[i] = Tup{keys[i], colS[i]};
  }
  std::shuffle(fkC.begin(), fkC.end(), rng);
  T._tuples.resize(cardFk);
  for (size_t i = 0; i < cardFk; ++i) {
    colT[i] = i < cardFkCommon ? fkC[i] : fkT[i - cardFkCommon];
    T._tuples[i] = Tup{keys[i], colT[i]};
  }
  const size_t nb = numFkCommon + numFkExcl;
  const Tup* rb = R._tuples.data();
  const Tup* sb = S._tuples.data();
  const Tup* tb = T._tuples.data();
  GS gs;

  std::printf("{\"exp\":4,\"log2R\":%u,\"alpha\":%u,\"multA\":%u,\"beta\":%u,\"multB\":%u,"
              "\"cardR\":%zu,\"cardS\":%zu,\"nb\":%zu,\"join_card1\":%zu,\"join_card2\":%zu,"
              "\"colsum_Sa\":%" PRIu64 ",\"colsum_Ta\":%" PRIu64 ",",
              log2R, alpha, mA, beta, mB, cardR, cardFk, nb, cardFk, numFkCommon * mA * mA,
              colsum(colS), colsum(colT));
  printHead("head_Sa", colS);
  std::printf(",");
  printHead("head_Ta", colT);
  std::printf(",");
  if (dump) {
    printAll("Sa", colS);
    std::printf(",");
    printAll("Ta", colT);
    std::printf(",");
  }
  std::printf("\"plans\":{");
  {  // Ndu (main_experiment4.cc:831-941)
    Agg agg;
    using top_t = AlgTop<Triple, GS>;
    using un2_t = AlgUnnestHt<top_t, UnS, nht_t>;
    using un1_t = AlgUnnestHt<un2_t, UnT, nht_t>;
    using pRT_t = AlgNestJoinProbe<un1_t, nbuild_t, HashNRS, PredNRS, CatNRST>;
    using pRS_t = AlgNestJoinProbe<pRT_t, nbuild_t, HashR, PredR, CatNRS>;
    nbuild_t bS(nb, 10, 10), bT(nb, 10, 10);
    AlgScan<nbuild_t> scS(&bS, &S), scT(&bT, &T);
    top_t top(gNull, true, [&](const Triple* x, std::ostream&) {
      agg.add3(uint64_t(x->_r - rb), uint64_t(x->_s - sb), uint64_t(x->_t - tb));
    });
    un2_t un2(&top);
    un1_t un1(&un2);
    pRT_t pRT(&un1, &bT);
    pRS_t pRS(&pRT, &bS);
    AlgScan<pRS_t> scR(&pRS, &R);
    scS.run(&gs);
    scT.run(&gs);
    scR.run(&gs);
    std::printf("\"Ndu\":{\"c_probe_RS\":%" PRIu64 ",\"c_probe_RS_cmp\":%" PRIu64
                ",\"c_probe_RT\":%" PRIu64 ",\"c_probe_RT_cmp\":%" PRIu64
                ",\"c_unnest_1\":%" PRIu64 ",\"c_unnest_2\":%" PRIu64 ",\"c_top\":%" PRIu64 ",",
                pRS.count(), pRS.numCmps(), pRT.count(), pRT.numCmps(), un1.count(), un2.count(), top.count());
    std::printf("\"stats_S\":{");
    { auto s = bS.hashtable().makeStatistics();
      std::printf("\"empty\":%zu,\"distinct\":%zu,\"cc1_max\":%zu,\"cc1_sum\":%zu}", s._numEmptyBuckets,
                  s._numDistinctKeys, s._collisionChainLenNonempty.max(), s._collisionChainLenNonempty.sum()); }
    std::printf(",");
    printAgg("out", agg);
    std::printf("},");
  }
  {  // Chj (main_experiment4.cc:943-1043)
    Agg agg;
    using cbuild_t = AlgHashJoinBuild<HashFk, EqFk, GS>;
    using top_t = AlgTop<Triple, GS>;
    using pRT_t = AlgHashJoinProbe<top_t, cbuild_t, HashRS, PredRS_T, CatRS_T>;
    using pRS_t = AlgHashJoinProbe<pRT_t, cbuild_t, HashR, PredR, CatRS>;
    cbuild_t bS(nb, 10), bT(nb, 10);
    AlgScan<cbuild_t> scS(&bS, &S), scT(&bT, &T);
    top_t top(gNull, true, [&](const Triple* x, std::ostream&) {
      agg.add3(uint64_t(x->_r - rb), uint64_t(x->_s - sb), uint64_t(x->_t - tb));
    });
    pRT_t pRT(&top, &bT);
    pRS_t pRS(&pRT, &bS);
    AlgScan<pRS_t> scR(&pRS, &R);
    scS.run(&gs);
    scT.run(&gs);
    scR.run(&gs);
    std::printf("\"Chj\":{\"c_probe_RS\":%" PRIu64 ",\"c_probe_RS_cmp\":%" PRIu64
                ",\"c_probe_RT\":%" PRIu64 ",\"c_probe_RT_cmp\":%" PRIu64 ",\"c_top\":%" PRIu64 ",",
                pRS.count(), pRS.numCmps(), pRT.count(), pRT.numCmps(), top.count());
    printAgg("out", agg);
    std::printf("}");
  }
  std::printf("}}\n");
  return 0;
}

// CPU baseline of config E (bench.py --workload E, kind "reference"): the reference's Ndu plan
// (main_experiment4.cc:831-941: two AlgNestJoinBuild on S.a, T.a; AlgScan(R) -> probe S -> probe
// T -> unnest T -> unnest S -> counting AlgTop) on the generation sequence of
// main_experiment4.cc:517-575 (as run() above). Builds and the probe strand timed separately.
int timeNdu(uint32_t log2R, uint32_t alpha, uint32_t mA, uint32_t beta, uint32_t mB, int reps) {
  const size_t cardR = size_t(1) << log2R;
  const size_t numFkCommon = cardR / (size_t(1) << alpha);
  const size_t numFkExcl = cardR / (size_t(1) << beta);
  const size_t cardFkCommon = numFkCommon * mA, cardFkExcl = numFkExcl * mB;
  const size_t cardFk = cardFkCommon + cardFkExcl;
  std::mt19937 rng;
  std::vector<uint32_t> keys(std::max(cardR, cardFk));
  std::iota(keys.begin(), keys.end(), 0u);
  std::vector<uint32_t> fkC(cardFkCommon), fkS(cardFkExcl), fkT(cardFkExcl);
  uint32_t v = 0;
  size_t idx = 0;
  for (; v < numFkCommon; ++v) for (uint32_t i = 0; i < mA; ++i) fkC[idx++] = v;
  idx = 0;
  for (; v < numFkCommon + numFkExcl; ++v) for (uint32_t i = 0; i < mB; ++i) fkS[idx++] = v;
  idx = 0;
  for (; v < numFkCommon + 2 * numFkExcl; ++v) for (uint32_t i = 0; i < mB; ++i) fkT[idx++] = v;
  RelationRS<Tup> R, S, T;
  R._tuples.resize(cardR);
  for (size_t i = 0; i < cardR; ++i) R._tuples[i] = Tup{keys[i], 0};
  std::shuffle(fkS.begin(), fkS.end(), rng);
  std::shuffle(fkT.begin(), fkT.end(), rng);
  std::shuffle(fkC.begin(), fkC.end(), rng);
  S._tuples.resize(cardFk);
  for (size_t i = 0; i < cardFk; ++i) S._tuples[i] = Tup{keys[i], i < cardFkCommon ? fkC[i] : fkS[i - cardFkCommon]};
  std::shuffle(fkC.begin(), fkC.end(), rng);
  T._tuples.resize(cardFk);
  for (size_t i = 0; i < cardFk; ++i) T._tuples[i] = Tup{keys[i], i < cardFkCommon ? fkC[i] : fkT[i - cardFkCommon]};
  const size_t nb = numFkCommon + numFkExcl;
  GS gs;
  using top_t = AlgTop<Triple, GS>;
  using un2_t = AlgUnnestHt<top_t, UnS, nht_t>;
  using un1_t = AlgUnnestHt<un2_t, UnT, nht_t>;
  using pRT_t = AlgNestJoinProbe<un1_t, nbuild_t, HashNRS, PredNRS, CatNRST>;
  using pRS_t = AlgNestJoinProbe<pRT_t, nbuild_t, HashR, PredR, CatNRS>;
  nbuild_t bS(nb, 10, 10), bT(nb, 10, 10);
  AlgScan<nbuild_t> scS(&bS, &S), scT(&bT, &T);
  top_t top(gNull, false);
  un2_t un2(&top);
  un1_t un1(&un2);
  pRT_t pRT(&un1, &bT);
  pRS_t pRS(&pRT, &bS);
  AlgScan<pRS_t> scR(&pRS, &R);
  using clk = std::chrono::steady_clock;
  std::chrono::nanoseconds tb{0}, tp{0};
  const size_t n = df::infra::repeat_mintime(
      std::chrono::milliseconds(300),
      [&]() {
        const auto t0 = clk::now();
        scS.run(&gs);
        scT.run(&gs);
        const auto t1 = clk::now();
        scR.run(&gs);
        const auto t2 = clk::now();
        tb += t1 - t0;
        tp += t2 - t1;
      },
      [&]() {
        bS.clear_ht();
        bT.clear_ht();
      },
      false, size_t(reps > 0 ? reps : 1)).second;
  std::printf("{\"plan\":\"Ndu\",\"cardR\":%zu,\"cardS\":%zu,\"nb\":%zu,\"reps\":%zu,\"build_ns\":%.1f,"
              "\"probe_ns\":%.1f,\"c_probe_rs\":%" PRIu64 ",\"c_probe_rt\":%" PRIu64 ",\"c_unnest_1\":%" PRIu64
              ",\"c_unnest_2\":%" PRIu64 ",\"c_top\":%" PRIu64 "}\n",
              cardR, cardFk, nb, n, double(tb.count()) / n, double(tp.count()) / n, pRS.count(),
              pRT.count(), un1.count(), un2.count(), top.count());
  return 0;
}
}  // namespace e4

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 8 && std::strcmp(argv[1], "exp1") == 0) {
    const bool dump = argc >= 9 && std::strcmp(argv[8], "dump") == 0;
    return e1::run(std::stoull(argv[2]), std::stoull(argv[3]), std::atoi(argv[4]) != 0, std::atof(argv[5]),
                   static_cast<uint32_t>(std::atoi(argv[6])), static_cast<uint32_t>(std::atoi(argv[7])), dump,
                   argc >= 10 ? std::string(argv[9]) : std::string());
  }
  if (argc >= 7 && std::strcmp(argv[1], "exp4") == 0) {
    const bool dump = argc >= 8 && std::strcmp(argv[7], "dump") == 0;
    return e4::run(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                   std::atoi(argv[6]), dump);
  }
  if (argc >= 5 && std::strcmp(argv[1], "time_csr") == 0)
    return e1::timeCsr(std::stoull(argv[2]), std::stoull(argv[3]), std::atoi(argv[4]),
                       argc >= 6 ? std::stoull(argv[5]) : 0);
  if (argc >= 8 && std::strcmp(argv[1], "time_ndu") == 0)
    return e4::timeNdu(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                       std::atoi(argv[6]), std::atoi(argv[7]));
  if (argc >= 6 && std::strcmp(argv[1], "time_nrs") == 0)
    return e1::timeNrs(std::stoull(argv[2]), std::stoull(argv[3]), std::atof(argv[4]), std::atoi(argv[5]));
  std::fprintf(stderr, "usage: ref_golden exp1 nR nS skew theta t b [dump|nodump [plan,plan...]] | exp4 log2R a A b B [dump]\n");
  return 2;
}

// The drop-in surface beyond the fused strands (tests/test_dropin.py runs it on the GPU):
//   A  HtChaining1::findDirEntryByOther + the reference's own chain walk (algebra.hh:625-659
//      restated below) per probe tuple: matches and comparisons equal the device probe operator's;
//   B  HtNested1::findMainNodeByOther + sub-chain walk per probe tuple: matches, main-chain
//      comparisons and unnested tuples equal the fused device strand probe -> unnest -> Top;
//   C  AlgNestJoinProbe -> AlgUnnestHt -> a custom consumer (no fused device strand): the host
//      probe path pushes exactly the pairs of a brute-force join, per probe tuple the key's first
//      build tuple first, then the others newest first (ht_nested.hh:299-311 order);
//   D  a relation modified in place at an unsampled tuple (same address, same size) is uploaded
//      again and the join result changes (RelationCache fingerprints every byte).
// Prints "PASS <name>" / "FAIL <name> ..." per check, exit status 0 iff all pass.
#include <algorithm>
#include <cstdint>
#include <iostream>
#include <map>
#include <unordered_map>
#include <vector>

#include "algebra.hh"

struct Tup { uint32_t k, a, b; };  // main_experiment1.cc:86

static inline uint32_t fmix32(uint32_t x) {  // util/hasht.hh:52-61
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}
struct HashK { using input_t = Tup; using output_t = uint32_t;
  static output_t eval(const input_t* t) { return fmix32(t->k); } };
struct HashA { using input_t = Tup; using output_t = uint32_t;
  static output_t eval(const input_t* t) { return fmix32(t->a); } };
struct EqK { using left_t = Tup; using right_t = Tup;
  static bool eval(const left_t* l, const right_t* r) { return l->k == r->k; } };
struct EqA { using left_t = Tup; using right_t = Tup;
  static bool eval(const left_t* l, const right_t* r) { return l->a == r->a; } };
struct PredAK { using left_t = Tup; using right_t = Tup;  // probe S.a = build R.k
  static bool eval(const left_t* l, const right_t* r) { return l->a == r->k; } };
struct PredKA { using left_t = Tup; using right_t = Tup;  // probe R.k = build S.a
  static bool eval(const left_t* l, const right_t* r) { return l->k == r->a; } };

struct pair_t { const Tup* l; const Tup* r; };
struct CatPair { using left_t = Tup; using right_t = Tup; using output_t = pair_t;
  static output_t eval(left_t* l, const right_t* r) { return {l, r}; } };
using HtN = HtNested1<Tup, HashA, EqA>;
struct nested_t { Tup* l; const HtN::MainNode* m; };
struct CatNested { using left_t = Tup; using right_t = HtN::MainNode; using output_t = nested_t;
  static output_t eval(left_t* l, const right_t* r) { return {l, r}; } };
struct Unnest { using input_t = nested_t; using output_t = pair_t; using MainNode = HtN::MainNode;
  using data_t = HtN::data_t;
  static const MainNode* getMainNode(input_t* n) { return n->m; }
  static void eval_left(output_t* o, input_t* i) { o->l = i->l; }
  static void eval_right(output_t* o, input_t*, const data_t* d) { o->r = d; } };

// a consumer the device strands do not know: collects the pairs it receives, in order
class Collect : public AlgBase {
 public:
  using globstat_t = GlobStat0;
  using input_t = pair_t;
  using output_t = void;
  Collect() : AlgBase("Collect") {}
  void init(globstat_t*) { reset(); got.clear(); }
  void step(input_t* t, globstat_t*) { inc(); got.push_back(*t); }
  void fin(globstat_t*) { stopTimer(); }
  std::vector<pair_t> got;
};

static int failures = 0;
static void check(bool ok, const char* name, const std::string& detail = "") {
  std::cout << (ok ? "PASS " : "FAIL ") << name << (ok ? "" : " " + detail) << "\n";
  failures += !ok;
}

int main() {
  try {
    const uint32_t nR = 30000, nS = 200000;
    RelationRS<Tup> R, S;
    R._tuples.resize(nR);
    S._tuples.resize(nS);
    uint64_t x = 88172645463325252ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (uint32_t i = 0; i < nR; ++i) R._tuples[i] = {i, 0, 0};
    for (uint32_t i = nR - 1; i > 0; --i) std::swap(R._tuples[i].k, R._tuples[rnd() % (i + 1)].k);
    for (uint32_t i = 0; i < nS; ++i) {  // FKs, 20 % dangling, a few hot keys
      const uint64_t r = rnd();
      uint32_t a = uint32_t(r % (nR + nR / 4));
      if ((r >> 40) % 10 == 0) a = uint32_t((r >> 20) % 8);
      S._tuples[i] = {i, a, 0};
    }
    GlobStat0 gs{nR, 10, 10, 10};

    // ---- A: chaining table on R.k, per-tuple probes of S ----
    {
      using build_t = AlgHashJoinBuild<HashK, EqK, GlobStat0>;
      using top_t = AlgTop<pair_t, GlobStat0>;
      using probe_t = AlgHashJoinProbe<top_t, build_t, HashA, PredAK, CatPair, true>;
      build_t build(nR, 10);
      AlgScan<build_t> scanR(&build, &R);
      top_t top(std::cout, false);
      probe_t probe(&top, &build);
      AlgScan<probe_t> scanS(&probe, &S);
      scanR.run(&gs);
      scanS.run(&gs);
      uint64_t match = 0, cmps = 0;
      const auto& ht = build.hashtable();
      for (auto& s : S._tuples) {  // AlgHashJoinProbe<unique>::step, tuple at a time
        const uint32_t h = HashA::eval(&s);
        auto it = ht.template findDirEntryByOther<Tup, HashA>(&s);
        if (it->isEmpty()) continue;
        for (; it != nullptr; ++it) {
          ++cmps;
          if (it->hashvalue() == h && PredAK::eval(&s, it->data())) {
            ++match;
            break;
          }
        }
      }
      check(match == probe.count() && cmps == probe.numCmps(), "chaining_per_tuple_walk",
            std::to_string(match) + "/" + std::to_string(probe.count()) + " " + std::to_string(cmps) + "/" +
                std::to_string(probe.numCmps()));
    }

    // ---- B and C: nested table on S.a (non-unique), probes of R ----
    {
      using build_t = AlgNestJoinBuild<HashA, EqA, GlobStat0>;
      build_t build(nR, 10, 10);
      AlgScan<build_t> scanS(&build, &S);
      scanS.run(&gs);
      // fused device strand: probe -> unnest -> Top
      using top_t = AlgTop<pair_t, GlobStat0>;
      using un_t = AlgUnnestHt<top_t, Unnest, HtN>;
      using probe_t = AlgNestJoinProbe<un_t, build_t, HashK, PredKA, CatNested>;
      top_t top(std::cout, false);
      un_t un(&top);
      probe_t probe(&un, &build);
      AlgScan<probe_t> scanR(&probe, &R);
      scanR.run(&gs);
      uint64_t match = 0, cmps = 0, unnested = 0;
      const auto& ht = build.hashtable();
      for (auto& r : R._tuples) {
        const auto [mn, c] = ht.template findMainNodeByOther<Tup, HashK, PredKA>(&r);
        cmps += c;
        if (!mn) continue;
        ++match;
        ++unnested;
        for (auto* sn = mn->child(); sn != nullptr; sn = sn->next()) ++unnested;
      }
      check(match == probe.count() && cmps == probe.numCmps() && unnested == un.count() && unnested == top.count(),
            "nested_per_tuple_walk",
            std::to_string(match) + "/" + std::to_string(probe.count()) + " " + std::to_string(cmps) + "/" +
                std::to_string(probe.numCmps()) + " " + std::to_string(unnested) + "/" + std::to_string(un.count()));

      // C: probe -> unnest -> a custom consumer (the host probe path)
      using unc_t = AlgUnnestHt<Collect, Unnest, HtN>;
      using probec_t = AlgNestJoinProbe<unc_t, build_t, HashK, PredKA, CatNested>;
      Collect col;
      unc_t unc(&col);
      probec_t probec(&unc, &build);
      AlgScan<probec_t> scanR2(&probec, &R);
      scanR2.run(&gs);
      std::unordered_map<uint32_t, std::vector<uint32_t>> byA;  // brute force: S rows per key
      for (uint32_t i = 0; i < nS; ++i) byA[S._tuples[i].a].push_back(i);
      std::vector<std::pair<uint32_t, uint32_t>> want;
      for (uint32_t i = 0; i < nR; ++i) {
        auto f = byA.find(R._tuples[i].k);
        if (f == byA.end()) continue;
        const auto& rows = f->second;  // ascending: first insert, then newest first
        want.emplace_back(i, rows[0]);
        for (size_t q = rows.size(); q-- > 1;) want.emplace_back(i, rows[q]);
      }
      std::vector<std::pair<uint32_t, uint32_t>> got;
      for (const auto& p : col.got) got.emplace_back(uint32_t(p.l - R._tuples.data()), uint32_t(p.r - S._tuples.data()));
      check(got == want && probec.count() == probe.count() && probec.numCmps() == probe.numCmps(),
            "nested_host_probe_custom_consumer",
            std::to_string(got.size()) + "/" + std::to_string(want.size()));
    }

    // ---- D: a relation modified in place at the same address ----
    {
      using build_t = AlgHashJoinBuild<HashK, EqK, GlobStat0>;
      using top_t = AlgTop<pair_t, GlobStat0>;
      using probe_t = AlgHashJoinProbe<top_t, build_t, HashA, PredAK, CatPair, true>;
      build_t build(nR, 10);
      AlgScan<build_t> scanR(&build, &R);
      top_t top(std::cout, false);
      probe_t probe(&top, &build);
      AlgScan<probe_t> scanS(&probe, &S);
      scanR.run(&gs);
      scanS.run(&gs);
      const uint64_t before = top.count();
      const uint64_t up0 = hj3d::host::RelationCache::get().uploads();
      scanS.run(&gs);  // unchanged: served from the device copy
      const uint64_t up1 = hj3d::host::RelationCache::get().uploads();
      // a tuple the 257-tuple sample never looks at, with a matching key, now dangling
      uint32_t i = nS / 2 + 17;
      while (S._tuples[i].a >= nR) ++i;
      S._tuples[i].a = 0xFFFFFFF0u;
      scanS.run(&gs);
      const uint64_t after = top.count();
      const uint64_t up2 = hj3d::host::RelationCache::get().uploads();
      check(after + 1 == before && up1 == up0 && up2 == up1 + 1, "relation_modified_in_place",
            std::to_string(before) + "->" + std::to_string(after) + " uploads " + std::to_string(up0) + "," +
                std::to_string(up1) + "," + std::to_string(up2));
    }
  } catch (const std::exception& e) {
    std::cerr << e.what() << "\n";
    return 2;
  }
  std::cout << (failures ? "SOME FAILED" : "ALL PASS") << "\n";
  return failures ? 1 : 0;
}

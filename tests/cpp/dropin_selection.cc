// Selection pushdown through the drop-in operator surface: scan(L) -> selection(L.b < 40) ->
// probe(L.a = R.c) [-> unnest] -> top, the plans of the reference's main_algebra_example.cc
// (algebra_test1..3) on its relations, once with the selection on the host (tuple at a time) and
// once pushed down (hj3d::device_predicate -> hj3d_select). Prints one line per plan and mode:
//   <plan> <mode> Top=<n> Probe=<n> Sel=<n> Scan=<n> Build=<n>
// and, for the chaining plan with a printing Top, the output tuples "(a,b,c,d)" in push order.
#include <cstdint>
#include <iostream>

#include "algebra.hh"

struct tuple_L_t { int a, b; };
struct tuple_R_t { int c, d; };

static inline uint32_t fmix32(uint32_t x) {  // util/hasht.hh:52-61
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}
struct HashR { using input_t = tuple_R_t; using output_t = uint32_t;
  static output_t eval(const input_t* t) { return fmix32(uint32_t(t->c)); } };
struct HashL { using input_t = tuple_L_t; using output_t = uint32_t;
  static output_t eval(const input_t* t) { return fmix32(uint32_t(t->a)); } };
struct EqR { using left_t = tuple_R_t; using right_t = tuple_R_t;
  static bool eval(const left_t* l, const right_t* r) { return l->c == r->c; } };
struct JoinLR { using left_t = tuple_L_t; using right_t = tuple_R_t;
  static bool eval(const left_t* l, const right_t* r) { return l->a == r->c; } };
struct SelL { using input_t = tuple_L_t; static bool eval(const input_t* t) { return t->b < 40; } };
struct DynSelL { using input_t = tuple_L_t; bool operator()(const input_t* t) { return t->b < 40; } };
// the same predicate on the host-only path (no device_predicate specialisation)
struct SelLHost { using input_t = tuple_L_t; static bool eval(const input_t* t) { return t->b < 40; } };

template <> struct hj3d::device_predicate<SelL> {
  static constexpr uint32_t npred = 1;
  static constexpr hj3d_sel_pred preds[1] = {{4, HJ3D_SEL_LT, 1, 0, 40, 0}};
};
template <> struct hj3d::device_predicate<DynSelL> {
  static constexpr uint32_t npred = 1;
  static constexpr hj3d_sel_pred preds[1] = {{4, HJ3D_SEL_LT, 1, 0, 40, 0}};
};

using HtN = HtNested1<tuple_R_t, HashR, EqR>;
struct nested_t { tuple_L_t* _left; const HtN::MainNode* _right; };
struct pair_t { const tuple_L_t* _left; const tuple_R_t* _right; };
struct ConcatN { using left_t = tuple_L_t; using right_t = HtN::MainNode; using output_t = nested_t;
  static output_t eval(left_t* l, const right_t* r) { return {l, r}; } };
struct ConcatC { using left_t = tuple_L_t; using right_t = tuple_R_t; using output_t = pair_t;
  static output_t eval(left_t* l, const right_t* r) { return {l, r}; } };
struct UnnestF { using input_t = nested_t; using output_t = pair_t; using MainNode = HtN::MainNode;
  using data_t = HtN::data_t;
  static const MainNode* getMainNode(input_t* n) { return n->_right; }
  static void eval_left(output_t* o, input_t* i) { o->_left = i->_left; }
  static void eval_right(output_t* o, input_t*, const data_t* d) { o->_right = d; } };

static RelationRS<tuple_L_t> relL() { return {._tuples{{1, 11}, {2, 21}, {3, 31}, {4, 41}}}; }
static RelationRS<tuple_R_t> relR() { return {._tuples{{1, -1}, {1, -2}, {1, -3}, {2, -1}, {2, -2}, {3, -1}}}; }

template <typename Tsel, bool Dyn = false>
void chaining(const char* mode, bool print) {
  GlobStat0 gs{4, 4, 4, 4};
  auto L = relL();
  auto R = relR();
  using build_t = AlgHashJoinBuild<HashR, EqR, GlobStat0>;
  using top_t = AlgTop<pair_t, GlobStat0>;
  using probe_t = AlgHashJoinProbe<top_t, build_t, HashL, JoinLR, ConcatC>;
  build_t build(4, 4);
  AlgScan<build_t> scanR(&build, &R);
  top_t top(std::cout, print, [](const pair_t* t, std::ostream& os) {
    os << "(" << t->_left->a << "," << t->_left->b << "," << t->_right->c << "," << t->_right->d << ")";
  });
  probe_t probe(&top, &build);
  auto run = [&](auto& sel) {
    AlgScan<std::remove_reference_t<decltype(sel)>> scanL(&sel, &L);
    scanR.run(&gs);
    scanL.run(&gs);
    std::cout << "chain " << mode << " Top=" << top.count() << " Probe=" << probe.count() << " Sel=" << sel.count()
              << " Scan=" << scanL.count() << " Build=" << build.count() << "\n";
  };
  if constexpr (Dyn) {
    AlgDynSelection<probe_t, Tsel> sel(&probe, Tsel());
    run(sel);
  } else {
    AlgSelection<probe_t, Tsel> sel(&probe);
    run(sel);
  }
}

template <typename Tsel, bool Unnest>
void nested(const char* mode) {
  GlobStat0 gs{4, 4, 4, 4};
  auto L = relL();
  auto R = relR();
  using build_t = AlgNestJoinBuild<HashR, EqR, GlobStat0>;
  build_t build(4, 4, 4);
  AlgScan<build_t> scanR(&build, &R);
  scanR.run(&gs);
  if constexpr (Unnest) {
    using top_t = AlgTop<pair_t, GlobStat0>;
    using un_t = AlgUnnestHt<top_t, UnnestF, HtN>;
    using probe_t = AlgNestJoinProbe<un_t, build_t, HashL, JoinLR, ConcatN>;
    top_t top(std::cout, false);
    un_t un(&top);
    probe_t probe(&un, &build);
    AlgSelection<probe_t, Tsel> sel(&probe);
    AlgScan<decltype(sel)> scanL(&sel, &L);
    scanL.run(&gs);
    std::cout << "unnest " << mode << " Top=" << top.count() << " Probe=" << probe.count() << " Sel=" << sel.count()
              << " Scan=" << scanL.count() << " Build=" << build.count() << "\n";
  } else {
    using top_t = AlgTop<nested_t, GlobStat0>;
    using probe_t = AlgNestJoinProbe<top_t, build_t, HashL, JoinLR, ConcatN>;
    top_t top(std::cout, false);
    probe_t probe(&top, &build);
    AlgSelection<probe_t, Tsel> sel(&probe);
    AlgScan<decltype(sel)> scanL(&sel, &L);
    scanL.run(&gs);
    std::cout << "nested " << mode << " Top=" << top.count() << " Probe=" << probe.count() << " Sel=" << sel.count()
              << " Scan=" << scanL.count() << " Build=" << build.count() << "\n";
  }
}

int main() {
  try {
    chaining<SelLHost>("host", false);
    chaining<SelL>("device", false);
    chaining<DynSelL, true>("device_dyn", false);
    chaining<SelL>("device_print", true);
    nested<SelLHost, false>("host");
    nested<SelL, false>("device");
    nested<SelLHost, true>("host");
    nested<SelL, true>("device");
  } catch (const std::exception& e) {
    std::cerr << e.what() << "\n";
    return 1;
  }
  return 0;
}

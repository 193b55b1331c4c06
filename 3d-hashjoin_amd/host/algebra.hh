// algebra.hh — the push-based operator algebra of the 3D hash join (reference: algebra.hh),
// with the join operators executed on the MI355X through libhj3d.so (include/hj3d.h).
//
// Drop-in: same operator names, template parameters, constructors and observers (count(),
// numCmps(), consumer(), hashtable(), clear_ht(), printResult(), print_strand,
// get_runtime_excl), so main_experiment1.cc / main_experiment4.cc compile unchanged against
// this directory. What changes is where the tuples go:
//   * AlgScan::run hands its whole relation to a build/probe consumer (consume_relation)
//     instead of pushing tuple by tuple (the batching seam, reference algebra.hh:259-269);
//     other consumers (Top, Selection) still get tuples one by one.
//   * Build operators record the input; the device build runs in fin(), inside the build
//     strand's timed scan like the reference's inserts.
//   * Probe operators record the input and run in fin(): probe -> Top, probe -> Unnest -> Top
//     and the experiment-4 strands (two probes + two unnests -> Top) run fused on the device
//     and only their counters come back (algebra.hh:435-459, 510-541, 625-659 semantics,
//     comparison counts included). A chaining probe into any other consumer materialises its
//     output pairs on the device and pushes concat(probe, build) tuples in the reference's
//     order. A nested probe into any other consumer runs the reference's tuple-at-a-time probe
//     over a host node view of the device table (correct, slow; ht_nested.hh findMainNodeByOther)
//     and AlgUnnestHt expands the nested tuples it receives on the host.
// No operator has a host-side join: without a GPU the engine cannot be created and the first
// build/probe throws.
#pragma once

#include <algorithm>
#include <cassert>
#include <chrono>
#include <concepts>
#include <cstdint>
#include <functional>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "concepts.hh"
#include "hj3d_host.hh"
#include "ht_chaining.hh"
#include "ht_nested.hh"

class AlgBase;

namespace hj3d::host {
struct OpAccess;
}

template <typename T>
concept alg_operator_c = std::derived_from<T, AlgBase> && requires {
  typename T::globstat_t;
  typename T::input_t;
  typename T::output_t;
};

template <typename T>
concept alg_consumer_c = alg_operator_c<T> && requires(T c) {
  { c.init(static_cast<typename T::globstat_t*>(nullptr)) } -> std::same_as<void>;
  { c.step(static_cast<typename T::input_t*>(nullptr), static_cast<typename T::globstat_t*>(nullptr)) }
      -> std::same_as<void>;
  { c.fin(static_cast<typename T::globstat_t*>(nullptr)) } -> std::same_as<void>;
};

template <typename T>
concept alg_producer_c = alg_operator_c<T> && requires(T c) {
  { c.run(static_cast<typename T::globstat*>(nullptr)) } -> std::same_as<void>;
};

template <typename T>
concept alg_buildop_c = alg_consumer_c<T> && requires(T t) {
  typename T::hashtable_t;
  { t.hashtable() } -> std::same_as<const typename T::hashtable_t&>;
};

// a row store relation (reference algebra.hh:97-106)
template <typename Ttuple>
struct RelationRS {
  using tuple_t = Ttuple;
  using tuple_vt = std::vector<tuple_t>;
  tuple_vt _tuples;
  inline size_t card() const { return _tuples.size(); }
};

template <typename Ttuple>
std::ostream& operator<<(std::ostream& os, const RelationRS<Ttuple>& aRel) {
  for (const auto& t : aRel._tuples) os << t << "\n";
  return os;
}

struct GlobStat0 {
  size_t _ht_num_buckets;
  size_t _ht_rsv_log2_chunksize_main;
  size_t _ht_rsv_log2_chunksize_sub;
  size_t _ht_rsv_log2_chunksize;
};

class AlgBase {
  friend struct hj3d::host::OpAccess;

 public:
  using clock_t = std::chrono::steady_clock;
  using time_point_t = std::chrono::time_point<clock_t>;
  using duration_t = std::chrono::nanoseconds;

  explicit AlgBase(const std::string& aName) : _name(aName) {}
  AlgBase() : AlgBase("") {}

  inline void reset() {
    _count = 0;
    _ok = true;
    startTimer();
    ++_runs;
  }
  inline void inc() { ++_count; }
  inline uint64_t count() const { return _count; }
  inline bool ok() const { return _ok; }
  inline bool ok(const bool b) { return (_ok = b); }
  inline void startTimer() { _startTime = clock_t::now(); }
  inline void stopTimer() { _stopTime = clock_t::now(); }
  inline const std::string& name() const { return _name; }
  inline uint64_t runs() const { return _runs; }
  // inclusive: an operator's runtime includes its consumers'
  inline duration_t getRuntime() const { return std::chrono::duration_cast<duration_t>(_stopTime - _startTime); }
  inline std::string getRuntimeStr() const { return std::to_string(getRuntime().count()) + " ns"; }

 protected:
  uint64_t _count = 0;
  bool _ok = true;
  time_point_t _startTime{};
  time_point_t _stopTime{};
  std::string _name;
  uint64_t _runs = 0;
};

template <alg_operator_c Toperator>
auto get_runtime_excl(const Toperator* aOp) -> typename Toperator::duration_t {
  assert(aOp != nullptr);
  if constexpr (requires(Toperator t) { t.consumer(); }) {
    return aOp->getRuntime() - aOp->consumer()->getRuntime();
  } else {
    return aOp->getRuntime();
  }
}

// name|count|exclusive runtime|runs, top-most operator first (reference algebra.hh:148-162)
template <alg_operator_c Toperator>
void print_strand(const Toperator* aOp, const size_t aIndentLvl = 0, std::ostream& os = std::cout) {
  assert(aOp != nullptr);
  if constexpr (requires(Toperator t) { t.consumer(); }) print_strand(aOp->consumer(), aIndentLvl, os);
  const auto ns = get_runtime_excl(aOp).count();
  std::ostringstream rt;
  if (ns >= 1000000) rt << (ns / 1000000) << "." << std::setw(3) << std::setfill('0') << (ns / 1000) % 1000 << " ms";
  else if (ns >= 1000) rt << (ns / 1000) << "." << std::setw(3) << std::setfill('0') << ns % 1000 << " us";
  else rt << ns << " ns";
  os << std::string(2 * aIndentLvl, ' ') << aOp->name() << "|" << aOp->count() << "|" << rt.str() << "|"
     << aOp->runs() << "\n";
}

namespace hj3d::host {
// Counter access for fused strands: the operator that runs a fused strand on the device sets
// the counters of the operators it absorbed.
struct OpAccess {
  static void add(AlgBase& op, uint64_t n) { op._count += n; }
};
}  // namespace hj3d::host

// Top operator (reference algebra.hh:203-243)
template <typename Tinput, typename Tglobstat>
class AlgTop : public AlgBase {
 public:
  using globstat_t = Tglobstat;
  using input_t = Tinput;
  using output_t = void;
  using print_fun_t = std::function<void(const input_t*, std::ostream& os)>;

  inline AlgTop() : AlgTop(std::cout, true) {}
  inline AlgTop(std::ostream& aOs, const bool aPrintResult) : AlgBase("AlgTop"), _os(aOs), _print_result(aPrintResult) {}
  inline AlgTop(std::ostream& aOs, const bool aPrintResult, print_fun_t aPrintFunction)
      : AlgBase("AlgTop"), _os(aOs), _print_result(aPrintResult), _print_fun(aPrintFunction) {}

  inline void init([[maybe_unused]] globstat_t* aGlobstat) { reset(); }
  inline void step(input_t* aInput, [[maybe_unused]] globstat_t* aGlobstat) {
    inc();
    if (prints()) {
      _print_fun(aInput, _os);
      _os << "\n";
    }
  }
  inline void fin([[maybe_unused]] globstat_t* aGlobstat) { stopTimer(); }

  bool printResult() const { return _print_result; }
  void printResult(const bool aPrint) { _print_result = aPrint; }
  // true when step() would print, i.e. the results must be materialised
  bool prints() const { return _print_result && runs() == 1; }

 private:
  std::ostream& _os;
  bool _print_result;
  print_fun_t _print_fun = [](const input_t* aInput, std::ostream& aOs) { aOs << aInput; };
};

// Table scan operator (reference algebra.hh:246-275)
template <alg_consumer_c Tconsumer>
class AlgScan : public AlgBase {
 public:
  using consumer_t = Tconsumer;
  using globstat_t = typename consumer_t::globstat_t;
  using input_t = typename consumer_t::input_t;
  using output_t = typename consumer_t::input_t;
  using input_rel_t = RelationRS<input_t>;

  inline AlgScan(consumer_t* aConsumer, input_rel_t* aRelation)
      : AlgBase("AlgScan"), _consumer(aConsumer), _relation(aRelation) {}

  inline void run(globstat_t* aGlobstat) {
    reset();
    _consumer->init(aGlobstat);
    if constexpr (requires(consumer_t c) { c.consume_relation(static_cast<input_t*>(nullptr), size_t(0), aGlobstat); }) {
      // the whole relation goes to the device operator at once
      _count += _relation->_tuples.size();
      _consumer->consume_relation(_relation->_tuples.data(), _relation->_tuples.size(), aGlobstat);
    } else {
      for (auto& t : _relation->_tuples) {
        inc();
        _consumer->step(&t, aGlobstat);
      }
    }
    _consumer->fin(aGlobstat);
    stopTimer();
  }
  inline const consumer_t* consumer() const { return _consumer; }

 private:
  consumer_t* _consumer;
  input_rel_t* _relation;
};

// Selection pushdown applies when the predicate has a device form (hj3d::device_predicate) and the
// consumer is a device probe operator that takes a selected relation.
template <typename Tpred, typename Tconsumer, typename Tinput, typename Tglobstat>
inline constexpr bool hj3d_pushdown_v =
    requires { hj3d::device_predicate<Tpred>::npred; } &&
    requires(Tconsumer c, Tinput* b, Tglobstat* g) { c.consume_selected(b, size_t(0), nullptr, 0u, g); };

// Selection operator (reference algebra.hh:278-315): host predicate, tuple at a time
template <alg_consumer_c Tconsumer, alg_predicate_c Tpredicate>
class AlgSelection : public AlgBase {
 public:
  using consumer_t = Tconsumer;
  using globstat_t = typename consumer_t::globstat_t;
  using input_t = typename consumer_t::input_t;
  using output_t = typename consumer_t::input_t;
  using predicate_t = Tpredicate;

  inline AlgSelection(Tconsumer* aConsumer) : AlgBase("AlgSelection"), _consumer(aConsumer) {}
  inline void init(globstat_t* g) {
    reset();
    _pushed = false;
    _consumer->init(g);
  }
  // Pushdown (hj3d::device_predicate<Tpredicate> specialised and a device probe consumer): the
  // whole relation goes to the consumer with the predicate, hj3d_select filters it on the device.
  inline void consume_relation(input_t* base, size_t n, globstat_t* g)
    requires(hj3d_pushdown_v<Tpredicate, Tconsumer, input_t, globstat_t>)
  {
    using P = hj3d::device_predicate<Tpredicate>;
    _pushed = true;
    _consumer->consume_selected(base, n, P::preds, P::npred, g);
  }
  inline void step(input_t* aInput, globstat_t* g) {
    if (predicate_t::eval(aInput)) {
      inc();
      _consumer->step(aInput, g);
    }
  }
  inline void fin(globstat_t* g) {
    _consumer->fin(g);
    if constexpr (hj3d_pushdown_v<Tpredicate, Tconsumer, input_t, globstat_t>)
      if (_pushed) _count += _consumer->selected_count();
    stopTimer();
  }
  inline const consumer_t* consumer() const { return _consumer; }

 private:
  consumer_t* _consumer;
  bool _pushed = false;
};

// Dynamic selection operator (reference algebra.hh:318-358)
template <alg_consumer_c Tconsumer, alg_dyn_predicate_c Tpredicate>
class AlgDynSelection : public AlgBase {
 public:
  using consumer_t = Tconsumer;
  using globstat_t = typename consumer_t::globstat_t;
  using input_t = typename consumer_t::input_t;
  using output_t = typename consumer_t::input_t;
  using predicate_t = Tpredicate;

  inline AlgDynSelection(consumer_t* aConsumer, predicate_t aPredicate)
      : AlgBase("AlgDynSelection"), _consumer(aConsumer), _pred(aPredicate) {}
  inline AlgDynSelection(consumer_t* aConsumer) : AlgDynSelection(aConsumer, predicate_t()) {}
  inline void init(globstat_t* g) {
    reset();
    _pushed = false;
    _consumer->init(g);
  }
  inline void consume_relation(input_t* base, size_t n, globstat_t* g)
    requires(hj3d_pushdown_v<Tpredicate, Tconsumer, input_t, globstat_t>)
  {
    using P = hj3d::device_predicate<Tpredicate>;
    _pushed = true;
    _consumer->consume_selected(base, n, P::preds, P::npred, g);
  }
  inline void step(input_t* aInput, globstat_t* g) {
    if (_pred(aInput)) {
      inc();
      _consumer->step(aInput, g);
    }
  }
  inline void fin(globstat_t* g) {
    _consumer->fin(g);
    if constexpr (hj3d_pushdown_v<Tpredicate, Tconsumer, input_t, globstat_t>)
      if (_pushed) _count += _consumer->selected_count();
    stopTimer();
  }
  inline const consumer_t* consumer() const { return _consumer; }

 private:
  consumer_t* _consumer;
  predicate_t _pred;
  bool _pushed = false;
};

// ---- build operators ----

// 3D hash join build (reference algebra.hh:361-401)
template <alg_hashfun_c Thashfun, alg_binary_predicate_c Tequalfun, typename Tglobstat>
class AlgNestJoinBuild : public AlgBase {
 public:
  using globstat_t = Tglobstat;
  using hashfun_t = Thashfun;
  using input_t = typename hashfun_t::input_t;
  using output_t = void;
  using eqfun_t = Tequalfun;
  using hashtable_t = HtNested1<input_t, hashfun_t, eqfun_t>;

  AlgNestJoinBuild(const size_t aHashDirSize, const uint32_t aHtLog2ChunkSizeMain, const uint32_t aHtLog2ChunkSizeSub)
      : AlgBase("AlgNestJoinBuild"), _hashtable(aHashDirSize, aHtLog2ChunkSizeMain, aHtLog2ChunkSizeSub) {}
  AlgNestJoinBuild(const globstat_t* g)
      : AlgNestJoinBuild(g->_ht_num_buckets, g->_ht_rsv_log2_chunksize_main, g->_ht_rsv_log2_chunksize_sub) {}

  inline void init([[maybe_unused]] globstat_t* g) { reset(); }
  inline void step(input_t* aInput, [[maybe_unused]] globstat_t* g) {
    inc();
    _hashtable.insert(aInput);
  }
  inline void consume_relation(input_t* base, size_t n, [[maybe_unused]] globstat_t* g) {
    _count += n;
    _hashtable.insert_batch(base, n);
  }
  inline void fin([[maybe_unused]] globstat_t* g) {
    _hashtable.device().table();  // device build of everything inserted
    stopTimer();
  }
  inline const hashtable_t& hashtable() const { return _hashtable; }
  inline void clear_ht() { _hashtable.clear(); }

 private:
  hashtable_t _hashtable;
};

// regular hash join build (reference algebra.hh:555-586)
template <alg_hashfun_c Thashfun, alg_binary_predicate_c Tequalfun, typename Tglobstat>
class AlgHashJoinBuild : public AlgBase {
 public:
  using globstat_t = Tglobstat;
  using hashfun_t = Thashfun;
  using input_t = typename hashfun_t::input_t;
  using output_t = void;
  using eqfun_t = Tequalfun;
  using hashtable_t = HtChaining1<input_t, hashfun_t, eqfun_t>;

  AlgHashJoinBuild(const size_t aHashDirSize, const uint32_t aHtLog2ChunkSize)
      : AlgBase("AlgHashJoinBuild"), _hashtable(aHashDirSize, aHtLog2ChunkSize) {}
  AlgHashJoinBuild(const globstat_t* g) : AlgHashJoinBuild(g->_ht_num_buckets, g->_ht_rsv_log2_chunksize) {}

  inline void init([[maybe_unused]] globstat_t* g) { reset(); }
  inline void step(input_t* aTuple, [[maybe_unused]] globstat_t* g) {
    inc();
    _hashtable.insert(aTuple);
  }
  inline void consume_relation(input_t* base, size_t n, [[maybe_unused]] globstat_t* g) {
    _count += n;
    _hashtable.insert_batch(base, n);
  }
  inline void fin([[maybe_unused]] globstat_t* g) {
    _hashtable.device().table();
    stopTimer();
  }
  inline const hashtable_t& hashtable() const { return _hashtable; }
  inline void clear_ht() { _hashtable.clear(); }

 private:
  hashtable_t _hashtable;
};

// ---- pipeline shape traits (which strands run fused on the device) ----
template <typename T>
struct hj3d_is_top : std::false_type {};
template <typename I, typename G>
struct hj3d_is_top<AlgTop<I, G>> : std::true_type {};

template <alg_consumer_c Tconsumer, alg_unnestfun_c Tunnestfun, typename Thtnested>
class AlgUnnestHt;
template <typename T>
struct hj3d_is_unnest : std::false_type {};
template <typename C, typename U, typename H>
struct hj3d_is_unnest<AlgUnnestHt<C, U, H>> : std::true_type {};

template <alg_consumer_c Tconsumer, alg_buildop_c Tbuild, alg_hashfun_c Thashfun, alg_binary_predicate_c Tjoinpred,
          alg_concatfun_c Tconcatfun>
class AlgNestJoinProbe;
template <typename T>
struct hj3d_is_nest_probe : std::false_type {};
template <typename C, typename B, typename H, typename J, typename K>
struct hj3d_is_nest_probe<AlgNestJoinProbe<C, B, H, J, K>> : std::true_type {};

template <alg_consumer_c Tconsumer, alg_buildop_c Tbuild, alg_hashfun_c Thashfun, alg_binary_predicate_c Tjoinpred,
          alg_concatfun_c Tconcatfun, bool IsBuildKeyUnique>
class AlgHashJoinProbe;
template <typename T>
struct hj3d_is_hash_probe : std::false_type {};
template <typename C, typename B, typename H, typename J, typename K, bool U>
struct hj3d_is_hash_probe<AlgHashJoinProbe<C, B, H, J, K, U>> : std::true_type {};

namespace hj3d::host {

inline hj3d_probe_res run_probe(hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out = nullptr, uint64_t cap = 0) {
  Engine& e = Engine::get();
  e.check(hj3d_probe(e.ctx(), t, &r, flags, out, cap), "hj3d_probe");
  hj3d_probe_res res{};
  e.check(hj3d_probe_result(e.ctx(), &res), "hj3d_probe");
  return res;
}

inline hj3d_probe_res run_probe_sel(hj3d_table* t, const hj3d_rel& r, const hj3d_sel_pred* preds, uint32_t npred,
                                    uint32_t flags) {
  Engine& e = Engine::get();
  e.check(hj3d_probe_sel(e.ctx(), t, &r, preds, npred, flags, nullptr, 0), "hj3d_probe_sel");
  hj3d_probe_res res{};
  e.check(hj3d_probe_result(e.ctx(), &res), "hj3d_probe_sel");
  return res;
}

inline hj3d_probe2_res run_probe2(hj3d_table* ts, hj3d_table* tt, const hj3d_rel& r) {
  Engine& e = Engine::get();
  e.check(hj3d_probe2(e.ctx(), ts, tt, &r, 0, nullptr, 0), "hj3d_probe2");
  hj3d_probe2_res res{};
  e.check(hj3d_probe2_result(e.ctx(), &res), "hj3d_probe2");
  return res;
}

// Two hash functors agree on `n` sampled inputs (used to check that the second probe of an
// experiment-4 strand is keyed on the first probe's attribute).
template <typename F, typename G>
inline bool same_hash_on_samples(uint64_t n, F&& f, G&& g) {
  const uint64_t k = n < 16 ? n : 16;
  for (uint64_t j = 0; j < k; ++j) {
    const uint64_t i = (k <= 1) ? 0 : (j * (n - 1)) / (k - 1);
    if (uint64_t(f(i)) != uint64_t(g(i))) return false;
  }
  return true;
}

}  // namespace hj3d::host

// ---- probe operators ----

/*
 * 3D hash join probe (reference algebra.hh:404-473). count() = probe tuples with a match;
 * numCmps() = main-chain comparisons (bit-exact).
 */
template <alg_consumer_c Tconsumer, alg_buildop_c Tbuild, alg_hashfun_c Thashfun, alg_binary_predicate_c Tjoinpred,
          alg_concatfun_c Tconcatfun>
class AlgNestJoinProbe : public AlgBase {
  template <alg_consumer_c, alg_buildop_c, alg_hashfun_c, alg_binary_predicate_c, alg_concatfun_c>
  friend class AlgNestJoinProbe;

 public:
  using consumer_t = Tconsumer;
  using build_t = Tbuild;
  using hashfun_t = Thashfun;
  using globstat_t = typename consumer_t::globstat_t;
  using input_t = typename hashfun_t::input_t;
  using output_t = typename consumer_t::input_t;
  using joinpred_t = Tjoinpred;
  using concatfun_t = Tconcatfun;

  AlgNestJoinProbe(consumer_t* aConsumer, build_t* aBuildOperator)
      : AlgBase("AlgNestJoinProbe"), _consumer(aConsumer), _buildOperator(aBuildOperator), _numCmps(0) {}

  inline void init(globstat_t* g) {
    reset();
    _numCmps = 0;
    _in.clear();
    _absorbed = false;
    _consumer->init(g);
  }
  inline void step(input_t* aProbeTuple, [[maybe_unused]] globstat_t* g) { _in.ptrs.push_back(aProbeTuple); }
  inline void consume_relation(input_t* base, size_t n, [[maybe_unused]] globstat_t* g) {
    _in.base = base;
    _in.n = n;
  }
  // the scanned relation behind a pushed-down selection (AlgSelection with hj3d::device_predicate)
  inline void consume_selected(input_t* base, size_t n, const hj3d_sel_pred* preds, uint32_t npred,
                               [[maybe_unused]] globstat_t* g) {
    _in.base = base;
    _in.n = n;
    _in.preds = preds;
    _in.npred = npred;
    _in.selecting = true;
  }
  inline uint64_t selected_count() const { return _dev.n_selected; }
  inline void fin(globstat_t* g) {
    if (!_absorbed) execute(g);
    _consumer->fin(g);
    stopTimer();
  }
  inline const consumer_t* consumer() const { return _consumer; }
  inline uint64_t numCmps() const { return _numCmps; }

 private:
  using ht_t = typename build_t::hashtable_t;

  void execute(globstat_t* g) {
    using namespace hj3d::host;
    auto& dt = _buildOperator->hashtable().device();
    hj3d_table* t = dt.table();
    _dev.make(_in, "AlgNestJoinProbe");
    _dev.ensure_selected();
    if (_dev.key_word && dt.key_word() && _in.size() && dt.rows())
      check_joinpred<joinpred_t>(_in.at(0), *_dev.key_word, dt.row_ptr(0), *dt.key_word(), "AlgNestJoinProbe");

    if constexpr (hj3d_is_top<consumer_t>::value) {
      // NrsNU: probe -> Top (main_experiment1.cc:1187-1285)
      if (!_consumer->prints()) {
        const hj3d_probe_res r = run_probe(t, _dev.rel, 0);
        absorb(r.n_matched, r.n_cmps);
        OpAccess::add(*_consumer, r.n_matched);
        return;
      }
    } else if constexpr (hj3d_is_unnest<consumer_t>::value) {
      if constexpr (hj3d_is_top<typename consumer_t::consumer_t>::value) {
        // Nsr / Nrs: probe -> unnest -> Top (main_experiment1.cc:969-1185)
        auto* top = const_cast<typename consumer_t::consumer_t*>(_consumer->consumer());
        if (!top->prints()) {
          const hj3d_probe_res r = run_probe(t, _dev.rel, HJ3D_PROBE_UNNEST);
          absorb(r.n_matched, r.n_cmps);
          OpAccess::add(*_consumer, r.n_out);
          OpAccess::add(*top, r.n_out);
          return;
        }
      }
    } else if constexpr (hj3d_is_nest_probe<consumer_t>::value) {
      // experiment 4 Ndu: probe(S) -> probe(T) -> unnest(T) -> unnest(S) -> Top
      // (main_experiment4.cc:831-927), deferred unnesting fused in one device strand
      using p2_t = consumer_t;
      using u1_t = typename p2_t::consumer_t;
      if constexpr (hj3d_is_unnest<u1_t>::value) {
        using u2_t = typename u1_t::consumer_t;
        if constexpr (hj3d_is_unnest<u2_t>::value) {
          using top_t = typename u2_t::consumer_t;
          if constexpr (hj3d_is_top<top_t>::value) {
            auto* p2 = _consumer;
            auto* u1 = const_cast<u1_t*>(p2->consumer());
            auto* u2 = const_cast<u2_t*>(u1->consumer());
            auto* top = const_cast<top_t*>(u2->consumer());
            auto& dt2 = p2->_buildOperator->hashtable().device();
            hj3d_table* t2 = dt2.table();
            if (!top->prints() && second_key_matches(dt)) {
              const hj3d_probe2_res r = run_probe2(t, t2, _dev.rel);
              absorb(r.c_probe_rs, r.c_probe_rs_cmp);
              p2->absorb(r.c_probe_rt, r.c_probe_rt_cmp);
              OpAccess::add(*u1, r.c_unnest_1);
              OpAccess::add(*u2, r.c_unnest_2);
              OpAccess::add(*top, r.c_top);
              return;
            }
          }
        }
      }
    }
    host_probe(g);
  }

  // Any other consumer pipeline (a printing Top, a custom consumer, an unnest into something
  // else): the reference's tuple-at-a-time probe (algebra.hh:435-459) over the host node view of
  // the device table (HtNested1::findMainNodeByOther), pushing nested tuples in probe order.
  // Correct but slow; the fused strands above are the fast path.
  void host_probe(globstat_t* g) {
    const auto& ht = _buildOperator->hashtable();
    auto push = [&](input_t* t) {
      const auto [mn, cmps] = ht.template findMainNodeByOther<input_t, hashfun_t, joinpred_t>(t);
      _numCmps += cmps;
      if (mn == nullptr) return;
      output_t o = concatfun_t::eval(t, mn);
      inc();
      _consumer->step(&o, g);
    };
    if (_dev.n_selected != _in.size() || _dev.rel.row_off != HJ3D_ROW_IMPLICIT) {
      // a device selection was applied: its passing rows, in scan order
      std::vector<uint32_t> pr(2 * _dev.rel.n);
      hj3d::host::Engine& e = hj3d::host::Engine::get();
      if (_dev.rel.n) e.check(hj3d_download(e.ctx(), pr.data(), _dev.rel.base, _dev.rel.n * 8), "hj3d_download (selection)");
      for (uint64_t i = 0; i < _dev.rel.n; ++i) push(_in.at(pr[2 * i + 1]));
    } else {
      for (uint64_t i = 0; i < _in.size(); ++i) push(_in.at(i));
    }
    _absorbed = true;
  }

  // the second probe's hash of concat(r, <a main node of this table>) equals this probe's hash of r
  template <typename Tdt>
  bool second_key_matches(Tdt& dt) {
    using p2_t = consumer_t;
    if (_in.size() == 0 || dt.rows() == 0) return true;  // nothing to probe
    typename ht_t::MainNode mn(dt.row_ptr(0));
    return hj3d::host::same_hash_on_samples(
        _in.size(), [&](uint64_t i) { return hashfun_t::eval(_in.at(i)); },
        [&](uint64_t i) {
          auto nested = concatfun_t::eval(_in.at(i), &mn);
          return p2_t::hashfun_t::eval(&nested);
        });
  }

  void absorb(uint64_t matched, uint64_t cmps) {
    _count += matched;
    _numCmps += cmps;
    _absorbed = true;
  }

  consumer_t* _consumer;
  build_t* _buildOperator;
  uint64_t _numCmps;
  hj3d::host::Input<input_t> _in;
  hj3d::host::DevInput<hashfun_t> _dev;
  bool _absorbed = false;
};

/*
 * 3D hash join unnest (reference algebra.hh:476-552). count() = unnested output tuples.
 * Runs fused inside the preceding AlgNestJoinProbe on the device; nested tuples pushed to step()
 * (the host probe path of AlgNestJoinProbe, or other code holding main nodes of HtNested1's host
 * node view) are expanded on the host as the reference does: the main node's tuple, then its
 * sub-chain.
 */
template <alg_consumer_c Tconsumer, alg_unnestfun_c Tunnestfun, typename Thtnested>
class AlgUnnestHt : public AlgBase {
 public:
  using consumer_t = Tconsumer;
  using globstat_t = typename consumer_t::globstat_t;
  using unnestfun_t = Tunnestfun;
  using output_t = typename consumer_t::input_t;
  using input_t = typename unnestfun_t::input_t;
  using ht_nested_t = Thtnested;
  static_assert(std::is_same_v<output_t, typename unnestfun_t::output_t>,
                "AlgUnnestHt::output_t (aka consumer_t::input_t) does not match unnestfun_t::output_t");

  inline AlgUnnestHt(consumer_t* aConsumer) : AlgBase("AlgUnnest"), _consumer(aConsumer) {}
  inline void init(globstat_t* g) {
    reset();
    _consumer->init(g);
  }
  inline void step(input_t* aNestedTuple, globstat_t* g) {
    const auto* mn = unnestfun_t::getMainNode(aNestedTuple);
    unnestfun_t::eval_left(&_outputTuple, aNestedTuple);
    unnestfun_t::eval_right(&_outputTuple, aNestedTuple, mn->data());
    _consumer->step(&_outputTuple, g);
    inc();
    for (auto* sn = mn->child(); sn != nullptr; sn = sn->next()) {
      unnestfun_t::eval_right(&_outputTuple, aNestedTuple, sn->data());
      _consumer->step(&_outputTuple, g);
      inc();
    }
  }
  inline void fin(globstat_t* g) {
    _consumer->fin(g);
    stopTimer();
  }
  inline const consumer_t* consumer() const { return _consumer; }

 private:
  consumer_t* _consumer;
  output_t _outputTuple{};
};

/*
 * Regular hash join probe (reference algebra.hh:589-672). count() = output tuples;
 * numCmps() = collision-chain comparisons (bit-exact, early exit when IsBuildKeyUnique).
 */
template <alg_consumer_c Tconsumer, alg_buildop_c Tbuild, alg_hashfun_c Thashfun, alg_binary_predicate_c Tjoinpred,
          alg_concatfun_c Tconcatfun, bool IsBuildKeyUnique = false>
class AlgHashJoinProbe : public AlgBase {
  template <alg_consumer_c, alg_buildop_c, alg_hashfun_c, alg_binary_predicate_c, alg_concatfun_c, bool>
  friend class AlgHashJoinProbe;

 public:
  using consumer_t = Tconsumer;
  using build_t = Tbuild;
  using hashfun_t = Thashfun;
  using globstat_t = typename consumer_t::globstat_t;
  using input_t = typename hashfun_t::input_t;
  using output_t = typename consumer_t::input_t;
  using hashvalue_t = typename hashfun_t::output_t;
  using joinpred_t = Tjoinpred;
  using concatfun_t = Tconcatfun;

  inline AlgHashJoinProbe(consumer_t* aConsumer, build_t* aBuildOperator)
      : AlgBase("AlgHashJoinProbe"), _consumer(aConsumer), _buildOperator(aBuildOperator), _numCmps(0) {}

  inline void init(globstat_t* g) {
    reset();
    _numCmps = 0;
    _in.clear();
    _absorbed = false;
    _consumer->init(g);
  }
  inline void step(input_t* aTuple, [[maybe_unused]] globstat_t* g) { _in.ptrs.push_back(aTuple); }
  inline void consume_relation(input_t* base, size_t n, [[maybe_unused]] globstat_t* g) {
    _in.base = base;
    _in.n = n;
  }
  // the scanned relation behind a pushed-down selection (AlgSelection with hj3d::device_predicate)
  inline void consume_selected(input_t* base, size_t n, const hj3d_sel_pred* preds, uint32_t npred,
                               [[maybe_unused]] globstat_t* g) {
    _in.base = base;
    _in.n = n;
    _in.preds = preds;
    _in.npred = npred;
    _in.selecting = true;
  }
  inline uint64_t selected_count() const { return _dev.n_selected; }
  inline void fin(globstat_t* g) {
    if (!_absorbed) execute(g);
    _consumer->fin(g);
    stopTimer();
  }
  inline const consumer_t* consumer() const { return _consumer; }
  inline uint64_t numCmps() const { return _numCmps; }

 private:
  static constexpr uint32_t kFlags = IsBuildKeyUnique ? HJ3D_PROBE_UNIQUE : 0u;

  void execute(globstat_t* g) {
    using namespace hj3d::host;
    auto& dt = _buildOperator->hashtable().device();
    hj3d_table* t = dt.table();
    _dev.make(_in, "AlgHashJoinProbe");
    if (_dev.key_word && dt.key_word() && _in.size() && dt.rows())
      check_joinpred<joinpred_t>(_in.at(0), *_dev.key_word, dt.row_ptr(0), *dt.key_word(), "AlgHashJoinProbe");

    if constexpr (hj3d_is_top<consumer_t>::value) {
      // Csr / CsrUU / Crs: probe -> Top (main_experiment1.cc:623-967)
      if (!_consumer->prints()) {
        // a pushed-down selection runs fused into the probe partitioner (hj3d_probe_sel)
        const hj3d_probe_res r = _dev.pending_sel ? run_probe_sel(t, _dev.rel, _dev.preds, _dev.npred, kFlags)
                                                  : run_probe(t, _dev.rel, kFlags);
        if (_dev.pending_sel) {
          _dev.pending_sel = false;
          _dev.n_selected = r.n_probe;
        }
        absorb(r.n_out, r.n_cmps);
        OpAccess::add(*_consumer, r.n_out);
        return;
      }
    }
    _dev.ensure_selected();  // the other pipelines take the selected pairs
    if constexpr (hj3d_is_hash_probe<consumer_t>::value) {
      // experiment 4 Chj: probe(S) -> probe(T) -> Top (main_experiment4.cc:929-1043)
      using p2_t = consumer_t;
      using top_t = typename p2_t::consumer_t;
      if constexpr (hj3d_is_top<top_t>::value && !IsBuildKeyUnique) {
        auto* p2 = _consumer;
        auto* top = const_cast<top_t*>(p2->consumer());
        auto& dt2 = p2->_buildOperator->hashtable().device();
        hj3d_table* t2 = dt2.table();
        if (!top->prints() && p2_t::kFlags == 0 && second_key_matches(dt)) {
          const hj3d_probe2_res r = run_probe2(t, t2, _dev.rel);
          absorb(r.c_probe_rs, r.c_probe_rs_cmp);
          p2->absorb(r.c_probe_rt, r.c_probe_rt_cmp);
          OpAccess::add(*top, r.c_top);
          return;
        }
      }
    }
    emit_and_push(t, dt, g);
  }

  // Materialise the output pairs on the device, then push concat(probe, build) tuples to the
  // consumer in the reference's order: probe order, and per probe tuple the chain walk order
  // (first inserted, then newest first; ht_chaining.hh:181-196).
  template <typename Tdt>
  void emit_and_push(hj3d_table* t, Tdt& dt, globstat_t* g) {
    using namespace hj3d::host;
    Engine& e = Engine::get();
    const uint64_t n = _dev.rel.n;  // probe tuples (the passing ones under a device selection)
    uint64_t cap = n;
    if (!IsBuildKeyUnique) cap = run_probe(t, _dev.rel, kFlags).n_out;
    DevBuffer buf;
    void* d = buf.ensure((cap ? cap : 1) * 8);
    const hj3d_probe_res r = run_probe(t, _dev.rel, kFlags | HJ3D_PROBE_EMIT, d, cap);
    const uint64_t slots = IsBuildKeyUnique ? n : r.n_out;
    std::vector<uint32_t> pairs(2 * slots);
    if (slots) e.check(hj3d_download(e.ctx(), pairs.data(), d, slots * 8), "hj3d_download (pairs)");
    std::vector<std::pair<uint32_t, uint32_t>> out;
    out.reserve(r.n_out);
    for (uint64_t i = 0; i < slots; ++i)
      if (pairs[2 * i + 1] != 0xFFFFFFFFu) out.emplace_back(pairs[2 * i], pairs[2 * i + 1]);
    // per probe tuple: smallest build row first, then descending
    std::sort(out.begin(), out.end(), [](const auto& x, const auto& y) {
      return x.first != y.first ? x.first < y.first : x.second > y.second;
    });
    for (size_t lo = 0; lo < out.size();) {
      size_t hi = lo;
      while (hi < out.size() && out[hi].first == out[lo].first) ++hi;
      std::rotate(out.begin() + lo, out.begin() + hi - 1, out.begin() + hi);
      lo = hi;
    }
    _numCmps += r.n_cmps;
    for (const auto& [a, b] : out) {
      output_t o = concatfun_t::eval(_in.at(a), dt.row_ptr(b));
      inc();
      _consumer->step(&o, g);
    }
  }

  template <typename Tdt>
  bool second_key_matches(Tdt& dt) {
    using p2_t = consumer_t;
    if (_in.size() == 0 || dt.rows() == 0) return true;
    return hj3d::host::same_hash_on_samples(
        _in.size(), [&](uint64_t i) { return hashfun_t::eval(_in.at(i)); },
        [&](uint64_t i) {
          auto rs = concatfun_t::eval(_in.at(i), dt.row_ptr(0));
          return p2_t::hashfun_t::eval(&rs);
        });
  }

  void absorb(uint64_t out, uint64_t cmps) {
    _count += out;
    _numCmps += cmps;
    _absorbed = true;
  }

  consumer_t* _consumer;
  build_t* _buildOperator;
  uint64_t _numCmps;
  hj3d::host::Input<input_t> _in;
  hj3d::host::DevInput<hashfun_t> _dev;
  bool _absorbed = false;
};

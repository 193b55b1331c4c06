// ht_nested.hh — HtNested1, the nested ("3D") hash table, on the MI355X (reference:
// ht_nested.hh:37-492).
//
// Same template signature and member types as the reference (MainNode, SubNode, data_t are
// named by the drivers' nested tuple and unnest functor types). The table lives on the device
// (one main record per distinct key + a row list per key); probe, unnest and
// deferred unnest run fused on the device through the algebra.hh operators. MainNode / SubNode
// are real nodes: findMainNodeByOther returns the reference's main node (with its sub-chain),
// rebuilt on the host from the device table, for per-tuple callers and host-side consumers.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

#include "concepts.hh"
#include "hj3d_host.hh"
#include "ht_iterators.hh"
#include "ht_statistics.hh"

template <typename Tdata, alg_hashfun_c Thashfun, alg_binary_predicate_c Tcontenteqfun>
class HtNested1 {
  static_assert(std::same_as<Tdata, typename Thashfun::input_t>, "Thashfun::input_t does not match Tdata");
  static_assert(std::same_as<Tdata, typename Tcontenteqfun::left_t> && std::same_as<Tdata, typename Tcontenteqfun::right_t>,
                "Tcontenteqfun::left_t/right_t do not match Tdata");

 public:
  struct MainNode;
  struct SubNode;
  using data_t = Tdata;
  using hashfun_t = Thashfun;
  using hashvalue_t = typename hashfun_t::output_t;
  using eqfun_t = Tcontenteqfun;
  using main_node_iterator = NodeIterator<MainNode, false>;
  using const_main_node_iterator = NodeIterator<MainNode, true>;
  using sub_node_iterator = NodeIterator<SubNode, false>;
  using const_sub_node_iterator = NodeIterator<SubNode, true>;
  using stats_t = HtStatistics;

  inline static MainNode* EMPTY_ENTRY = reinterpret_cast<MainNode*>(0x1);
  inline static SubNode* UNINITIALIZED_SUBNODE = reinterpret_cast<SubNode*>(0x1);

  // One distinct key: its first tuple + the list of the others (ht_nested.hh:111-160).
  struct MainNode {
    MainNode* _next;
    SubNode* _subchain_head;
    data_t* _data;
    hashvalue_t _hashvalue;

    MainNode(data_t* d) : _next(nullptr), _subchain_head(nullptr), _data(d), _hashvalue(0) {}
    MainNode() : _next(EMPTY_ENTRY), _subchain_head(nullptr), _data(nullptr), _hashvalue(0) {}
    const data_t* data() const { return _data; }
    hashvalue_t hashvalue() const { return _hashvalue; }
    MainNode* next() const { return isEmpty() ? nullptr : _next; }
    SubNode* child() const { return _subchain_head; }
    bool isEmpty() const { return _next == EMPTY_ENTRY; }
    bool hasNext() const { return !isEmpty() && next() != nullptr; }
    bool hasChild() const { return child() != nullptr; }
    void init(data_t* d, const hashvalue_t h) {
      _next = nullptr;
      _subchain_head = nullptr;
      _data = d;
      _hashvalue = h;
    }
    void clear() { _next = EMPTY_ENTRY; }
    main_node_iterator begin() { return main_node_iterator(this); }
    main_node_iterator end() { return main_node_iterator(nullptr); }
    const_main_node_iterator cbegin() const { return const_main_node_iterator(this); }
    const_main_node_iterator cend() const { return const_main_node_iterator(nullptr); }
  };

  // A further tuple of one key (ht_nested.hh:163-183).
  struct SubNode {
    SubNode* _next;
    data_t* _data;

    SubNode() : _next(UNINITIALIZED_SUBNODE), _data(nullptr) {}
    SubNode(data_t* d, SubNode* next) : _next(next), _data(d) {}
    SubNode(data_t* d) : SubNode(d, nullptr) {}
    const data_t* data() const { return _data; }
    bool hasNext() const { return _next != nullptr; }
    SubNode* next() const { return _next; }
    void init(data_t* d, SubNode* next) {
      _data = d;
      _next = next;
    }
    void init(data_t* d) { init(d, nullptr); }
    sub_node_iterator begin() { return sub_node_iterator(this); }
    sub_node_iterator end() { return sub_node_iterator(nullptr); }
    const_sub_node_iterator cbegin() const { return const_sub_node_iterator(this); }
    const_sub_node_iterator cend() const { return const_sub_node_iterator(nullptr); }
  };

 public:
  HtNested1(const size_t aNumBuckets, [[maybe_unused]] const uint32_t aMainRsvLog2ChunkSize,
            [[maybe_unused]] const uint32_t aSubRsvLog2ChunkSize)
      : _dev(HJ3D_NESTED, aNumBuckets), _size(0) {}

  size_t numBuckets() const { return _dev.num_buckets(); }
  hashvalue_t hash(const data_t* d) const { return hashfun_t::eval(d); }
  size_t size() const { return _size; }
  size_t getRsvMainSize() const { return 0; }
  size_t getRsvSubSize() const { return 0; }
  size_t memoryConsupmtion() const { return memoryConsupmtionDir() + memoryConsupmtionSubChains(); }
  size_t memoryConsupmtionDir() const { return (numBuckets() + 1) * 4; }
  size_t memoryConsupmtionMainChains() const { return 0; }
  size_t memoryConsupmtionSubChains() const { return _dev.rows() * 4; }

  // HtNested1::insert (ht_nested.hh:287-311): recorded, built on the device on first use
  void insert(data_t* d) {
    _dev.add_one(d);
    ++_size;
  }
  void insert_batch(data_t* base, size_t n) {
    _dev.add_batch(base, n);
    _size += n;
  }
  void clear() { _dev.clear(); }

  stats_t makeStatistics() const { return HtStatistics::from(_dev.stats(), _size); }

  // HtNested1::findMainNodeByOther (ht_nested.hh:354-382): the main node of the probe tuple's key
  // and the main-chain comparisons, walked as the reference walks them. Correct but slow: the
  // first call after a build copies the device table to the host and materialises the reference's
  // node layout (main nodes in first-occurrence order, each key's further tuples as a sub-chain,
  // newest first), whose MainNode / SubNode pointers an unnest functor can then follow.
  template <typename Tprobedata, alg_hashfun_c Tprobehashfun, alg_binary_predicate_c Tjoinpred>
  const std::tuple<const MainNode*, const uint64_t> findMainNodeByOther(const Tprobedata* aProbeTuple) const {
    static_assert(std::is_same_v<hashvalue_t, typename Tprobehashfun::output_t>);
    const hashvalue_t h = Tprobehashfun::eval(aProbeTuple);
    nodes();
    const MainNode* n = &_dir[size_t(h) % numBuckets()];
    uint64_t cmps = 0;
    do {
      if (n->isEmpty()) return {nullptr, cmps};
      ++cmps;
      if (n->hashvalue() == h && Tjoinpred::eval(aProbeTuple, n->data())) return {n, cmps};
      n = n->next();
    } while (n != nullptr);
    return {nullptr, cmps};
  }

  // the device table is built lazily, hence mutable behind the const observers
  hj3d::host::DeviceTable<data_t, hashfun_t>& device() const { return _dev; }

 private:
  // the reference's node layout rebuilt from the host mirror of the device table
  void nodes() const {
    auto& dev = _dev;
    const auto& m = dev.mirror();
    if (_nodes_version == dev.version()) return;
    const size_t nb = numBuckets();
    _dir.assign(nb, MainNode());
    _mains.clear();
    _mains.reserve(m.n_payload);
    _subs.clear();
    _subs.reserve(m.sub.size());
    std::vector<std::pair<uint32_t, uint32_t>> mains;  // (first row, main record) of one bucket
    std::vector<uint32_t> rows;
    for (size_t k = 0; k < nb; ++k) {
      const uint32_t s = m.off[k], e = m.off[k + 1];
      if (s == e) continue;
      mains.clear();
      for (uint32_t i = s; i < e; ++i) mains.emplace_back(m.payload[4 * i + 1], i);
      std::sort(mains.begin(), mains.end());  // first-occurrence order of the keys
      MainNode* prev = nullptr;
      for (size_t j = 0; j < mains.size(); ++j) {
        const uint32_t* rec = &m.payload[4 * size_t(mains[j].second)];
        MainNode* mn = j == 0 ? &_dir[k] : &_mains.emplace_back();
        mn->init(dev.row_ptr(rec[1]), hashvalue_t(rec[0]));
        // sub-chain: the key's other tuples, head-inserted, so the newest comes first
        rows.assign(m.sub.begin() + rec[2], m.sub.begin() + rec[2] + rec[3]);
        std::sort(rows.begin(), rows.end());
        SubNode* head = nullptr;
        for (size_t q = 1; q < rows.size(); ++q) head = &_subs.emplace_back(dev.row_ptr(rows[q]), head);
        mn->_subchain_head = head;
        if (prev) prev->_next = mn;
        prev = mn;
      }
    }
    _nodes_version = dev.version();
  }

  mutable hj3d::host::DeviceTable<data_t, hashfun_t> _dev;
  size_t _size;
  mutable std::vector<MainNode> _dir, _mains;
  mutable std::vector<SubNode> _subs;
  mutable uint64_t _nodes_version = 0;
};

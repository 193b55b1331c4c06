// ht_chaining.hh — HtChaining1 on the MI355X (reference: ht_chaining.hh:37-294).
//
// Same template signature, member types and observers as the reference, so plans that name
// HtChaining1<...>::Node / data_t / hashvalue_t or call numBuckets()/size()/makeStatistics()
// compile unchanged. The table itself lives on the device (CSR buckets of {hash, row}, see
// DESIGN.md §3): insert() records tuples, the device build runs at the first probe or
// statistics call after an insert, and probing is done by the algebra.hh probe operators
// through the C ABI. Node (24 B, as the reference prints it) is a real node: per-tuple callers
// of findDirEntryByOther get the reference's directory slot and chain, rebuilt on the host from
// the device table.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <type_traits>
#include <utility>
#include <vector>

#include "concepts.hh"
#include "hj3d_host.hh"
#include "ht_iterators.hh"
#include "ht_statistics.hh"

template <typename Tdata, alg_hashfun_c Thashfun, alg_binary_predicate_c Tcontenteqfun>
class HtChaining1 {
  static_assert(std::same_as<Tdata, typename Thashfun::input_t>, "Thashfun::input_t does not match Tdata");
  static_assert(std::same_as<Tdata, typename Tcontenteqfun::left_t> && std::same_as<Tdata, typename Tcontenteqfun::right_t>,
                "Tcontenteqfun::left_t/right_t do not match Tdata");

 public:
  struct Node;
  using data_t = Tdata;
  using hashfun_t = Thashfun;
  using hashvalue_t = typename hashfun_t::output_t;
  using eqfun_t = Tcontenteqfun;
  using node_iterator = NodeIterator<Node, false>;
  using const_node_iterator = NodeIterator<Node, true>;
  using stats_t = HtStatistics;

  inline static Node* EMPTY_ENTRY = reinterpret_cast<Node*>(0x1);

  // A bucket node as the reference lays it out (ht_chaining.hh:69-103).
  struct Node {
    Node* _next;
    data_t* _data;
    hashvalue_t _hashvalue;

    Node(data_t* d) : _next(nullptr), _data(d), _hashvalue() {}
    Node() : _next(EMPTY_ENTRY), _data(), _hashvalue() {}
    void init(data_t* d, const hashvalue_t h, Node* next) {
      _data = d;
      _next = next;
      _hashvalue = h;
    }
    void init(data_t* d, const hashvalue_t h) { init(d, h, nullptr); }
    data_t* data() const { return _data; }
    Node* next() const { return isEmpty() ? nullptr : _next; }
    hashvalue_t hashvalue() const { return _hashvalue; }
    bool isEmpty() const { return _next == EMPTY_ENTRY; }
    bool hasNext() const { return !isEmpty() && _next != nullptr; }
    void clear() { _next = EMPTY_ENTRY; }
    node_iterator begin() { return node_iterator(this); }
    node_iterator end() { return node_iterator(nullptr); }
    const_node_iterator cbegin() const { return const_node_iterator(this); }
    const_node_iterator cend() const { return const_node_iterator(nullptr); }
  };

 public:
  HtChaining1(const size_t aNumBuckets, [[maybe_unused]] const uint32_t aReservoirLog2ChunkSize)
      : _dev(HJ3D_CHAIN, aNumBuckets), _size(0) {}

  size_t numBuckets() const { return _dev.num_buckets(); }
  hashvalue_t hash(const data_t* d) const { return hashfun_t::eval(d); }
  // inserts since construction: like the reference, clear() does not reset it
  size_t size() const { return _size; }
  size_t getRsvSize() const { return 0; }
  size_t memoryConsupmtion() const { return (numBuckets() + 1) * 4 + _dev.rows() * 8; }
  size_t memoryConsupmtionDir() const { return (numBuckets() + 1) * 4; }
  size_t memoryConsupmtionChains() const { return _dev.rows() * 8; }

  // HtChaining1::insert (ht_chaining.hh:181-196): recorded, built on the device on first use
  void insert(data_t* d) {
    _dev.add_one(d);
    ++_size;
  }
  // the whole scanned relation at once (AlgScan -> AlgHashJoinBuild)
  void insert_batch(data_t* base, size_t n) {
    _dev.add_batch(base, n);
    _size += n;
  }
  void clear() { _dev.clear(); }

  stats_t makeStatistics() const { return HtStatistics::from(_dev.stats(), _size); }

  // HtChaining1::findDirEntryByOther (ht_chaining.hh:236-248): the directory slot of the probe
  // tuple's bucket as the reference lays it out, walked through the reference's node iterator.
  // Correct but slow: the first call after a build copies the device table to the host and
  // materialises the reference's node layout from it (directory node = the bucket's first insert,
  // then the chain newest first), so per-tuple callers that walk the table themselves run
  // unchanged; the algebra.hh probe operators never take this path.
  template <typename Tprobedata, alg_hashfun_c Tprobehashfun>
  const_node_iterator findDirEntryByOther(const Tprobedata* aProbeTuple) const {
    static_assert(std::is_same_v<hashvalue_t, typename Tprobehashfun::output_t>);
    const hashvalue_t h = Tprobehashfun::eval(aProbeTuple);
    nodes();
    return const_node_iterator(&_dir[size_t(h) % numBuckets()]);
  }

  // ---- device access for the algebra.hh operators ----
  // the device table is built lazily, hence mutable behind the const observers
  hj3d::host::DeviceTable<data_t, hashfun_t>& device() const { return _dev; }

 private:
  // the reference's node layout rebuilt from the host mirror of the device table
  void nodes() const {
    auto& dev = _dev;
    const auto& m = dev.mirror();
    if (_nodes_version == dev.version()) return;
    const size_t nb = numBuckets();
    _dir.assign(nb, Node());
    _chain.clear();
    _chain.reserve(m.n_payload);
    std::vector<std::pair<uint32_t, uint32_t>> b;  // (row, hash) of one bucket
    for (size_t k = 0; k < nb; ++k) {
      const uint32_t s = m.off[k], e = m.off[k + 1];
      if (s == e) continue;
      b.clear();
      for (uint32_t i = s; i < e; ++i) b.emplace_back(m.payload[2 * i + 1], m.payload[2 * i]);
      std::sort(b.begin(), b.end());  // row order = insertion order
      Node* next = nullptr;
      for (size_t j = 1; j < b.size(); ++j) {  // chain: head-inserted, so the newest comes first
        _chain.emplace_back(dev.row_ptr(b[j].first));
        _chain.back().init(dev.row_ptr(b[j].first), hashvalue_t(b[j].second), next);
        next = &_chain.back();
      }
      _dir[k].init(dev.row_ptr(b[0].first), hashvalue_t(b[0].second), next);
    }
    _nodes_version = dev.version();
  }

  mutable hj3d::host::DeviceTable<data_t, hashfun_t> _dev;
  size_t _size;
  mutable std::vector<Node> _dir, _chain;
  mutable uint64_t _nodes_version = 0;
};

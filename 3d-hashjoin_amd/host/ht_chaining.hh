// ht_chaining.hh — HtChaining1 on the MI355X (reference: ht_chaining.hh:37-294).
//
// Same template signature, member types and observers as the reference, so plans that name
// HtChaining1<...>::Node / data_t / hashvalue_t or call numBuckets()/size()/makeStatistics()
// compile unchanged. The table itself lives on the device (CSR buckets of {hash, row}, see
// DESIGN.md §3): insert() records tuples, the device build runs at the first probe or
// statistics call after an insert, and probing is done by the algebra.hh probe operators
// through the C ABI. Node is kept as a type (24 B, as the reference prints it) for drivers
// that name it.
#pragma once

#include <cstddef>
#include <cstdint>
#include <type_traits>

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

  // Per-tuple probing of the device table is not offered; the probe operators of algebra.hh
  // probe whole inputs on the device.
  template <typename Tprobedata, alg_hashfun_c Tprobehashfun>
  const_node_iterator findDirEntryByOther(const Tprobedata*) const {
    throw hj3d::host::Error("hj3d: HtChaining1::findDirEntryByOther: per-tuple probes are not supported by the "
                            "device table; use AlgHashJoinProbe");
  }

  // ---- device access for the algebra.hh operators ----
  // the device table is built lazily, hence mutable behind the const observers
  hj3d::host::DeviceTable<data_t, hashfun_t>& device() const { return _dev; }

 private:
  mutable hj3d::host::DeviceTable<data_t, hashfun_t> _dev;
  size_t _size;
};

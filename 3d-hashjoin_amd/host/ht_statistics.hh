// ht_statistics.hh — HtStatistics as the drivers read it (reference: ht_statistics.hh:18-54),
// filled from hj3d_table_stats (device-side bucket scan, csrc/stats.hip) instead of a host walk
// over pointer chains.
#pragma once

#include <cstddef>
#include <cstdint>
#include <iostream>
#include <limits>
#include <ostream>
#include <sstream>
#include <string>
#include <vector>

#include "hj3d.h"

namespace hj3d::host {

// min / max / sum / count of one per-bucket quantity (the reference's Aggregate<size_t>,
// util/aggregate.hh: empty => min = max value of Num, max = 0).
template <typename Num>
struct BucketAggregate {
  Num _min = std::numeric_limits<Num>::max();
  Num _max = 0;
  Num _sum = 0;
  Num _count = 0;
  void step(Num x) {
    if (x < _min) _min = x;
    if (x > _max) _max = x;
    _sum += x;
    _count += 1;
  }
  void set(Num mn, Num mx, Num sum, Num count) {
    _count = count;
    _sum = sum;
    _min = count ? mn : std::numeric_limits<Num>::max();
    _max = count ? mx : 0;
  }
  Num count() const { return _count; }
  Num min() const { return _min; }
  Num max() const { return _max; }
  Num sum() const { return _sum; }
  double avg() const { return double(sum()) / double(count()); }
};

}  // namespace hj3d::host

struct HtBucketStatistics {
  size_t _bucketIndex = 0;
  size_t _numEntries = 0;
  size_t _chainLen = 0;
  std::string toCsvString() const {
    return std::to_string(_bucketIndex) + "," + std::to_string(_numEntries) + "," + std::to_string(_chainLen);
  }
};

struct HtStatistics {
  size_t _numBuckets = 0;
  size_t _numEmptyBuckets = 0;
  size_t _numEntries = 0;       // #stored key/data pairs (HtChaining1/HtNested1::size())
  size_t _numDistinctKeys = 0;
  hj3d::host::BucketAggregate<size_t> _collisionChainLen;          // over all buckets (cc0)
  hj3d::host::BucketAggregate<size_t> _collisionChainLenNonempty;  // over non-empty buckets (cc1)
  hj3d::host::BucketAggregate<size_t> _numDistinctKeysPerBucket;
  hj3d::host::BucketAggregate<size_t> _numDistinctKeysPerNonemptyBucket;
  std::vector<HtBucketStatistics> _bucketStats;

  double numEntriesPerKey() const { return (_numEntries + 0.0) / _numDistinctKeys; }
  double fracEmptyBuckets() const { return (_numEmptyBuckets + 0.0) / _numBuckets; }

  void reset() { *this = HtStatistics(); }

  // from the device statistics; `entries` is the table's size() (the reference keeps counting
  // inserts across clear(), ht_chaining.hh:250-258, and reports that)
  static HtStatistics from(const hj3d_stats& s, size_t entries) {
    HtStatistics h;
    h._numBuckets = s.nb;
    h._numEmptyBuckets = s.empty;
    h._numEntries = entries;
    h._numDistinctKeys = s.distinct;
    h._collisionChainLen.set(s.cc0_min, s.cc0_max, s.cc0_sum, s.cc0_cnt);
    h._collisionChainLenNonempty.set(s.cc1_min, s.cc1_max, s.cc1_sum, s.cc1_cnt);
    return h;
  }

  static std::string toCsvStringHeader() {
    return "numBuckets,numEmptyBuckets,fracEmpty,numEntries,numDistinctKeys,cc0_min,cc0_avg,cc0_max,cc1_min,cc1_avg,cc1_max";
  }
  std::string toCsvString() const {
    std::ostringstream os;
    os << _numBuckets << "," << _numEmptyBuckets << "," << fracEmptyBuckets() << "," << _numEntries << ","
       << _numDistinctKeys << "," << _collisionChainLen.min() << "," << _collisionChainLen.avg() << ","
       << _collisionChainLen.max() << "," << _collisionChainLenNonempty.min() << ","
       << _collisionChainLenNonempty.avg() << "," << _collisionChainLenNonempty.max();
    return os.str();
  }
  static std::string bucketStatToCsvStringHeader() { return "bucketIndex,numEntries,chainLen"; }
  std::string bucketStatToCsvString() const {
    std::string s;
    for (const auto& b : _bucketStats) s += b.toCsvString() + "\n";
    return s;
  }
  void print(std::ostream& os = std::cout) const {
    os << "buckets " << _numBuckets << ", empty " << _numEmptyBuckets << " (" << fracEmptyBuckets() << "), entries "
       << _numEntries << ", distinct keys " << _numDistinctKeys << ", chain length all [" << _collisionChainLen.min()
       << ", " << _collisionChainLen.avg() << ", " << _collisionChainLen.max() << "], non-empty ["
       << _collisionChainLenNonempty.min() << ", " << _collisionChainLenNonempty.avg() << ", "
       << _collisionChainLenNonempty.max() << "]\n";
  }
  void printCsv(std::ostream& os = std::cout) const { os << toCsvString() << "\n"; }
  static void printCsvHeader(std::ostream& os = std::cout) { os << toCsvStringHeader() << "\n"; }
};

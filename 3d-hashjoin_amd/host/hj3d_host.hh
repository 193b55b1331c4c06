// hj3d_host.hh — C++ host plumbing of the drop-in layer (algebra.hh / ht_chaining.hh /
// ht_nested.hh in this directory) over the C ABI of libhj3d.so (include/hj3d.h).
//
// The reference's operators push one tuple at a time through std::function-free templates
// (algebra.hh:259-269 AlgScan::run). Here every build/probe operator collects its whole input —
// the scanned relation (one batch) or the pushed tuple pointers — and hands it to the GPU at
// fin() through the C ABI. What this header provides:
//   * Engine: the process-wide hj3d context (device from $HJ3D_DEVICE, default 0). No GPU, no
//     engine: creation throws hj3d::host::Error. There is no CPU fallback.
//   * key_word_of<Thashfun>(): locates the u32 join attribute inside an opaque tuple type by
//     fingerprinting the hash functor (murmur3 fmix32 is a bijection, util/hasht.hh:52-61), and
//     check_joinpred<>() verifies that a join predicate is key equality on the located words.
//   * RelationCache: device copies of the host relations, re-uploaded when their contents change
//     (a full 64-bit fingerprint of every byte, computed in parallel; HJ3D_TRUST_RELATIONS=1
//     checks a 257-tuple sample instead, for drivers that never modify a relation in place).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "hj3d.h"

namespace hj3d {
// Opt-in selection pushdown. Specialise for a selection predicate (AlgSelection's Tpredicate or
// AlgDynSelection's functor type) with the same condition as hj3d_sel_pred terms, e.g. for
// `L.b < 40` on tuple {int a, b}:
//   template <> struct hj3d::device_predicate<SelectionL> {
//     static constexpr uint32_t npred = 1;
//     static constexpr hj3d_sel_pred preds[1] = {{4, HJ3D_SEL_LT, 1, 0, 40, 0}};
//   };
// Then a scanned relation flowing AlgScan -> AlgSelection -> a join probe operator is filtered by
// hj3d_select on the device; without it the selection runs on the host, tuple at a time.
template <typename Tpredicate>
struct device_predicate;
}  // namespace hj3d

namespace hj3d::host {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline uint32_t murmur32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// inverse of murmur32 (each step of fmix32 is invertible)
inline uint32_t murmur32_inv(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7ed1b41du;  // inverse of 0xc2b2ae35 mod 2^32
  x ^= (x >> 13) ^ (x >> 26);
  x *= 0xa5cb9243u;  // inverse of 0x85ebca6b mod 2^32
  x ^= x >> 16;
  return x;
}

class Engine {
 public:
  static Engine& get() {
    static Engine e;
    return e;
  }
  hj3d_ctx* ctx() const { return _ctx; }
  void check(hj3d_status s, const char* what) const {
    if (s != HJ3D_OK)
      throw Error(std::string("hj3d: ") + what + " failed (status " + std::to_string(int(s)) + "): " +
                  hj3d_last_error(_ctx));
  }
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

 private:
  Engine() {
    const char* d = std::getenv("HJ3D_DEVICE");
    const int dev = d ? std::atoi(d) : 0;
    const hj3d_status s = hj3d_ctx_create(dev, nullptr, &_ctx);
    if (s != HJ3D_OK)
      throw Error("hj3d: no usable MI355X device (hj3d_ctx_create status " + std::to_string(int(s)) +
                  "); the drop-in layer has no CPU path");
  }
  ~Engine() { hj3d_ctx_destroy(_ctx); }
  hj3d_ctx* _ctx = nullptr;
};

// Grow-only device buffer owned by the host layer.
class DevBuffer {
 public:
  DevBuffer() = default;
  DevBuffer(const DevBuffer&) = delete;
  DevBuffer& operator=(const DevBuffer&) = delete;
  ~DevBuffer() {
    if (_p) hj3d_dev_free(Engine::get().ctx(), _p);
  }
  void* ensure(uint64_t bytes) {
    if (bytes <= _bytes && _p) return _p;
    Engine& e = Engine::get();
    if (_p) e.check(hj3d_dev_free(e.ctx(), _p), "hj3d_dev_free");
    _p = nullptr;
    _bytes = 0;
    const uint64_t cap = bytes + bytes / 8 + 256;
    e.check(hj3d_dev_alloc(e.ctx(), cap, &_p), "hj3d_dev_alloc");
    _bytes = cap;
    return _p;
  }
  void* get() const { return _p; }

 private:
  void* _p = nullptr;
  uint64_t _bytes = 0;
};

// Device copies of host relations keyed by their address. A relation is re-uploaded when its
// size, stride or contents change: the fingerprint covers every byte (8-byte words folded by
// several threads for large relations), so a relation regenerated or modified in place at the
// same address is never joined from a stale device copy. HJ3D_TRUST_RELATIONS=1 fingerprints a
// 257-tuple sample instead (faster, unsafe under in-place modification); invalidate() forces the
// next upload either way.
class RelationCache {
 public:
  static RelationCache& get() {
    static RelationCache c;
    return c;
  }
  const void* upload(const void* host, uint64_t n, uint32_t stride) {
    Entry& e = _m[host];
    const uint64_t sig = trust_sample() ? sample(host, n, stride) : fingerprint(host, n * stride);
    if (e.buf && e.n == n && e.stride == stride && e.sig == sig && e.valid) return e.buf->get();
    if (!e.buf) e.buf = new DevBuffer();
    Engine& g = Engine::get();
    void* d = e.buf->ensure(n * stride);
    g.check(hj3d_upload(g.ctx(), d, host, n * stride), "hj3d_upload (relation)");
    e.n = n;
    e.stride = stride;
    e.sig = sig;
    e.valid = true;
    ++_uploads;
    return d;
  }
  void invalidate(const void* host) {
    auto it = _m.find(host);
    if (it != _m.end()) it->second.valid = false;
  }
  uint64_t uploads() const { return _uploads; }  // uploads so far (tests)
  ~RelationCache() {
    for (auto& kv : _m) delete kv.second.buf;
  }

  // 64-bit fingerprint of `bytes` bytes: per 8-byte word w at index i, mix(w ^ i * K) summed (order-
  // free, so the word ranges of the threads combine by addition).
  static uint64_t fingerprint(const void* host, uint64_t bytes) {
    const unsigned char* p = static_cast<const unsigned char*>(host);
    const uint64_t words = bytes / 8;
    auto range = [p](uint64_t a, uint64_t b) {
      uint64_t s0 = 0, s1 = 0;
      uint64_t i = a;
      for (; i + 1 < b; i += 2) {
        uint64_t w0, w1;
        std::memcpy(&w0, p + 8 * i, 8);
        std::memcpy(&w1, p + 8 * i + 8, 8);
        s0 += mix(w0 ^ (i * 0x9e3779b97f4a7c15ull));
        s1 += mix(w1 ^ ((i + 1) * 0x9e3779b97f4a7c15ull));
      }
      if (i < b) {
        uint64_t w;
        std::memcpy(&w, p + 8 * i, 8);
        s0 += mix(w ^ (i * 0x9e3779b97f4a7c15ull));
      }
      return s0 + s1;
    };
    uint64_t h = 0;
    const unsigned nt = words >= (uint64_t(1) << 22) ? std::min(16u, std::max(1u, std::thread::hardware_concurrency())) : 1u;
    if (nt > 1) {
      std::vector<uint64_t> part(nt, 0);
      std::vector<std::thread> th;
      for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] { part[t] = range(words * t / nt, words * (t + 1) / nt); });
      for (auto& x : th) x.join();
      for (uint64_t v : part) h += v;
    } else {
      h = range(0, words);
    }
    for (uint64_t b = words * 8; b < bytes; ++b) h += mix(uint64_t(p[b]) ^ (b << 8) ^ 0xa5a5a5a5ull);
    return mix(h ^ bytes);
  }

 private:
  struct Entry {
    DevBuffer* buf = nullptr;
    uint64_t n = 0, sig = 0;
    uint32_t stride = 0;
    bool valid = false;
  };
  static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  static bool trust_sample() {
    static const bool t = [] {
      const char* v = std::getenv("HJ3D_TRUST_RELATIONS");
      return v && v[0] == '1';
    }();
    return t;
  }
  static uint64_t sample(const void* host, uint64_t n, uint32_t stride) {
    uint64_t h = 0xcbf29ce484222325ull ^ n;
    const unsigned char* p = static_cast<const unsigned char*>(host);
    const uint64_t k = n < 257 ? n : 257;
    for (uint64_t j = 0; j < k; ++j) {
      const uint64_t i = (k <= 1) ? 0 : (j * (n - 1)) / (k - 1);
      for (uint32_t b = 0; b < stride; ++b) h = (h ^ p[i * stride + b]) * 0x100000001b3ull;
    }
    return h;
  }
  std::map<const void*, Entry> _m;
  uint64_t _uploads = 0;
};

// ---- locating the join attribute behind opaque functors ----
// All probing is done on REAL tuples of the relation (copies), never on fabricated ones, so a
// functor that dereferences pointer members stays safe.
template <typename T>
constexpr bool word_tuple_v = std::is_trivially_copyable_v<T> && sizeof(T) % 4 == 0 && sizeof(T) >= 4;

template <typename T>
inline uint32_t word_of(const T& t, uint32_t word) {
  uint32_t v;
  std::memcpy(&v, reinterpret_cast<const char*>(&t) + 4 * word, 4);
  return v;
}

template <typename T>
inline void set_word(T& t, uint32_t word, uint32_t v) {
  std::memcpy(reinterpret_cast<char*>(&t) + 4 * word, &v, 4);
}

// Word w of T such that hash(t) == murmur32(word w of t) for every sampled tuple (and no other
// word qualifies), or nothing. `hash` maps const T* -> hash value.
template <typename T, typename Hash>
inline std::optional<uint32_t> key_word_from_samples(const T* base, uint64_t n, Hash&& hash) {
  if constexpr (!word_tuple_v<T>) {
    return std::nullopt;
  } else {
    constexpr uint32_t kWords = sizeof(T) / 4;
    bool cand[kWords];
    for (uint32_t i = 0; i < kWords; ++i) cand[i] = true;
    const uint64_t k = n < 64 ? n : 64;
    if (k == 0) return std::nullopt;
    for (uint64_t j = 0; j < k; ++j) {
      const T& t = base[(k <= 1) ? 0 : (j * (n - 1)) / (k - 1)];
      const uint64_t h = uint64_t(hash(&t));
      for (uint32_t i = 0; i < kWords; ++i) cand[i] = cand[i] && uint64_t(murmur32(word_of(t, i))) == h;
    }
    std::optional<uint32_t> w;
    for (uint32_t i = 0; i < kWords; ++i) {
      if (!cand[i]) continue;
      if (w) return std::nullopt;  // ambiguous on this sample
      w = i;
    }
    return w;
  }
}

// Throws unless joinpred(p, b') is true for a copy b' of b with its key word set to p's key
// word, and false with it set to a different value (real sample tuples, key words known).
template <typename Tjoinpred, typename Tprobe, typename Tbuild>
inline void check_joinpred(const Tprobe* p, uint32_t pk, const Tbuild* b, uint32_t bk, const char* op) {
  if constexpr (word_tuple_v<Tbuild>) {
    Tbuild c = *b;
    set_word(c, bk, word_of(*p, pk));
    const bool eq = Tjoinpred::eval(p, &c);
    set_word(c, bk, word_of(*p, pk) + 1u);
    const bool ne = Tjoinpred::eval(p, &c);
    if (!eq || ne)
      throw Error(std::string("hj3d: ") + op + ": the join predicate is not equality of the hashed attributes; "
                  "only equi-joins on the hashed u32 attribute run on the device");
  }
}

// The input of one GPU operator: either a contiguous batch (the scanned relation) or the tuple
// pointers pushed through step().
// A batch may carry a device selection (AlgSelection pushed down, hj3d::device_predicate):
// then only its passing tuples are the operator's input, still addressed by their row in the batch.
template <typename T>
struct Input {
  T* base = nullptr;
  uint64_t n = 0;
  std::vector<T*> ptrs;
  const hj3d_sel_pred* preds = nullptr;
  uint32_t npred = 0;
  bool selecting = false;
  uint64_t size() const { return base ? n : ptrs.size(); }
  T* at(uint64_t row) const { return base ? base + row : ptrs[row]; }
  void clear() {
    base = nullptr;
    n = 0;
    ptrs.clear();
    preds = nullptr;
    npred = 0;
    selecting = false;
  }
};

// A device relation for `in`, keyed by Thashfun. A batch whose key is one u32 word is uploaded
// whole (cached) and keyed by that word (key_word). Otherwise the host reduces the input to a
// u32 key column, key = murmur32^-1(Thashfun::eval(t)) (key_word = nothing). Row i of the
// device relation is in.at(i).
template <typename Thashfun>
struct DevInput {
  using T = typename Thashfun::input_t;
  DevBuffer keys;
  hj3d_rel rel{};
  std::optional<uint32_t> key_word;

  void make(const Input<T>& in, const char* op) {
    Engine& e = Engine::get();
    rel = hj3d_rel{};
    rel.row_off = HJ3D_ROW_IMPLICIT;
    rel.n = in.size();
    pending_sel = false;
    n_selected = rel.n;
    key_word.reset();
    if (in.base && in.n) key_word = key_word_from_samples(in.base, in.n, [](const T* t) { return Thashfun::eval(t); });
    if (key_word) {
      rel.base = RelationCache::get().upload(in.base, in.n, sizeof(T));
      rel.stride = sizeof(T);
      rel.key_off = 4 * *key_word;
      pending_sel = in.selecting;  // applied by the probe (fused) or by ensure_selected()
      preds = in.preds;
      npred = in.npred;
      n_selected = in.selecting ? 0 : rel.n;
      return;
    }
    if (in.selecting)
      throw Error(std::string("hj3d: ") + op + ": a device selection needs the join key to be one u32 word of "
                  "the tuple");
    std::vector<uint32_t> k(rel.n);
    for (uint64_t i = 0; i < rel.n; ++i) {
      const uint64_t h = uint64_t(Thashfun::eval(in.at(i)));
      if (h >> 32)
        throw Error(std::string("hj3d: ") + op + ": the hash functor is not murmur3 fmix32 (util/hasht.hh:52-61); "
                    "no other hash runs on the device");
      k[i] = murmur32_inv(uint32_t(h));
    }
    void* d = keys.ensure(rel.n * 4 + 4);
    if (rel.n) e.check(hj3d_upload(e.ctx(), d, k.data(), rel.n * 4), "hj3d_upload (keys)");
    rel.base = d;
    rel.stride = 4;
    rel.key_off = 0;
  }

  // AlgSelection on the device (hj3d_select), for the paths that do not fuse it: rel becomes the
  // passing tuples' (key, row) pairs, rows still index the batch.
  void ensure_selected() {
    if (!pending_sel) return;
    Engine& e = Engine::get();
    void* d = sel.ensure(rel.n * 8 + 16);
    uint64_t* cnt = reinterpret_cast<uint64_t*>(static_cast<char*>(d) + rel.n * 8 + 8);
    e.check(hj3d_select(e.ctx(), &rel, preds, npred, d, cnt), "hj3d_select");
    uint64_t n_sel = 0;
    e.check(hj3d_download(e.ctx(), &n_sel, cnt, 8), "hj3d_download (selection count)");
    rel = hj3d_rel{d, n_sel, 8, 0, 4, 0, 0};
    pending_sel = false;
    n_selected = n_sel;
  }
  DevBuffer sel;
  bool pending_sel = false;  // rel is the whole batch; the selection below is still to apply
  const hj3d_sel_pred* preds = nullptr;
  uint32_t npred = 0;
  uint64_t n_selected = 0;   // the selection's count() once applied
};

// The device table behind HtChaining1 / HtNested1. Inserted tuples are kept as segments (the
// scanned relation of a build operator, or pointers pushed one by one) and built into the
// device table at the first use after an insert; build rows index the concatenation of the
// segments, so the reference's insertion order (chain order, first occurrence) is row order.
template <typename Tdata, typename Thashfun>
class DeviceTable {
 public:
  DeviceTable(uint32_t kind, size_t num_buckets) : _kind(kind), _nb(num_buckets) {
    if (num_buckets == 0 || num_buckets >= (uint64_t(1) << 32))
      throw Error("hj3d: the number of buckets must be in [1, 2^32)");
    Engine& e = Engine::get();
    hj3d_table_desc d{};
    d.num_buckets = num_buckets;
    d.bucket_lo = 0;
    d.bucket_hi = num_buckets;
    d.kind = kind;
    e.check(hj3d_table_create(e.ctx(), &d, &_t), "hj3d_table_create");
  }
  DeviceTable(const DeviceTable&) = delete;
  DeviceTable& operator=(const DeviceTable&) = delete;
  ~DeviceTable() { hj3d_table_destroy(_t); }

  size_t num_buckets() const { return _nb; }
  void add_batch(Tdata* base, uint64_t n) {
    Input<Tdata> s;
    s.base = base;
    s.n = n;
    _segs.push_back(std::move(s));
    _dirty = true;
  }
  void add_one(Tdata* t) {
    if (_segs.empty() || _segs.back().base) _segs.emplace_back();
    _segs.back().ptrs.push_back(t);
    _dirty = true;
  }
  void clear() {
    _segs.clear();
    _rows.clear();
    _dirty = false;
    ++_version;
    Engine& e = Engine::get();
    e.check(hj3d_table_clear(e.ctx(), _t), "hj3d_table_clear");
  }
  // device table, built from every segment inserted since the last clear
  hj3d_table* table() {
    if (_dirty) flush();
    return _t;
  }
  Tdata* row_ptr(uint64_t row) const { return _rows.at(row); }
  uint64_t rows() const { return _rows.size(); }
  const std::optional<uint32_t>& key_word() const { return _dev.key_word; }
  // Host copy of the device arrays (hj3d_table_export), fetched once per build: the per-tuple
  // probe API (findDirEntryByOther / findMainNodeByOther) walks node views made from it.
  struct Mirror {
    std::vector<uint32_t> off, payload, sub;  // payload: {hash, row} or {hash, first_row, sub_off, sub_len}
    uint64_t n_payload = 0;
  };
  const Mirror& mirror() {
    hj3d_table* t = table();
    if (_mirror_version == _version) return _mirror;
    Engine& e = Engine::get();
    uint64_t np = 0, ns = 0;
    e.check(hj3d_table_export(e.ctx(), t, nullptr, nullptr, nullptr, &np, &ns), "hj3d_table_export");
    _mirror.off.assign(_nb + 1, 0);
    _mirror.payload.assign(np * (_kind == HJ3D_NESTED ? 4 : 2), 0);
    _mirror.sub.assign(ns, 0);
    _mirror.n_payload = np;
    e.check(hj3d_table_export(e.ctx(), t, _mirror.off.data(), _mirror.payload.data(), _mirror.sub.data(), &np, &ns),
            "hj3d_table_export");
    _mirror_version = _version;
    return _mirror;
  }
  uint64_t version() const { return _version; }  // bumped by every build / clear
  hj3d_stats stats() {
    hj3d_table* t = table();
    Engine& e = Engine::get();
    hj3d_stats s{};
    e.check(hj3d_table_stats(e.ctx(), t, &s), "hj3d_table_stats");
    return s;
  }

 private:
  void flush() {
    Input<Tdata> all;
    if (_segs.size() == 1) {
      all = _segs[0];
    } else {
      for (const auto& s : _segs)
        for (uint64_t i = 0; i < s.size(); ++i) all.ptrs.push_back(s.at(i));
    }
    if (all.size() >= (uint64_t(1) << 32)) throw Error("hj3d: more than 2^32-1 build tuples");
    _rows.resize(all.size());
    for (uint64_t i = 0; i < all.size(); ++i) _rows[i] = all.at(i);
    _dev.make(all, "build");
    Engine& e = Engine::get();
    e.check(hj3d_build(e.ctx(), _t, &_dev.rel), "hj3d_build");
    e.check(hj3d_ctx_sync(e.ctx()), "hj3d_build (sync)");
    _dirty = false;
    ++_version;
  }
  uint32_t _kind;
  size_t _nb;
  hj3d_table* _t = nullptr;
  std::vector<Input<Tdata>> _segs;
  std::vector<Tdata*> _rows;
  DevInput<Thashfun> _dev;
  bool _dirty = false;
  uint64_t _version = 1, _mirror_version = 0;
  Mirror _mirror;
};

}  // namespace hj3d::host

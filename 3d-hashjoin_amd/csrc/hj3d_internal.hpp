// hj3d_internal.hpp — host-side internals shared by the C-ABI implementation and the kernel
// translation units. Not installed; the public surface is include/hj3d.h.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "hj3d.h"
#include "hj3d_device.hpp"

namespace hj3d {
// Kernel launches of this library, process-wide (hj3d_launch_count: the bench reports launches per
// step). Every launch site goes through hipLaunchKernelGGL (redefined below) or KernelSpan::launch.
void note_launch();
uint64_t launch_total();
}  // namespace hj3d
#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(kernelName, ...)                   \
  do {                                                        \
    ::hj3d::note_launch();                                    \
    hipLaunchKernelGGLInternal((kernelName), __VA_ARGS__);    \
  } while (0)

namespace hj3d {

constexpr int kBlock = 256;           // 4 waves; the default workgroup of every streaming kernel
constexpr uint32_t kInvalid = 0xFFFFFFFFu;

// Grow-only device buffer (allocation happens outside timed loops once sizes are warm).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t need) {
    if (need <= bytes) return hipSuccess;
    if (p) {
      (void)hipDeviceSynchronize();  // the old buffer may still be in use by enqueued work
      hipError_t e = hipFree(p);
      if (e != hipSuccess) return e;
      p = nullptr;
      bytes = 0;
    }
    size_t cap = need + need / 8 + 256;  // headroom so small growth does not reallocate
    hipError_t e = hipMalloc(&p, cap);
    if (e != hipSuccess) return e;
    bytes = cap;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

// comm.hip: false (and why) when two HIP runtimes are mapped into the process
bool runtime_check(std::string* msg);

}  // namespace hj3d

struct hj3d_comm_state;  // comm.hip: RCCL communicator, exchange stream, tickets

// ctl word (u64 index) of exclusive_scan_u32's tile ticket; words 0..4 belong to chain_pk.hip
constexpr int kCtlScanTicket = 6;

// Opaque handles of the C ABI.
struct hj3d_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int num_cus = 256;
  std::string last_error;
  // scratch arena slots (see api for their use)
  hj3d::DevBuf scratch[15];
  hj3d::DevBuf res;       // device result slot (u64 fields) for probe / probe2
  hj3d::DevBuf misc;      // small device reductions (statistics)
  uint32_t res_flags = 0;     // flags of the last probe (overflow check in hj3d_probe_result)
  bool res_dense = false;     // last probe emitted one slot per probe tuple
  uint64_t res_cap = ~0ull;   // output capacity of the last probe
  uint64_t res_nprobe = 0;    // probe tuples of the last probe (strand, when accumulating)
  bool res_overflow = false;  // a dense-output probe of the strand had fewer slots than tuples
  bool res_accumulated = false;
  // phase timers
  int timing = 0;  // hj3d_ctx_timing: 0 off, 1 every timer, 2 dispatch-carried kernel spans only
  bool force_direct = false;  // HJ3D_OPT_FORCE_DIRECT: never use the radix-partitioned paths
  uint64_t radix_min = 1u << 20;  // HJ3D_OPT_RADIX_MIN: smallest input that takes the radix paths
  bool nested_sort = false;       // HJ3D_OPT_NESTED_SORT
  bool sel_unfused = false;       // HJ3D_OPT_SEL_UNFUSED
  hj3d::DevBuf sel;               // hj3d_probe_sel: passing (key, row) pairs when not fused
  int pk_items = 0;                // HJ3D_OPT_PROBE_ITEMS: packed probe pairs per lane and chunk (0 = chosen per probe)
  bool pk_off = false;            // HJ3D_OPT_PACKED_PROBE = 0: the unique chaining probe on (hash, row) pairs
  uint32_t pk_slice_max = 0;      // HJ3D_OPT_PK_SLICE: cap on the packed probe's slice width (0 = LDS-sized)
  uint32_t pk_stage = 0;          // HJ3D_OPT_PK_STAGE: carry-flush threshold of its partitioner (0 = the stage)
  bool pk_build = false;          // HJ3D_OPT_PK_BUILD: the slice build (pk_build) for every chaining table it takes
  bool nested_pk = false;         // HJ3D_OPT_NESTED_PK: the nested aggregation build on pk_slices always
  bool rp_unfused = false;        // HJ3D_OPT_RP_UNFUSED: small build partitions as histogram + scatter launches
  bool sync_build = false;        // HJ3D_OPT_SYNC_BUILD: nested builds resolved before hj3d_build returns
  // control words of the packed probe (chain_pk.hip): zero between probes (its last workgroup
  // restores them), zeroed once here; words 64..127 are the sink of its unconditional stores
  hj3d::DevBuf ctl;
  uint32_t scan_epoch = 0;  // tags the look-back status words of exclusive_scan_u32 (scan.hip)
  hj3d::DevBuf scan_status;  // its per-tile status words (no other use)
  // partition cursors of the build partitioner (radix.hip partition_pairs): two sets of 2049 words,
  // call k counts into set k & 1 and clears set (k + 1) & 1 for the next call; zeroed once here
  hj3d::DevBuf part_cur;
  uint32_t part_parity = 0;
  // grid barrier of the fused partition (radix.hip k_rp_fused): word 0 a monotonic arrival counter
  // (each launch waits for the running sum of the grids launched on it), word 1 the timeout flag
  // (the timeout flag is also written into the built table's counts word 3, tagged with the launch's
  // sequence number gbar_seq, and checked by the table's getters)
  hj3d::DevBuf gbar;
  // the slice-path nested build's decoupled look-back (nested_agg.hip): words 0-1 ticket and finish
  // counters (zeroed by the launch before k_nagg), then one status word per partition tagged with
  // nagg_epoch (no other use; cleared when allocated)
  hj3d::DevBuf nagg_lb;
  uint32_t nagg_epoch = 0;
  uint64_t gbar_target = 0;
  uint64_t gbar_seq = 0;
  uint64_t diag_lb = 0;    // HJ3D_OPT_DIAG_LOOKBACK: slice-path look-back wait limit in 100 MHz ticks, partition 0 silent
  uint64_t diag_gbar = 0;  // HJ3D_OPT_DIAG_GBAR: barrier timeout in 100 MHz ticks, workgroup 0 never arrives
  hipError_t ensure_ctl() {
    if (ctl.p) return hipSuccess;
    hipError_t e = ctl.ensure(128 * sizeof(uint64_t));  // 8 control words; [64, 128): store sink
    if (e == hipSuccess) e = hipMemsetAsync(ctl.p, 0, ctl.bytes, stream);
    return e;
  }
  hj3d_comm_state* comm = nullptr;  // hj3d_comm_init
  struct Span { hipEvent_t a, b; };
  std::vector<Span> spans[HJ3D_T_NTIMERS];
  std::vector<hipEvent_t> event_pool;
  size_t pool_used = 0;
};

struct hj3d_table {
  hj3d_table_desc desc{};
  uint32_t nb_local = 0;  // bucket_hi - bucket_lo
  hj3d::FastMod fm{};
  uint64_t n_build = 0;   // tuples in the last build (host-known)
  uint64_t n_mains = 0;   // nested: main records (distinct keys) of the last build (host-known)
  bool built = false;
  const char* path = "none";  // which build made the table (hj3d_table_build_path)
  char path_buf[40] = {0};    // hj3d_table_build_path of a table not resolved yet: path + "?"
  // nested builds: the counts (main records, give-up flag) are copied to pinned host memory behind
  // the build and read at the table's next use (table_resolve), not waited for inside hj3d_build
  bool pending = false, pending_agg = false;
  hj3d_rel pending_rel{};
  hj3d_ctx* pending_ctx = nullptr;
  uint64_t* hc = nullptr;  // pinned host copy of counts[4]
  hipEvent_t hc_ev = nullptr;
  // chaining: off[nb_local+1] (u32 CSR offsets), ent[n] = {hash, row}
  // nested:   off[nb_local+1] over mains, main[d] = {hash, first_row, sub_off, sub_len},
  //           sub[n] = build rows grouped per key (first occurrence first, then row order)
  hj3d::DevBuf off, ent, main, sub;
  hj3d::DevBuf counts;    // device u64[4]: {entries, distinct, max_sub_len, give-up flag (nested) /
                          // fused-partition barrier timeout tag (chaining)}
  uint64_t gbar_tag = 0;  // chaining tables built by the fused partition: its launch tag (0: none)
};

namespace hj3d {

// Selection predicate (hj3d_sel_pred conjunction) as a kernel argument, and its evaluation on the
// u32 tuple word(s) it reads (AlgSelection::step, algebra.hh:295-300).
struct SelArgs {
  uint32_t npred = 0;
  hj3d_sel_pred p[HJ3D_SEL_MAX];
};
__device__ __forceinline__ bool sel_one(const hj3d_sel_pred& p, uint32_t w) {
  const int64_t v = p.is_signed ? int64_t(int32_t(w)) : int64_t(w);
  switch (p.op) {
    case HJ3D_SEL_LT: return v < p.lo;
    case HJ3D_SEL_LE: return v <= p.lo;
    case HJ3D_SEL_GT: return v > p.lo;
    case HJ3D_SEL_GE: return v >= p.lo;
    case HJ3D_SEL_EQ: return v == p.lo;
    case HJ3D_SEL_NE: return v != p.lo;
    default: return v >= p.lo && v < p.hi;  // HJ3D_SEL_RANGE
  }
}
__device__ __forceinline__ bool sel_eval(const RelView& r, const SelArgs& a, uint64_t i) {
  const char* t = r.base + i * r.stride;
  bool ok = true;
  for (uint32_t k = 0; k < a.npred; ++k)
    ok = ok && sel_one(a.p[k], *reinterpret_cast<const uint32_t*>(t + a.p[k].word_off));
  return ok;
}
// One predicate as an inclusive range test on the word read as int32 / uint32 (inverted for !=):
// the form the probe partitioner evaluates in its hot loop.
struct SelRange {
  uint32_t word_off = 0, is_signed = 0, invert = 0, pad = 0;
  int64_t lo = 0, hi = -1;
  __device__ __forceinline__ bool test(uint32_t w) const {
    const int64_t v = is_signed ? int64_t(int32_t(w)) : int64_t(w);
    return (v >= lo && v <= hi) != (invert != 0);
  }
  static bool from(const SelArgs& a, SelRange* r) {
    if (a.npred != 1) return false;
    const hj3d_sel_pred& p = a.p[0];
    const int64_t mn = p.is_signed ? INT32_MIN : 0, mx = p.is_signed ? INT32_MAX : int64_t(UINT32_MAX);
    r->word_off = p.word_off;
    r->is_signed = p.is_signed != 0;
    r->invert = 0;
    switch (p.op) {
      case HJ3D_SEL_LT: r->lo = mn; r->hi = p.lo - 1; break;
      case HJ3D_SEL_LE: r->lo = mn; r->hi = p.lo; break;
      case HJ3D_SEL_GT: r->lo = p.lo + 1; r->hi = mx; break;
      case HJ3D_SEL_GE: r->lo = p.lo; r->hi = mx; break;
      case HJ3D_SEL_EQ: r->lo = p.lo; r->hi = p.lo; break;
      case HJ3D_SEL_NE: r->lo = p.lo; r->hi = p.lo; r->invert = 1; break;
      default: r->lo = p.lo; r->hi = p.hi - 1; break;  // RANGE
    }
    return true;
  }
};
inline SelArgs sel_args(const hj3d_sel_pred* preds, uint32_t npred) {
  SelArgs a{};
  a.npred = npred;
  for (uint32_t k = 0; k < npred; ++k) a.p[k] = preds[k];
  return a;
}

// ---- decoupled look-back (exclusive_scan_u32, k_pk_build) ----
// Status word of item t: epoch << 34 | flag << 32 | value, flag 1 = the item's own sum, 2 = its
// inclusive prefix; words of other epochs read as unpublished (nothing is cleared between calls).
// The value travels inside the word, so relaxed device-scope atomics suffice.
constexpr uint64_t kLbAgg = 1ull << 32, kLbInc = 2ull << 32;
__device__ __forceinline__ void lb_publish(uint64_t* status, uint32_t t, uint32_t epoch, uint64_t flag, uint32_t v) {
  __hip_atomic_store(status + t, (uint64_t(epoch) << 34) | flag | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Called by one whole wave: the sum of items [0, t) from their status words, 64 predecessors per
// step (lane k reads item q - k; the nearest inclusive prefix ends the walk). Items below t must
// be published by running workgroups (taken by ticket), which never wait for later items.
__device__ __forceinline__ uint32_t lb_exclusive(const uint64_t* status, uint32_t t, uint32_t epoch) {
  const int lane = threadIdx.x & 63;
  uint32_t excl = 0;
  int64_t hi = int64_t(t) - 1;
  while (hi >= 0) {
    const int64_t q = hi - lane;
    const uint64_t w = q >= 0 ? __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : ((uint64_t(epoch) << 34) | kLbInc);  // before item 0: prefix 0
    const uint32_t f = uint32_t(w >> 32) & 3u;
    const bool ready = (w >> 34) == epoch && f != 0;
    const uint64_t inc = __ballot(ready && f == 2u), nready = __ballot(!ready);
    const int fi = inc ? __ffsll((unsigned long long)inc) - 1 : 63;  // nearest inclusive (or the whole step)
    const uint64_t need = fi >= 63 ? ~0ull : ((2ull << fi) - 1);
    if (nready & need) continue;  // a predecessor in range has not published yet: read again
    uint32_t v = lane <= fi ? uint32_t(w) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += uint32_t(__shfl_xor(int(v), o, 64));
    excl += v;
    if (inc) break;
    hi -= 64;
  }
  return excl;
}

// ---- launchers (defined in the .hip translation units); all asynchronous on `s` ----
// scan.hip: exclusive prefix sum of n values into out[0..n], out[n] = total. in may alias out.
hipError_t exclusive_scan_u32(hj3d_ctx* ctx, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t s);
hipError_t exclusive_scan_u64(hj3d_ctx* ctx, const uint64_t* in, uint64_t* out, uint64_t n, hipStream_t s);
// scan.hip: up to four arrays of u64 words zeroed by one launch (instead of a runtime fill each,
// ~5 us apiece between the kernels of a short strand)
struct ZeroList {
  uint64_t* p[4] = {nullptr, nullptr, nullptr, nullptr};
  uint32_t n[4] = {0, 0, 0, 0};
  bool add(uint64_t* q, uint32_t words) {  // false: the list is full
    for (int k = 0; k < 4; ++k)
      if (!p[k]) {
        p[k] = q;
        n[k] = words;
        return true;
      }
    return false;
  }
};
hipError_t zero_words(const ZeroList& z, hipStream_t s);
// sort.hip: stable LSD radix sort of (key,val) u32 pairs on key bits [0, bits). Result lands in
// (k0,v0); (k1,v1) is a same-size scratch double buffer. With in_alt, an odd number of passes
// leaves the result in (k1,v1) and sets *in_alt instead of copying it back.
hipError_t radix_sort_pairs(hj3d_ctx* ctx, uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint64_t n,
                            int bits, hipStream_t s, bool* in_alt = nullptr);
// radix.hip: partitioned (LDS-slice) build / probe of the chaining table
bool radix_probe_applicable(const hj3d_ctx* ctx, const hj3d_table* t, uint64_t n_probe);
// rows_sorted (optional): set when the small buckets already come out sorted by row.
hipError_t radix_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s, bool* rows_sorted = nullptr);
// Partition r into (hash, row) pairs by ranges of W local buckets (LDS-histogram pass, scan,
// LDS-staged scatter): partition p is out[ps[p] .. ps[p+1]), *nparts = ceil(nb_local / W).
// Uses scratch kScrPHist. hipErrorNotSupported beyond 2048 partitions.
// r1 (optional): a second relation of the same geometry in the same two launches; its partitions are
// P .. 2P - 1 (ps[P .. 2P]), its pairs follow r's.
hipError_t radix_partition_pairs(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t W, uint2* out,
                                 uint32_t* ps, uint32_t* nparts, hipStream_t s, const hj3d_rel* r1 = nullptr);
// after every chaining build: buckets of <= 32 entries sorted by row (single-pass probe order)
hipError_t sort_small_buckets(hj3d_ctx* ctx, hj3d_table* t, hipStream_t s);
// sel (nullable, <= 2 predicates): the selection fused into the probe-side partitioner; tuples
// failing it are dropped there and res[0] (n_probe) = the passing tuples. hipErrorNotSupported
// when the fused form does not apply (the caller then selects first).
hipError_t radix_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                       uint64_t out_cap, uint64_t* res_dev, hipStream_t s, const SelArgs* sel = nullptr);
// The probe side partitioned by bucket range for a table slice of W buckets per partition
// (k_rp_part1 + output-slot scan; layout in radix_seg.hpp). Output slots: regions first
// (seg[P * G] of them), then the overflow list (*novf pairs). Uses scratch kScrPairs,
// kScrPHist, kScrSortV. hipErrorNotSupported: more than 2048 partitions.
struct ProbeParts {
  uint32_t W = 0, P = 0, G = 0, cap = 0, splits = 1;
  bool flat = false;  // short regions: walk them as one flattened stream (radix_seg.hpp)
  const uint2* region = nullptr;
  const uint32_t* counts = nullptr;
  const uint32_t* seg = nullptr;  // seg[P * G] = slots taken by the regions
  const uint2* ovf = nullptr;
  const unsigned long long* novf = nullptr;
};
// slots = false: the caller never writes output (the dense output slots of the regions, a
// transpose + scan of the region counts, are not computed; pp->seg is then undefined)
// also (optional): words the caller needs zeroed before the strand, cleared by the same launch as
// the partitioner's overflow counters (only on success: on hipErrorNotSupported nothing was launched)
hipError_t radix_partition_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t W, ProbeParts* pp,
                                 hipStream_t s, const SelArgs* sel = nullptr, unsigned long long** npass = nullptr,
                                 bool slots = true, const ZeroList* also = nullptr);
// chain_pk.hip: the unique chaining probe on packed pairs (partitioner + probe, two launches; the
// result slot is set, or added to with HJ3D_PROBE_ACCUMULATE, by the probe kernel itself: no fill
// before it). hipErrorNotSupported when the geometry does not pack (use radix_probe).
bool pk_probe_applicable(const hj3d_ctx* ctx, const hj3d_table* t, uint64_t n_probe, uint32_t flags);
hipError_t pk_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                    uint64_t out_cap, uint64_t* res_dev, hipStream_t s, const SelArgs* sel = nullptr);
// Slice geometry of the packed probe: P slices of W buckets (a slice's directory + entries fit the
// probe workgroup's LDS); above 1024 slices, two partition levels: k_pk_part into P1 coarse ranges
// of C slices (W1 = C * W buckets), then k_pk_split by slice.
struct PkPlan {
  uint32_t W = 0, P = 0, C = 1, W1 = 0, P1 = 0;
};
PkPlan pk_plan(const hj3d_ctx* ctx, uint32_t nb_local, uint64_t n_build);
// Packed-pair geometry of P slices of W buckets: a pair of slice p carries v = (bucket in the slice)
// << qbits | h / NB, from which the hash follows without a division (chain_pk.hip).
struct PkGeom {
  FastDiv32 dnb, dw;  // / NB, / W
  uint32_t nb, lo, nbl, W, P, qbits, qmask;
  // hash of a packed pair in slice p
  __device__ __forceinline__ uint32_t hash_of(uint32_t v, uint32_t p) const {
    return (v & qmask) * nb + lo + p * W + (v >> qbits);
  }
};
// A relation partitioned into slices of W local buckets by the packed partitioner's two levels
// (k_pk_part into coarse ranges, k_pk_split into slices): slice p's pairs {v, row} lie in S2 fine
// regions fine[(s * P + p) * cap2 ...], fcnt[s * P + p] pairs each; ps[p] = exclusive scan of the
// slices' totals (ps[P] = all pairs in the slices). Pairs that overflowed a region are not in any
// slice: pk_overflow_check (synchronous) reports their number and restores the control words.
struct PkSlices {
  PkGeom pk{};
  uint32_t P = 0, S2 = 0, cap2 = 0;
  const uint2* fine = nullptr;
  const uint32_t* fcnt = nullptr;
  const uint32_t* ps = nullptr;             // (sums = false: not computed)
  const uint2* ovf = nullptr;               // region-overflow pairs {h, row}
  const unsigned long long* novf = nullptr;  // their count: control word kCtlNovf (reset by the caller)
};
hipError_t pk_slices(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t W, PkSlices* o, hipStream_t s,
                     bool sums = true);
// The probe side of a nested table wider than the one-level partitioner's 2048 LDS slices: pk_slices
// (two levels, packed pairs) into slices of W buckets, plus the dense output slots of its fine
// regions (seg, partition-major); pp's region layout is radix_seg.hpp's with G = S2 regions per
// slice. Overflow pairs: pp->ovf / pp->novf (the packed probe's control word: the caller resets the
// control words after the probe, pk_ctl_reset).
hipError_t pk_probe_slices(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t W, ProbeParts* pp,
                           PkGeom* pk, hipStream_t s);
hipError_t pk_ctl_reset(hj3d_ctx* ctx, hipStream_t s);
hipError_t pk_overflow_check(hj3d_ctx* ctx, hipStream_t s, uint64_t* novf);
// The chaining build of tables beyond the radix build's range (> 2048 x 16384 buckets): R
// partitioned by the packed partitioner's two levels into 8192-bucket slices, each built in LDS
// (rows sorted inside buckets of <= 32). Synchronous (checks for region overflow);
// hipErrorNotSupported when not applicable or on overflow (use chain_build).
hipError_t pk_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s);
// chain.hip
hipError_t chain_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s);
hipError_t chain_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                       uint64_t out_cap, uint64_t* res_dev, hipStream_t s);
// nested.hip
hipError_t nested_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s);
// nested_agg.hip: the nested build by bucket-range partition + per-partition LDS aggregation.
// hipErrorNotSupported when not applicable (small inputs / tables): use nested_build.
// *path (optional): "nested_agg" or "nested_agg_slices" (the pk_slices form, > 2048 partitions).
hipError_t nested_build_agg(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& r, hipStream_t s,
                            const char** path = nullptr);
// The same for nt <= 2 tables of one geometry (equal NB and bucket range) in one launch sequence:
// both relations partitioned, one k_nagg grid over both tables' partitions, one scan, one compaction.
hipError_t nested_build_agg_many(hj3d_ctx* ctx, hj3d_table* const* t, const hj3d_rel* r, uint32_t nt, hipStream_t s,
                                 const char** path = nullptr);
hipError_t nested_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                        uint64_t out_cap, uint64_t* res_dev, hipStream_t s);
// partitioned nested probe (every mode of nested_probe); needs t->n_mains
bool radix_nested_applicable(const hj3d_ctx* ctx, const hj3d_table* t, uint64_t n_probe);
// also (optional): words to zero before the strand (a fresh result slot), in the partitioner's
// counter-clearing launch; on hipErrorNotSupported nothing was launched
hipError_t radix_nested_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel& r, uint32_t flags, void* out,
                              uint64_t out_cap, uint64_t* res_dev, hipStream_t s, const SelArgs* sel = nullptr,
                              const ZeroList* also = nullptr);
// exp4.hip
hipError_t probe2(hj3d_ctx* ctx, const hj3d_table* ts, const hj3d_table* tt, const hj3d_rel& r, uint32_t flags,
                  void* out, uint64_t out_cap, uint64_t* res_dev, hipStream_t s);
// stats.hip
hipError_t table_stats(hj3d_ctx* ctx, const hj3d_table* t, hj3d_stats* out, hipStream_t s);
// part.hip
hipError_t partition(hj3d_ctx* ctx, const hj3d_rel& r, uint64_t nb, uint32_t nparts, void* out_pairs,
                     void* counts, hipStream_t s, const SelArgs* sel = nullptr);
// single pass, no order kept inside a destination: destination p's pairs at out_pairs + p * stride
// (stride >= r.n), counts (u64) zeroed here and then filled by the run claims
hipError_t partition_strided(hj3d_ctx* ctx, const hj3d_rel& r, uint64_t nb, uint32_t parts, void* out_pairs,
                             uint64_t stride, void* counts, hipStream_t s, const SelArgs* sel = nullptr);
hipError_t select_pairs(hj3d_ctx* ctx, const hj3d_rel& rel, const hj3d_sel_pred* preds, uint32_t npred, void* out,
                        void* count, hipStream_t s);
hipError_t key_bitmap(hj3d_ctx* ctx, const hj3d_rel& r, uint64_t domain, void* bitmap, void* outside, hipStream_t s);
hipError_t bitmap_or_popcount(hj3d_ctx* ctx, const void* bitmaps, uint32_t rows, uint64_t words, void* count,
                              hipStream_t s);
hipError_t gen_keys(void* tuples, uint64_t n, uint32_t stride, uint32_t key_off, uint64_t row_base,
                    uint64_t n_keys, uint64_t seed, hipStream_t s);
hipError_t gen_fk(void* tuples, uint64_t n, uint32_t stride, uint32_t key_off, uint64_t row_base, uint32_t fk_max,
                  uint64_t seed, hipStream_t s);
hipError_t gen_zipf(void* tuples, uint64_t n, uint32_t stride, uint32_t key_off, uint64_t row_base, uint32_t fk_max,
                    double theta, uint64_t seed, hipStream_t s);
hipError_t expected_fk_join(hj3d_ctx* ctx, const hj3d_rel& build, const hj3d_rel& probe, uint64_t n_keys,
                            bool swap, void* res, hipStream_t s);
hipError_t expected_fk_join_gen(hj3d_ctx* ctx, const hj3d_rel& probe, uint64_t n_keys, uint64_t seed, bool swap,
                                void* res, hipStream_t s);

// api.cpp: completes a nested build whose counts are still in flight (reads them; runs the sort
// build when the aggregation build gave up). Every use of a table's content calls it first.
hipError_t table_resolve(hj3d_ctx* ctx, hj3d_table* t);

// Scratch slot ids in hj3d_ctx::scratch.
enum ScratchSlot {
  kScrScan = 0, kScrSlot = 1, kScrSortK = 2, kScrSortV = 3, kScrA = 4, kScrB = 5, kScrC = 6, kScrD = 7,
  kScrPairs = 8,    // radix-partitioned (hash, row) pairs
  kScrPHist = 9,    // radix partition histograms / offsets
  kScrPartial = 10, // per-block result partials
  kScrPStart = 11,  // partition starts of the probe side
  kScrPk2 = 12,     // packed probe, second partition level: fine regions
  kScrPk2Cnt = 13,  // and their pair counts
  kScrSink = 14,    // 1024 pairs: target of the stores of lanes without a pair (fixed store counts)
  kScrSlots = 15
};

// Per-block result partials: kernels store their block totals (block_store) to
// partials[block * nf ...]; reduce_partials adds the column sums into res (stream-ordered).
// set0 != ~0: res[0] is set to set0 (+ *base0 when given) instead of accumulated (the scanned-tuple
// count is known on the host; base0 = res[0] before this probe, for accumulating probes).
hipError_t reduce_partials(const uint64_t* partials, uint32_t nblocks, int nf, int nxor, uint64_t* res, hipStream_t s,
                           uint64_t set0 = ~0ull, const uint64_t* base0 = nullptr);

// timer events: no system-scope fence when recorded (a default event writes the L2 back and left the
// GPU idle ~10 us between the kernels around it: config B probe 0.887 -> 0.881 ms, r05z_ev_ab)
constexpr unsigned HJ3D_TIMER_EVENT_FLAGS = hipEventDisableSystemFence;
// Event spans on the context stream when timing is enabled (hj3d_ctx_timer): a PhaseTimer
// brackets whatever is enqueued during its lifetime.
inline hipEvent_t take_event(hj3d_ctx* ctx) {
  if (ctx->pool_used == ctx->event_pool.size()) {
    hipEvent_t ev;
    // timing only: no system-scope fence when the event is recorded (a fence writes the L2 back
    // and leaves the GPU idle ~10 us between the kernels around the event)
    if (hipEventCreateWithFlags(&ev, HJ3D_TIMER_EVENT_FLAGS) != hipSuccess) return nullptr;
    ctx->event_pool.push_back(ev);
  }
  return ctx->event_pool[ctx->pool_used++];
}

struct PhaseTimer {
  hj3d_ctx* ctx;
  int phase;
  hipEvent_t a = nullptr;
  PhaseTimer(hj3d_ctx* c, int p) : ctx(c), phase(p) {
    if (ctx->timing == 1 && p >= 0 && (a = take_event(ctx))) (void)hipEventRecord(a, ctx->stream);
  }
  ~PhaseTimer() {
    if (!a) return;
    hipEvent_t b = take_event(ctx);
    if (!b) return;
    (void)hipEventRecord(b, ctx->stream);
    ctx->spans[phase].push_back({a, b});
  }
};

// One kernel's span for the per-kernel timers: the two events travel with the dispatch
// (hipExtLaunchKernel), so timing a kernel puts no marker packet between it and its neighbours.
// launch(kernel, grid, block, stream, args...) launches with or without them.
struct KernelSpan {
  hj3d_ctx* ctx;
  int phase;
  hipEvent_t a = nullptr, b = nullptr;
  KernelSpan(hj3d_ctx* c, int p) : ctx(c), phase(p) {
    if (!ctx->timing || p < 0) return;
    a = take_event(ctx);
    b = a ? take_event(ctx) : nullptr;
    if (!b) a = nullptr;
  }
  ~KernelSpan() {
    if (a && b) ctx->spans[phase].push_back({a, b});
  }
  template <typename F, typename... Args>
  void launch(F kernel, dim3 grid, dim3 block, hipStream_t s, Args... args) {
    if (a) note_launch();
    if (a) hipExtLaunchKernelGGL(kernel, grid, block, 0, s, a, b, 0, args...);
    else hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
  }
};

inline RelView view_of(const hj3d_rel& r) {
  RelView v;
  v.base = static_cast<const char*>(r.base);
  v.n = r.n;
  v.stride = r.stride;
  v.key_off = r.key_off;
  v.row_off = r.row_off;
  v.pad = 0;
  v.row_base = r.row_base;
  return v;
}

// Grid for grid-stride streaming kernels: enough blocks to fill the chip (>= 8 per CU),
// bounded so that per-block result flushes stay cheap.
// the sink of fixed-count store loops (garbage, shared by every workgroup)
inline hipError_t store_sink(hj3d_ctx* ctx, uint2** sink) {
  const hipError_t e = ctx->scratch[kScrSink].ensure(1024 * sizeof(uint2));
  *sink = ctx->scratch[kScrSink].as<uint2>();
  return e;
}

inline unsigned grid_for(const hj3d_ctx* ctx, uint64_t items, unsigned items_per_block) {
  const uint64_t want = (items + items_per_block - 1) / items_per_block;
  const uint64_t cap = uint64_t(ctx->num_cus) * 8;
  uint64_t g = want < cap ? want : cap;
  return unsigned(g < 1 ? 1 : g);
}

}  // namespace hj3d

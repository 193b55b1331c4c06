/* hj3d.h — C ABI of the MI355X-native 3D hash-join engine (libhj3d.so).
 *
 * The reference (dflaxx/3d-hashjoin) has no FFI: its boundary is the compile-time
 * template surface of algebra.hh / ht_chaining.hh / ht_nested.hh. This ABI is what
 * that surface binds to. Each entry point replaces one reference interface:
 *
 *   hj3d_build  (HJ3D_CHAIN)   HtChaining1::insert            ht_chaining.hh:181-196
 *                              driven by AlgScan -> AlgHashJoinBuild::step  algebra.hh:259-269, 574-577
 *   hj3d_build  (HJ3D_NESTED)  HtNested1::insert              ht_nested.hh:287-311, 386-436
 *                              driven by AlgNestJoinBuild::step            algebra.hh:386-389
 *   hj3d_probe  (chain table)  AlgHashJoinProbe::step         algebra.hh:625-659
 *                              (+ HtChaining1::findDirEntryByOther ht_chaining.hh:236-248)
 *   hj3d_probe  (nested table) AlgNestJoinProbe::step         algebra.hh:435-459
 *                              (+ HtNested1::findMainNodeByOther ht_nested.hh:354-382)
 *                              and with HJ3D_PROBE_UNNEST also AlgUnnestHt::step  algebra.hh:510-541
 *   hj3d_probe2                the experiment-4 probe strand: two probes keyed on the same
 *                              probe attribute + deferred unnesting   main_experiment4.cc:831-1043
 *   hj3d_table_stats           HtChaining1/HtNested1::makeStatistics  ht_chaining.hh:260-292,
 *                                                                     ht_nested.hh:450-482
 *   hj3d_table_clear           HtChaining1/HtNested1::clear           ht_chaining.hh:250-258,
 *                                                                     ht_nested.hh:438-447
 *   hj3d_select                AlgSelection / AlgDynSelection::step   algebra.hh:278-358
 *   hj3d_probe_sel             AlgScan -> AlgSelection -> AlgHashJoinProbe / AlgNestJoinProbe
 *
 * Semantics kept bit-exact with the reference: hash = murmur3 fmix32 (util/hasht.hh:52-61),
 * bucket = hash % num_buckets, and every counter the reference reports (match counts,
 * collision-chain comparisons c_htProbeCmp, unnest counts, HT statistics). The physical
 * layout is NOT the reference's pointer chains: tables are CSR-bucketized arrays, and the
 * reference's chain order (chaining: directory entry first, then newest-first; nested:
 * main nodes in first-occurrence order) is reproduced arithmetically from row ids.
 *
 * Join predicate: the engine joins on EQUALITY OF THE u32 JOIN ATTRIBUTE, tested as equality of
 * its fmix32 hash. fmix32 is a bijection on u32 (every step is invertible), so equal hashes are
 * equal keys and the reference's joinpred after the hash compare (algebra.hh:647-648) is implied
 * (SURVEY App. B item 7). A caller whose join predicate is anything else must not use this ABI;
 * the drop-in layer checks this on sample tuples (hj3d_host.hh check_joinpred) and refuses.
 *
 * Conventions: all relation/pair pointers are DEVICE pointers; every call is enqueued on the
 * context's stream (asynchronous) unless documented as synchronous. Calls return hj3d_status;
 * nothing throws. One host thread per context.
 */
#ifndef HJ3D_H
#define HJ3D_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  HJ3D_OK = 0,
  HJ3D_EINVAL = 1,       /* bad argument (null pointer, misaligned stride, ...)          */
  HJ3D_ENOMEM = 2,       /* device allocation failed                                      */
  HJ3D_EDEVICE = 3,      /* a HIP runtime call failed (see hj3d_last_error)               */
  HJ3D_EUNSUPPORTED = 4, /* a request outside what the engine implements                 */
  HJ3D_EOVERFLOW = 5     /* output buffer too small (counters are still complete)         */
} hj3d_status;

typedef struct hj3d_ctx hj3d_ctx;     /* device, stream, scratch arena, event timers        */
typedef struct hj3d_table hj3d_table; /* a device-resident hash table (chaining or nested)  */

#define HJ3D_ROW_IMPLICIT 0xFFFFFFFFu

/* A relation in device memory: array of structs. The join attribute is the u32 at
 * key_off of every tuple (main_experiment1.cc:86 tuple {k,a,b} -> stride 12, key_off 0 for
 * R.k, 4 for S.a). Row id of tuple i: row_base + i, or the u32 at row_off when
 * row_off != HJ3D_ROW_IMPLICIT (exchanged (key,row) pairs on multi-GPU). Row ids are the
 * identity of tuples: they are what the reference's tuple pointers become. The chain orders the
 * counters follow are derived from row order, so a build relation's explicit row ids must ascend in
 * its scan order (the reference's insertion order), as received pairs do: the exchange keeps each
 * source's pairs in row order and concatenates the sources in rank order. */
typedef struct {
  const void* base;
  uint64_t n;
  uint32_t stride;  /* bytes between consecutive tuples, multiple of 4, > 0 */
  uint32_t key_off; /* byte offset of the u32 join attribute, multiple of 4  */
  uint32_t row_off; /* byte offset of a u32 row id, or HJ3D_ROW_IMPLICIT     */
  uint32_t reserved;
  uint64_t row_base;
} hj3d_rel;

enum { HJ3D_CHAIN = 0, HJ3D_NESTED = 1 };

typedef struct {
  uint64_t num_buckets; /* global NB: bucket(key) = murmur32(key) % NB, 1 <= NB < 2^32     */
  uint64_t bucket_lo;   /* this table holds buckets [bucket_lo, bucket_hi) (a multi-GPU    */
  uint64_t bucket_hi;   /* shard); 0 / num_buckets on one GPU. Keys of other buckets are  */
                        /* ignored by build and never match in probe.                      */
  uint32_t kind;        /* HJ3D_CHAIN or HJ3D_NESTED                                        */
  uint32_t reserved;
} hj3d_table_desc;

/* probe flags */
#define HJ3D_PROBE_UNIQUE 0x1u /* IsBuildKeyUnique: stop at the first match (algebra.hh:653-655) */
#define HJ3D_PROBE_UNNEST 0x2u /* nested table: expand main + sub-chain (AlgUnnestHt)           */
#define HJ3D_PROBE_EMIT   0x4u /* write output tuples to out_dev (else aggregate only)          */
#define HJ3D_PROBE_ACCUMULATE 0x10u /* add to the result slot of the previous probe instead of
                                       restarting it (one probe strand issued in chunks) */
#define HJ3D_PROBE_CHECKSUM 0x8u /* fold sum_a/sum_b/sum_h/xor_h over the output (verification;
                                    the reference itself only counts); counts are always exact */

/* Result of one probe strand. Orientation follows the reference's concat functors:
 * a = probe-side row, b = build-side row (for a nested probe without unnest, b = the row of
 * the matched key's first build tuple, i.e. MainNode::data()). */
typedef struct {
  uint64_t n_probe;   /* probe tuples scanned                    (c_scanProbe)             */
  uint64_t n_matched; /* probe tuples with >= 1 match            (nested c_htProbe)         */
  uint64_t n_out;     /* output tuples: chaining c_htProbe, nested c_unnest / c_top         */
  uint64_t n_cmps;    /* collision-chain comparisons             (c_htProbeCmp, bit-exact)  */
  uint64_t sum_a, sum_b, sum_c; /* sum of row ids over output tuples (c only for triples)   */
  uint64_t sum_h, xor_h;        /* sum / xor of HJ3D pair (triple) hashes over output tuples */
} hj3d_probe_res;

/* Result of the experiment-4 probe strand (main_experiment4.cc:831-1043 counter columns).
 * Output triples (r, s, t) rows; a = r, b = s, c = t in the checksums. */
typedef struct {
  uint64_t c_probe_rs, c_probe_rs_cmp, c_probe_rt, c_probe_rt_cmp;
  uint64_t c_unnest_1, c_unnest_2, c_top;
  uint64_t sum_a, sum_b, sum_c, sum_h, xor_h;
} hj3d_probe2_res;

/* HtStatistics (ht_statistics.hh:18-54): cc0 over all buckets, cc1 over non-empty ones.
 * Chain length = #entries (chaining) or #main nodes = distinct keys (nested) per bucket. */
typedef struct {
  uint64_t nb, empty, entries, distinct;
  uint64_t cc0_min, cc0_max, cc0_sum, cc0_cnt;
  uint64_t cc1_min, cc1_max, cc1_sum, cc1_cnt;
} hj3d_stats;

/* ---- checksums (definitions shared with oracle/ and tests) ----
 * mix64 = splitmix64 finalizer; pair(a,b) = mix64(a<<32 | b); triple(a,b,c) = mix64(pair(a,b) ^ c) */
uint64_t hj3d_mix64(uint64_t z);

/* ---- context ---- */
/* hip_stream: the stream every call of this context is enqueued on; NULL = the device's null
 * (default) stream, i.e. the stream torch uses unless told otherwise. */
hj3d_status hj3d_ctx_create(int device, void* hip_stream, hj3d_ctx** out);
void        hj3d_ctx_destroy(hj3d_ctx* ctx);
hj3d_status hj3d_ctx_set_stream(hj3d_ctx* ctx, void* hip_stream);
void*       hj3d_ctx_stream(const hj3d_ctx* ctx);
hj3d_status hj3d_ctx_sync(hj3d_ctx* ctx); /* synchronous: waits for the stream */
const char* hj3d_last_error(const hj3d_ctx* ctx);
/* Engine options. HJ3D_OPT_FORCE_DIRECT (0/1): probe / build the chaining table without the
 * radix-partitioned (LDS-slice) kernels, i.e. with one random table access chain per tuple
 * (kept for small inputs and for A/B measurements). */
enum {
  HJ3D_OPT_FORCE_DIRECT = 1,
  /* HJ3D_OPT_RADIX_MIN (tuples): probes of at least this many tuples (builds of at least 1/16 of
   * it) use the radix-partitioned kernels; default 2^20. */
  HJ3D_OPT_RADIX_MIN = 2,
  /* 3: reserved (a nested build from the radix bucket CSR with per-bucket key grouping: faster at low
   * bucket fill, slower under Zipf skew than the aggregation build; removed in round 6) */
  /* HJ3D_OPT_NESTED_SORT (0/1, default 0): build nested tables by the LSD key sort (nested.hip)
   * instead of the bucket-range partition + per-partition LDS aggregation (nested_agg.hip, the
   * default for large inputs). */
  HJ3D_OPT_NESTED_SORT = 4,
  /* HJ3D_OPT_SEL_UNFUSED (0/1, default 0): hj3d_probe_sel always selects first (hj3d_select) and
   * probes the passing pairs, instead of fusing the selection into the probe partitioner. */
  HJ3D_OPT_SEL_UNFUSED = 5,
  /* HJ3D_OPT_PACKED_PROBE (0/1, default 1): the unique chaining probe partitions the probe side into
   * packed {bucket-in-slice | hash / NB, row} pairs and finishes in two launches; 0 keeps the
   * {hash, row} partitioned probe (A/B measurements). */
  HJ3D_OPT_PACKED_PROBE = 6,
  /* HJ3D_OPT_PROBE_ITEMS (0 or 5..8, default 0): pairs per lane and chunk in the packed probe's
   * region walk; 0 picks it from the expected region length (tests and A/B measurements). */
  HJ3D_OPT_PROBE_ITEMS = 7,
  /* HJ3D_OPT_PK_SLICE (buckets, 0 or >= 2; default 0): upper bound on the packed probe's slice
   * width (normally the largest that fits one workgroup's LDS). Tables of more than 1024 slices
   * take the two-level partition (k_pk_part into coarse ranges, k_pk_split by slice), so a small
   * bound puts small tables on that path (tests). It bounds the partitioned nested probe's slice
   * width too: beyond 2048 slices that probe takes the same two-level partition. */
  HJ3D_OPT_PK_SLICE = 8,
  /* HJ3D_OPT_PK_STAGE (pairs, default 0 = the whole LDS stage): the packed partitioner writes its
   * carried partial segments out early once the carries plus a tile exceed this many pairs
   * (tests: 1 flushes after every tile). */
  HJ3D_OPT_PK_STAGE = 9,
  /* HJ3D_OPT_PK_BUILD (0/1, default 0): chaining builds take the slice build of tables beyond the
   * radix build's range (R through the packed partitioner's two levels into 8192-bucket slices,
   * each built in LDS; synchronous, region overflow falls back to the direct build) whenever it
   * applies, not only above 2048 x 16384 buckets (tests). */
  HJ3D_OPT_PK_BUILD = 10,
  /* HJ3D_OPT_NESTED_PK (0/1, default 0): the nested aggregation build partitions by the packed
   * partitioner's slices (k_pk_part + k_pk_split, the form tables of more than 2048 partitions take,
   * e.g. config D's 1e8-bucket Nrs table) whenever it applies, not only above 2048 partitions
   * (tests). Region overflow (skewed keys) falls back to the sort build. */
  HJ3D_OPT_NESTED_PK = 11,
  /* 12: reserved (a compact slice image for the packed probe, measured slower: 0.61 against 0.49 ms
   * at config B; removed in round 6) */
  /* HJ3D_OPT_SYNC_BUILD (0/1, default 0): hj3d_build / hj3d_build_many finish a nested table before
   * they return (they wait for its counts and run the sort build there if the LDS aggregation build
   * gave up), so the build relation's device memory may be released as soon as the call returns.
   * Default: the table finishes at its next use (see hj3d_build). */
  HJ3D_OPT_SYNC_BUILD = 13,
  /* 14: retired (the two-level nested partition, measured slower than the one-level one) */
  /* HJ3D_OPT_RP_UNFUSED (0/1, default 0): small implicit-row build partitions run as two launches
   * (histogram, then scatter) instead of the fused one-launch partition with its grid barrier
   * (A/B measurements and the parity test of both forms). The fused form runs only when the
   * occupancy API confirms all its workgroups are resident (another stream holding CUs can still
   * delay some); should a barrier not complete within 0.2 s, its workgroups go on with partial
   * partition sizes and the table is invalid: hj3d_table_stats / _size / _export / _finish of that
   * table and the next hj3d_probe_result / hj3d_probe2_result return HJ3D_EDEVICE. A rebuild of the
   * table replaces it. */
  HJ3D_OPT_RP_UNFUSED = 15,
  /* HJ3D_OPT_DIAG_GBAR (ticks of the 100 MHz clock, default 0 = off): diagnostic for the failure path
   * above. The fused partition's barrier then times out after this many ticks, and its workgroup 0
   * never arrives, so every barrier of such a build times out (tests). */
  HJ3D_OPT_DIAG_GBAR = 16,
  /* HJ3D_OPT_DIAG_LOOKBACK (ticks of the 100 MHz clock, default 0 = off): diagnostic of the nested
   * build on the packed slices (the aggregation form that finishes by decoupled look-back: each
   * partition's main-record base waits on its predecessors' published counts, at most 0.2 s, after
   * which the build gives up and the sort build replaces the table). Partition 0 then never
   * publishes and the wait limit is this many ticks, so every such build gives up (tests). */
  HJ3D_OPT_DIAG_LOOKBACK = 17
};
hj3d_status hj3d_ctx_set_option(hj3d_ctx* ctx, int option, int64_t value);
/* Timing events for a host's own phase timers (the bench's build / probe boundaries): HIP events
 * created without the system-scope fence (hipEventDisableSystemFence), recorded on the context
 * stream. A default event writes the L2 back when it is recorded, which leaves the GPU idle
 * ~10 us between the kernels around it. hj3d_tevent_elapsed waits for b, then gives b - a in ms. */
hj3d_status hj3d_tevent_create(hj3d_ctx* ctx, void** ev);
hj3d_status hj3d_tevent_record(hj3d_ctx* ctx, void* ev);
hj3d_status hj3d_tevent_elapsed(void* a, void* b, float* ms);
void hj3d_tevent_destroy(void* ev);
/* Kernel-phase timers: HIP events recorded on the context stream around every phase
 * (phase ids below). hj3d_ctx_timer reads (synchronously) the summed milliseconds and the
 * number of recorded intervals since the last reset. hj3d_ctx_timing(ctx, mode): 0 off; 1 every
 * timer (whole-call phases are marker events between the kernels on the stream); 2 only the timers
 * whose events travel with a kernel's dispatch (the packed probe's k_pk_part / k_pk_split /
 * k_pk_probe), so timing puts no packet between the kernels. */
enum {
  HJ3D_T_BUILD = 0,         /* hj3d_build, whole call */
  HJ3D_T_PROBE = 1,         /* hj3d_probe / hj3d_probe2, whole call */
  HJ3D_T_PROBE_KERNEL = 2,  /* the join-probe kernel launches only (radix path: k_rp_probe) */
  HJ3D_T_PARTITION = 3,     /* hj3d_partition (multi-GPU exchange partitioner) */
  HJ3D_T_SCATTER = 4,       /* radix probe path: probe-side partition scatter kernel */
  HJ3D_T_HIST = 5,          /* radix probe path: probe-side partition histogram kernel; packed probe
                             * of more than 1024 slices: its second partition level (k_pk_split) */
  HJ3D_T_NTIMERS = 6
};
/* Kernel launches issued by this library so far, all contexts of the process (diagnostic: the bench
 * reports launches per step). */
uint64_t hj3d_launch_count(void);
/* Diagnostic: per-partition phase clocks of the last k_nagg launch (library built with
 * -DHJ3D_NAGG_CLK=1; otherwise HJ3D_EUNSUPPORTED). 8 u64 words per partition: 0 entry, 1 table
 * cleared, 2 pass A done, 3 main records written, 4 pass B done, 5 exit (100 MHz wall clock), 7 the
 * workgroup's dispatch index. parts <= 16384. */
hj3d_status hj3d_diag_nagg_clk(uint64_t* host, uint32_t parts);
hj3d_status hj3d_ctx_timing(hj3d_ctx* ctx, int mode);
hj3d_status hj3d_ctx_timer(hj3d_ctx* ctx, int phase, double* ms_total, uint64_t* count);
hj3d_status hj3d_ctx_timer_reset(hj3d_ctx* ctx);

/* ---- device memory for hosts that link only this ABI (the C++ drop-in layer) ---- */
hj3d_status hj3d_dev_alloc(hj3d_ctx* ctx, uint64_t bytes, void** dev);
hj3d_status hj3d_dev_free(hj3d_ctx* ctx, void* dev);
/* synchronous copies (host <-> device) on the context stream */
hj3d_status hj3d_upload(hj3d_ctx* ctx, void* dev, const void* host, uint64_t bytes);
hj3d_status hj3d_download(hj3d_ctx* ctx, void* host, const void* dev, uint64_t bytes);

/* ---- tables ---- */
hj3d_status hj3d_table_create(hj3d_ctx* ctx, const hj3d_table_desc* desc, hj3d_table** out);
void        hj3d_table_destroy(hj3d_table* t);
/* Pre-size device storage for builds of up to max_build tuples (allocation outside timed loops). */
hj3d_status hj3d_table_reserve(hj3d_ctx* ctx, hj3d_table* t, uint64_t max_build);
hj3d_status hj3d_table_clear(hj3d_ctx* ctx, hj3d_table* t);
/* Build: replaces the table content with the tuples of `build` (asynchronous). A nested table's
 * build finishes at the table's next use (probe, statistics, export): its counts are read then, and
 * when the LDS aggregation build gave up on a key range too dense for it, the sort build runs then,
 * from `build` again -- so the build relation's device memory must stay valid until that use (or set
 * HJ3D_OPT_SYNC_BUILD). That fallback build is timed as HJ3D_T_BUILD, not as part of the probe. */
hj3d_status hj3d_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel* build);
/* Builds several tables, tables[k] from builds[k] (asynchronous; as hj3d_build for each). Two nested
 * tables of one geometry (equal num_buckets and bucket range: experiment 4's S and T tables,
 * main_experiment4.cc:832-859) take ONE launch sequence: both relations partitioned, one
 * aggregation grid over both tables' partitions, one scan, one compaction. Otherwise the tables
 * are built one after another. Replaces the reference's consecutive AlgScan -> AlgNestJoinBuild
 * runs (main_experiment4.cc:856-859, 879-881). */
hj3d_status hj3d_build_many(hj3d_ctx* ctx, hj3d_table* const* tables, const hj3d_rel* builds, uint32_t count);
/* Host copy of a table's device arrays (synchronous): what the drop-in layer's per-tuple probes
 * walk (HtChaining1::findDirEntryByOther ht_chaining.hh:236-248, HtNested1::findMainNodeByOther
 * ht_nested.hh:354-382). Call with NULL arrays first to get the sizes: *n_payload = entries
 * (chaining) or main records (nested), *n_sub = build rows of a nested table (0 for chaining).
 * Then off[nb_local + 1] receives the CSR offsets of the local buckets into the payload, payload
 * the chaining entries {u32 hash, u32 row} or the nested main records {u32 hash, first_row,
 * sub_off, sub_len}, and sub (nested) the build rows grouped per key, sub[sub_off .. + sub_len).
 * Entry order: chaining buckets of <= 32 entries come sorted by row (the reference's chain order is
 * then [first, newest, ..., second], arithmetic in that order); longer buckets are in no defined
 * order (the builds claim their runs with atomics) -- a consumer that needs the reference's chain
 * order there sorts by row, as the drop-in host view does. Nested: mains and sub rows in no defined
 * order (the reference's order follows from first_row and the rows). */
hj3d_status hj3d_table_export(hj3d_ctx* ctx, const hj3d_table* t, uint32_t* off, void* payload, uint32_t* sub,
                              uint64_t* n_payload, uint64_t* n_sub);
/* Which build made the table's current content (diagnostic, static string): chaining "radix",
 * "slices" (pk_slices, tables beyond the radix build's range) or "direct"; nested "nested_agg",
 * "nested_agg_slices" (more than 2048 partitions), each with "_reg" appended when the register form
 * aggregated them, or "nested_sort"; "none" before a
 * build. A nested table whose build has not been resolved yet (no use since hj3d_build) reports the
 * path that was started, with "?" appended ("nested_agg?"): the getter never waits or builds. Replaces
 * nothing of the reference (which has one insert path). */
const char* hj3d_table_build_path(const hj3d_table* t);
/* Finishes a nested table's build now (waits for its counts; runs the sort build from the build
 * relation if the LDS aggregation build gave up), as its next use would. No-op for a finished table.
 * Replaces nothing of the reference (whose insert is synchronous). */
hj3d_status hj3d_table_finish(hj3d_ctx* ctx, hj3d_table* t);
/* Synchronous statistics (makeStatistics). */
hj3d_status hj3d_table_stats(hj3d_ctx* ctx, const hj3d_table* t, hj3d_stats* out);
/* Number of tuples / distinct keys currently stored (synchronous). */
hj3d_status hj3d_table_size(hj3d_ctx* ctx, const hj3d_table* t, uint64_t* n_entries, uint64_t* n_distinct);

/* ---- probe ----
 * Asynchronous: counters accumulate in a device-side result slot; hj3d_probe_result reads it
 * (synchronous). With HJ3D_PROBE_EMIT, output pairs {u32 a, u32 b} are written to out_dev
 * (at most out_cap pairs; n_out still counts all and HJ3D_EOVERFLOW is reported by
 * hj3d_probe_result if n_out > out_cap). Pair order in out_dev is unspecified. */
hj3d_status hj3d_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel* probe, uint32_t flags,
                       void* out_dev, uint64_t out_cap);
hj3d_status hj3d_probe_result(hj3d_ctx* ctx, hj3d_probe_res* out);

/* Experiment-4 probe strand over two tables built on S and T (both HJ3D_NESTED: Ndu with deferred
 * unnesting; both HJ3D_CHAIN: Chj). With HJ3D_PROBE_EMIT, triples {u32 r, s, t} go to out_dev.
 * The row sums sum_a / sum_b / sum_c are always folded (the unnest reads every output triple's
 * rows); the triple hashes sum_h / xor_h only with HJ3D_PROBE_CHECKSUM (else 0). */
hj3d_status hj3d_probe2(hj3d_ctx* ctx, const hj3d_table* ts, const hj3d_table* tt, const hj3d_rel* probe,
                        uint32_t flags, void* out_dev, uint64_t out_cap);
hj3d_status hj3d_probe2_result(hj3d_ctx* ctx, hj3d_probe2_res* out);

/* ---- multi-GPU exchange helpers (bucket-range radix partition) ----
 * Destination of a tuple: owner(bucket) = bucket * nparts / num_buckets. Writes (key,row)
 * pairs grouped by destination into out_pairs_dev (capacity rel->n pairs) and the per
 * destination counts into counts_dev[nparts] (device u64). Order within a destination
 * follows input order (stable). */
hj3d_status hj3d_partition(hj3d_ctx* ctx, const hj3d_rel* rel, uint64_t num_buckets, uint32_t nparts,
                           void* out_pairs_dev, void* counts_dev);
/* The same with a selection below the exchange (AlgSelection, algebra.hh:278-358): only the tuples
 * passing the predicate conjunction (hj3d_sel_pred, below) are partitioned and shipped; row ids
 * stay those of `rel`, so the probe downstream reports the reference's rows. */
typedef struct hj3d_sel_pred hj3d_sel_pred;
hj3d_status hj3d_partition_sel(hj3d_ctx* ctx, const hj3d_rel* rel, const hj3d_sel_pred* preds, uint32_t npred,
                               uint64_t num_buckets, uint32_t nparts, void* out_pairs_dev, void* counts_dev);
/* Single-pass form for the probe side of the exchange (no order kept inside a destination: the
 * probe's counters are per tuple; the build side keeps hj3d_partition's stable order, which fixes
 * the chain order of buckets longer than the sorted build handles). The relation is read once
 * (hj3d_partition reads it twice); destination p's pairs go to out_pairs_dev + p * stride pairs
 * (stride >= 1, nparts <= 256; out_pairs_dev holds nparts * stride pairs), counts_dev[p] (device
 * u64) = the number of tuples destined to p. Pairs past a destination's stride are NOT written
 * (a spill): when any counts_dev[p] > stride the caller re-partitions with hj3d_partition (the
 * counts are the same). hj3d_partition_stride gives a bounded stride that distinct keys spill with
 * negligible probability (mean + max(8 sigma of the binomial destination count, mean / 64) + 2
 * tiles; the mean / 64 covers keys repeated ~10 times, as config D's S.a), so the send
 * buffer is ~|rel| pairs instead of nparts x |rel| (stride = rel->n never spills). preds / npred:
 * an optional selection as in hj3d_partition_sel (npred = 0: none). Send it with
 * hj3d_comm_exchange_strided (same stride). Replaces the same seam as hj3d_partition
 * (the reference itself runs on one node, main_experiment1.cc:623-848). */
hj3d_status hj3d_partition_strided(hj3d_ctx* ctx, const hj3d_rel* rel, const hj3d_sel_pred* preds, uint32_t npred,
                                   uint64_t num_buckets, uint32_t nparts, void* out_pairs_dev, uint64_t stride,
                                   void* counts_dev);
uint64_t hj3d_partition_stride(uint64_t n, uint32_t nparts);
/* Owned bucket range of part p: [lo, hi) with lo = ceil(p*NB/nparts). */
void hj3d_part_range(uint64_t num_buckets, uint32_t nparts, uint32_t part, uint64_t* lo, uint64_t* hi);
/* Slice geometry the packed unique probe takes for a chaining table of nb_local buckets holding
 * n_build entries (diagnostic; no device work): out = {W, P, C, W1, P1}: P slices of W buckets
 * (one slice's directory + entries fill one probe workgroup's LDS); C > 1: two partition levels,
 * P1 coarse ranges of W1 = C * W buckets. Replaces nothing of the reference (whose chains are not
 * partitioned); bench.py reports it beside config D's line. */
hj3d_status hj3d_probe_geometry(hj3d_ctx* ctx, uint64_t nb_local, uint64_t n_build, uint32_t out[5]);

/* ---- the exchange itself: RCCL over xGMI, one communicator per context ----
 * One process (or host thread) per GPU, one context per process. RCCL is resolved at run time: a
 * librccl already mapped into the process (torch's) is used, else /opt/rocm's (hj3d_runtime_info
 * names the files). Collective calls must be made by every rank in the same order.
 *   hj3d_comm_unique_id  rank 0 creates the 128-byte communicator id; the host hands it to the
 *                        other ranks by any side channel (torch.distributed broadcast, a file, MPI);
 *   hj3d_comm_init       every rank joins (synchronous; collective);
 *   hj3d_comm_counts     all-to-all of per-destination counts of `chunks` partitioned chunks at once:
 *                        counts_dev = device i64 [chunks][world] (the counts hj3d_partition wrote,
 *                        one row per chunk); send_host / recv_host = host i64 [chunks][world],
 *                        recv[c][p] = elements rank p sends this rank in chunk c (synchronous: the
 *                        one host synchronisation of an exchange strand; collective);
 *   hj3d_comm_counts_cap the same, with this rank's receive capacity (elements it can take over
 *                        the chunks): the ranks agree by an all-reduce whether any rank's total
 *                        exceeds its capacity, and then EVERY rank returns HJ3D_EOVERFLOW, before
 *                        any pair collective (recv_cap = UINT64_MAX: hj3d_comm_counts);
 *   hj3d_comm_exchange   grouped send / recv of one chunk: send_dev holds send_counts[p] elements of
 *                        elem_bytes for every peer p back to back (hj3d_partition's layout), recv_dev
 *                        receives recv_counts[p] elements from every peer in rank order. A receive
 *                        total above recv_cap returns HJ3D_EOVERFLOW BEFORE the collective: every
 *                        rank knows its totals from hj3d_comm_counts, so size recv_dev from them
 *                        (a rank that skips the call leaves its peers waiting; hj3d_comm_counts_cap
 *                        makes that refusal collective). ticket == NULL:
 *                        enqueued on the context stream. ticket != NULL: enqueued on the context's
 *                        exchange stream after the work already on the context stream, so probes of
 *                        earlier chunks overlap it; hj3d_comm_wait(ticket) orders the context stream
 *                        after it (tickets count up; a ticket older than the 64 latest waits for a
 *                        later exchange of the same stream, never too early). Collective;
 *   hj3d_comm_allreduce_u64 / hj3d_comm_allgather  merge the per-rank result slots and statistics
 *                        (u64 counters add, extremes max / min; xor via all-gather), on the context
 *                        stream. Collective. */
#define HJ3D_COMM_ID_BYTES 128
enum { HJ3D_RED_SUM = 0, HJ3D_RED_MAX = 1, HJ3D_RED_MIN = 2 };
hj3d_status hj3d_comm_unique_id(hj3d_ctx* ctx, uint8_t* id);
hj3d_status hj3d_comm_init(hj3d_ctx* ctx, const uint8_t* id, int rank, int world);
hj3d_status hj3d_comm_destroy(hj3d_ctx* ctx);
hj3d_status hj3d_comm_rank(const hj3d_ctx* ctx, int* rank, int* world);
hj3d_status hj3d_comm_counts(hj3d_ctx* ctx, const void* counts_dev, uint32_t chunks, int64_t* send_host,
                             int64_t* recv_host);
hj3d_status hj3d_comm_counts_cap(hj3d_ctx* ctx, const void* counts_dev, uint32_t chunks, uint64_t recv_cap,
                                 int64_t* send_host, int64_t* recv_host);
hj3d_status hj3d_comm_exchange(hj3d_ctx* ctx, const void* send_dev, const int64_t* send_counts, void* recv_dev,
                               const int64_t* recv_counts, uint64_t recv_cap, uint32_t elem_bytes,
                               uint32_t* ticket);
/* The same with peer p's elements at send_dev + p * send_stride elements (hj3d_partition_strided's
 * layout; send_stride = 0: back to back); a send count above send_stride is HJ3D_EINVAL.
 * MANDATORY before this call on every rank: check the partitioner's counts against the stride and
 * re-partition a spilled chunk (hj3d_partition_strided above). The EINVAL is local to the rank
 * that spilled; its peers, already inside the collective, would wait for it forever. */
hj3d_status hj3d_comm_exchange_strided(hj3d_ctx* ctx, const void* send_dev, uint64_t send_stride,
                                       const int64_t* send_counts, void* recv_dev, const int64_t* recv_counts,
                                       uint64_t recv_cap, uint32_t elem_bytes, uint32_t* ticket);
hj3d_status hj3d_comm_wait(hj3d_ctx* ctx, uint32_t ticket);
hj3d_status hj3d_comm_allreduce_u64(hj3d_ctx* ctx, void* buf_dev, uint64_t n, int op);
hj3d_status hj3d_comm_allgather(hj3d_ctx* ctx, const void* send_dev, void* recv_dev, uint64_t bytes);
/* Which HIP runtime (and RCCL) this library runs on: file names and versions, as text. hj3d_ctx_create
 * fails with HJ3D_EDEVICE (reason on stderr) when two HIP runtimes are mapped into the process. */
hj3d_status hj3d_runtime_info(char* buf, uint64_t cap);

/* ---- #dv pre-pass (the number of distinct join-attribute values sizes the build-on-S.a plans:
 * NB = #dv(S.a) / b, main_experiment1.cc:453-454 counts it with an unordered_set, 875, 1001,
 * 1214 use it). One GPU: key_bitmap + or_popcount with rows = 1. Multi-GPU (SURVEY §8e step 1,
 * hj3d/dist.py num_distinct): each rank builds the bitmap of its slice, the ranks all-to-all
 * the bitmap in nranks equal slices, each ORs the slices it received (rows = nranks) and
 * popcounts, and the counts are summed. ----
 * hj3d_key_bitmap: sets bit k of bitmap_dev (u32 words, ceil(domain / 32) of them, zeroed by the
 * caller) for every key k < domain of rel; outside_dev (u64, may be NULL) += #keys >= domain. */
hj3d_status hj3d_key_bitmap(hj3d_ctx* ctx, const hj3d_rel* rel, uint64_t domain, void* bitmap_dev,
                            void* outside_dev);
/* count_dev (u64) += popcount of the OR of `rows` bitmaps of `words` u32 words each, stored
 * back to back at bitmaps_dev. */
hj3d_status hj3d_bitmap_or_popcount(hj3d_ctx* ctx, const void* bitmaps_dev, uint32_t rows, uint64_t words,
                                    void* count_dev);

/* ---- measurement: the box's streaming-copy peak, measured in the same run as the
 * kernels whose roofline fractions are quoted. Replaces nothing of the reference. ----
 * Synchronous: copies `bytes` (a multiple of 16) from src_dev to dst_dev `reps` times for each of
 * six variants (plain / non-temporal 16-B vectors, 4 / 8 / 16 workgroups per CU), each launch timed
 * by HIP events on the context stream; out[0] = the best rate in GB/s (read + write bytes), out[1] =
 * the median launch of that variant, out[2] = its id (workgroups per CU, + 100 when non-temporal). */
hj3d_status hj3d_stream_copy(hj3d_ctx* ctx, void* dst_dev, const void* src_dev, uint64_t bytes, uint32_t reps,
                             double out[3]);

/* ---- selection pushdown: AlgSelection / AlgDynSelection (algebra.hh:278-358) on the device ----
 * The predicate is a conjunction of `npred` (<= HJ3D_SEL_MAX) comparisons of one u32 tuple word
 * (byte offset word_off, compared as int32 when is_signed, else as uint32) against lo (and hi for
 * HJ3D_SEL_RANGE: lo <= v < hi). The passing tuples of `rel` are written, in scan order, to
 * out_pairs_dev as {u32 key, u32 row} (row = the tuple's row id in rel, capacity rel->n pairs);
 * count_dev (device u64) receives their number. The pairs are a relation {out, n, stride 8,
 * key_off 0, row_off 4} that hj3d_build / hj3d_probe take as the selection's consumer would:
 * same order, same row identities. Asynchronous. */
#define HJ3D_SEL_MAX 4
enum { HJ3D_SEL_LT = 0, HJ3D_SEL_LE, HJ3D_SEL_GT, HJ3D_SEL_GE, HJ3D_SEL_EQ, HJ3D_SEL_NE, HJ3D_SEL_RANGE };
struct hj3d_sel_pred {
  uint32_t word_off;  /* byte offset of the compared u32 word, multiple of 4, < stride */
  uint32_t op;        /* HJ3D_SEL_*                                                    */
  uint32_t is_signed; /* compare as int32 (the reference's attrval_t is int)           */
  uint32_t reserved;
  int64_t lo, hi;
};
hj3d_status hj3d_select(hj3d_ctx* ctx, const hj3d_rel* rel, const hj3d_sel_pred* preds, uint32_t npred,
                        void* out_pairs_dev, void* count_dev);
/* Probe strand behind a selection: scan(probe) -> AlgSelection -> probe, as hj3d_probe of the
 * passing tuples (rows = their rows in `probe`). On the partitioned probe path (chaining or nested
 * table) with one predicate the selection is fused into the probe-side partitioner (the failing tuples are
 * dropped where the tuples are read; no extra pass); otherwise hj3d_select runs first
 * (synchronous count read). Result: n_probe = passing tuples (the selection's count()), the
 * other fields as hj3d_probe. Dense output (chaining + HJ3D_PROBE_UNIQUE) fills n_probe slots
 * and needs out_cap >= probe->n. */
hj3d_status hj3d_probe_sel(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel* probe, const hj3d_sel_pred* preds,
                           uint32_t npred, uint32_t flags, void* out_dev, uint64_t out_cap);

/* ---- synthetic key/FK relations generated on the device (bench / full-size checks) ----
 * R.k = a seeded bijective permutation of [0, n_keys) (keys for global rows
 * [row_base, row_base+n)), written into tuple word key_off of an AoS buffer;
 * S.a = uniform in [0, fk_max) from a counter-based RNG of the global row id. */
hj3d_status hj3d_gen_keys(hj3d_ctx* ctx, void* tuples_dev, uint64_t n, uint32_t stride, uint32_t key_off,
                          uint64_t row_base, uint64_t n_keys, uint64_t seed);
hj3d_status hj3d_gen_fk(hj3d_ctx* ctx, void* tuples_dev, uint64_t n, uint32_t stride, uint32_t key_off,
                        uint64_t row_base, uint32_t fk_max, uint64_t seed);
/* S.a ~ Zipf(theta) over [0, fk_max) (value 0 the most frequent; P(v) ~ (v+1)^-theta), sampled by
 * rejection-inversion (the method of util/zipf_distribution.hh) from a counter-based RNG of the
 * global row id: config C (nested table, Zipf 0.8 duplicates) at full size. */
hj3d_status hj3d_gen_zipf(hj3d_ctx* ctx, void* tuples_dev, uint64_t n, uint32_t stride, uint32_t key_off,
                          uint64_t row_base, uint32_t fk_max, double theta, uint64_t seed);
/* ---- the reference's own input generators (host, synchronous, bit-exact) ----
 * hj3d_gen_exp1_ref replaces Experiment1::init (main_experiment1.cc:415-457): one std::mt19937
 * stream (seed 5489) shuffles R.k = iota(nR) (std::shuffle), draws S.a uniform over [0, fkMax)
 * (GenRandIntVec::generate_uni, util/GenRandIntVec.cc:72-98) or Zipf(theta) - 1
 * (generate_zipf :167-200, util/zipf_distribution.hh:48-58), then permutes S.a (vec_permute
 * :335-340); fkMax = nR >> t (main_experiment1.cc:190). Writes the columns Rk[nR], Sa[nS] to
 * HOST memory; S.k is the row id. theta: the reference's experiment 1 fixes 1.0 (:444); config C
 * uses 0.8. threads: workers for the Zipf attempts (0 = min(hardware threads, 16)); the result does
 * not depend on it.
 * hj3d_gen_exp4_ref replaces Experiment4::init (main_experiment4.cc:517-575): S.a, T.a of
 * card = (2^log2R >> alpha) * mult_a + (2^log2R >> beta) * mult_b tuples each (R.k, S.k, T.k =
 * iota). With Sa or Ta NULL only *card is written. */
hj3d_status hj3d_gen_exp1_ref(uint64_t nR, uint64_t nS, int skew, double theta, uint32_t t, uint32_t* Rk,
                              uint32_t* Sa, int threads);
hj3d_status hj3d_gen_exp4_ref(uint32_t log2R, uint32_t alpha, uint32_t mult_a, uint32_t beta, uint32_t mult_b,
                              uint32_t* Sa, uint32_t* Ta, uint64_t* card);
/* Expected key/FK join aggregates WITHOUT a hash table (full-size verification of the
 * key/FK plans): `build` holds unique keys in [0, n_keys); every probe tuple's partner row is
 * inv[key], inv being the inverse of the build key column. Accumulates {n_out, sum_a, sum_b,
 * sum_h, xor_h} (u64 each) into res_dev (zero it first). Orientation: a = probe row,
 * b = build row; with swap != 0, a = build row, b = probe row (plans that build on the FK side). */
hj3d_status hj3d_expected_fk_join(hj3d_ctx* ctx, const hj3d_rel* build, const hj3d_rel* probe, uint64_t n_keys,
                                  int swap, void* res_dev);
/* The same expectation when the build keys were made by hj3d_gen_keys(n_keys, key_seed): the
 * partner row of key k is the inverse permutation of k (per-rank verification on multi-GPU). */
hj3d_status hj3d_expected_fk_join_gen(hj3d_ctx* ctx, const hj3d_rel* probe, uint64_t n_keys, uint64_t key_seed,
                                      int swap, void* res_dev);

#ifdef __cplusplus
}
#endif
#endif /* HJ3D_H */

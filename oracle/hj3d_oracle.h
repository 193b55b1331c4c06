/* hj3d_oracle.h — CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so, and only as the checker / the timed CPU baseline. The product
 * (libhj3d.so) never links or calls it.
 *
 * Parity pinning: every function here is checked against golden fixtures that
 * oracle/_ref/ref_golden.out produced by running the REAL reference code
 * (tests/golden/exp*.json, made by tests/golden/make_golden.py).
 *
 * Relations are array-of-structs of u32 words: tuple i starts at base + i*stride
 * (stride in u32 words); its join attribute is word `key` of the tuple.
 */
#ifndef HJ3D_ORACLE_H
#define HJ3D_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { uint32_t mt[624]; int idx; } orc_mt19937;

#define ORC_ROW_IMPLICIT 0xFFFFFFFFu

typedef struct {
  const uint32_t* base;
  uint64_t n;
  uint32_t stride; /* u32 words per tuple */
  uint32_t key;    /* word index of the join attribute */
  uint32_t row;    /* word index of an explicit row id (exchanged (key,row) pairs of the
                      multi-GPU path), or ORC_ROW_IMPLICIT: row id = index in the relation */
  uint32_t pad;
} orc_rel;

typedef struct {
  uint64_t nb, empty, entries, distinct;
  uint64_t cc0_min, cc0_max, cc0_sum, cc0_cnt;
  uint64_t cc1_min, cc1_max, cc1_sum, cc1_cnt;
} orc_stats;

typedef struct { uint64_t n, sum_a, sum_b, sum_c, sum_h, xor_h; } orc_agg;

typedef struct {
  uint64_t c_build, c_probe, c_cmp, c_unnest, c_top;
  uint64_t reps;
  double build_ns, probe_ns; /* mean per rep (repeat_mintime protocol) */
  orc_stats stats;
  orc_agg out;
} orc_plan_res;

typedef struct {
  uint64_t c_probe_rs, c_probe_rs_cmp, c_probe_rt, c_probe_rt_cmp, c_unnest_1, c_unnest_2, c_top;
  uint64_t reps;
  double build_s_ns, build_t_ns, probe_ns;
  orc_agg out;
} orc_exp4_res;

/* ---- checksums (identical definitions in include/hj3d.h) ---- */
uint64_t orc_mix64(uint64_t z);
uint64_t orc_colsum(const uint32_t* v, uint64_t n);

/* ---- input generation (bit-exact restatement of the reference generators) ---- */
void     orc_mt_seed(orc_mt19937* g, uint32_t seed);
uint32_t orc_mt_next(orc_mt19937* g);
/* experiment 1: R.k = shuffle(iota(nR)), S.a = uniform/zipf FKs in [0, nR>>t) then permuted.
 * Returns fkMax. main_experiment1.cc:415-457. */
uint32_t orc_gen_exp1(uint64_t nR, uint64_t nS, int skew, double theta, uint32_t t,
                      uint32_t* Rk, uint32_t* Sa);
/* experiment 4: S.a / T.a foreign-key columns (R.k = S.k = T.k = iota). main_experiment4.cc:517-575.
 * Returns |S| (= |T|). Pass NULL outputs to query the size only. */
uint64_t orc_gen_exp4(uint32_t log2R, uint32_t alpha, uint32_t multA, uint32_t beta, uint32_t multB,
                      uint32_t* Sa, uint32_t* Ta);
uint64_t orc_num_distinct(const uint32_t* v, uint64_t n);

/* ---- plans (one build + one probe strand; repeated per repeat_mintime) ----
 * agg != 0: fold every emitted tuple into res->out (parity mode).
 * min_ms / min_reps: util/measure_helpers.hh:15-41 protocol; (0, 1) = single run. */
int orc_chain_plan(const orc_rel* build, const orc_rel* probe, uint64_t num_buckets, int unique,
                   int agg, double min_ms, uint64_t min_reps, orc_plan_res* res);
int orc_nested_plan(const orc_rel* build, const orc_rel* probe, uint64_t num_buckets, int unnest,
                    int agg, double min_ms, uint64_t min_reps, orc_plan_res* res);
/* experiment 4: nested (Ndu, deferred unnesting) or chaining (Chj); R/S/T are {k,a} tuples. */
int orc_exp4_plan(const orc_rel* R, const orc_rel* S, const orc_rel* T, uint64_t num_buckets,
                  int nested, int agg, double min_ms, uint64_t min_reps, orc_exp4_res* res);

#ifdef __cplusplus
}
#endif
#endif

/* hj3d_oracle.c — clean-room single-thread C restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py (as the checker and the timed "port" CPU baseline).
 * It is deliberately a pointer-chasing, tuple-at-a-time structure like the
 * reference (24-B chain nodes, 32-B main nodes, 16-B sub nodes, chunked node
 * reservoirs), so that its timing is representative of the reference's CPU path.
 *
 * Pinned against fixtures produced by the real reference (oracle/ref_golden.cc).
 *
 * Reference entities restated here (file:line under /root/reference):
 *   murmur_hash<uint32_t>            util/hasht.hh:52-61
 *   HtChaining1 insert / probe dir   ht_chaining.hh:181-196, 236-248
 *   HtChaining1::makeStatistics      ht_chaining.hh:260-292
 *   HtNested1 insert & helpers       ht_nested.hh:287-311, 386-436
 *   HtNested1::findMainNodeByOther   ht_nested.hh:354-382
 *   HtNested1::makeStatistics        ht_nested.hh:450-482
 *   AlgHashJoinProbe::step           algebra.hh:625-659
 *   AlgNestJoinProbe::step           algebra.hh:435-459
 *   AlgUnnestHt::step                algebra.hh:510-541
 *   repeat_mintime                   util/measure_helpers.hh:15-41
 *   Experiment1::init                main_experiment1.cc:415-457
 *   GenRandIntVec uni / zipf / perm  util/GenRandIntVec.cc:72-98, 167-200, 290-293, 335-340
 *   zipf_distribution                util/zipf_distribution.hh:22-147
 *   Experiment4::init                main_experiment4.cc:517-575
 *   Experiment4 Ndu / Chj plans      main_experiment4.cc:831-1043
 * Third-party algorithms the reference delegates to (libstdc++ 11.4 from GCC 11.4.0,
 * glibc libm of this image):
 *   std::mt19937                     bits/random.tcc (MT19937, seed 5489)
 *   uniform_int_distribution (Lemire) bits/uniform_int_dist.h:241-330
 *   std::shuffle                     bits/stl_algo.h:3706-3792
 *   generate_canonical<double,53>    bits/random.tcc:3348-3380
 */
#define _POSIX_C_SOURCE 200809L
#include "hj3d_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ */
/* hashing & checksums                                                 */
/* ------------------------------------------------------------------ */
static inline uint32_t murmur32(uint32_t x) { /* util/hasht.hh:52-61 */
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

uint64_t orc_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static inline uint64_t pair_hash(uint64_t a, uint64_t b) { return orc_mix64((a << 32) | (b & 0xffffffffULL)); }
static inline uint64_t triple_hash(uint64_t a, uint64_t b, uint64_t c) { return orc_mix64(pair_hash(a, b) ^ c); }

uint64_t orc_colsum(const uint32_t* v, uint64_t n) {
  uint64_t s = 0;
  for (uint64_t i = 0; i < n; ++i) s += pair_hash(i, v[i]);
  return s;
}

static inline void agg2(orc_agg* a, uint64_t x, uint64_t y) {
  const uint64_t h = pair_hash(x, y);
  a->n++; a->sum_a += x; a->sum_b += y; a->sum_h += h; a->xor_h ^= h;
}
static inline void agg3(orc_agg* a, uint64_t x, uint64_t y, uint64_t z) {
  const uint64_t h = triple_hash(x, y, z);
  a->n++; a->sum_a += x; a->sum_b += y; a->sum_c += z; a->sum_h += h; a->xor_h ^= h;
}

static double now_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e9 + (double)ts.tv_nsec;
}

/* ------------------------------------------------------------------ */
/* std::mt19937 and the libstdc++ 11 distributions                      */
/* ------------------------------------------------------------------ */
void orc_mt_seed(orc_mt19937* g, uint32_t seed) {
  g->mt[0] = seed;
  for (int i = 1; i < 624; ++i) g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
  g->idx = 624;
}

uint32_t orc_mt_next(orc_mt19937* g) {
  if (g->idx >= 624) {
    for (int k = 0; k < 624; ++k) {
      const uint32_t y = (g->mt[k] & 0x80000000u) | (g->mt[(k + 1) % 624] & 0x7fffffffu);
      g->mt[k] = g->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    g->idx = 0;
  }
  uint32_t y = g->mt[g->idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

/* uniform_int_distribution downscaling for a 32-bit engine: Lemire's nearly divisionless
 * method on the 32-bit range `range` (= b - a + 1, 1 <= range <= 2^32 - 1).
 * bits/uniform_int_dist.h:241-271 (_S_nd) and :296-330 (dispatch). */
static inline uint32_t uni_range(orc_mt19937* g, uint32_t range) {
  uint64_t product = (uint64_t)orc_mt_next(g) * (uint64_t)range;
  uint32_t low = (uint32_t)product;
  if (low < range) {
    const uint32_t threshold = (uint32_t)(-range) % range;
    while (low < threshold) {
      product = (uint64_t)orc_mt_next(g) * (uint64_t)range;
      low = (uint32_t)product;
    }
  }
  return (uint32_t)(product >> 32);
}

/* std::shuffle over u32 elements (bits/stl_algo.h:3729-3792). */
static void std_shuffle(uint32_t* v, uint64_t n, orc_mt19937* g) {
  if (n == 0) return;
  const uint64_t urngrange = 0xffffffffULL;
  if (urngrange / n >= n) {
    uint64_t i = 1;
    if ((n % 2) == 0) { /* one up-front swap with a {0,1} draw */
      const uint32_t j = uni_range(g, 2);
      const uint32_t t = v[i]; v[i] = v[j]; v[j] = t;
      ++i;
    }
    while (i != n) { /* two positions from one draw: __gen_two_uniform_ints */
      const uint64_t b0 = i + 1, b1 = i + 2;
      const uint64_t x = uni_range(g, (uint32_t)(b0 * b1));
      const uint64_t p0 = x / b1, p1 = x % b1;
      uint32_t t = v[i]; v[i] = v[p0]; v[p0] = t;
      ++i;
      t = v[i]; v[i] = v[p1]; v[p1] = t;
      ++i;
    }
    return;
  }
  for (uint64_t i = 1; i < n; ++i) {
    const uint64_t j = uni_range(g, (uint32_t)(i + 1));
    const uint32_t t = v[i]; v[i] = v[j]; v[j] = t;
  }
}

/* generate_canonical<double, 53>(mt19937): two draws (bits/random.tcc:3348-3380). */
static inline double canonical53(orc_mt19937* g) {
  double sum = (double)orc_mt_next(g);
  sum += (double)orc_mt_next(g) * 4294967296.0;
  double r = sum / 18446744073709551616.0;
  if (r >= 1.0) r = nextafter(1.0, 0.0);
  return r;
}

/* GenRandIntVec::vec_permute (util/GenRandIntVec.cc:335-340). */
static void vec_permute(uint32_t* v, uint64_t n, orc_mt19937* g) {
  if (n == 0) return;
  for (uint64_t i = n - 1; i > 0; --i) {
    const uint64_t j = (uint64_t)orc_mt_next(g) % i;
    const uint32_t t = v[i]; v[i] = v[j]; v[j] = t;
  }
}

/* zipf_distribution<uint, double> (util/zipf_distribution.hh:22-147). */
typedef struct { uint32_t n; double q, H_x1, H_n; } zipf_t;
static const double ZIPF_EPS = 1e-8;
static inline double expxm1bx(double x) {
  return (fabs(x) > ZIPF_EPS) ? expm1(x) / x : (1.0 + x / 2.0 * (1.0 + x / 3.0 * (1.0 + x / 4.0)));
}
static inline double log1pxbx(double x) {
  return (fabs(x) > ZIPF_EPS) ? log1p(x) / x : 1.0 - x * ((1 / 2.0) - x * ((1 / 3.0) - x * (1 / 4.0)));
}
static inline double zH(const zipf_t* z, double x) {
  const double log_x = log(x);
  return expxm1bx((1.0 - z->q) * log_x) * log_x;
}
static inline double zH_inv(const zipf_t* z, double x) {
  const double a = -1.0, b = x * (1.0 - z->q);
  const double t = (a < b) ? b : a; /* std::max(-1.0, ...) */
  return exp(log1pxbx(t) * x);
}
static inline double zh(const zipf_t* z, double x) { return exp(-z->q * log(x)); }
static void zipf_init(zipf_t* z, uint32_t n, double q) {
  z->n = n;
  z->q = q;
  z->H_x1 = zH(z, 1.5) - 1.0;
  z->H_n = zH(z, (double)n + 0.5);
}
static uint32_t zipf_draw(const zipf_t* z, orc_mt19937* g) {
  for (;;) {
    const double u = (canonical53(g) * (z->H_n - z->H_x1)) + z->H_x1; /* uniform_real_distribution */
    const double x = zH_inv(z, u);
    uint32_t k = (uint32_t)round(x);
    if (k > z->n) k = z->n; /* clamp<IntType>(round(x), 1, n) */
    if (k < 1) k = 1;
    if (u >= zH(z, (double)k + 0.5) - zh(z, (double)k)) return k;
  }
}

uint32_t orc_gen_exp1(uint64_t nR, uint64_t nS, int skew, double theta, uint32_t t, uint32_t* Rk, uint32_t* Sa) {
  orc_mt19937 g;
  orc_mt_seed(&g, 5489u);
  for (uint64_t i = 0; i < nR; ++i) Rk[i] = (uint32_t)i;
  std_shuffle(Rk, nR, &g);
  const uint32_t fkMax = (uint32_t)(nR >> t);
  if (!skew) {
    for (uint64_t i = 0; i < nS; ++i) Sa[i] = uni_range(&g, fkMax); /* uniform_int_distribution<int>(0, max-1) */
  } else {
    zipf_t z;
    zipf_init(&z, fkMax, theta);
    for (uint64_t i = 0; i < nS; ++i) Sa[i] = (zipf_draw(&z, &g) - 1u) % fkMax; /* genval_zipf */
  }
  vec_permute(Sa, nS, &g);
  return fkMax;
}

uint64_t orc_gen_exp4(uint32_t log2R, uint32_t alpha, uint32_t multA, uint32_t beta, uint32_t multB,
                      uint32_t* Sa, uint32_t* Ta) {
  const uint64_t cardR = 1ULL << log2R;
  const uint64_t nC = cardR >> alpha, nE = cardR >> beta;
  const uint64_t cardC = nC * multA, cardE = nE * multB, card = cardC + cardE;
  if (!Sa || !Ta) return card;
  uint32_t* fkC = (uint32_t*)malloc(sizeof(uint32_t) * (cardC ? cardC : 1));
  uint32_t* fkS = (uint32_t*)malloc(sizeof(uint32_t) * (cardE ? cardE : 1));
  uint32_t* fkT = (uint32_t*)malloc(sizeof(uint32_t) * (cardE ? cardE : 1));
  uint64_t v = 0, idx = 0;
  for (; v < nC; ++v) for (uint32_t i = 0; i < multA; ++i) fkC[idx++] = (uint32_t)v;
  idx = 0;
  for (; v < nC + nE; ++v) for (uint32_t i = 0; i < multB; ++i) fkS[idx++] = (uint32_t)v;
  idx = 0;
  for (; v < nC + 2 * nE; ++v) for (uint32_t i = 0; i < multB; ++i) fkT[idx++] = (uint32_t)v;
  orc_mt19937 g;
  orc_mt_seed(&g, 5489u);
  std_shuffle(fkS, cardE, &g);
  std_shuffle(fkT, cardE, &g);
  std_shuffle(fkC, cardC, &g);
  for (uint64_t i = 0; i < card; ++i) Sa[i] = i < cardC ? fkC[i] : fkS[i - cardC];
  std_shuffle(fkC, cardC, &g);
  for (uint64_t i = 0; i < card; ++i) Ta[i] = i < cardC ? fkC[i] : fkT[i - cardC];
  free(fkC); free(fkS); free(fkT);
  return card;
}

static int cmp_u32(const void* a, const void* b) {
  const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return (x > y) - (x < y);
}

uint64_t orc_num_distinct(const uint32_t* v, uint64_t n) {
  if (n == 0) return 0;
  uint32_t mx = 0;
  for (uint64_t i = 0; i < n; ++i) mx = v[i] > mx ? v[i] : mx;
  if (mx < (1u << 31)) {
    const uint64_t words = ((uint64_t)mx >> 6) + 1;
    uint64_t* bits = (uint64_t*)calloc(words, sizeof(uint64_t));
    for (uint64_t i = 0; i < n; ++i) bits[v[i] >> 6] |= 1ULL << (v[i] & 63);
    uint64_t c = 0;
    for (uint64_t w = 0; w < words; ++w) c += (uint64_t)__builtin_popcountll(bits[w]);
    free(bits);
    return c;
  }
  uint32_t* s = (uint32_t*)malloc(sizeof(uint32_t) * n);
  memcpy(s, v, sizeof(uint32_t) * n);
  qsort(s, n, sizeof(uint32_t), cmp_u32);
  uint64_t c = 1;
  for (uint64_t i = 1; i < n; ++i) c += s[i] != s[i - 1];
  free(s);
  return c;
}

/* ------------------------------------------------------------------ */
/* node reservoir (util/reservoir.hh semantics: chunks of 2^10 stable nodes) */
/* ------------------------------------------------------------------ */
typedef struct { char** chunks; size_t nchunks, cap, used_in_last, esz; } reservoir;
enum { RSV_LOG2 = 10, RSV_CHUNK = 1 << RSV_LOG2 };
static void rsv_init(reservoir* r, size_t esz) { memset(r, 0, sizeof(*r)); r->esz = esz; r->used_in_last = RSV_CHUNK; }
static void* rsv_new(reservoir* r) {
  if (r->used_in_last == RSV_CHUNK) {
    if (r->nchunks == r->cap) {
      r->cap = r->cap ? 2 * r->cap : 64;
      r->chunks = (char**)realloc(r->chunks, r->cap * sizeof(char*));
    }
    r->chunks[r->nchunks++] = (char*)malloc(RSV_CHUNK * r->esz);
    r->used_in_last = 0;
  }
  return r->chunks[r->nchunks - 1] + (r->used_in_last++) * r->esz;
}
static void rsv_erase(reservoir* r) { /* Reservoir::erase: release every chunk */
  for (size_t i = 0; i < r->nchunks; ++i) free(r->chunks[i]);
  free(r->chunks);
  rsv_init(r, r->esz);
}

static inline uint32_t key_of(const orc_rel* r, const uint32_t* t) { return t[r->key]; }
static inline uint64_t row_of(const orc_rel* r, const uint32_t* t) {
  return r->row == ORC_ROW_IMPLICIT ? (uint64_t)(t - r->base) / r->stride : t[r->row];
}

static void stats_init(orc_stats* s, uint64_t nb) {
  memset(s, 0, sizeof(*s));
  s->nb = nb;
  s->cc0_min = s->cc1_min = UINT64_MAX;
}
static inline void stats_step(orc_stats* s, uint64_t len) {
  if (len < s->cc0_min) s->cc0_min = len;
  if (len > s->cc0_max) s->cc0_max = len;
  s->cc0_sum += len; s->cc0_cnt++;
  if (len == 0) { s->empty++; return; }
  if (len < s->cc1_min) s->cc1_min = len;
  if (len > s->cc1_max) s->cc1_max = len;
  s->cc1_sum += len; s->cc1_cnt++;
}

/* ------------------------------------------------------------------ */
/* HtChaining1: 24-B node {next, data, hash}; dir slot holds the 1st entry  */
/* ------------------------------------------------------------------ */
typedef struct cnode { struct cnode* next; const uint32_t* data; uint32_t hash; } cnode;
#define CEMPTY ((cnode*)(uintptr_t)1)

typedef struct { cnode* dir; uint64_t nb, size; reservoir rsv; } chain_ht;

static void cht_init(chain_ht* h, uint64_t nb) {
  h->nb = nb; h->size = 0;
  h->dir = (cnode*)malloc(sizeof(cnode) * nb);
  for (uint64_t i = 0; i < nb; ++i) { h->dir[i].next = CEMPTY; h->dir[i].data = NULL; h->dir[i].hash = 0; }
  rsv_init(&h->rsv, sizeof(cnode));
}
static void cht_clear(chain_ht* h) { /* ht_chaining.hh:250-258 (size not reset: quirk) */
  rsv_erase(&h->rsv);
  for (uint64_t i = 0; i < h->nb; ++i) h->dir[i].next = CEMPTY;
}
static void cht_free(chain_ht* h) { rsv_erase(&h->rsv); free(h->dir); }

static inline void cht_insert(chain_ht* h, const uint32_t* t, uint32_t key) { /* ht_chaining.hh:181-196 */
  const uint32_t hv = murmur32(key);
  cnode* d = &h->dir[hv % h->nb];
  if (d->next == CEMPTY) {
    d->data = t; d->hash = hv; d->next = NULL;
  } else {
    cnode* n = (cnode*)rsv_new(&h->rsv);
    n->data = t; n->hash = hv; n->next = d->next;
    d->next = n;
  }
  h->size++;
}

static void cht_stats(const chain_ht* h, orc_stats* s) { /* ht_chaining.hh:260-292 */
  stats_init(s, h->nb);
  s->entries = h->size;
  uint32_t* hv = (uint32_t*)malloc(sizeof(uint32_t) * (h->size ? h->size : 1));
  uint64_t nh = 0;
  for (uint64_t b = 0; b < h->nb; ++b) {
    const cnode* d = &h->dir[b];
    if (d->next == CEMPTY) { stats_step(s, 0); continue; }
    uint64_t len = 0;
    for (const cnode* n = d; n; n = n->next) { ++len; if (nh < h->size) hv[nh++] = n->hash; }
    stats_step(s, len);
  }
  s->distinct = orc_num_distinct(hv, nh); /* distinct hash values == distinct keys (murmur32 is a bijection) */
  free(hv);
}

int orc_chain_plan(const orc_rel* build, const orc_rel* probe, uint64_t num_buckets, int unique, int agg,
                   double min_ms, uint64_t min_reps, orc_plan_res* res) {
  if (!build || !probe || !res || num_buckets == 0) return 1;
  memset(res, 0, sizeof(*res));
  chain_ht h;
  cht_init(&h, num_buckets);
  uint64_t n = min_reps ? min_reps : 1;
  double tb = 0, tp = 0;
  for (uint64_t rep = 0; rep < n; ++rep) {
    memset(&res->out, 0, sizeof(res->out));
    const double t0 = now_ns();
    for (uint64_t i = 0; i < build->n; ++i) { /* AlgScan -> AlgHashJoinBuild::step */
      const uint32_t* t = build->base + i * build->stride;
      cht_insert(&h, t, key_of(build, t));
    }
    const double t1 = now_ns();
    uint64_t cnt = 0, cmps = 0;
    for (uint64_t i = 0; i < probe->n; ++i) { /* AlgScan -> AlgHashJoinProbe::step (algebra.hh:625-659) */
      const uint32_t* t = probe->base + i * probe->stride;
      const uint32_t pk = key_of(probe, t);
      const uint32_t hv = murmur32(pk);
      const cnode* it = &h.dir[hv % h.nb];
      if (it->next == CEMPTY) continue;
      uint64_t c = 0;
      for (; it; it = it->next) {
        ++c;
        if (it->hash == hv && pk == key_of(build, it->data)) {
          ++cnt;
          if (agg) agg2(&res->out, row_of(probe, t), row_of(build, it->data));
          if (unique) break;
        }
      }
      cmps += c;
    }
    const double t2 = now_ns();
    tb += t1 - t0; tp += t2 - t1;
    res->c_probe = cnt; res->c_cmp = cmps;
    if (rep == n - 1 && (tb + tp) < min_ms * 1e6) n *= 2; /* repeat_mintime */
    if (rep != n - 1) cht_clear(&h);
  }
  res->reps = n;
  res->build_ns = tb / (double)n;
  res->probe_ns = tp / (double)n;
  res->c_build = build->n;
  res->c_top = res->c_probe;
  h.size = build->n; /* report entries of one build (the reference inflates this by reps) */
  cht_stats(&h, &res->stats);
  cht_free(&h);
  return 0;
}

/* ------------------------------------------------------------------ */
/* HtNested1: MainNode {next, sub, data, hash} (32 B), SubNode {next, data} */
/* ------------------------------------------------------------------ */
typedef struct snode { struct snode* next; const uint32_t* data; } snode;
typedef struct mnode { struct mnode* next; snode* sub; const uint32_t* data; uint32_t hash; } mnode;
#define MEMPTY ((mnode*)(uintptr_t)1)

typedef struct { mnode* dir; uint64_t nb, size; reservoir mrsv, srsv; const orc_rel* rel; } nest_ht;

static void nht_init(nest_ht* h, uint64_t nb, const orc_rel* rel) {
  h->nb = nb; h->size = 0; h->rel = rel;
  h->dir = (mnode*)malloc(sizeof(mnode) * nb);
  for (uint64_t i = 0; i < nb; ++i) { h->dir[i].next = MEMPTY; h->dir[i].sub = NULL; h->dir[i].data = NULL; h->dir[i].hash = 0; }
  rsv_init(&h->mrsv, sizeof(mnode));
  rsv_init(&h->srsv, sizeof(snode));
}
static void nht_clear(nest_ht* h) { /* ht_nested.hh:438-447 */
  rsv_erase(&h->srsv);
  rsv_erase(&h->mrsv);
  for (uint64_t i = 0; i < h->nb; ++i) h->dir[i].next = MEMPTY;
}
static void nht_free(nest_ht* h) { rsv_erase(&h->srsv); rsv_erase(&h->mrsv); free(h->dir); }

static inline int nht_match(const nest_ht* h, const mnode* m, uint32_t hv, uint32_t key) { /* isMainNodeMatch */
  return m->hash == hv && key == key_of(h->rel, m->data);
}
static inline void nht_at_main(nest_ht* h, mnode* m, const uint32_t* t, uint32_t hv) { /* :386-412 */
  if (m->next == MEMPTY) {
    m->next = NULL; m->sub = NULL; m->data = t; m->hash = hv;
  } else {
    snode* s = (snode*)rsv_new(&h->srsv);
    s->data = t; s->next = m->sub; /* head insert into the sub-chain */
    m->sub = s;
  }
}
static inline void nht_insert(nest_ht* h, const uint32_t* t) { /* ht_nested.hh:287-311 */
  const uint32_t key = key_of(h->rel, t);
  const uint32_t hv = murmur32(key);
  mnode* d = &h->dir[hv % h->nb];
  if (d->next == MEMPTY || nht_match(h, d, hv, key)) {
    nht_at_main(h, d, t, hv);
  } else {
    mnode* it = d; /* findMainNode (:414-436): walk the main chain */
    mnode* found = NULL;
    for (; it->next != NULL; it = it->next) {
      if (nht_match(h, it->next, hv, key)) { found = it->next; break; }
    }
    if (found) {
      nht_at_main(h, found, t, hv);
    } else {
      mnode* m = (mnode*)rsv_new(&h->mrsv); /* tail-append a new main node */
      m->next = MEMPTY;
      it->next = m;
      nht_at_main(h, m, t, hv);
    }
  }
  h->size++;
}
/* findMainNodeByOther (ht_nested.hh:354-382): returns the match (or NULL), counts comparisons. */
static inline const mnode* nht_find(const nest_ht* h, uint32_t pkey, uint64_t* cmps) {
  const uint32_t hv = murmur32(pkey);
  const mnode* m = &h->dir[hv % h->nb];
  uint64_t c = 0;
  do {
    if (m->next == MEMPTY) { *cmps += c; return NULL; }
    ++c;
    if (m->hash == hv && pkey == key_of(h->rel, m->data)) { *cmps += c; return m; }
    m = m->next;
  } while (m);
  *cmps += c;
  return NULL;
}
static void nht_stats(const nest_ht* h, orc_stats* s) { /* ht_nested.hh:450-482 */
  stats_init(s, h->nb);
  s->entries = h->size;
  for (uint64_t b = 0; b < h->nb; ++b) {
    const mnode* d = &h->dir[b];
    if (d->next == MEMPTY) { stats_step(s, 0); continue; }
    uint64_t len = 0;
    for (const mnode* m = d; m; m = m->next) { ++len; s->distinct++; }
    stats_step(s, len);
  }
}

int orc_nested_plan(const orc_rel* build, const orc_rel* probe, uint64_t num_buckets, int unnest, int agg,
                    double min_ms, uint64_t min_reps, orc_plan_res* res) {
  if (!build || !probe || !res || num_buckets == 0) return 1;
  memset(res, 0, sizeof(*res));
  nest_ht h;
  nht_init(&h, num_buckets, build);
  uint64_t n = min_reps ? min_reps : 1;
  double tb = 0, tp = 0;
  for (uint64_t rep = 0; rep < n; ++rep) {
    memset(&res->out, 0, sizeof(res->out));
    const double t0 = now_ns();
    for (uint64_t i = 0; i < build->n; ++i) nht_insert(&h, build->base + i * build->stride);
    const double t1 = now_ns();
    uint64_t cnt = 0, cmps = 0, un = 0;
    for (uint64_t i = 0; i < probe->n; ++i) { /* AlgNestJoinProbe::step (algebra.hh:435-459) */
      const uint32_t* t = probe->base + i * probe->stride;
      const mnode* m = nht_find(&h, key_of(probe, t), &cmps);
      if (!m) continue;
      ++cnt;
      if (unnest) { /* AlgUnnestHt::step (algebra.hh:510-541): main datum, then sub-chain */
        ++un;
        if (agg) agg2(&res->out, row_of(probe, t), row_of(build, m->data));
        for (const snode* s = m->sub; s; s = s->next) {
          ++un;
          if (agg) agg2(&res->out, row_of(probe, t), row_of(build, s->data));
        }
      } else if (agg) {
        agg2(&res->out, row_of(probe, t), row_of(build, m->data));
      }
    }
    const double t2 = now_ns();
    tb += t1 - t0; tp += t2 - t1;
    res->c_probe = cnt; res->c_cmp = cmps; res->c_unnest = unnest ? un : 0;
    res->c_top = unnest ? un : cnt;
    if (rep == n - 1 && (tb + tp) < min_ms * 1e6) n *= 2;
    if (rep != n - 1) nht_clear(&h);
  }
  res->reps = n;
  res->build_ns = tb / (double)n;
  res->probe_ns = tp / (double)n;
  res->c_build = build->n;
  h.size = build->n;
  nht_stats(&h, &res->stats);
  nht_free(&h);
  return 0;
}

/* ------------------------------------------------------------------ */
/* experiment 4: Ndu (two nested probes + deferred unnesting) and Chj    */
/* ------------------------------------------------------------------ */
int orc_exp4_plan(const orc_rel* R, const orc_rel* S, const orc_rel* T, uint64_t num_buckets, int nested, int agg,
                  double min_ms, uint64_t min_reps, orc_exp4_res* res) {
  if (!R || !S || !T || !res || num_buckets == 0) return 1;
  memset(res, 0, sizeof(*res));
  uint64_t n = min_reps ? min_reps : 1;
  double ts = 0, tt = 0, tp = 0;
  if (nested) { /* main_experiment4.cc:831-941 */
    nest_ht hs, ht;
    nht_init(&hs, num_buckets, S);
    nht_init(&ht, num_buckets, T);
    for (uint64_t rep = 0; rep < n; ++rep) {
      memset(&res->out, 0, sizeof(res->out));
      const double t0 = now_ns();
      for (uint64_t i = 0; i < S->n; ++i) nht_insert(&hs, S->base + i * S->stride);
      const double t1 = now_ns();
      for (uint64_t i = 0; i < T->n; ++i) nht_insert(&ht, T->base + i * T->stride);
      const double t2 = now_ns();
      uint64_t prs = 0, crs = 0, prt = 0, crt = 0, u1 = 0, u2 = 0;
      for (uint64_t i = 0; i < R->n; ++i) {
        const uint32_t* r = R->base + i * R->stride;
        const uint32_t k = key_of(R, r);
        const mnode* ms = nht_find(&hs, k, &crs);
        if (!ms) continue;
        ++prs;
        const mnode* mt = nht_find(&ht, k, &crt); /* probe T keyed through the nested tuple's r */
        if (!mt) continue;
        ++prt;
        /* unnest #1 expands T, unnest #2 expands S (deferred until both joins matched) */
        const uint32_t* td = mt->data;
        const snode* tsub = mt->sub;
        for (;;) {
          ++u1;
          const uint32_t* sd = ms->data;
          const snode* ssub = ms->sub;
          for (;;) {
            ++u2;
            if (agg) agg3(&res->out, row_of(R, R->base + i * R->stride), row_of(S, sd), row_of(T, td));
            if (!ssub) break;
            sd = ssub->data; ssub = ssub->next;
          }
          if (!tsub) break;
          td = tsub->data; tsub = tsub->next;
        }
      }
      const double t3 = now_ns();
      ts += t1 - t0; tt += t2 - t1; tp += t3 - t2;
      res->c_probe_rs = prs; res->c_probe_rs_cmp = crs; res->c_probe_rt = prt; res->c_probe_rt_cmp = crt;
      res->c_unnest_1 = u1; res->c_unnest_2 = u2; res->c_top = u2;
      if (rep == n - 1 && (ts + tt + tp) < min_ms * 1e6) n *= 2;
      if (rep != n - 1) { nht_clear(&hs); nht_clear(&ht); }
    }
    nht_free(&hs);
    nht_free(&ht);
  } else { /* main_experiment4.cc:943-1043 */
    chain_ht hs, ht;
    cht_init(&hs, num_buckets);
    cht_init(&ht, num_buckets);
    for (uint64_t rep = 0; rep < n; ++rep) {
      memset(&res->out, 0, sizeof(res->out));
      const double t0 = now_ns();
      for (uint64_t i = 0; i < S->n; ++i) { const uint32_t* t = S->base + i * S->stride; cht_insert(&hs, t, key_of(S, t)); }
      const double t1 = now_ns();
      for (uint64_t i = 0; i < T->n; ++i) { const uint32_t* t = T->base + i * T->stride; cht_insert(&ht, t, key_of(T, t)); }
      const double t2 = now_ns();
      uint64_t prs = 0, crs = 0, prt = 0, crt = 0;
      for (uint64_t i = 0; i < R->n; ++i) {
        const uint32_t* r = R->base + i * R->stride;
        const uint32_t k = key_of(R, r);
        const uint32_t hv = murmur32(k);
        const cnode* a = &hs.dir[hv % hs.nb];
        if (a->next == CEMPTY) continue;
        for (; a; a = a->next) {
          ++crs;
          if (a->hash != hv || k != key_of(S, a->data)) continue;
          ++prs; /* (r, s) pair pushed into the second probe */
          const cnode* b = &ht.dir[hv % ht.nb];
          if (b->next == CEMPTY) continue;
          for (; b; b = b->next) {
            ++crt;
            if (b->hash == hv && k == key_of(T, b->data)) {
              ++prt;
              if (agg) agg3(&res->out, row_of(R, r), row_of(S, a->data), row_of(T, b->data));
            }
          }
        }
      }
      const double t3 = now_ns();
      ts += t1 - t0; tt += t2 - t1; tp += t3 - t2;
      res->c_probe_rs = prs; res->c_probe_rs_cmp = crs; res->c_probe_rt = prt; res->c_probe_rt_cmp = crt;
      res->c_top = prt;
      if (rep == n - 1 && (ts + tt + tp) < min_ms * 1e6) n *= 2;
      if (rep != n - 1) { cht_clear(&hs); cht_clear(&ht); }
    }
    cht_free(&hs);
    cht_free(&ht);
  }
  res->reps = n;
  res->build_s_ns = ts / (double)n;
  res->build_t_ns = tt / (double)n;
  res->probe_ns = tp / (double)n;
  return 0;
}

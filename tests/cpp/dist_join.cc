// A C++ host of the multi-GPU bucket-range partitioned join on the C ABI alone (include/hj3d.h):
// the same hj3d_partition -> hj3d_comm_counts -> hj3d_comm_exchange -> build / chunked probe ->
// hj3d_comm_allreduce_u64 strand bench.py runs through hj3d/dist.py, so the Python and C++ hosts
// share one exchange implementation (libhj3d over RCCL).
//
// One process per GPU: RANK / WORLD_SIZE / LOCAL_RANK from the environment (defaults 0 / 1 / 0);
// rank 0 writes the communicator id to $HJ3D_COMM_ID_FILE, the others wait for it.
// Usage: dist_join <nR> <nS> <Csr|Nsr> [chunks]
// Inputs: the reference's experiment-1 relations (hj3d_gen_exp1_ref, main_experiment1.cc:415-457),
// generated whole by every rank, which keeps its contiguous slice of R and S.
// Rank 0 prints "c_build=.. c_top=.. c_cmp=.. n=.. sum_a=.. sum_b=.. sum_h=.. xor_h=.. nb=.. empty=.."
// with the counters, checksums and statistics merged over the ranks.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "hj3d.h"

#define CHECK(call)                                                                      \
  do {                                                                                   \
    hj3d_status s_ = (call);                                                             \
    if (s_ != HJ3D_OK) {                                                                 \
      std::fprintf(stderr, "%s failed (%d): %s\n", #call, int(s_), hj3d_last_error(ctx)); \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

static int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v ? std::atoi(v) : d;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <nR> <nS> <Csr|Nsr> [chunks]\n", argv[0]);
    return 2;
  }
  const uint64_t nR = std::strtoull(argv[1], nullptr, 10), nS = std::strtoull(argv[2], nullptr, 10);
  const std::string plan = argv[3];
  const uint32_t C = argc > 4 ? uint32_t(std::atoi(argv[4])) : 1;
  const bool unique = plan == "Csr";
  if (!(plan == "Csr" || plan == "Nsr") || C == 0) return 2;
  const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1), local = env_int("LOCAL_RANK", 0);

  hj3d_ctx* ctx = nullptr;
  if (hj3d_ctx_create(local, nullptr, &ctx) != HJ3D_OK) {
    std::fprintf(stderr, "hj3d_ctx_create failed: no GPU (there is no CPU path)\n");
    return 1;
  }
  // communicator id: rank 0 -> file -> other ranks
  uint8_t id[HJ3D_COMM_ID_BYTES];
  const char* idf = std::getenv("HJ3D_COMM_ID_FILE");
  if (rank == 0) {
    CHECK(hj3d_comm_unique_id(ctx, id));
    if (world > 1) {
      if (!idf) return 2;
      const std::string tmp = std::string(idf) + ".tmp";
      std::ofstream(tmp, std::ios::binary).write(reinterpret_cast<const char*>(id), sizeof(id));
      std::rename(tmp.c_str(), idf);
    }
  } else {
    if (!idf) return 2;
    for (int i = 0;; ++i) {
      std::ifstream f(idf, std::ios::binary);
      if (f && f.read(reinterpret_cast<char*>(id), sizeof(id))) break;
      if (i > 6000) return 3;  // 60 s
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
  CHECK(hj3d_comm_init(ctx, id, rank, world));

  // inputs: this rank's slices of the reference's relations, uploaded as {k, a, b} tuples
  std::vector<uint32_t> Rk(nR), Sa(nS ? nS : 1);
  CHECK(hj3d_gen_exp1_ref(nR, nS, 0, 1.0, 0, Rk.data(), Sa.data(), 0));
  const uint64_t r_lo = rank * nR / world, r_hi = (rank + 1) * nR / world;
  const uint64_t s_lo = rank * nS / world, s_hi = (rank + 1) * nS / world;
  const uint64_t nr = r_hi - r_lo, ns = s_hi - s_lo;
  std::vector<uint32_t> Rh(3 * nr, 0), Sh(3 * ns, 0);
  for (uint64_t i = 0; i < nr; ++i) Rh[3 * i] = Rk[r_lo + i];
  for (uint64_t i = 0; i < ns; ++i) {
    Sh[3 * i] = uint32_t(s_lo + i);
    Sh[3 * i + 1] = Sa[s_lo + i];
  }
  void *dR, *dS, *sendB, *recvB, *sendP, *recvP, *cnt, *res;
  CHECK(hj3d_dev_alloc(ctx, 12 * nr + 4, &dR));
  CHECK(hj3d_dev_alloc(ctx, 12 * ns + 4, &dS));
  CHECK(hj3d_upload(ctx, dR, Rh.data(), 12 * nr));
  CHECK(hj3d_upload(ctx, dS, Sh.data(), 12 * ns));
  CHECK(hj3d_dev_alloc(ctx, 8 * nr + 8, &sendB));
  CHECK(hj3d_dev_alloc(ctx, 8 * ns + 8, &sendP));
  CHECK(hj3d_dev_alloc(ctx, 8 * size_t(C + 1) * world, &cnt));
  CHECK(hj3d_dev_alloc(ctx, 8 * 16, &res));

  const uint64_t nb = nR ? nR : 1;  // main_experiment1.cc:651 (b = 1)
  uint64_t lo, hi;
  hj3d_part_range(nb, uint32_t(world), uint32_t(rank), &lo, &hi);
  hj3d_table_desc desc{nb, lo, hi, unique ? uint32_t(HJ3D_CHAIN) : uint32_t(HJ3D_NESTED), 0};
  hj3d_table* t = nullptr;
  CHECK(hj3d_table_create(ctx, &desc, &t));

  // build side: partition, counts, exchange, explicit-row build of the owned bucket range
  std::vector<uint8_t> zero(8 * size_t(C + 1) * world, 0);
  CHECK(hj3d_upload(ctx, cnt, zero.data(), zero.size()));
  hj3d_rel rR{dR, nr, 12, 0, HJ3D_ROW_IMPLICIT, 0, r_lo};
  CHECK(hj3d_partition(ctx, &rR, nb, uint32_t(world), sendB, cnt));
  std::vector<int64_t> sc(size_t(C) * world), rc(size_t(C) * world);
  CHECK(hj3d_comm_counts(ctx, cnt, 1, sc.data(), rc.data()));
  uint64_t nrecvB = 0;
  for (int p = 0; p < world; ++p) nrecvB += uint64_t(rc[p]);
  CHECK(hj3d_dev_alloc(ctx, 8 * nrecvB + 8, &recvB));
  CHECK(hj3d_comm_exchange(ctx, sendB, sc.data(), recvB, rc.data(), nrecvB, 8, nullptr));
  hj3d_rel rB{recvB, nrecvB, 8, 0, 4, 0, 0};
  CHECK(hj3d_build(ctx, t, &rB));

  // probe side in C chunks: partition all, one count collective, exchanges in flight, probe each
  // chunk once its pairs have landed (accumulated into one strand)
  CHECK(hj3d_upload(ctx, cnt, zero.data(), zero.size()));
  std::vector<uint64_t> sb(C + 1);
  for (uint32_t c = 0; c <= C; ++c) sb[c] = ns * c / C;
  for (uint32_t c = 0; c < C; ++c) {
    hj3d_rel rS{static_cast<const char*>(dS) + 12 * sb[c], sb[c + 1] - sb[c], 12, 4, HJ3D_ROW_IMPLICIT, 0,
                s_lo + sb[c]};
    CHECK(hj3d_partition(ctx, &rS, nb, uint32_t(world), static_cast<char*>(sendP) + 8 * sb[c],
                         static_cast<int64_t*>(cnt) + size_t(c) * world));
  }
  CHECK(hj3d_comm_counts(ctx, cnt, C, sc.data(), rc.data()));
  uint64_t nrecvP = 0;
  for (auto v : rc) nrecvP += uint64_t(v);
  CHECK(hj3d_dev_alloc(ctx, 8 * nrecvP + 8, &recvP));
  std::vector<uint32_t> tickets(C);
  std::vector<uint64_t> roff(C + 1, 0);
  for (uint32_t c = 0; c < C; ++c) {
    uint64_t n = 0;
    for (int p = 0; p < world; ++p) n += uint64_t(rc[size_t(c) * world + p]);
    roff[c + 1] = roff[c] + n;
    CHECK(hj3d_comm_exchange(ctx, static_cast<char*>(sendP) + 8 * sb[c], &sc[size_t(c) * world],
                             static_cast<char*>(recvP) + 8 * roff[c], &rc[size_t(c) * world], n, 8, &tickets[c]));
  }
  for (uint32_t c = 0; c < C; ++c) {
    CHECK(hj3d_comm_wait(ctx, tickets[c]));
    hj3d_rel rP{static_cast<char*>(recvP) + 8 * roff[c], roff[c + 1] - roff[c], 8, 0, 4, 0, 0};
    uint32_t flags = (unique ? HJ3D_PROBE_UNIQUE : HJ3D_PROBE_UNNEST) | HJ3D_PROBE_CHECKSUM |
                     (c ? HJ3D_PROBE_ACCUMULATE : 0);
    CHECK(hj3d_probe(ctx, t, &rP, flags, nullptr, 0));
  }
  hj3d_probe_res pr;
  CHECK(hj3d_probe_result(ctx, &pr));
  hj3d_stats st;
  CHECK(hj3d_table_stats(ctx, t, &st));

  // merge over ranks: counters and sums add, xor via all-gather, statistics extremes max / min
  uint64_t add[14] = {nrecvB, pr.n_out, pr.n_cmps, pr.n_out, pr.sum_a, pr.sum_b, pr.sum_h,
                      st.nb, st.empty, st.entries, st.cc0_sum, st.cc0_cnt, st.cc1_sum, st.cc1_cnt};
  CHECK(hj3d_upload(ctx, res, add, sizeof(add)));
  CHECK(hj3d_comm_allreduce_u64(ctx, res, 14, HJ3D_RED_SUM));
  CHECK(hj3d_download(ctx, add, res, sizeof(add)));
  uint64_t mx[2] = {st.cc0_max, st.cc1_max}, mn[2] = {st.cc0_min, st.cc1_cnt ? st.cc1_min : ~0ull};
  CHECK(hj3d_upload(ctx, res, mx, sizeof(mx)));
  CHECK(hj3d_comm_allreduce_u64(ctx, res, 2, HJ3D_RED_MAX));
  CHECK(hj3d_download(ctx, mx, res, sizeof(mx)));
  CHECK(hj3d_upload(ctx, res, mn, sizeof(mn)));
  CHECK(hj3d_comm_allreduce_u64(ctx, res, 2, HJ3D_RED_MIN));
  CHECK(hj3d_download(ctx, mn, res, sizeof(mn)));
  std::vector<uint64_t> xs(world);
  void* xd;
  CHECK(hj3d_dev_alloc(ctx, 8 * size_t(world) + 8, &xd));
  CHECK(hj3d_upload(ctx, res, &pr.xor_h, 8));
  CHECK(hj3d_comm_allgather(ctx, res, xd, 8));
  CHECK(hj3d_download(ctx, xs.data(), xd, 8 * size_t(world)));
  uint64_t x = 0;
  for (auto v : xs) x ^= v;
  if (rank == 0)
    std::printf("c_build=%llu c_top=%llu c_cmp=%llu n=%llu sum_a=%llu sum_b=%llu sum_h=%llu xor_h=%llu nb=%llu "
                "empty=%llu entries=%llu cc0_sum=%llu cc0_cnt=%llu cc1_sum=%llu cc1_cnt=%llu cc0_max=%llu "
                "cc1_max=%llu cc0_min=%llu cc1_min=%llu\n",
                (unsigned long long)add[0], (unsigned long long)add[1], (unsigned long long)add[2],
                (unsigned long long)add[3], (unsigned long long)add[4], (unsigned long long)add[5],
                (unsigned long long)add[6], (unsigned long long)x, (unsigned long long)add[7],
                (unsigned long long)add[8], (unsigned long long)add[9], (unsigned long long)add[10],
                (unsigned long long)add[11], (unsigned long long)add[12], (unsigned long long)add[13],
                (unsigned long long)mx[0], (unsigned long long)mx[1], (unsigned long long)mn[0],
                (unsigned long long)mn[1]);
  hj3d_table_destroy(t);
  for (void* p : {dR, dS, sendB, recvB, sendP, recvP, cnt, res, xd}) hj3d_dev_free(ctx, p);
  hj3d_ctx_destroy(ctx);
  return 0;
}

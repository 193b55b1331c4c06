// comm.hip — the exchange step of the multi-GPU bucket-range partitioned join
// inside libhj3d, over RCCL (xGMI): one communicator per context, grouped point-to-point
// send / recv of the (key, row) pairs hj3d_partition grouped by destination, the per-chunk count
// all-to-all, and the u64 counter all-reduce / all-gather of the result merge. Python
// (hj3d/dist.py) and the C++ drop-in hosts call the same entry points.
//
// RCCL is resolved at run time: a librccl.so.1 already mapped into the process (torch's, whose HIP
// runtime this library then shares) is reused, otherwise the one next to the HIP runtime this
// library was built against is loaded (RUNPATH). Nothing links RCCL at build time, so a
// single-GPU process never maps it.
//
// The reference has no multi-GPU path (the exchange is new; the per-bucket semantics
// stay the reference's because every bucket lives on exactly one GPU).
#include <dlfcn.h>
#include <link.h>
#include <rccl/rccl.h>
#include <sys/stat.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <utility>

#include "hj3d_internal.hpp"

namespace hj3d {
namespace {

// ---- the RCCL entry points this file uses, resolved once ----
struct Rccl {
  void* h = nullptr;
  std::string path, err;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRank) commInitRank = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclAllReduce) allReduce = nullptr;
  decltype(&ncclAllGather) allGather = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  decltype(&ncclGetVersion) getVersion = nullptr;
};

template <typename F> bool sym(void* h, const char* name, F* f) {
  *f = reinterpret_cast<F>(dlsym(h, name));
  return *f != nullptr;
}

Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      r.err = std::string("librccl.so.1 not loadable: ") + (e ? e : "?");
      return;
    }
    bool ok = sym(h, "ncclGetUniqueId", &r.getUniqueId) && sym(h, "ncclCommInitRank", &r.commInitRank) &&
              sym(h, "ncclCommDestroy", &r.commDestroy) && sym(h, "ncclGroupStart", &r.groupStart) &&
              sym(h, "ncclGroupEnd", &r.groupEnd) && sym(h, "ncclSend", &r.send) && sym(h, "ncclRecv", &r.recv) &&
              sym(h, "ncclAllReduce", &r.allReduce) && sym(h, "ncclAllGather", &r.allGather) &&
              sym(h, "ncclGetErrorString", &r.errorString) && sym(h, "ncclGetVersion", &r.getVersion);
    if (!ok) {
      r.err = "librccl.so.1 lacks an entry point libhj3d needs";
      return;
    }
    Dl_info di{};
    if (dladdr(reinterpret_cast<void*>(r.send), &di) && di.dli_fname) r.path = di.dli_fname;
    r.h = h;
  });
  return &r;
}

// distinct files mapped into the process whose name starts with `stem` (e.g. two HIP runtimes:
// torch's torch/lib/libamdhip64.so and /opt/rocm's libamdhip64.so.7 carry the same SONAME)
std::set<std::string> mapped(const char* stem) {
  struct Arg { const char* stem; std::set<std::pair<uint64_t, uint64_t>> ids; std::set<std::string> names; } a{stem, {}, {}};
  dl_iterate_phdr(
      [](dl_phdr_info* info, size_t, void* p) -> int {
        auto* a = static_cast<Arg*>(p);
        const char* name = info->dlpi_name;
        if (!name || !*name) return 0;
        const char* base = std::strrchr(name, '/');
        base = base ? base + 1 : name;
        if (std::strncmp(base, a->stem, std::strlen(a->stem)) != 0) return 0;
        struct stat st{};
        if (stat(name, &st) == 0) {
          if (!a->ids.insert({uint64_t(st.st_dev), uint64_t(st.st_ino)}).second) return 0;
        }
        a->names.insert(name);
        return 0;
      },
      &a);
  return a.names;
}

std::string joined(const std::set<std::string>& s) {
  std::string o;
  for (const auto& x : s) o += (o.empty() ? "" : ", ") + x;
  return o;
}

// counts[c][p] (device, chunks x world) -> blocks[p][c], the block for peer p contiguous
__global__ void k_comm_transpose(const int64_t* __restrict__ in, int64_t* __restrict__ out, uint32_t chunks,
                                 uint32_t world) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= chunks * world) return;
  const uint32_t c = i / world, p = i % world;
  out[size_t(p) * chunks + c] = in[i];
}

}  // namespace

// The HIP runtime check of hj3d_ctx_create: exactly one libamdhip64 mapped, the one whose
// hipMalloc this library calls.
bool runtime_check(std::string* msg) {
  const auto hips = mapped("libamdhip64.so");
  if (hips.size() > 1) {
    *msg = "two HIP runtimes are mapped into this process (" + joined(hips) +
           "): device pointers and streams of one are invalid in the other. Load torch before libhj3d.so "
           "(python: import torch first; hj3d does) or keep one runtime on the library path";
    return false;
  }
  return true;
}

std::string runtime_info() {
  std::string s;
  Dl_info di{};
  hipError_t (*malloc_fn)(void**, size_t) = &hipMalloc;
  if (dladdr(reinterpret_cast<void*>(malloc_fn), &di) && di.dli_fname) s += std::string("hip=") + di.dli_fname;
  int v = 0;
  if (hipRuntimeGetVersion(&v) == hipSuccess) s += " (runtime " + std::to_string(v) + ")";
  const auto hips = mapped("libamdhip64.so");
  s += "; hip mapped=" + std::to_string(hips.size());
  const auto rcs = mapped("librccl.so");
  if (!rcs.empty()) s += "; rccl=" + joined(rcs);
  return s;
}

}  // namespace hj3d

using namespace hj3d;

struct hj3d_comm_state {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  hipStream_t xstream = nullptr;     // exchange stream (asynchronous exchanges)
  hipEvent_t ready = nullptr;        // "the context stream reached this exchange"
  static constexpr uint32_t kTickets = 64;
  hipEvent_t done[kTickets] = {};    // "exchange t has landed", on xstream (slot t % kTickets)
  uint32_t next_ticket = 0;          // tickets count up; slot t % kTickets holds the latest one
  DevBuf counts;                     // transposed send / received counts
};

namespace {

hj3d_status comm_fail(hj3d_ctx* ctx, hj3d_status st, const std::string& what) {
  if (ctx) ctx->last_error = what;
  return st;
}

hj3d_status nccl_ok(hj3d_ctx* ctx, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return HJ3D_OK;
  return comm_fail(ctx, HJ3D_EDEVICE, std::string(what) + ": " + rccl()->errorString(r) + " (" + std::to_string(int(r)) + ")");
}

hj3d_status hip_ok(hj3d_ctx* ctx, hipError_t e, const char* what) {
  if (e == hipSuccess) return HJ3D_OK;
  return comm_fail(ctx, e == hipErrorOutOfMemory ? HJ3D_ENOMEM : HJ3D_EDEVICE,
                   std::string(what) + ": " + hipGetErrorString(e));
}

bool rccl_ready(hj3d_ctx* ctx) {
  Rccl* r = rccl();
  if (!r->h) {
    comm_fail(ctx, HJ3D_EUNSUPPORTED, r->err);
    return false;
  }
  return true;
}

hj3d_comm_state* st(hj3d_ctx* ctx) { return ctx ? ctx->comm : nullptr; }

// grouped send / recv of per-peer blocks (an all-to-all with per-peer sizes); counts in elements
// of elem bytes, displacements = prefix sums of the counts. Blocks move as 8- or 4-byte words
// when their size allows, in pieces of at most kPieceBytes = 2^28 bytes (matched in order per
// peer). A single RCCL message of ~1 GiB and more arrived with its second half corrupted
// (profiles/r03d_rccl_limits.jsonl, r04 sweep), so pieces stay a factor 4 below that, whatever the
// word size.
// send_stride (elements): peer p's elements start at send + p * send_stride (0: back to back)
constexpr size_t kPieceBytes = size_t(1) << 28;
ncclResult_t alltoallv(hj3d_comm_state* c, const char* send, const int64_t* sc, char* recv, const int64_t* rc,
                       size_t elem, hipStream_t s, uint64_t send_stride = 0) {
  Rccl* r = rccl();
#ifdef HJ3D_COMM_DIAG
  // diagnostic builds only (scripts/rccl_limits.sh builds a variant library with -DHJ3D_COMM_DIAG):
  // HJ3D_COMM_WORD=1 forces byte words, HJ3D_COMM_PIECE_LOG2 sets the piece size in BYTES
  static const size_t force_word = [] {
    const char* e = getenv("HJ3D_COMM_WORD");
    return size_t(e && *e ? atoi(e) : 0);
  }();
  static const size_t piece_bytes = [] {
    const char* e = getenv("HJ3D_COMM_PIECE_LOG2");
    const int l = e && *e ? atoi(e) : 28;
    return size_t(1) << (l < 3 ? 3 : l > 40 ? 40 : l);
  }();
#else
  constexpr size_t force_word = 0, piece_bytes = kPieceBytes;
#endif
  const size_t word = force_word == 1 ? 1 : elem % 8 == 0 ? 8 : elem % 4 == 0 ? 4 : 1;
  const size_t kPiece = piece_bytes / word;  // words per piece
  const ncclDataType_t dt = word == 8 ? ncclUint64 : word == 4 ? ncclUint32 : ncclUint8;
  ncclResult_t e = r->groupStart();
  if (e != ncclSuccess) return e;
  size_t so = 0, ro = 0;
  for (int p = 0; p < c->world && e == ncclSuccess; ++p) {
    const size_t ns = size_t(sc[p]) * elem / word, nr = size_t(rc[p]) * elem / word;
    if (send_stride) so = size_t(p) * send_stride * elem;
    for (size_t k = 0; k < ns && e == ncclSuccess; k += kPiece)
      e = r->send(send + so + k * word, ns - k < kPiece ? ns - k : kPiece, dt, p, c->comm, s);
    for (size_t k = 0; k < nr && e == ncclSuccess; k += kPiece)
      e = r->recv(recv + ro + k * word, nr - k < kPiece ? nr - k : kPiece, dt, p, c->comm, s);
    so += ns * word;
    ro += nr * word;
  }
  const ncclResult_t g = r->groupEnd();
  return e != ncclSuccess ? e : g;
}

}  // namespace

extern "C" {

hj3d_status hj3d_runtime_info(char* buf, uint64_t cap) {
  if (!buf || !cap) return HJ3D_EINVAL;
  const std::string s = runtime_info();
  std::snprintf(buf, cap, "%s", s.c_str());
  return s.size() < cap ? HJ3D_OK : HJ3D_EOVERFLOW;
}

hj3d_status hj3d_comm_unique_id(hj3d_ctx* ctx, uint8_t* id) {
  if (!ctx || !id) return HJ3D_EINVAL;
  if (!rccl_ready(ctx)) return HJ3D_EUNSUPPORTED;
  ncclUniqueId u;
  hj3d_status s = nccl_ok(ctx, rccl()->getUniqueId(&u), "ncclGetUniqueId");
  if (s == HJ3D_OK) std::memcpy(id, u.internal, HJ3D_COMM_ID_BYTES);
  return s;
}

hj3d_status hj3d_comm_init(hj3d_ctx* ctx, const uint8_t* id, int rank, int world) {
  if (!ctx || !id || world < 1 || rank < 0 || rank >= world) return HJ3D_EINVAL;
  if (ctx->comm) return comm_fail(ctx, HJ3D_EINVAL, "hj3d_comm_init: the context already has a communicator");
  if (!rccl_ready(ctx)) return HJ3D_EUNSUPPORTED;
  const auto rcs = mapped("librccl.so");
  if (rcs.size() > 1)
    return comm_fail(ctx, HJ3D_EDEVICE, "two RCCL libraries are mapped into this process (" + joined(rcs) + ")");
  std::string msg;
  if (!runtime_check(&msg)) return comm_fail(ctx, HJ3D_EDEVICE, msg);
  hj3d_status s = hip_ok(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  if (s != HJ3D_OK) return s;
  auto* c = new (std::nothrow) hj3d_comm_state();
  if (!c) return HJ3D_ENOMEM;
  c->rank = rank;
  c->world = world;
  ncclUniqueId u;
  std::memcpy(u.internal, id, HJ3D_COMM_ID_BYTES);
  s = nccl_ok(ctx, rccl()->commInitRank(&c->comm, world, u, rank), "ncclCommInitRank");
  if (s == HJ3D_OK) s = hip_ok(ctx, hipStreamCreateWithFlags(&c->xstream, hipStreamNonBlocking), "hipStreamCreate");
  if (s == HJ3D_OK) s = hip_ok(ctx, hipEventCreateWithFlags(&c->ready, hipEventDisableTiming), "hipEventCreate");
  for (uint32_t t = 0; s == HJ3D_OK && t < hj3d_comm_state::kTickets; ++t)
    s = hip_ok(ctx, hipEventCreateWithFlags(&c->done[t], hipEventDisableTiming), "hipEventCreate");
  ctx->comm = c;
  if (s != HJ3D_OK) hj3d_comm_destroy(ctx);
  return s;
}

hj3d_status hj3d_comm_destroy(hj3d_ctx* ctx) {
  if (!ctx) return HJ3D_EINVAL;
  hj3d_comm_state* c = ctx->comm;
  if (!c) return HJ3D_OK;
  (void)hipSetDevice(ctx->device);
  if (c->xstream) (void)hipStreamSynchronize(c->xstream);
  (void)hipStreamSynchronize(ctx->stream);
  if (c->comm) (void)rccl()->commDestroy(c->comm);
  for (auto& e : c->done)
    if (e) (void)hipEventDestroy(e);
  if (c->ready) (void)hipEventDestroy(c->ready);
  if (c->xstream) (void)hipStreamDestroy(c->xstream);
  c->counts.release();
  delete c;
  ctx->comm = nullptr;
  return HJ3D_OK;
}

hj3d_status hj3d_comm_rank(const hj3d_ctx* ctx, int* rank, int* world) {
  if (!ctx || !ctx->comm) return HJ3D_EINVAL;
  if (rank) *rank = ctx->comm->rank;
  if (world) *world = ctx->comm->world;
  return HJ3D_OK;
}

hj3d_status hj3d_comm_counts(hj3d_ctx* ctx, const void* counts_dev, uint32_t chunks, int64_t* send_host,
                             int64_t* recv_host) {
  return hj3d_comm_counts_cap(ctx, counts_dev, chunks, ~0ull, send_host, recv_host);
}

hj3d_status hj3d_comm_counts_cap(hj3d_ctx* ctx, const void* counts_dev, uint32_t chunks, uint64_t recv_cap,
                                 int64_t* send_host, int64_t* recv_host) {
  hj3d_comm_state* c = st(ctx);
  if (!c || !counts_dev || !chunks || !recv_host) return HJ3D_EINVAL;
  const uint32_t P = uint32_t(c->world);
  const size_t n = size_t(chunks) * P;
  hj3d_status s = hip_ok(ctx, c->counts.ensure(2 * n * sizeof(int64_t)), "comm counts buffer");
  if (s != HJ3D_OK) return s;
  int64_t* tx = c->counts.as<int64_t>();
  int64_t* rx = tx + n;
  hipLaunchKernelGGL(k_comm_transpose, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, ctx->stream,
                     static_cast<const int64_t*>(counts_dev), tx, chunks, P);
  if ((s = hip_ok(ctx, hipGetLastError(), "k_comm_transpose")) != HJ3D_OK) return s;
  std::vector<int64_t> per(P, int64_t(chunks) * int64_t(sizeof(int64_t)));
  ncclResult_t e = alltoallv(c, reinterpret_cast<const char*>(tx), per.data(), reinterpret_cast<char*>(rx),
                             per.data(), 1, ctx->stream);
  if ((s = nccl_ok(ctx, e, "count all-to-all")) != HJ3D_OK) return s;
  std::vector<int64_t> h(2 * n);
  s = hip_ok(ctx, hipMemcpyAsync(h.data(), tx, 2 * n * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream),
             "count download");
  if (s == HJ3D_OK) s = hip_ok(ctx, hipStreamSynchronize(ctx->stream), "count download");
  if (s != HJ3D_OK) return s;
  uint64_t total = 0;
  for (uint32_t p = 0; p < P; ++p)
    for (uint32_t k = 0; k < chunks; ++k) {  // back to [chunk][peer]
      if (send_host) send_host[size_t(k) * P + p] = h[size_t(p) * chunks + k];
      recv_host[size_t(k) * P + p] = h[n + size_t(p) * chunks + k];
      total += uint64_t(h[n + size_t(p) * chunks + k]);
    }
  if (recv_cap == ~0ull) return HJ3D_OK;
  // every rank learns whether ANY rank's receive buffer is short, so all refuse together before
  // the first pair collective (a one-sided refusal would leave the peers waiting in it)
  int64_t* flag = tx;  // the transposed counts are downloaded already
  const int64_t mine = total > recv_cap ? 1 : 0;
  s = hip_ok(ctx, hipMemcpyAsync(flag, &mine, sizeof(mine), hipMemcpyHostToDevice, ctx->stream), "overflow flag");
  if (s != HJ3D_OK) return s;
  if ((s = nccl_ok(ctx, rccl()->allReduce(flag, flag, 1, ncclInt64, ncclMax, c->comm, ctx->stream),
                   "overflow flag all-reduce")) != HJ3D_OK)
    return s;
  int64_t any = 0;
  s = hip_ok(ctx, hipMemcpyAsync(&any, flag, sizeof(any), hipMemcpyDeviceToHost, ctx->stream), "overflow flag");
  if (s == HJ3D_OK) s = hip_ok(ctx, hipStreamSynchronize(ctx->stream), "overflow flag");
  if (s != HJ3D_OK) return s;
  if (any)
    return comm_fail(ctx, HJ3D_EOVERFLOW,
                     mine ? "hj3d_comm_counts_cap: " + std::to_string(total) + " elements arrive at this rank, its "
                                "receive buffer holds " + std::to_string(recv_cap)
                          : std::string("hj3d_comm_counts_cap: another rank's receive buffer is short"));
  return HJ3D_OK;
}

hj3d_status hj3d_comm_exchange(hj3d_ctx* ctx, const void* send_dev, const int64_t* send_counts, void* recv_dev,
                               const int64_t* recv_counts, uint64_t recv_cap, uint32_t elem_bytes,
                               uint32_t* ticket) {
  return hj3d_comm_exchange_strided(ctx, send_dev, 0, send_counts, recv_dev, recv_counts, recv_cap, elem_bytes, ticket);
}

hj3d_status hj3d_comm_exchange_strided(hj3d_ctx* ctx, const void* send_dev, uint64_t send_stride,
                                       const int64_t* send_counts, void* recv_dev, const int64_t* recv_counts,
                                       uint64_t recv_cap, uint32_t elem_bytes, uint32_t* ticket) {
  hj3d_comm_state* c = st(ctx);
  if (!c || !send_counts || !recv_counts || !elem_bytes) return HJ3D_EINVAL;
  uint64_t ns = 0, nr = 0;
  for (int p = 0; p < c->world; ++p) {
    // a count above the stride means hj3d_partition_strided spilled (a bounded stride, skewed
    // keys): the caller must check every count against the stride and re-partition BEFORE any rank
    // calls this (hj3d.h). Refused here only on this rank, so a caller that skipped the check
    // leaves its peers waiting in the collective.
    if (send_counts[p] < 0 || recv_counts[p] < 0 || (send_stride && uint64_t(send_counts[p]) > send_stride))
      return HJ3D_EINVAL;
    ns += uint64_t(send_counts[p]);
    nr += uint64_t(recv_counts[p]);
  }
  if ((ns && !send_dev) || (nr && !recv_dev)) return HJ3D_EINVAL;
  if (nr > recv_cap)
    return comm_fail(ctx, HJ3D_EOVERFLOW, "hj3d_comm_exchange: " + std::to_string(nr) + " elements arrive, the "
                                              "receive buffer holds " + std::to_string(recv_cap) +
                                              " (size it from hj3d_comm_counts before any rank exchanges)");
  hipStream_t s = ctx->stream;
  hj3d_status r;
  if (ticket) {  // on the exchange stream, after everything enqueued so far on the context stream
    if ((r = hip_ok(ctx, hipEventRecord(c->ready, ctx->stream), "hipEventRecord")) != HJ3D_OK) return r;
    if ((r = hip_ok(ctx, hipStreamWaitEvent(c->xstream, c->ready, 0), "hipStreamWaitEvent")) != HJ3D_OK) return r;
    s = c->xstream;
  }
  r = nccl_ok(ctx,
              alltoallv(c, static_cast<const char*>(send_dev), send_counts, static_cast<char*>(recv_dev), recv_counts,
                        elem_bytes, s, send_stride),
              "pair exchange");
  if (r != HJ3D_OK || !ticket) return r;
  const uint32_t t = c->next_ticket++;
  if ((r = hip_ok(ctx, hipEventRecord(c->done[t % hj3d_comm_state::kTickets], s), "hipEventRecord")) != HJ3D_OK)
    return r;
  *ticket = t;
  return HJ3D_OK;
}

hj3d_status hj3d_comm_wait(hj3d_ctx* ctx, uint32_t ticket) {
  hj3d_comm_state* c = st(ctx);
  // a ticket never issued is refused; an older one whose slot a later exchange took waits for that
  // later exchange instead: the exchanges run in issue order on the exchange stream, so the event
  // in the slot is recorded after the ticket's own exchange (waits on it are never too early)
  if (!c || ticket >= c->next_ticket) return HJ3D_EINVAL;
  return hip_ok(ctx, hipStreamWaitEvent(ctx->stream, c->done[ticket % hj3d_comm_state::kTickets], 0),
                "hipStreamWaitEvent");
}

hj3d_status hj3d_comm_allreduce_u64(hj3d_ctx* ctx, void* buf_dev, uint64_t n, int op) {
  hj3d_comm_state* c = st(ctx);
  if (!c || (n && !buf_dev)) return HJ3D_EINVAL;
  ncclRedOp_t o;
  switch (op) {
    case HJ3D_RED_SUM: o = ncclSum; break;
    case HJ3D_RED_MAX: o = ncclMax; break;
    case HJ3D_RED_MIN: o = ncclMin; break;
    default: return HJ3D_EINVAL;
  }
  if (!n) return HJ3D_OK;
  return nccl_ok(ctx, rccl()->allReduce(buf_dev, buf_dev, n, ncclUint64, o, c->comm, ctx->stream), "ncclAllReduce");
}

hj3d_status hj3d_comm_allgather(hj3d_ctx* ctx, const void* send_dev, void* recv_dev, uint64_t bytes) {
  hj3d_comm_state* c = st(ctx);
  if (!c || (bytes && (!send_dev || !recv_dev))) return HJ3D_EINVAL;
  if (!bytes) return HJ3D_OK;
  return nccl_ok(ctx, rccl()->allGather(send_dev, recv_dev, bytes, ncclUint8, c->comm, ctx->stream), "ncclAllGather");
}

}  // extern "C"

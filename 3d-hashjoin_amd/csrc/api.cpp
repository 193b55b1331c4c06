// api.cpp — the extern "C" surface of libhj3d.so (declared in include/hj3d.h).
//
// Argument checking, context / table lifetime, device result slots and HIP-event phase
// timers live here; the kernels are in the .hip translation units. Every entry point
// returns an hj3d_status and never throws.
#include <cmath>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <new>

#include "hj3d_internal.hpp"

#include <atomic>
#include <chrono>
#include <sched.h>

namespace hj3d {
static std::atomic<uint64_t> g_launches{0};
void note_launch() { g_launches.fetch_add(1, std::memory_order_relaxed); }
uint64_t launch_total() { return g_launches.load(std::memory_order_relaxed); }
}  // namespace hj3d

using namespace hj3d;

namespace {

hj3d_status fail(hj3d_ctx* ctx, hj3d_status st, const char* what, hipError_t e = hipSuccess) {
  if (ctx) {
    char buf[512];
    if (e != hipSuccess)
      std::snprintf(buf, sizeof(buf), "%s: %s (%d)", what, hipGetErrorString(e), int(e));
    else
      std::snprintf(buf, sizeof(buf), "%s", what);
    ctx->last_error = buf;
  }
  return st;
}

hj3d_status from_hip(hj3d_ctx* ctx, hipError_t e, const char* what) {
  if (e == hipSuccess) return HJ3D_OK;
  if (e == hipErrorOutOfMemory) return fail(ctx, HJ3D_ENOMEM, what, e);
  if (e == hipErrorNotSupported) return fail(ctx, HJ3D_EUNSUPPORTED, what, e);
  if (e == hipErrorInvalidValue) return fail(ctx, HJ3D_EINVAL, what, e);
  return fail(ctx, HJ3D_EDEVICE, what, e);
}

bool rel_ok(const hj3d_rel* r) {
  if (!r) return false;
  if (r->n && !r->base) return false;
  if (r->stride == 0 || (r->stride & 3) || (r->key_off & 3) || r->key_off + 4 > r->stride) return false;
  if (r->row_off != HJ3D_ROW_IMPLICIT && ((r->row_off & 3) || r->row_off + 4 > r->stride)) return false;
  if (r->row_off == HJ3D_ROW_IMPLICIT && r->n && r->row_base + r->n - 1 > 0xFFFFFFFFull) return false;
  return true;
}

// (kResFields: hj3d_device.hpp)
// result-slot words beyond the counters: n_out before the current probe call, and a sticky flag
// set when a call's non-dense output exceeded its own buffer (accumulated strands included)
constexpr int kResOutMark = 14, kResOvf = 15;

__global__ void k_out_overflow(uint64_t* res, uint64_t cap) {
  if (threadIdx.x == 0 && res[2] - res[kResOutMark] > cap) res[kResOvf] = 1;
}

bool dense_output(const hj3d_table* t, uint32_t flags) {
  return (t->desc.kind == HJ3D_CHAIN) ? (flags & HJ3D_PROBE_UNIQUE) != 0 : !(flags & HJ3D_PROBE_UNNEST);
}

// Non-dense EMIT probes (chains without early exit, unnest) write as many pairs as they find; the
// kernels drop pairs past out_cap. Mark n_out before the call and compare after it, on the stream.
hipError_t out_mark(hj3d_ctx* ctx, const hj3d_table* t, uint32_t flags) {
  if (!(flags & HJ3D_PROBE_EMIT) || dense_output(t, flags)) return hipSuccess;
  // a fresh strand's result slot was just zeroed: its mark (word 14) equals n_out (word 2) = 0
  if (!(flags & HJ3D_PROBE_ACCUMULATE)) return hipSuccess;
  uint64_t* res = ctx->res.as<uint64_t>();
  return hipMemcpyAsync(res + kResOutMark, res + 2, sizeof(uint64_t), hipMemcpyDeviceToDevice, ctx->stream);
}

hipError_t out_check(hj3d_ctx* ctx, const hj3d_table* t, uint32_t flags, uint64_t out_cap) {
  if (!(flags & HJ3D_PROBE_EMIT) || dense_output(t, flags)) return hipSuccess;
  hipLaunchKernelGGL(k_out_overflow, dim3(1), dim3(64), 0, ctx->stream, ctx->res.as<uint64_t>(), out_cap);
  return hipGetLastError();
}

// The fused build partition's grid barrier (radix.hip k_rp_fused) sets word 1 of ctx->gbar when a
// barrier did not complete in time (its workgroups then went on, so the build is not valid). Result
// reads copy the word with the result slot and report it.
hipError_t gbar_copy(hj3d_ctx* ctx, uint64_t* word) {
  *word = 0;
  return ctx->gbar.p ? hipMemcpyAsync(word, ctx->gbar.as<uint64_t>() + 1, sizeof(uint64_t), hipMemcpyDeviceToHost,
                                      ctx->stream)
                     : hipSuccess;
}
hj3d_status gbar_check(hj3d_ctx* ctx, uint64_t word) {
  if (!word) return HJ3D_OK;
  (void)hipMemsetAsync(ctx->gbar.as<uint64_t>() + 1, 0, sizeof(uint64_t), ctx->stream);
  return fail(ctx, HJ3D_EDEVICE, "fused build partition: a grid barrier timed out, a build since the last result is invalid");
}
// The same for one table, in every getter that hands out its content: a chaining table built by the
// fused partition carries its launch tag (gbar_tag), and a timed-out barrier wrote that tag into the
// table's counts word 3 (synchronous; tables of other builds skip the read).
hj3d_status table_gbar_check(hj3d_ctx* ctx, const hj3d_table* t) {
  if (!t->gbar_tag) return HJ3D_OK;
  uint64_t w = 0;
  hipError_t e = hipMemcpyAsync(&w, t->counts.as<const uint64_t>() + 3, sizeof(w), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return from_hip(ctx, e, "fused build partition flag");
  if (w != t->gbar_tag) return HJ3D_OK;
  return fail(ctx, HJ3D_EDEVICE, "fused build partition: a grid barrier timed out, the table is invalid (rebuild it)");
}

}  // namespace

extern "C" {

uint64_t hj3d_mix64(uint64_t z) { return mix64(z); }

hj3d_status hj3d_ctx_create(int device, void* stream, hj3d_ctx** out) {
  if (!out) return HJ3D_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return HJ3D_EDEVICE;
  if (hipSetDevice(device) != hipSuccess) return HJ3D_EDEVICE;
  std::string why;
  if (!runtime_check(&why)) {
    std::fprintf(stderr, "hj3d_ctx_create: %s\n", why.c_str());
    return HJ3D_EDEVICE;
  }
  hj3d_ctx* ctx = new (std::nothrow) hj3d_ctx();
  if (!ctx) return HJ3D_ENOMEM;
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->num_cus = prop.multiProcessorCount;
  ctx->stream = static_cast<hipStream_t>(stream);  // NULL: the null stream
  ctx->own_stream = false;
  if (ctx->res.ensure(kResFields * sizeof(uint64_t)) != hipSuccess) {
    delete ctx;
    return HJ3D_ENOMEM;
  }
  *out = ctx;
  return HJ3D_OK;
}

void hj3d_ctx_destroy(hj3d_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hj3d_comm_destroy(ctx);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& b : ctx->scratch) b.release();
  ctx->res.release();
  ctx->misc.release();
  ctx->ctl.release();
  ctx->scan_status.release();
  ctx->part_cur.release();
  ctx->gbar.release();
  for (auto ev : ctx->event_pool) (void)hipEventDestroy(ev);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

hj3d_status hj3d_ctx_set_stream(hj3d_ctx* ctx, void* stream) {
  if (!ctx) return HJ3D_EINVAL;
  if (ctx->own_stream) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
    ctx->own_stream = false;
  }
  ctx->stream = static_cast<hipStream_t>(stream);
  return HJ3D_OK;
}

void* hj3d_ctx_stream(const hj3d_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

hj3d_status hj3d_ctx_sync(hj3d_ctx* ctx) {
  if (!ctx) return HJ3D_EINVAL;
  return from_hip(ctx, hipStreamSynchronize(ctx->stream), "hj3d_ctx_sync");
}

const char* hj3d_last_error(const hj3d_ctx* ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

hj3d_status hj3d_ctx_set_option(hj3d_ctx* ctx, int option, int64_t value) {
  if (!ctx) return HJ3D_EINVAL;
  switch (option) {
    case HJ3D_OPT_FORCE_DIRECT: ctx->force_direct = value != 0; return HJ3D_OK;
    case HJ3D_OPT_RADIX_MIN: ctx->radix_min = value < 0 ? 0 : uint64_t(value); return HJ3D_OK;
    case HJ3D_OPT_NESTED_SORT: ctx->nested_sort = value != 0; return HJ3D_OK;
    case HJ3D_OPT_SEL_UNFUSED: ctx->sel_unfused = value != 0; return HJ3D_OK;
    case HJ3D_OPT_PACKED_PROBE: ctx->pk_off = value == 0; return HJ3D_OK;
    case HJ3D_OPT_PROBE_ITEMS:
      if (value != 0 && (value < 5 || value > 8)) return fail(ctx, HJ3D_EINVAL, "HJ3D_OPT_PROBE_ITEMS: 0 or 5..8");
      ctx->pk_items = int(value);
      return HJ3D_OK;
    case HJ3D_OPT_PK_SLICE:
      if (value < 0 || value == 1 || value > 0xFFFFFFFFll) return fail(ctx, HJ3D_EINVAL, "HJ3D_OPT_PK_SLICE: 0 or >= 2");
      ctx->pk_slice_max = uint32_t(value);
      return HJ3D_OK;
    case HJ3D_OPT_PK_BUILD: ctx->pk_build = value != 0; return HJ3D_OK;
    case HJ3D_OPT_NESTED_PK: ctx->nested_pk = value != 0; return HJ3D_OK;
    case HJ3D_OPT_SYNC_BUILD: ctx->sync_build = value != 0; return HJ3D_OK;
    case HJ3D_OPT_RP_UNFUSED: ctx->rp_unfused = value != 0; return HJ3D_OK;
    case HJ3D_OPT_DIAG_GBAR:
      if (value < 0) return fail(ctx, HJ3D_EINVAL, "HJ3D_OPT_DIAG_GBAR: >= 0");
      ctx->diag_gbar = uint64_t(value);
      return HJ3D_OK;
    case HJ3D_OPT_DIAG_LOOKBACK:
      if (value < 0 || value > 0xFFFFFFFFll) return fail(ctx, HJ3D_EINVAL, "HJ3D_OPT_DIAG_LOOKBACK: 0 .. 2^32-1");
      ctx->diag_lb = uint64_t(value);
      return HJ3D_OK;
    case HJ3D_OPT_PK_STAGE:
      if (value < 0 || value > 0xFFFFFFFFll) return fail(ctx, HJ3D_EINVAL, "HJ3D_OPT_PK_STAGE: >= 0");
      ctx->pk_stage = uint32_t(value);
      return HJ3D_OK;
    default: return fail(ctx, HJ3D_EINVAL, "hj3d_ctx_set_option: unknown option");
  }
}

hj3d_status hj3d_ctx_timing(hj3d_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 2) return HJ3D_EINVAL;
  ctx->timing = mode;
  return HJ3D_OK;
}

hj3d_status hj3d_ctx_timer(hj3d_ctx* ctx, int phase, double* ms_total, uint64_t* count) {
  if (!ctx || phase < 0 || phase >= HJ3D_T_NTIMERS) return HJ3D_EINVAL;
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return from_hip(ctx, e, "hj3d_ctx_timer");
  double sum = 0;
  for (const auto& sp : ctx->spans[phase]) {
    float ms = 0;
    if ((e = hipEventElapsedTime(&ms, sp.a, sp.b)) != hipSuccess) return from_hip(ctx, e, "hipEventElapsedTime");
    sum += ms;
  }
  if (ms_total) *ms_total = sum;
  if (count) *count = ctx->spans[phase].size();
  return HJ3D_OK;
}

hj3d_status hj3d_tevent_create(hj3d_ctx* ctx, void** ev) {
  if (!ctx || !ev) return HJ3D_EINVAL;
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreateWithFlags(&e, HJ3D_TIMER_EVENT_FLAGS);
  *ev = r == hipSuccess ? e : nullptr;
  return from_hip(ctx, r, "hj3d_tevent_create");
}

hj3d_status hj3d_tevent_record(hj3d_ctx* ctx, void* ev) {
  if (!ctx || !ev) return HJ3D_EINVAL;
  return from_hip(ctx, hipEventRecord(static_cast<hipEvent_t>(ev), ctx->stream), "hj3d_tevent_record");
}

hj3d_status hj3d_tevent_elapsed(void* a, void* b, float* ms) {
  if (!a || !b || !ms) return HJ3D_EINVAL;
  if (hipEventSynchronize(static_cast<hipEvent_t>(b)) != hipSuccess) return HJ3D_EDEVICE;
  return hipEventElapsedTime(ms, static_cast<hipEvent_t>(a), static_cast<hipEvent_t>(b)) == hipSuccess ? HJ3D_OK
                                                                                                      : HJ3D_EDEVICE;
}

void hj3d_tevent_destroy(void* ev) {
  if (ev) (void)hipEventDestroy(static_cast<hipEvent_t>(ev));
}

hj3d_status hj3d_ctx_timer_reset(hj3d_ctx* ctx) {
  if (!ctx) return HJ3D_EINVAL;
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& v : ctx->spans) v.clear();
  ctx->pool_used = 0;
  return HJ3D_OK;
}

hj3d_status hj3d_dev_alloc(hj3d_ctx* ctx, uint64_t bytes, void** dev) {
  if (!ctx || !dev) return HJ3D_EINVAL;
  *dev = nullptr;
  return from_hip(ctx, hipMalloc(dev, bytes ? bytes : 1), "hj3d_dev_alloc");
}

hj3d_status hj3d_dev_free(hj3d_ctx* ctx, void* dev) {
  if (!ctx) return HJ3D_EINVAL;
  if (!dev) return HJ3D_OK;
  (void)hipStreamSynchronize(ctx->stream);
  return from_hip(ctx, hipFree(dev), "hj3d_dev_free");
}

hj3d_status hj3d_upload(hj3d_ctx* ctx, void* dev, const void* host, uint64_t bytes) {
  if (!ctx || (bytes && (!dev || !host))) return HJ3D_EINVAL;
  if (!bytes) return HJ3D_OK;
  hipError_t e = hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  return from_hip(ctx, e, "hj3d_upload");
}

hj3d_status hj3d_download(hj3d_ctx* ctx, void* host, const void* dev, uint64_t bytes) {
  if (!ctx || (bytes && (!dev || !host))) return HJ3D_EINVAL;
  if (!bytes) return HJ3D_OK;
  hipError_t e = hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  return from_hip(ctx, e, "hj3d_download");
}

hj3d_status hj3d_table_create(hj3d_ctx* ctx, const hj3d_table_desc* desc, hj3d_table** out) {
  if (!ctx || !desc || !out) return HJ3D_EINVAL;
  *out = nullptr;
  if (desc->kind != HJ3D_CHAIN && desc->kind != HJ3D_NESTED) return fail(ctx, HJ3D_EINVAL, "unknown table kind");
  if (desc->num_buckets == 0 || desc->num_buckets >= (1ull << 32))
    return fail(ctx, HJ3D_EINVAL, "num_buckets must be in [1, 2^32)");
  if (desc->bucket_lo > desc->bucket_hi || desc->bucket_hi > desc->num_buckets)
    return fail(ctx, HJ3D_EINVAL, "bucket range outside [0, num_buckets]");
  hj3d_table* t = new (std::nothrow) hj3d_table();
  if (!t) return HJ3D_ENOMEM;
  t->desc = *desc;
  t->nb_local = uint32_t(desc->bucket_hi - desc->bucket_lo);
  t->fm = FastMod::make(uint32_t(desc->num_buckets));
  (void)hipSetDevice(ctx->device);
  hipError_t e = t->off.ensure((uint64_t(t->nb_local) + 1) * sizeof(uint32_t));
  if (e == hipSuccess) e = t->counts.ensure(4 * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMemsetAsync(t->off.p, 0, (uint64_t(t->nb_local) + 1) * sizeof(uint32_t), ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(t->counts.p, 0, 4 * sizeof(uint64_t), ctx->stream);
  if (e != hipSuccess) {
    hj3d_table_destroy(t);
    return from_hip(ctx, e, "hj3d_table_create");
  }
  *out = t;
  return HJ3D_OK;
}

void hj3d_table_destroy(hj3d_table* t) {
  if (!t) return;
  if (t->hc_ev) {
    (void)hipEventSynchronize(t->hc_ev);  // the counts copy into t->hc has landed
    (void)hipEventDestroy(t->hc_ev);
  }
  if (t->hc) (void)hipHostFree(t->hc);
  t->off.release();
  t->ent.release();
  t->main.release();
  t->sub.release();
  t->counts.release();
  delete t;
}

hj3d_status hj3d_table_reserve(hj3d_ctx* ctx, hj3d_table* t, uint64_t max_build) {
  if (!ctx || !t) return HJ3D_EINVAL;
  const uint64_t n = max_build ? max_build : 1;
  hipError_t e = hipSuccess;
  if (t->desc.kind == HJ3D_CHAIN) {
    e = t->ent.ensure(n * sizeof(uint2));
    if (e == hipSuccess) e = ctx->scratch[kScrSlot].ensure(n * sizeof(uint32_t));
  } else {
    e = t->main.ensure(n * sizeof(uint4));
    if (e == hipSuccess) e = t->sub.ensure(n * sizeof(uint32_t));
    if (e == hipSuccess) e = ctx->scratch[kScrSortK].ensure(3 * n * sizeof(uint32_t));
    if (e == hipSuccess) e = ctx->scratch[kScrB].ensure((5 * n + 2) * sizeof(uint32_t));
  }
  return from_hip(ctx, e, "hj3d_table_reserve");
}

hj3d_status hj3d_table_clear(hj3d_ctx* ctx, hj3d_table* t) {
  if (!ctx || !t) return HJ3D_EINVAL;
  t->pending = false;
  t->gbar_tag = 0;
  hipError_t e = hipMemsetAsync(t->off.p, 0, (uint64_t(t->nb_local) + 1) * sizeof(uint32_t), ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(t->counts.p, 0, 4 * sizeof(uint64_t), ctx->stream);
  t->n_build = 0;
  t->n_mains = 0;
  return from_hip(ctx, e, "hj3d_table_clear");
}

// The partitioned probe sizes its LDS slices by the number of main records: a nested build's counts
// (word 1 = main records; word 3 = the aggregation build's give-up flag) travel to pinned host
// memory behind the build and are read at the table's next use (table_resolve), so consecutive
// builds (experiment 4's two tables) do not wait for each other.
// The aggregation builds write the host copy from their last kernel (k_nagg_mains), so their pinned
// mirror must exist before the build (nested_host_counts); the other nested builds copy it.
static hipError_t nested_host_counts(hj3d_table* t) {
  hipError_t e = hipSuccess;
  if (!t->hc) {
    e = hipHostMalloc(reinterpret_cast<void**>(&t->hc), 4 * sizeof(uint64_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->hc_ev, hipEventDisableTiming);
  }
  return e;
}
static hipError_t nested_pending(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel& build, bool agg) {
  hipError_t e = nested_host_counts(t);
  // (agg: k_nagg_mains wrote the mirror)
  if (e == hipSuccess && !agg)
    e = hipMemcpyAsync(t->hc, t->counts.p, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipEventRecord(t->hc_ev, ctx->stream);
  t->pending = e == hipSuccess;
  t->pending_agg = agg;
  t->pending_rel = build;
  t->pending_ctx = ctx;
  t->n_mains = 0;
  return e;
}

hj3d_status hj3d_build_many(hj3d_ctx* ctx, hj3d_table* const* tables, const hj3d_rel* builds, uint32_t count) {
  if (!ctx || (count && (!tables || !builds))) return HJ3D_EINVAL;
  for (uint32_t k = 0; k < count; ++k) {
    if (!tables[k]) return HJ3D_EINVAL;
    if (!rel_ok(&builds[k])) return fail(ctx, HJ3D_EINVAL, "hj3d_build_many: invalid relation");
    for (uint32_t j = 0; j < k; ++j)
      if (tables[j] == tables[k]) return fail(ctx, HJ3D_EINVAL, "hj3d_build_many: a table given twice");
  }
  // two nested tables of one geometry: one launch sequence (the aggregation build over both)
  if (count == 2 && tables[0]->desc.kind == HJ3D_NESTED && tables[1]->desc.kind == HJ3D_NESTED &&
      !ctx->nested_sort && !ctx->nested_pk) {
    hipError_t e;
    const char* path = "nested_agg";
    {
      PhaseTimer tm(ctx, HJ3D_T_BUILD);
      for (uint32_t k = 0; k < 2; ++k) tables[k]->pending = false;
      e = nested_host_counts(tables[0]);
      if (e == hipSuccess) e = nested_host_counts(tables[1]);
      if (e == hipSuccess) e = nested_build_agg_many(ctx, tables, builds, 2, ctx->stream, &path);
    }
    if (e == hipErrorOutOfMemory) {
      (void)hipGetLastError();
      e = hipErrorNotSupported;
    }
    if (e != hipErrorNotSupported) {
      for (uint32_t k = 0; k < 2 && e == hipSuccess; ++k) {
        tables[k]->path = path;
        e = nested_pending(ctx, tables[k], builds[k], true);
      }
      for (uint32_t k = 0; k < 2; ++k) tables[k]->built = e == hipSuccess;
      for (uint32_t k = 0; k < 2 && e == hipSuccess && ctx->sync_build; ++k) e = table_resolve(ctx, tables[k]);
      return from_hip(ctx, e, "hj3d_build_many");
    }
  }
  for (uint32_t k = 0; k < count; ++k) {
    const hj3d_status st = hj3d_build(ctx, tables[k], &builds[k]);
    if (st != HJ3D_OK) return st;
  }
  return HJ3D_OK;
}

}  // extern "C"

static hipError_t build_one(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel* build) {
  PhaseTimer tm(ctx, HJ3D_T_BUILD);
  hipError_t e;
  t->pending = false;  // a build in flight for the old content is replaced (its copy stays stream-ordered)
  t->gbar_tag = 0;     // (set again by a fused build partition)
  if (t->desc.kind == HJ3D_CHAIN) {
    bool sorted = false;
    t->path = "radix";
    e = (!ctx->force_direct && !ctx->pk_build && build->n >= (ctx->radix_min >> 4) && build->n > 0 &&
         t->nb_local >= 64)
            ? radix_build(ctx, t, *build, ctx->stream, &sorted)
            : hipErrorNotSupported;
    if (e == hipErrorNotSupported && build->n >= (ctx->radix_min >> 4)) {
      t->path = "slices";
      e = pk_build(ctx, t, *build, ctx->stream);  // tables beyond the radix build's 2048 x 16384 buckets
      if (e == hipErrorOutOfMemory) {  // its region scratch did not fit: the direct build needs far less
        (void)hipGetLastError();
        e = hipErrorNotSupported;
      }
      sorted = e == hipSuccess;
    }
    if (e == hipErrorNotSupported) {
      t->path = "direct";
      e = chain_build(ctx, t, *build, ctx->stream);
    }
    if (e == hipSuccess && !sorted) e = sort_small_buckets(ctx, t, ctx->stream);
  } else {
    e = hipErrorNotSupported;
    bool agg = false;
    if (!ctx->nested_sort) {
      e = nested_host_counts(t);
      if (e == hipSuccess) e = nested_build_agg(ctx, t, *build, ctx->stream, &t->path);
      if (e == hipErrorOutOfMemory) {  // partition / slice scratch did not fit: the sort build
        (void)hipGetLastError();
        e = hipErrorNotSupported;
      }
      agg = e == hipSuccess;
    }
    if (e == hipErrorNotSupported) {
      t->path = "nested_sort";
      e = nested_build(ctx, t, *build, ctx->stream);
    }
    if (e == hipSuccess) e = nested_pending(ctx, t, *build, agg);
  }
  t->built = e == hipSuccess;
  return e;
}

extern "C" {

hj3d_status hj3d_build(hj3d_ctx* ctx, hj3d_table* t, const hj3d_rel* build) {
  if (!ctx || !t) return HJ3D_EINVAL;
  if (!rel_ok(build)) return fail(ctx, HJ3D_EINVAL, "hj3d_build: invalid relation");
  if (build->n >= (1ull << 32)) return fail(ctx, HJ3D_EUNSUPPORTED, "hj3d_build: more than 2^32-1 build tuples");
  hipError_t e = build_one(ctx, t, build);
  // HJ3D_OPT_SYNC_BUILD: finished here (its own timer interval if the sort build has to run)
  if (e == hipSuccess && ctx->sync_build) e = table_resolve(ctx, t);
  return from_hip(ctx, e, "hj3d_build");
}

}  // extern "C"

namespace hj3d {
hipError_t table_resolve(hj3d_ctx* ctx, hj3d_table* t) {
  if (!t->pending) return hipSuccess;
  t->pending = false;
  // polled, not waited for: the build is short (config E: ~0.3 ms) and the probe's launches follow
  // as soon as it lands (a blocking wait's wake-up left the GPU idle for ~20 us)
  // A short build lands within the spin; past 50 us the loop yields its core to other host threads
  // (an RCCL proxy, other ranks), and past 20 ms it blocks.
  hipError_t e;
  const auto t0 = std::chrono::steady_clock::now();
  while ((e = hipEventQuery(t->hc_ev)) == hipErrorNotReady) {
    const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    if (us > 20000) {
      e = hipEventSynchronize(t->hc_ev);
      break;
    }
    if (us > 50) sched_yield();
  }
  if (e != hipSuccess) {
    t->built = false;
    return e;
  }
  uint64_t hc[4];
  std::memcpy(hc, t->hc, sizeof(hc));
  if (t->pending_agg && uint32_t(hc[3]) != 0) {  // a key range too dense for the LDS table
    // the rest of the build: timed as build work (not inside the probe that triggered it)
    PhaseTimer tm(ctx, HJ3D_T_BUILD);
    t->path = "nested_sort";
    e = nested_build(ctx, t, t->pending_rel, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(hc, t->counts.p, sizeof(hc), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  }
  t->n_mains = e == hipSuccess ? hc[1] : 0;
  t->built = e == hipSuccess;
  return e;
}
}  // namespace hj3d

static hipError_t resolve(hj3d_ctx* ctx, const hj3d_table* t) {
  return table_resolve(ctx, const_cast<hj3d_table*>(t));
}

extern "C" {

const char* hj3d_table_build_path(const hj3d_table* t) {
  if (!t || !t->built) return "none";
  if (!t->pending) return t->path;
  // not resolved yet: the started path, marked (no wait, no build from a read-only getter)
  hj3d_table* w = const_cast<hj3d_table*>(t);
  std::snprintf(w->path_buf, sizeof(w->path_buf), "%s?", t->path);
  return w->path_buf;
}

uint64_t hj3d_launch_count(void) { return hj3d::launch_total(); }

hj3d_status hj3d_table_finish(hj3d_ctx* ctx, hj3d_table* t) {
  if (!ctx || !t) return HJ3D_EINVAL;
  if (const hj3d_status gs = table_gbar_check(ctx, t); gs != HJ3D_OK) return gs;
  return from_hip(ctx, table_resolve(ctx, t), "hj3d_table_finish");
}

hj3d_status hj3d_table_export(hj3d_ctx* ctx, const hj3d_table* t, uint32_t* off, void* payload, uint32_t* sub,
                              uint64_t* n_payload, uint64_t* n_sub) {
  if (!ctx || !t || !n_payload || !n_sub) return HJ3D_EINVAL;
  const uint64_t nbl = t->nb_local;
  uint32_t last = 0;  // off[nb_local] = the payload count
  if (const hj3d_status gs = table_gbar_check(ctx, t); gs != HJ3D_OK) return gs;
  hipError_t e = resolve(ctx, t);
  if (e != hipSuccess) return from_hip(ctx, e, "hj3d_table_export");
  e = hipMemcpyAsync(&last, t->off.as<uint32_t>() + nbl, sizeof(last), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return from_hip(ctx, e, "hj3d_table_export");
  const bool nested = t->desc.kind == HJ3D_NESTED;
  *n_payload = t->built ? last : 0;
  *n_sub = nested && t->built ? t->n_build : 0;
  if (!off && !payload && !sub) return HJ3D_OK;
  if (!off || (*n_payload && !payload) || (*n_sub && !sub)) return fail(ctx, HJ3D_EINVAL, "hj3d_table_export: null array");
  e = hipMemcpyAsync(off, t->off.p, (nbl + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess && *n_payload)
    e = hipMemcpyAsync(payload, nested ? t->main.p : t->ent.p, *n_payload * (nested ? 16 : 8), hipMemcpyDeviceToHost,
                       ctx->stream);
  if (e == hipSuccess && *n_sub) e = hipMemcpyAsync(sub, t->sub.p, *n_sub * 4, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  return from_hip(ctx, e, "hj3d_table_export");
}

hj3d_status hj3d_table_stats(hj3d_ctx* ctx, const hj3d_table* t, hj3d_stats* out) {
  if (!ctx || !t || !out) return HJ3D_EINVAL;
  std::memset(out, 0, sizeof(*out));
  if (const hj3d_status gs = table_gbar_check(ctx, t); gs != HJ3D_OK) return gs;
  hipError_t e = resolve(ctx, t);
  if (e == hipSuccess) e = table_stats(ctx, t, out, ctx->stream);
  return from_hip(ctx, e, "hj3d_table_stats");
}

hj3d_status hj3d_table_size(hj3d_ctx* ctx, const hj3d_table* t, uint64_t* n_entries, uint64_t* n_distinct) {
  if (!ctx || !t) return HJ3D_EINVAL;
  hj3d_stats st;
  const hj3d_status s = hj3d_table_stats(ctx, t, &st);
  if (s != HJ3D_OK) return s;
  if (n_entries) *n_entries = st.entries;
  if (n_distinct) *n_distinct = st.distinct;
  return HJ3D_OK;
}

// remember what an overflow check needs (hj3d_probe_result)
static void note_probe(hj3d_ctx* ctx, const hj3d_table* t, uint64_t n, uint32_t flags, uint64_t out_cap) {
  const bool acc = flags & HJ3D_PROBE_ACCUMULATE;
  ctx->res_flags = flags;
  ctx->res_dense = dense_output(t, flags);
  ctx->res_cap = (flags & HJ3D_PROBE_EMIT) ? out_cap : ~0ull;
  ctx->res_nprobe = acc ? ctx->res_nprobe + n : n;
  // dense output: each call needs one slot per probe tuple of its own buffer
  const bool ovf_dense = ctx->res_dense && (flags & HJ3D_PROBE_EMIT) && n > out_cap;
  ctx->res_overflow = (acc && ctx->res_overflow) || ovf_dense;
  ctx->res_accumulated = acc;
}

static bool sel_ok(const hj3d_rel* rel, const hj3d_sel_pred* preds, uint32_t npred) {
  if (npred > HJ3D_SEL_MAX || (npred && !preds)) return false;
  for (uint32_t k = 0; k < npred; ++k)
    if ((preds[k].word_off & 3) || preds[k].word_off + 4 > rel->stride || preds[k].op > HJ3D_SEL_RANGE) return false;
  return true;
}

hj3d_status hj3d_probe(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel* probe, uint32_t flags, void* out_dev,
                       uint64_t out_cap) {
  if (!ctx || !t) return HJ3D_EINVAL;
  if (!rel_ok(probe)) return fail(ctx, HJ3D_EINVAL, "hj3d_probe: invalid relation");
  if ((flags & HJ3D_PROBE_EMIT) && !out_dev && out_cap) return fail(ctx, HJ3D_EINVAL, "hj3d_probe: EMIT without buffer");
  if ((flags & HJ3D_PROBE_UNNEST) && t->desc.kind != HJ3D_NESTED)
    return fail(ctx, HJ3D_EINVAL, "hj3d_probe: UNNEST needs a nested table");
  if (hipError_t re = resolve(ctx, t); re != hipSuccess) return from_hip(ctx, re, "hj3d_probe");
  PhaseTimer tm(ctx, HJ3D_T_PROBE);
  uint64_t* res = ctx->res.as<uint64_t>();
  const bool acc = flags & HJ3D_PROBE_ACCUMULATE;
  if (pk_probe_applicable(ctx, t, probe->n, flags)) {  // the packed unique probe sets res itself
    hipError_t e = pk_probe(ctx, t, *probe, flags, out_dev, out_cap, res, ctx->stream);
    if (e != hipErrorNotSupported) {
      note_probe(ctx, t, probe->n, flags, out_cap);
      return from_hip(ctx, e, "hj3d_probe");
    }
  }
  // the partitioned nested probe zeroes a fresh strand's result slot in the launch that clears its
  // partitioner's counters (no runtime fill); the other paths with a fill here
  const bool nested_radix = t->desc.kind == HJ3D_NESTED && radix_nested_applicable(ctx, t, probe->n);
  ZeroList zres;
  zres.add(res, kResFields);
  hipError_t e = acc || nested_radix ? hipSuccess : hipMemsetAsync(res, 0, kResFields * sizeof(uint64_t), ctx->stream);
  if (e == hipSuccess) e = out_mark(ctx, t, flags);
  if (e == hipSuccess) {
    e = hipErrorNotSupported;
    if (t->desc.kind == HJ3D_CHAIN && radix_probe_applicable(ctx, t, probe->n))
      e = radix_probe(ctx, t, *probe, flags, out_dev, out_cap, res, ctx->stream);  // times its own kernels
    else if (nested_radix)
      e = radix_nested_probe(ctx, t, *probe, flags, out_dev, out_cap, res, ctx->stream, nullptr, acc ? nullptr : &zres);
    if (e == hipErrorNotSupported && nested_radix && !acc) {  // (nothing was launched: the slot is still to clear)
      const hipError_t z = hipMemsetAsync(res, 0, kResFields * sizeof(uint64_t), ctx->stream);
      if (z != hipSuccess) e = z;
    }
    if (e == hipErrorNotSupported) {
      PhaseTimer tk(ctx, HJ3D_T_PROBE_KERNEL);
      e = (t->desc.kind == HJ3D_CHAIN) ? chain_probe(ctx, t, *probe, flags, out_dev, out_cap, res, ctx->stream)
                                       : nested_probe(ctx, t, *probe, flags, out_dev, out_cap, res, ctx->stream);
    }
  }
  if (e == hipSuccess) e = out_check(ctx, t, flags, out_cap);
  note_probe(ctx, t, probe->n, flags, out_cap);
  return from_hip(ctx, e, "hj3d_probe");
}

hj3d_status hj3d_probe_sel(hj3d_ctx* ctx, const hj3d_table* t, const hj3d_rel* probe, const hj3d_sel_pred* preds,
                           uint32_t npred, uint32_t flags, void* out_dev, uint64_t out_cap) {
  if (!ctx || !t) return HJ3D_EINVAL;
  if (npred == 0) return hj3d_probe(ctx, t, probe, flags, out_dev, out_cap);
  if (!rel_ok(probe)) return fail(ctx, HJ3D_EINVAL, "hj3d_probe_sel: invalid relation");
  if (!sel_ok(probe, preds, npred)) return fail(ctx, HJ3D_EINVAL, "hj3d_probe_sel: invalid predicate");
  if ((flags & HJ3D_PROBE_EMIT) && !out_dev && out_cap) return fail(ctx, HJ3D_EINVAL, "hj3d_probe_sel: EMIT without buffer");
  if ((flags & HJ3D_PROBE_UNNEST) && t->desc.kind != HJ3D_NESTED)
    return fail(ctx, HJ3D_EINVAL, "hj3d_probe_sel: UNNEST needs a nested table");
  if (hipError_t re = resolve(ctx, t); re != hipSuccess) return from_hip(ctx, re, "hj3d_probe_sel");
  const bool chain_radix = t->desc.kind == HJ3D_CHAIN && radix_probe_applicable(ctx, t, probe->n);
  const bool nested_radix = t->desc.kind == HJ3D_NESTED && radix_nested_applicable(ctx, t, probe->n);
  if (!ctx->sel_unfused && pk_probe_applicable(ctx, t, probe->n, flags)) {
    PhaseTimer tm(ctx, HJ3D_T_PROBE);
    const SelArgs a = sel_args(preds, npred);
    hipError_t e = pk_probe(ctx, t, *probe, flags, out_dev, out_cap, ctx->res.as<uint64_t>(), ctx->stream, &a);
    if (e != hipErrorNotSupported) {
      note_probe(ctx, t, probe->n, flags, out_cap);
      return from_hip(ctx, e, "hj3d_probe_sel");
    }
  }
  if (!(flags & HJ3D_PROBE_ACCUMULATE) && !ctx->sel_unfused && (chain_radix || nested_radix)) {
    // the selection fused into the probe-side partitioner
    PhaseTimer tm(ctx, HJ3D_T_PROBE);
    uint64_t* res = ctx->res.as<uint64_t>();
    hipError_t e = hipMemsetAsync(res, 0, kResFields * sizeof(uint64_t), ctx->stream);
    const SelArgs a = sel_args(preds, npred);
    if (e == hipSuccess)
      e = chain_radix ? radix_probe(ctx, t, *probe, flags, out_dev, out_cap, res, ctx->stream, &a)
                      : radix_nested_probe(ctx, t, *probe, flags, out_dev, out_cap, res, ctx->stream, &a);
    if (e == hipSuccess) e = out_check(ctx, t, flags, out_cap);
    if (e != hipErrorNotSupported) {
      note_probe(ctx, t, probe->n, flags, out_cap);
      return from_hip(ctx, e, "hj3d_probe_sel");
    }
  }
  // select first (stable (key, row) pairs), then probe the passing tuples
  hipError_t e = ctx->sel.ensure(probe->n * sizeof(uint2) + 16);
  if (e != hipSuccess) return from_hip(ctx, e, "hj3d_probe_sel");
  uint64_t* cnt = reinterpret_cast<uint64_t*>(ctx->sel.as<char>() + probe->n * sizeof(uint2) + 8);
  e = select_pairs(ctx, *probe, preds, npred, ctx->sel.p, cnt, ctx->stream);
  uint64_t n_sel = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&n_sel, cnt, sizeof(n_sel), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return from_hip(ctx, e, "hj3d_probe_sel");
  const hj3d_rel pairs{ctx->sel.p, n_sel, 8, 0, 4, 0, 0};
  return hj3d_probe(ctx, t, &pairs, flags, out_dev, out_cap);
}

hj3d_status hj3d_probe_result(hj3d_ctx* ctx, hj3d_probe_res* out) {
  if (!ctx || !out) return HJ3D_EINVAL;
  uint64_t h[kResFields], gw = 0;
  hipError_t e = hipMemcpyAsync(h, ctx->res.p, sizeof(h), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = gbar_copy(ctx, &gw);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return from_hip(ctx, e, "hj3d_probe_result");
  if (const hj3d_status gs = gbar_check(ctx, gw); gs != HJ3D_OK) return gs;
  out->n_probe = h[0];
  out->n_matched = h[1];
  out->n_out = h[2];
  out->n_cmps = h[3];
  out->sum_a = h[4];
  out->sum_b = h[5];
  out->sum_c = h[6];
  out->sum_h = h[7];
  out->xor_h = h[8];
  const bool ovf = ctx->res_dense ? ctx->res_overflow : h[kResOvf] != 0;
  if ((ctx->res_flags & HJ3D_PROBE_EMIT) && ovf) return fail(ctx, HJ3D_EOVERFLOW, "hj3d_probe: output buffer too small");
  return HJ3D_OK;
}

hj3d_status hj3d_probe2(hj3d_ctx* ctx, const hj3d_table* ts, const hj3d_table* tt, const hj3d_rel* probe,
                        uint32_t flags, void* out_dev, uint64_t out_cap) {
  if (!ctx || !ts || !tt) return HJ3D_EINVAL;
  if (!rel_ok(probe)) return fail(ctx, HJ3D_EINVAL, "hj3d_probe2: invalid relation");
  if (ts->desc.kind != tt->desc.kind) return fail(ctx, HJ3D_EINVAL, "hj3d_probe2: both tables must be of one kind");
  if (flags & HJ3D_PROBE_EMIT) return fail(ctx, HJ3D_EUNSUPPORTED, "hj3d_probe2: triple materialisation not implemented");
  if (hipError_t re = resolve(ctx, ts); re != hipSuccess) return from_hip(ctx, re, "hj3d_probe2");
  if (hipError_t re = resolve(ctx, tt); re != hipSuccess) return from_hip(ctx, re, "hj3d_probe2");
  PhaseTimer tm(ctx, HJ3D_T_PROBE);
  uint64_t* res = ctx->res.as<uint64_t>();
  hipError_t e;
  {
    PhaseTimer tk(ctx, HJ3D_T_PROBE_KERNEL);
    e = probe2(ctx, ts, tt, *probe, flags, out_dev, out_cap, res, ctx->stream);  // (clears res itself)
  }
  return from_hip(ctx, e, "hj3d_probe2");
}

hj3d_status hj3d_probe2_result(hj3d_ctx* ctx, hj3d_probe2_res* out) {
  if (!ctx || !out) return HJ3D_EINVAL;
  uint64_t h[kResFields], gw = 0;
  hipError_t e = hipMemcpyAsync(h, ctx->res.p, sizeof(h), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = gbar_copy(ctx, &gw);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return from_hip(ctx, e, "hj3d_probe2_result");
  if (const hj3d_status gs = gbar_check(ctx, gw); gs != HJ3D_OK) return gs;
  static_assert(sizeof(hj3d_probe2_res) == 12 * sizeof(uint64_t), "probe2 result layout");
  std::memcpy(out, h, sizeof(hj3d_probe2_res));
  return HJ3D_OK;
}

hj3d_status hj3d_probe_geometry(hj3d_ctx* ctx, uint64_t nb_local, uint64_t n_build, uint32_t out[5]) {
  if (!ctx || !out || nb_local == 0 || nb_local >= (1ull << 32)) return HJ3D_EINVAL;
  const PkPlan pl = pk_plan(ctx, uint32_t(nb_local), n_build);
  out[0] = pl.W;
  out[1] = pl.P;
  out[2] = pl.C;
  out[3] = pl.W1;
  out[4] = pl.P1;
  return HJ3D_OK;
}

void hj3d_part_range(uint64_t nb, uint32_t parts, uint32_t part, uint64_t* lo, uint64_t* hi) {
  // owner(b) = b * parts / nb  =>  part p owns b in [ceil(p*nb/parts), ceil((p+1)*nb/parts))
  const auto first = [&](uint64_t p) -> uint64_t {
    const unsigned __int128 x = (unsigned __int128)p * nb;
    return uint64_t((x + parts - 1) / parts);
  };
  if (lo) *lo = parts ? first(part) : 0;
  if (hi) *hi = parts ? first(uint64_t(part) + 1) : nb;
}

uint64_t hj3d_partition_stride(uint64_t n, uint32_t parts) {
  // Each tuple's destination is a bucket range of equal width: its count is ~ Binomial(n, 1/parts)
  // for distinct keys. Repeated keys (config D's S.a: ~10 rows per key) widen that by the spread of
  // the keys over the ranges: at 1e9 tuples into 8 ranges a destination held ~280 K more than 8
  // sigma of the binomial (profiles/r04c_ab_xpart.log). Area = mean + max(8 sigma, mean / 64) + 2
  // tiles of slack (the tile claims), capped at n; a spill is still reported by the counts.
  if (parts <= 1) return n;
  const double m = double(n) / parts, sd = std::sqrt(m * (1.0 - 1.0 / parts));
  const double slack = 8.0 * sd > m / 64.0 ? 8.0 * sd : m / 64.0;
  const uint64_t s = uint64_t(std::ceil(m + slack)) + 16384;
  return s < n ? s : n;
}

hj3d_status hj3d_partition(hj3d_ctx* ctx, const hj3d_rel* rel, uint64_t nb, uint32_t parts, void* out_pairs,
                           void* counts) {
  if (!ctx || !rel_ok(rel) || !counts || (rel->n && !out_pairs)) return HJ3D_EINVAL;
  PhaseTimer tm(ctx, HJ3D_T_PARTITION);
  return from_hip(ctx, partition(ctx, *rel, nb, parts, out_pairs, counts, ctx->stream), "hj3d_partition");
}

hj3d_status hj3d_partition_sel(hj3d_ctx* ctx, const hj3d_rel* rel, const hj3d_sel_pred* preds, uint32_t npred,
                               uint64_t nb, uint32_t parts, void* out_pairs, void* counts) {
  if (!ctx || !rel_ok(rel) || !counts || (rel->n && !out_pairs)) return HJ3D_EINVAL;
  if (!sel_ok(rel, preds, npred)) return fail(ctx, HJ3D_EINVAL, "hj3d_partition_sel: invalid predicate");
  PhaseTimer tm(ctx, HJ3D_T_PARTITION);
  const SelArgs a = sel_args(preds, npred);
  return from_hip(ctx, partition(ctx, *rel, nb, parts, out_pairs, counts, ctx->stream, &a), "hj3d_partition_sel");
}

hj3d_status hj3d_partition_strided(hj3d_ctx* ctx, const hj3d_rel* rel, const hj3d_sel_pred* preds, uint32_t npred,
                                   uint64_t nb, uint32_t parts, void* out_pairs, uint64_t stride, void* counts) {
  if (!ctx || !rel_ok(rel) || !counts || (rel->n && !out_pairs)) return HJ3D_EINVAL;
  if (stride == 0 && rel->n) return fail(ctx, HJ3D_EINVAL, "hj3d_partition_strided: stride 0");
  if (parts == 0 || parts > 256) return fail(ctx, HJ3D_EINVAL, "hj3d_partition_strided: nparts outside [1, 256]");
  if (npred && !sel_ok(rel, preds, npred)) return fail(ctx, HJ3D_EINVAL, "hj3d_partition_strided: invalid predicate");
  PhaseTimer tm(ctx, HJ3D_T_PARTITION);
  const SelArgs a = npred ? sel_args(preds, npred) : SelArgs{};
  return from_hip(ctx, partition_strided(ctx, *rel, nb, parts, out_pairs, stride, counts, ctx->stream, &a),
                  "hj3d_partition_strided");
}

hj3d_status hj3d_key_bitmap(hj3d_ctx* ctx, const hj3d_rel* rel, uint64_t domain, void* bitmap, void* outside) {
  if (!ctx || !rel_ok(rel) || domain == 0 || domain > (1ull << 32) || !bitmap) return HJ3D_EINVAL;
  return from_hip(ctx, key_bitmap(ctx, *rel, domain, bitmap, outside, ctx->stream), "hj3d_key_bitmap");
}

hj3d_status hj3d_bitmap_or_popcount(hj3d_ctx* ctx, const void* bitmaps, uint32_t rows, uint64_t words, void* count) {
  if (!ctx || !count || (words && rows && !bitmaps)) return HJ3D_EINVAL;
  return from_hip(ctx, bitmap_or_popcount(ctx, bitmaps, rows, words, count, ctx->stream), "hj3d_bitmap_or_popcount");
}

hj3d_status hj3d_select(hj3d_ctx* ctx, const hj3d_rel* rel, const hj3d_sel_pred* preds, uint32_t npred, void* out,
                        void* count) {
  if (!ctx) return HJ3D_EINVAL;
  if (!rel_ok(rel) || !count || (rel->n && !out)) return fail(ctx, HJ3D_EINVAL, "hj3d_select: invalid argument");
  if (!sel_ok(rel, preds, npred)) return fail(ctx, HJ3D_EINVAL, "hj3d_select: invalid predicate");
  if (rel->n >= (1ull << 32)) return fail(ctx, HJ3D_EUNSUPPORTED, "hj3d_select: more than 2^32-1 tuples");
  return from_hip(ctx, select_pairs(ctx, *rel, preds, npred, out, count, ctx->stream), "hj3d_select");
}

hj3d_status hj3d_gen_keys(hj3d_ctx* ctx, void* tuples, uint64_t n, uint32_t stride, uint32_t key_off,
                          uint64_t row_base, uint64_t n_keys, uint64_t seed) {
  if (!ctx || (n && !tuples) || stride == 0 || (stride & 3) || (key_off & 3) || key_off + 4 > stride)
    return HJ3D_EINVAL;
  return from_hip(ctx, gen_keys(tuples, n, stride, key_off, row_base, n_keys, seed, ctx->stream), "hj3d_gen_keys");
}

hj3d_status hj3d_gen_fk(hj3d_ctx* ctx, void* tuples, uint64_t n, uint32_t stride, uint32_t key_off,
                        uint64_t row_base, uint32_t fk_max, uint64_t seed) {
  if (!ctx || (n && !tuples) || stride == 0 || (stride & 3) || (key_off & 3) || key_off + 4 > stride || fk_max == 0)
    return HJ3D_EINVAL;
  return from_hip(ctx, gen_fk(tuples, n, stride, key_off, row_base, fk_max, seed, ctx->stream), "hj3d_gen_fk");
}

hj3d_status hj3d_gen_zipf(hj3d_ctx* ctx, void* tuples, uint64_t n, uint32_t stride, uint32_t key_off,
                          uint64_t row_base, uint32_t fk_max, double theta, uint64_t seed) {
  if (!ctx || (n && !tuples) || stride == 0 || (stride & 3) || (key_off & 3) || key_off + 4 > stride || fk_max == 0 ||
      !(theta > 0.0) || theta > 10.0)
    return HJ3D_EINVAL;
  return from_hip(ctx, gen_zipf(tuples, n, stride, key_off, row_base, fk_max, theta, seed, ctx->stream),
                  "hj3d_gen_zipf");
}

hj3d_status hj3d_expected_fk_join(hj3d_ctx* ctx, const hj3d_rel* build, const hj3d_rel* probe, uint64_t n_keys,
                                  int swap, void* res_dev) {
  if (!ctx || !rel_ok(build) || !rel_ok(probe) || !res_dev) return HJ3D_EINVAL;
  return from_hip(ctx, expected_fk_join(ctx, *build, *probe, n_keys, swap != 0, res_dev, ctx->stream),
                  "hj3d_expected_fk_join");
}

hj3d_status hj3d_expected_fk_join_gen(hj3d_ctx* ctx, const hj3d_rel* probe, uint64_t n_keys, uint64_t key_seed,
                                      int swap, void* res_dev) {
  if (!ctx || !rel_ok(probe) || !res_dev || n_keys == 0) return HJ3D_EINVAL;
  return from_hip(ctx, expected_fk_join_gen(ctx, *probe, n_keys, key_seed, swap != 0, res_dev, ctx->stream),
                  "hj3d_expected_fk_join_gen");
}

}  // extern "C"

// api.hip — libtsdbhip.so: the C-ABI declared in include/tsdbhip.h and the
// host orchestration of the gfx950 kernels. One unity translation unit.
//
// Pipeline of tsdbhip_spangroup_run (all on the ctx stream):
//   k_assemble        Span.addRow / RowSeq.addRow rules, S7 keep rule, E caps
//   scans             kept-span list, E offsets                     [sync 1]
//   k_decode_*        RowSeq decode (+ greedy downsampling) -> E_s   (HBM-bound)
//   k_span_summary    grid range, F*
//   k_grid_*          union grid G as bitmap + ranks                 [sync 2]
//   k_reduce          per (tile, span chunk) lerp/rate + aggregation
//   k_finalize_*      chunk combine, int/double select, NaN check   [sync 3]
// With TSDBHIP_SHARDED the grid bitmap and the per-t partials are exchanged
// over RCCL (allgather, then a rank-ordered combine on every rank).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tsdbhip.h"
#include "dev_common.h"
#include "k_assemble.hip"
#include "k_decode.hip"
#include "k_grid.hip"
#include "k_reduce.hip"
#include "k_util.hip"
#include "k_decode_fast.hip"
#include "k_ds_chunks.hip"
#include "k_ds_reg.hip"
#include "k_compact.hip"
#include "k_direct.hip"
#include "k_lockstep.hip"
#include "k_group.hip"

using namespace tsdb;

namespace {

struct Buf {
  void* p = nullptr;
  size_t n = 0;
};

struct Fail {
  int code;
};

}  // namespace

// Path / diagnostic options of a context (tsdbhip_set_option): which kernel
// variant takes a span or a row. Results never depend on them; the tests set
// them to run every variant. No environment variable is read.
enum { DEC_AUTO = 0, DEC_GENERAL, DEC_FAST, DEC_CHUNKS, DEC_SPANS, DEC_DIRECT };
struct Options {
  int decode = DEC_AUTO;       // "decode": the decode / downsample path forced
  bool aligned_group = true;   // "aligned_group": k_ds_reg's aligned-group reduction may be tried
  int lockstep = 1;            // "lockstep": "off" (0), "on" (1: groups big enough), "always" (2)
  bool timing_detail = false;  // "timing_detail": decode / grid event pairs (tsdbhip_timing)
  bool check_clean = false;    // "check_clean": verify the zero-on-entry invariants (stderr)
  int events = 0;              // "events": timing events on kernel launches (0), marker packets (1), none (2)
};

// Per-call resources. A call takes a free slot of its context (or a new
// one), so calls from several host threads on one context run concurrently,
// each on its own stream with its own scratch (the reference's Netty workers
// and gnuplot pool call SpanGroup concurrently, GraphHandler.java:182,285).
struct Xchg;
// The mapped output block's header: the call-state snapshot (Small), the
// call's end stamp in its last word (small_snap / check_stamp)
constexpr size_t OUT_HDR = 1024;

struct Slot {
  int device = 0;
  hipStream_t stream = nullptr;
  std::map<std::string, Buf> bufs;  // grow-only named scratch (HBM)
  void* host_small = nullptr;       // pinned readback area
  // mapped pinned host memory the kernels write directly: the call state at
  // the two sizing round trips (host_publish + a spin on the flag instead of
  // a copy and a stream sync), and the results with their header
  uint64_t* map_state = nullptr;  // [0, 511]: state words, [512]: flag
  uint64_t* map_state_dev = nullptr;
  uint64_t pub_seq = 0;
  uint32_t timing_late = 0;  // this call's end stamp arrived after the stream sync (check_stamp)
  uint8_t* map_out = nullptr;
  uint8_t* map_out_dev = nullptr;
  size_t map_out_n = 0;
  void* host_big = nullptr;         // grow-only pinned staging (group-by batches)
  size_t host_big_n = 0;
  hipEvent_t ev[10] = {};  // [8],[9] bracket the dominant kernel
  int8_t ev_alias[10] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1};  // "kernel" events: a start no kernel carried reads as this one (-1: none)
  bool time_reduce = false;  // the dominant kernel is k_reduce (direct path)
  uint32_t hot_kernel = 0;
  tsdbhip_timing timing = {};
  Xchg* x = nullptr;  // the exchange of a sharded call (its rank / nranks)
  Options opt;        // the context's options, copied at the lease
  bool want_output = true;  // false: a non-zero rank of an in-process sharded call
  // a rerun of the same call (spangroup_run): the host-resident inputs are
  // already in HBM (stage() copies nothing); h2d_bytes: this call's copies
  bool reuse_inputs = false;
  uint64_t h2d_bytes = 0;
  // left by the previous spangroup_run that completed: its call state reset
  // to the initial values, its grid bitmap all zero (k_call_end)
  bool sm_ready = false, bitmap_clean = false;
  bool bitmapx_clean = false;  // the same for "gbitmap_x" (sharded calls whose grids differ)
  bool tgdone_clean = false;   // the same for k_reduce's tile-group counters ("tg_done")
  std::map<std::string, Buf> zeroed;  // scratch_zero_kept: allocation last zeroed whole (not owned)
};

struct Multi;
struct tsdbhip_ctx {
  int device = 0;
  std::mutex mu;                   // slot pool, owned buffers, last timing
  std::vector<Slot*> slots, free_slots;
  std::map<std::string, Buf> owned;  // tsdbhip_synth_generate datasets
  tsdbhip_timing last = {};
  tsdbhip_timing sum = {};  // tsdbhip_timing_totals
  Options opt;              // tsdbhip_set_option
  uint64_t n_sum = 0;
  // one process per GPU (tsdbhip_comm_init): sharded calls serialise on the
  // communicator (every rank must issue its collectives in the same order)
  std::mutex comm_mu;
  ncclComm_t comm = nullptr;
  Xchg* rccl = nullptr;
  // one process, several GPUs / shards (tsdbhip_open_devices): member
  // contexts, one per rank
  Multi* multi = nullptr;
};

static thread_local std::string g_thread_err;
static thread_local const tsdbhip_ctx* g_last_ctx = nullptr;  // this thread's last call
static thread_local tsdbhip_timing g_last_timing = {};

static void set_error(const void*, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_thread_err = buf;
}

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      set_error(ctx, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, \
                __LINE__);                                                         \
      throw Fail{TSDBHIP_E_HIP};                                                   \
    }                                                                              \
  } while (0)

#define NCCLCHK(x)                                                              \
  do {                                                                          \
    ncclResult_t r_ = (x);                                                      \
    if (r_ != ncclSuccess) {                                                    \
      set_error(ctx, "%s failed: %s (%s:%d)", #x, ncclGetErrorString(r_),       \
                __FILE__, __LINE__);                                            \
      throw Fail{TSDBHIP_E_RCCL};                                               \
    }                                                                           \
  } while (0)

// grow-only named scratch
template <typename T>
static T* scratch(Slot* ctx, const char* name, size_t count, bool zero = false) {
  size_t bytes = std::max<size_t>(count * sizeof(T), 16) + 64;
  Buf& b = ctx->bufs[name];
  if (b.n < bytes) {
    if (b.p) HIPCHK(hipFree(b.p));
    b.p = nullptr;
    size_t alloc = std::max(bytes, b.n + b.n / 4);
    HIPCHK(hipMalloc(&b.p, alloc));
    b.n = alloc;
  }
  if (zero) HIPCHK(hipMemsetAsync(b.p, 0, bytes, ctx->stream));
  return (T*)b.p;
}

static unsigned grid_for(uint64_t work, unsigned per_block, unsigned cap = 1u << 20) {
  uint64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// Timing events (tsdbhip_timing). "kernel" (the default): a start event rides
// on the next kernel launched through LAUNCH (hipExtLaunchKernel's start
// event) and a stop event on the kernel it follows (LAUNCH_STOP), so no
// marker packet stands between two kernels: in the C3* shard trace each
// hipEventRecord between kernels left the GPU idle ~5 us. "marker": events
// recorded in the stream (hipEventRecord). "none": no events (timings 0).
static thread_local hipEvent_t g_ev_pend = nullptr;
static thread_local int g_ev_pend_i = -1;
static inline hipEvent_t ev_take() {
  hipEvent_t e = g_ev_pend;
  g_ev_pend = nullptr;
  g_ev_pend_i = -1;
  return e;
}
static void EV_START(Slot* ctx, int i) {
  if (ctx->opt.events == 0) {
    // (a start no kernel took reads as this one: both mark the next kernel's
    // start, and a marker would cost a host call and a GPU-side gap)
    if (g_ev_pend && g_ev_pend_i >= 0) ctx->ev_alias[g_ev_pend_i] = (int8_t)i;
    g_ev_pend = ctx->ev[i];
    g_ev_pend_i = i;
  } else if (ctx->opt.events == 1) {
    HIPCHK(hipEventRecord(ctx->ev[i], ctx->stream));
  }
}
// the stop event for LAUNCH_STOP ("kernel"), then EV_STOP_M after it ("marker")
#define EV_STOP_K(ctx, i) ((ctx)->opt.events == 0 ? (ctx)->ev[i] : (hipEvent_t) nullptr)
#define EV_STOP_M(ctx, i)                                                             \
  do {                                                                                \
    if ((ctx)->opt.events == 1) HIPCHK(hipEventRecord((ctx)->ev[i], (ctx)->stream)); \
  } while (0)
// The call's last event, a marker in every mode: its system-scope release
// makes the call-end kernels' writes into mapped host memory (the state
// snapshot, small results) visible to the host after the stream sync.
#define EV_FINAL(ctx, i) HIPCHK(hipEventRecord((ctx)->ev[i], (ctx)->stream))
// (a launch without an event goes the plain way: hipExtLaunchKernel costs
// more host time a call)
#define LAUNCH(k, g, b, sh, st, ...)                                          \
  do {                                                                        \
    hipEvent_t e_ = ev_take();                                                \
    if (e_) hipExtLaunchKernelGGL(k, g, b, sh, st, e_, nullptr, 0, ##__VA_ARGS__); \
    else hipLaunchKernelGGL(k, g, b, sh, st, ##__VA_ARGS__);                  \
  } while (0)
#define LAUNCH_STOP(ev, k, g, b, sh, st, ...) hipExtLaunchKernelGGL(k, g, b, sh, st, ev_take(), ev, 0, ##__VA_ARGS__)
static float ev_ms(Slot* ctx, int a, int b) {
  float ms = 0;
  for (int n = 0; n < 10 && ctx->ev_alias[a] >= 0; n++) a = ctx->ev_alias[a];
  for (int n = 0; n < 10 && ctx->ev_alias[b] >= 0; n++) b = ctx->ev_alias[b];
  if (ctx->opt.events == 2 || hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]) != hipSuccess) {
    (void)hipGetLastError();
    return ctx->opt.events == 2 ? 0.f : -1.f;
  }
  return ms;
}

#include "xchg.hip"

static void dscan_u64(Slot* ctx, const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* d_total,
                      const char* tag) {
  const uint64_t nb = (n + 1023) / 1024;
  std::string key = std::string("scan_blocks_") + tag;
  uint64_t* bs = scratch<uint64_t>(ctx, key.c_str(), nb + 1);
  if (n == 0) {
    HIPCHK(hipMemsetAsync(d_total, 0, 8, ctx->stream));
    return;
  }
  LAUNCH(k_scan_block_u64, dim3((unsigned)nb), dim3(256), 0, ctx->stream, in, out, n, bs);
  LAUNCH(k_scan_blocks_u64, dim3(1), dim3(256), 0, ctx->stream, bs, nb, d_total);
  LAUNCH(k_scan_add_u64, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, out, n, bs);
}

// ------------------------------------------------------------ slot pool ----
static void slot_free(Slot* s) {
  if (!s) return;
  hipSetDevice(s->device);
  if (s->stream) hipStreamSynchronize(s->stream);
  for (auto& kv : s->bufs)
    if (kv.second.p) hipFree(kv.second.p);
  for (auto& e : s->ev)
    if (e) hipEventDestroy(e);
  if (s->host_small) hipHostFree(s->host_small);
  if (s->map_state) hipHostFree(s->map_state);
  if (s->map_out) hipHostFree(s->map_out);
  if (s->host_big) hipHostFree(s->host_big);
  if (s->stream) hipStreamDestroy(s->stream);
  delete s;
}

static Slot* slot_new(int device) {
  Slot* ctx = new Slot();
  ctx->device = device;
  try {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    HIPCHK(hipHostMalloc(&ctx->host_small, 4096, hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&ctx->map_state, 8 * 520, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void**)&ctx->map_state_dev, ctx->map_state, 0));
    std::memset(ctx->map_state, 0, 8 * 520);
    // Timing events inside a call: no system-scope fence (no L2 writeback /
    // invalidate between kernels). The call's last events ([5] spangroup,
    // [1] compaction) keep it: the call-end kernels write the state snapshot
    // and small results into mapped host memory, and that release is what
    // makes them visible to the host after the stream sync (without it a
    // host read of the snapshot came back stale about once in five suites).
    for (int i = 0; i < 10; i++)
      HIPCHK(hipEventCreateWithFlags(&ctx->ev[i], (i == 5 || i == 1) ? hipEventDefault : hipEventDisableSystemFence));
  } catch (Fail&) {
    slot_free(ctx);
    throw;
  }
  return ctx;
}

static constexpr size_t MAX_SLOTS = 64;  // concurrent calls per context

static void timing_add(tsdbhip_ctx* c, const tsdbhip_timing& t) {  // (c->mu held)
  c->sum.total_ms += t.total_ms;
  c->sum.decode_ms += t.decode_ms;
  c->sum.grid_ms += t.grid_ms;
  c->sum.reduce_ms += t.reduce_ms;
  c->sum.exchange_ms += t.exchange_ms;
  c->sum.hot_ms += t.hot_ms;
  c->sum.hot_kernel = t.hot_kernel;
  c->sum.n_collectives += t.n_collectives;
  c->sum.decode_bytes += t.decode_bytes;
  c->sum.alg_bytes += t.alg_bytes;
  c->sum.n_grid += t.n_grid;
  c->sum.n_emitted += t.n_emitted;
  c->sum.paths |= t.paths;
  c->sum.x_bytes += t.x_bytes;
  c->sum.late_stamp += t.late_stamp;
  c->sum.h2d_bytes += t.h2d_bytes;
  c->n_sum++;
}

// A slot held for the duration of one call.
struct Lease {
  tsdbhip_ctx* c;
  Slot* s = nullptr;
  explicit Lease(tsdbhip_ctx* c_) : c(c_) {
    {
      std::lock_guard<std::mutex> lk(c->mu);
      if (!c->free_slots.empty()) {
        s = c->free_slots.back();
        c->free_slots.pop_back();
      } else if (c->slots.size() >= MAX_SLOTS) {
        set_error(c, "more than %zu concurrent calls on one context", MAX_SLOTS);
        throw Fail{TSDBHIP_E_INVALID_ARG};
      }
    }
    if (!s) {
      s = slot_new(c->device);
      std::lock_guard<std::mutex> lk(c->mu);
      c->slots.push_back(s);
    }
    s->x = nullptr;
    s->want_output = true;
    // (no start event pending from an earlier call on this thread that threw
    // between EV_START and its LAUNCH: ADVICE r4)
    g_ev_pend = nullptr;
    g_ev_pend_i = -1;
    {
      std::lock_guard<std::mutex> lk(c->mu);
      s->opt = c->opt;
    }
    if (hipSetDevice(c->device) != hipSuccess) {  // (the destructor will not run: hand the slot back here)
      set_error(c, "hipSetDevice(%d) failed", c->device);
      std::lock_guard<std::mutex> lk(c->mu);
      c->free_slots.push_back(s);
      throw Fail{TSDBHIP_E_HIP};
    }
  }
  ~Lease() {
    s->x = nullptr;
    g_last_ctx = c;
    g_last_timing = s->timing;
    std::lock_guard<std::mutex> lk(c->mu);
    c->last = s->timing;
    timing_add(c, s->timing);
    c->free_slots.push_back(s);
  }
};

// ---------------------------------------------- in-process multi-device ----
// tsdbhip_open_devices: rank r is member context r (device devs[r]); a
// SpanGroup is split into contiguous span ranges, one per rank, run by one
// host thread each through the sharded path.
struct Multi {
  int n = 0;
  std::vector<int> devs;
  std::vector<tsdbhip_ctx*> members;
  std::vector<std::unique_ptr<Xchg>> xs;
  std::vector<ncclComm_t> comms;
  LocalGroup local;
  bool rccl = false;
  std::mutex call_mu;  // one sharded call at a time (collectives in lockstep)
  // per rank > 0: result buffers of its (unused) copy of the output
  std::vector<std::vector<int64_t>> ts, bits;
  std::vector<std::vector<uint8_t>> isint;
};

// plain context of a call: a multi-device context's non-sharded work
// (inputs, compaction, probes) runs on its first member
static tsdbhip_ctx* plain_of(tsdbhip_ctx* c) { return c->multi ? c->multi->members[0] : c; }

// ----------------------------------------------------------------------------
extern "C" int tsdbhip_abi_version(void) { return TSDBHIP_ABI_VERSION; }

extern "C" const char* tsdbhip_last_error(tsdbhip_ctx*) { return g_thread_err.c_str(); }

static int ctx_open(int32_t device, tsdbhip_ctx** out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    set_error(nullptr, "no HIP device available");
    return TSDBHIP_E_NO_DEVICE;
  }
  if (device < 0 || device >= n) {
    set_error(nullptr, "device %d out of range (%d devices)", device, n);
    return TSDBHIP_E_INVALID_ARG;
  }
  tsdbhip_ctx* c = new tsdbhip_ctx();
  c->device = device;
  try {
    Slot* s = slot_new(device);  // the first slot (and a check that the device works)
    c->slots.push_back(s);
    c->free_slots.push_back(s);
  } catch (Fail& f) {
    delete c;
    return f.code;
  }
  *out = c;
  return TSDBHIP_OK;
}

extern "C" int tsdbhip_open(int32_t device, tsdbhip_ctx** out) {
  if (!out) return TSDBHIP_E_INVALID_ARG;
  *out = nullptr;
  return ctx_open(device, out);
}

extern "C" void tsdbhip_close(tsdbhip_ctx* ctx) {
  if (!ctx) return;
  if (ctx->multi) {
    Multi* m = ctx->multi;
    for (int r = 0; r < m->n; r++) {
      hipSetDevice(m->devs[r]);
      if (r < (int)m->local.ready.size() && m->local.ready[r]) hipEventDestroy(m->local.ready[r]);
      if (r < (int)m->local.done.size() && m->local.done[r]) hipEventDestroy(m->local.done[r]);
    }
    for (ncclComm_t cm : m->comms)
      if (cm) ncclCommDestroy(cm);
    for (tsdbhip_ctx* mc : m->members) tsdbhip_close(mc);
    delete m;
    delete ctx;
    return;
  }
  hipSetDevice(ctx->device);
  for (Slot* s : ctx->slots) slot_free(s);
  for (auto& kv : ctx->owned)
    if (kv.second.p) hipFree(kv.second.p);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  delete ctx->rccl;
  delete ctx;
}

// One context over several devices; devs may repeat (several shards on one
// GPU exchange through device copies, LocalXchg); distinct devices exchange
// over RCCL (one communicator per device, ncclCommInitAll) unless
// TSDBHIP_XCHG=local.
extern "C" int tsdbhip_open_devices(const int32_t* devs, uint32_t n, tsdbhip_ctx** out) {
  if (!out || !devs || n == 0 || n > 64) return TSDBHIP_E_INVALID_ARG;
  *out = nullptr;
  if (n == 1) return ctx_open(devs[0], out);
  tsdbhip_ctx* ctx = new tsdbhip_ctx();
  Multi* m = new Multi();
  ctx->multi = m;
  ctx->device = devs[0];
  m->n = (int)n;
  m->devs.assign(devs, devs + n);
  int rc = TSDBHIP_OK;
  for (uint32_t r = 0; r < n && !rc; r++) {
    tsdbhip_ctx* mc = nullptr;
    rc = ctx_open(devs[r], &mc);
    if (!rc) m->members.push_back(mc);
  }
  bool distinct = true;
  for (uint32_t a = 0; a < n; a++)
    for (uint32_t b = a + 1; b < n; b++) distinct = distinct && devs[a] != devs[b];
  m->rccl = distinct;
  try {
    if (rc) throw Fail{rc};
    if (m->rccl) {
      m->comms.assign(n, nullptr);
      std::vector<int> dl(devs, devs + n);
      NCCLCHK(ncclCommInitAll(m->comms.data(), (int)n, dl.data()));
      for (uint32_t r = 0; r < n; r++) {
        RcclXchg* x = new RcclXchg();
        x->comm = m->comms[r];
        x->nranks = (int)n;
        x->rank = (int)r;
        m->xs.emplace_back(x);
      }
    } else {
      LocalGroup& G = m->local;
      G.n = (int)n;
      G.dev = m->devs;
      G.ptr.assign(n, nullptr);
      G.ready.assign(n, nullptr);
      G.done.assign(n, nullptr);
      for (uint32_t r = 0; r < n; r++) {
        HIPCHK(hipSetDevice(devs[r]));
        HIPCHK(hipEventCreateWithFlags(&G.ready[r], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&G.done[r], hipEventDisableTiming));
        if (!distinct) continue;
        for (uint32_t q = 0; q < n; q++) {  // peer copies between distinct devices
          int can = 0;
          if (devs[q] != devs[r] && hipDeviceCanAccessPeer(&can, devs[r], devs[q]) == hipSuccess && can)
            (void)hipDeviceEnablePeerAccess(devs[q], 0);
        }
      }
      (void)hipGetLastError();  // (peer access already enabled is not an error here)
      for (uint32_t r = 0; r < n; r++) {
        LocalXchg* x = new LocalXchg();
        x->G = &G;
        x->nranks = (int)n;
        x->rank = (int)r;
        m->xs.emplace_back(x);
      }
    }
  } catch (Fail& f) {
    tsdbhip_close(ctx);
    return f.code;
  }
  m->ts.resize(n);
  m->bits.resize(n);
  m->isint.resize(n);
  *out = ctx;
  return TSDBHIP_OK;
}

extern "C" int tsdbhip_open_mask(uint32_t gpu_mask, tsdbhip_ctx** out) {
  int32_t devs[32];
  uint32_t n = 0;
  for (int d = 0; d < 32; d++)
    if (gpu_mask & (1u << d)) devs[n++] = d;
  if (!n) return TSDBHIP_E_INVALID_ARG;
  return tsdbhip_open_devices(devs, n, out);
}

extern "C" int tsdbhip_set_option(tsdbhip_ctx* ctx, const char* name, const char* value) {
  if (!ctx || !name || !value) return TSDBHIP_E_INVALID_ARG;
  const std::string n(name), v(value);
  auto on_off = [&](bool& f) {
    if (v == "on") f = true;
    else if (v == "off") f = false;
    else return false;
    return true;
  };
  Options o;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    o = ctx->opt;
  }
  bool ok = true;
  if (n == "decode") {
    static const char* names[] = {"auto", "general", "fast", "chunks", "spans", "direct"};
    ok = false;
    for (int i = 0; i < 6; i++)
      if (v == names[i]) { o.decode = i; ok = true; }
  } else if (n == "aligned_group") ok = on_off(o.aligned_group);
  else if (n == "lockstep") {
    ok = v == "on" || v == "off" || v == "always";
    o.lockstep = v == "off" ? 0 : (v == "on" ? 1 : 2);
  }
  else if (n == "timing_detail") ok = on_off(o.timing_detail);
  else if (n == "check_clean") ok = on_off(o.check_clean);
  else if (n == "events") {
    static const char* names[] = {"kernel", "marker", "none"};
    ok = false;
    for (int i = 0; i < 3; i++)
      if (v == names[i]) { o.events = i; ok = true; }
  } else ok = false;
  if (!ok) {
    set_error(ctx, "tsdbhip_set_option: unknown option %s=%s", name, value);
    return TSDBHIP_E_INVALID_ARG;
  }
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->opt = o;
  }
  if (ctx->multi)  // (every rank's member context runs with them)
    for (tsdbhip_ctx* m : ctx->multi->members) {
      std::lock_guard<std::mutex> lk(m->mu);
      m->opt = o;
    }
  return TSDBHIP_OK;
}

extern "C" int tsdbhip_ranks(tsdbhip_ctx* ctx) {
  if (!ctx) return TSDBHIP_E_INVALID_ARG;
  return ctx->multi ? ctx->multi->n : 1;
}

// The registered host ranges [p, p + n): the in-kernel finalize writes a long
// result through a mapped pointer only into a range that holds all of it
// (mapped_dev_ptr). A HIP registration is process-wide, so contexts share it:
// each entry counts its tsdbhip_host_register calls, and the range is
// unregistered from HIP (and dropped here) only by the last unregister
// (ADVICE r5).
struct RegEntry {
  size_t n;
  uint32_t refs;
};
static std::mutex g_reg_mu;
static std::map<uintptr_t, RegEntry> g_reg;

extern "C" int tsdbhip_host_register(tsdbhip_ctx* ctx, void* p, size_t n) {
  if (!ctx || !p || !n) return TSDBHIP_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find((uintptr_t)p);
  if (it != g_reg.end()) {  // (registered by this library already: the same range, shared)
    if (it->second.n != n) {
      set_error(ctx, "host_register: %p is registered with %zu bytes, not %zu", p, it->second.n, n);
      return TSDBHIP_E_INVALID_ARG;
    }
    it->second.refs++;
    return TSDBHIP_OK;
  }
  try {
    HIPCHK(hipSetDevice(ctx->device));
    // (portable: pinned for every device of a multi-device context)
    // (mapped: a long result is then written by the reduce straight into it)
    HIPCHK(hipHostRegister(p, n, hipHostRegisterMapped | (ctx->multi ? hipHostRegisterPortable : 0u)));
  } catch (Fail& f) {
    return f.code;
  }
  g_reg[(uintptr_t)p] = RegEntry{n, 1};
  return TSDBHIP_OK;
}

extern "C" int tsdbhip_host_unregister(tsdbhip_ctx* ctx, void* p) {
  if (!ctx || !p) return TSDBHIP_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find((uintptr_t)p);
  if (it != g_reg.end() && it->second.refs > 1) {
    it->second.refs--;
    return TSDBHIP_OK;
  }
  try {
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipHostUnregister(p));
  } catch (Fail& f) {
    return f.code;
  }
  if (it != g_reg.end()) g_reg.erase(it);
  return TSDBHIP_OK;
}

// The timings of this thread's last call on ctx (else of the ctx's last call).
extern "C" int tsdbhip_last_timing(tsdbhip_ctx* ctx, tsdbhip_timing* t) {
  if (!ctx || !t) return TSDBHIP_E_INVALID_ARG;
  if (g_last_ctx == ctx) {
    *t = g_last_timing;
    return TSDBHIP_OK;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  *t = ctx->last;
  return TSDBHIP_OK;
}

extern "C" int tsdbhip_timing_totals(tsdbhip_ctx* ctx, tsdbhip_timing* sum, uint64_t* n_calls, int32_t reset) {
  if (!ctx) return TSDBHIP_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (sum) *sum = ctx->sum;
  if (n_calls) *n_calls = ctx->n_sum;
  if (reset) {
    ctx->sum = tsdbhip_timing();
    ctx->n_sum = 0;
  }
  return TSDBHIP_OK;
}

// ---------------------------------------------------------------- comm ----
extern "C" int tsdbhip_comm_unique_id(uint8_t out[TSDBHIP_UNIQUE_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) <= TSDBHIP_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    set_error(nullptr, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    return TSDBHIP_E_RCCL;
  }
  std::memset(out, 0, TSDBHIP_UNIQUE_ID_BYTES);
  std::memcpy(out, &id, sizeof id);
  return TSDBHIP_OK;
}

extern "C" int tsdbhip_comm_init(tsdbhip_ctx* ctx, int32_t nranks, int32_t rank,
                                 const uint8_t id[TSDBHIP_UNIQUE_ID_BYTES]) {
  if (!ctx || ctx->multi || nranks < 1 || rank < 0 || rank >= nranks) return TSDBHIP_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(ctx->comm_mu);
  try {
    HIPCHK(hipSetDevice(ctx->device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    if (ctx->comm) {
      ncclCommDestroy(ctx->comm);
      ctx->comm = nullptr;
    }
    NCCLCHK(ncclCommInitRank(&ctx->comm, nranks, uid, rank));
    delete ctx->rccl;
    RcclXchg* x = new RcclXchg();
    x->comm = ctx->comm;
    x->nranks = nranks;
    x->rank = rank;
    ctx->rccl = x;
  } catch (Fail& f) {
    return f.code;
  }
  return TSDBHIP_OK;
}

// ------------------------------------------------------------- helpers ----
static int err_code(uint64_t key) { return key == ERR_NONE ? 0 : -(int)(key & 0xFFu); }

template <typename T>
static const T* stage(Slot* ctx, const char* name, const T* src, size_t count, bool on_device,
                      size_t pad = 0) {
  if (on_device) return src;
  T* d = scratch<T>(ctx, name, count + pad);
  if (ctx->reuse_inputs) return d;  // (the same call's earlier attempt staged it)
  if (count) HIPCHK(hipMemcpyAsync(d, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  if (pad) HIPCHK(hipMemsetAsync((char*)d + count * sizeof(T), 0, pad * sizeof(T), ctx->stream));
  ctx->h2d_bytes += count * sizeof(T);
  return d;
}

// grow-only pinned host staging
static void* host_buf(Slot* ctx, size_t bytes) {
  if (ctx->host_big_n < bytes) {
    if (ctx->host_big) HIPCHK(hipHostFree(ctx->host_big));
    ctx->host_big = nullptr;
    size_t n = std::max(bytes, ctx->host_big_n + ctx->host_big_n / 4);
    HIPCHK(hipHostMalloc(&ctx->host_big, n, hipHostMallocDefault));
    ctx->host_big_n = n;
  }
  return ctx->host_big;
}

static void readback(Slot* ctx, void* host, const void* dev, size_t bytes) {
  HIPCHK(hipMemcpyAsync(ctx->host_small, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  std::memcpy(host, ctx->host_small, bytes);
}

// The next host_publish of `bytes` of device state (a kernel argument).
static HostPub next_pub(Slot* ctx, size_t bytes) {
  HostPub p;
  p.dst = ctx->map_state_dev;
  p.flag = ctx->map_state_dev + 512;
  p.seq = ++ctx->pub_seq;
  p.nwords = (uint32_t)((bytes + 7) / 8);
  return p;
}
// Waits for that publish and copies the state out: a spin on the mapped flag
// (the stream is queried now and then: a stream that drained without the
// flag means the producing kernel did not run).
static void wait_pub(Slot* ctx, const HostPub& p, void* host, size_t bytes) {
  const uint64_t* flag = ctx->map_state + 512;
  for (uint32_t i = 1;; i++) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == p.seq) break;
    if ((i & 1023) == 0) {
      const hipError_t e = hipStreamQuery(ctx->stream);
      if (e == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) != p.seq) {
        set_error(ctx, "host publish %llu never arrived", (unsigned long long)p.seq);
        throw Fail{TSDBHIP_E_HIP};
      }
      if (e != hipSuccess && e != hipErrorNotReady) HIPCHK(e);
    }
    __builtin_ia32_pause();
  }
  std::memcpy(host, ctx->map_state, bytes);
}

// The call-end stamp (small_snap) after the stream sync: the snapshot, and
// every result the call wrote into host memory, are this call's iff it reads
// `seq`. A stamp that is late (the stream has drained, so the writes are on
// their way) is waited for briefly; one that never comes is an error, never a
// stale result (the red test_nan_in_a_long_grid run).
static void check_stamp(Slot* ctx, uint64_t seq) {
  const uint64_t* stamp = (const uint64_t*)(ctx->map_out + OUT_HDR - 8);
  uint64_t v = __atomic_load_n(stamp, __ATOMIC_ACQUIRE);
  if (v == seq) return;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1; v != seq; i++) {
    __builtin_ia32_pause();
    v = __atomic_load_n(stamp, __ATOMIC_ACQUIRE);
    if ((i & 1023) == 0 && v != seq && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
      set_error(ctx, "stale snapshot: seq %llu, expected %llu", (unsigned long long)v, (unsigned long long)seq);
      throw Fail{TSDBHIP_E_HIP};
    }
  }
  ctx->timing_late = 1;
}

// grow-only mapped pinned result area (device pointer in map_out_dev)
static void map_out_reserve(Slot* ctx, size_t bytes) {
  if (ctx->map_out_n >= bytes) return;
  const size_t n = std::max(bytes, ctx->map_out_n + ctx->map_out_n / 4);
  if (ctx->map_out) HIPCHK(hipHostFree(ctx->map_out));
  ctx->map_out = nullptr;
  ctx->map_out_n = 0;
  HIPCHK(hipHostMalloc((void**)&ctx->map_out, n, hipHostMallocMapped | hipHostMallocCoherent));
  HIPCHK(hipHostGetDevicePointer((void**)&ctx->map_out_dev, ctx->map_out, 0));
  ctx->map_out_n = n;
  *(volatile uint64_t*)(ctx->map_out + OUT_HDR - 8) = 0;  // (no call's stamp)
}

// runtime aggregator id -> F::template run<AGG>(args...)
template <typename F, typename... A>
static void launch_agg(int agg, A&&... args) {
  switch (agg) {
    case 0: F::template run<0>(args...); break;
    case 1: F::template run<1>(args...); break;
    case 2: F::template run<2>(args...); break;
    case 3: F::template run<3>(args...); break;
    default: F::template run<4>(args...); break;
  }
}

struct LaunchGeneralDs {
  template <int AGG>
  static void run(Slot* ctx, unsigned blocks, const DecodeArgs& a) {
    LAUNCH(k_decode_ds<AGG>, dim3(blocks), dim3(256), 0, ctx->stream, a);
  }
};

struct LaunchFastDs {
  template <int AGG>
  static void run(Slot* ctx, unsigned blocks, const DecodeArgs& a, const uint32_t* ncells,
                  const uint32_t* vlen) {
    LAUNCH((k_decode_fast<AGG, true>), dim3(blocks), dim3(256), 0, ctx->stream, a, ncells, vlen);
  }
};
// (a leftover list: the general code inline, one launch)
struct LaunchFastDsInl {
  template <int AGG>
  static void run(Slot* ctx, unsigned blocks, const DecodeArgs& a, const uint32_t* ncells,
                  const uint32_t* vlen) {
    LAUNCH((k_decode_fast<AGG, true, true>), dim3(blocks), dim3(256), 0, ctx->stream, a, ncells, vlen);
  }
};

// Streaming downsampling: constant-step spans by formula (k_ds_reg, up to 4
// waves per span), then chain-proved regular-cadence spans (k_ds_spans,
// integer, then float); leaves the spans neither took in fa.span_list for
// k_decode_fast.
constexpr uint32_t CK_NSEG = 64;
// an aligned-group reduction of this call (k_ds_reg.hip FapArgs) and what its
// rerun needs
struct FapPlan {
  FapArgs a = {};
  SpanDsArgs g = {};
  unsigned blocks = 0, pad = 0;
};
struct LaunchChunks {
  template <int AGG>
  static void run(Slot* ctx, const DecodeArgs& da, DecodeArgs& fa, const uint32_t* ncells,
                  const uint32_t* vlen, SpanDsArgs g, uint64_t n_rows, bool use_reg = true,
                  uint32_t* zeroed2 = nullptr, uint32_t* zeroed_seg = nullptr, uint32_t* zeroed_seg2 = nullptr,
                  FapPlan* fp = nullptr) {
    if (AGG == 4) return;  // dev: Welford is order-dependent, serial kernels only
    hipStream_t st = ctx->stream;
    const uint32_t n_kept = da.n_kept;
    // (zeroed*: list counters already zero on the device, no memsets)
    // k_ds_reg: a span's rows split over 1 << wps_log2 waves of a block
    const uint64_t rps = n_rows / std::max<uint32_t>(n_kept, 1);
    const uint32_t wps_log2 = rps >= 12 ? 2 : (rps >= 6 ? 1 : 0);
    const uint32_t rblocks = (uint32_t)(((uint64_t)n_kept * (1u << wps_log2) + 3) / 4);
    SpanDsArgs gr = g;
    gr.nseg = CK_NSEG;
    gr.seg_cap = (4u >> wps_log2) * ((rblocks + CK_NSEG - 1) / CK_NSEG);
    gr.list = scratch<uint32_t>(ctx, "cr_list", (uint64_t)gr.seg_cap * CK_NSEG);
    gr.list_count = zeroed_seg2 ? zeroed_seg2 : scratch<uint32_t>(ctx, "cr_seg_count", CK_NSEG, true);
    gr.in_list = nullptr;
    gr.in_count = nullptr;
    gr.in_nseg = gr.in_seg_cap = 0;
    // k_ds_spans (integer and float spans, one launch) over k_ds_reg's
    // leftovers (usually few: a capped, grid-stride launch), or over every
    // kept span without k_ds_reg; its own leftovers to k_decode_fast
    const unsigned iblocks = use_reg ? std::min(grid_for(n_kept, 4, 1u << 20), 4096u) : grid_for(n_kept, 4, 1u << 20);
    g.in_list = use_reg ? gr.list : nullptr;
    g.in_count = use_reg ? gr.list_count : nullptr;
    g.in_nseg = use_reg ? gr.nseg : 0;
    g.in_seg_cap = use_reg ? gr.seg_cap : 0;
    g.nseg = g.seg_cap = 0;
    g.list = scratch<uint32_t>(ctx, "ck_list2", n_kept);
    g.list_count = zeroed2 ? zeroed2 + 1 : scratch<uint32_t>(ctx, "ck_list2_count", 1, true);
    EV_START(ctx, 8);
    // one wave per span (long rows, C3*): 4 resident blocks per CU (LDS
    // padding) measured faster than the 6 its registers allow; split spans
    // (C2) prefer the full occupancy
    // (the padding brings the block's LDS to 40 KB whatever the kernel's own
    // static LDS: a few bytes more would leave room for only 3 blocks)
    static const unsigned stat_lds = [] {
      hipFuncAttributes fa = {};
      return hipFuncGetAttributes(&fa, (const void*)k_ds_reg<AGG>) == hipSuccess ? (unsigned)fa.sharedSizeBytes
                                                                                 : 18960u;
    }();
    const unsigned pad = wps_log2 == 0 ? (stat_lds < 40960u ? 40960u - stat_lds : 0u) : 0u;
    // the aligned-group reduction (one wave per span): a partial row per block
    FapArgs fa0 = {};
    fa0.op = -1;
    if (fp && (!use_reg || wps_log2 != 0)) fp->a.op = -1;
    if (fp && fp->a.op >= 0) {
      fp->a.nrows = rblocks;
      fp->a.part = scratch<int64_t>(ctx, "fap_part", (uint64_t)rblocks * WAVE);
      fp->g = gr;  // (the rerun after a broken FAP pass: the same launch, E only)
      fp->blocks = rblocks;
      fp->pad = pad;
    }
    if (use_reg)
      LAUNCH((k_ds_reg<AGG>), dim3(rblocks), dim3(256), pad, st, da, gr, ncells, vlen, wps_log2,
                         fp ? fp->a : fa0);
    LAUNCH_STOP(EV_STOP_K(ctx, 9), (k_ds_spans<AGG, 2>), dim3(iblocks), dim3(256), 0, st, da, g, ncells, vlen);
    EV_STOP_M(ctx, 9);
    ctx->hot_kernel = TSDBHIP_HOT_DS_CHUNKS;
    fa.span_list = g.list;
    fa.span_count = g.list_count;
  }
};

// the rerun of k_ds_reg after a broken aligned-group pass: E of the spans it
// takes (the FAP members), no list, no marks, no flags
struct LaunchRegRerun {
  template <int AGG>
  static void run(Slot* ctx, const DecodeArgs& da, const FapPlan& fp, const uint32_t* ncells, const uint32_t* vlen) {
    if (AGG == 4) return;
    FapArgs a = fp.a;
    a.op = -1;
    a.rewrite = 1;
    LAUNCH((k_ds_reg<AGG>), dim3(fp.blocks), dim3(256), fp.pad, ctx->stream, da, fp.g, ncells, vlen, 0u,
                       a);
  }
};

template <int AGG, int MODE, bool RATE>
static void launch_reduce(Slot* ctx, unsigned blocks, const ReduceArgs& r, const FinalArgs& f,
                          bool par, bool finalize) {
  if (ctx->time_reduce) EV_START(ctx, 8);
  if (r.d_info && r.chunk_e)
    LAUNCH((k_reduce<AGG, MODE, RATE, true>), dim3(blocks), dim3(256), 0, ctx->stream, r);
  const unsigned lds = r.lds_state ? 4 * red_lds_stride(r.spans_per_chunk, RATE) : 0;
  const hipEvent_t stop = ctx->time_reduce ? EV_STOP_K(ctx, 9) : nullptr;
  if constexpr (AGG == TSDBHIP_AGG_DEV)
    LAUNCH_STOP(stop, (k_reduce<AGG, MODE, RATE, false>), dim3(blocks), dim3(256), lds, ctx->stream, r);
  else
    LAUNCH_STOP(stop, (k_reduce_w4<AGG, MODE, RATE, false>), dim3(blocks), dim3(256), lds, ctx->stream, r);
  if (ctx->time_reduce) EV_STOP_M(ctx, 9);
  if (!finalize) return;
  if (par && f.T >= 1024)  // (large T: coalesced columns)
    LAUNCH((k_chunks_cols<AGG, MODE, RATE, true>), dim3((unsigned)((f.T + 63) / 64)), dim3(64 * COLW), 0,
                       ctx->stream, r, r, f, f.T, f.n_chunks);
  else if (par)
    LAUNCH((k_finalize_par<AGG, MODE, RATE>), dim3((unsigned)f.T), dim3(256), 0, ctx->stream, r, f);
  else
    LAUNCH((k_finalize_seq<AGG, MODE, RATE>), dim3(grid_for(f.T, 256)), dim3(256), 0, ctx->stream,
                       r, f);
}

// k_lockstep over the group (one instantiation per value width and type; the
// mode follows: rate or float values reduce doubles, int values longs), then
// the finalize of launch_reduce
struct LsPlan {
  LockstepArgs a;
  bool w8, flt;
};
#ifndef LS_MIN_SPC
#define LS_MIN_SPC 128  // fewest spans a lockstep chunk (the n_chunks x T partials the combine reads; 64: the C3 rate-sum 8-way shard 1.07 ms, 128: 0.98-1.00, 256: 0.99-1.00; 1M spans unchanged)
#endif
template <int AGG, bool RATE, uint32_t W, bool FLT>
static void launch_lockstep_wf(Slot* ctx, unsigned blocks, const ReduceArgs& r, const LockstepArgs& a,
                               const FinalArgs& f, bool finalize) {
  constexpr int MODE = (RATE || FLT) ? MODE_DBL : MODE_INT;
  if (AGG == 4 && MODE == MODE_INT) return;  // (integer dev reduces in one span-ordered pass: never lockstep)
  EV_START(ctx, 8);
  LAUNCH_STOP(EV_STOP_K(ctx, 9), (k_lockstep<AGG, MODE, RATE, W, FLT>), dim3(blocks), dim3(256), 0, ctx->stream, r, a);
  EV_STOP_M(ctx, 9);
  if (!finalize) return;
  if (f.n_chunks >= 64 && f.T >= 1024)
    LAUNCH((k_chunks_cols<AGG, MODE, RATE, true>), dim3((unsigned)((f.T + 63) / 64)), dim3(64 * COLW), 0,
                       ctx->stream, r, r, f, f.T, f.n_chunks);
  else if (f.n_chunks >= 64)
    LAUNCH((k_finalize_par<AGG, MODE, RATE>), dim3((unsigned)f.T), dim3(256), 0, ctx->stream, r, f);
  else
    LAUNCH((k_finalize_seq<AGG, MODE, RATE>), dim3(grid_for(f.T, 256)), dim3(256), 0, ctx->stream, r, f);
}
template <int AGG>
static void launch_lockstep(Slot* ctx, bool rate, unsigned blocks, const ReduceArgs& r, const LsPlan& p,
                            const FinalArgs& f, bool fin) {
#define LS_GO(RT, W, F) launch_lockstep_wf<AGG, RT, W, F>(ctx, blocks, r, p.a, f, fin)
  if (rate) {
    if (p.w8) { if (p.flt) LS_GO(true, 8, true); else LS_GO(true, 8, false); }
    else { if (p.flt) LS_GO(true, 4, true); else LS_GO(true, 4, false); }
  } else {
    if (p.w8) { if (p.flt) LS_GO(false, 8, true); else LS_GO(false, 8, false); }
    else { if (p.flt) LS_GO(false, 4, true); else LS_GO(false, 4, false); }
  }
#undef LS_GO
}
static void dispatch_lockstep(Slot* ctx, int agg, bool rate, unsigned blocks, const ReduceArgs& r, const LsPlan& p,
                              const FinalArgs& f, bool fin) {
  switch (agg) {
    case 0: return launch_lockstep<0>(ctx, rate, blocks, r, p, f, fin);
    case 1: return launch_lockstep<1>(ctx, rate, blocks, r, p, f, fin);
    case 2: return launch_lockstep<2>(ctx, rate, blocks, r, p, f, fin);
    case 3: return launch_lockstep<3>(ctx, rate, blocks, r, p, f, fin);
    default: return launch_lockstep<4>(ctx, rate, blocks, r, p, f, fin);
  }
}

// the uniform path's E variant: k_ug_reduce, then launch_reduce's finalize
template <int AGG, int MODE>
static void launch_ug_reduce(Slot* ctx, const ReduceArgs& r, const FinalArgs& f) {
  const uint64_t n_waves = (r.T + WAVE - 1) / WAVE * r.n_chunks;
  LAUNCH((k_ug_reduce<AGG, MODE>), dim3((unsigned)((n_waves + 3) / 4)), dim3(256), 0, ctx->stream, r);
  if (f.n_chunks >= 64 && f.T >= 1024)
    LAUNCH((k_chunks_cols<AGG, MODE, false, true>), dim3((unsigned)((f.T + 63) / 64)), dim3(64 * COLW), 0,
           ctx->stream, r, r, f, f.T, f.n_chunks);
  else if (f.n_chunks >= 64)
    LAUNCH((k_finalize_par<AGG, MODE, false>), dim3((unsigned)f.T), dim3(256), 0, ctx->stream, r, f);
  else
    LAUNCH((k_finalize_seq<AGG, MODE, false>), dim3(grid_for(f.T, 256)), dim3(256), 0, ctx->stream, r, f);
}
template <int AGG>
static void ug_reduce_mode(Slot* ctx, int mode, const ReduceArgs& r, const FinalArgs& f) {
  if (mode == MODE_INT) launch_ug_reduce<AGG, MODE_INT>(ctx, r, f);
  else launch_ug_reduce<AGG, MODE_DBL>(ctx, r, f);
}
static void dispatch_ug_reduce(Slot* ctx, int agg, int mode, const ReduceArgs& r, const FinalArgs& f) {
  switch (agg) {
    case 0: return ug_reduce_mode<0>(ctx, mode, r, f);
    case 1: return ug_reduce_mode<1>(ctx, mode, r, f);
    case 2: return ug_reduce_mode<2>(ctx, mode, r, f);
    case 3: return ug_reduce_mode<3>(ctx, mode, r, f);
    default: return ug_reduce_mode<4>(ctx, mode, r, f);
  }
}

template <int AGG>
static void dispatch_mode(Slot* ctx, int mode, bool rate, unsigned blocks, const ReduceArgs& r,
                          const FinalArgs& f, bool par, bool fin) {
  if (rate) return launch_reduce<AGG, MODE_DBL, true>(ctx, blocks, r, f, par, fin);
  if (mode == MODE_INT) return launch_reduce<AGG, MODE_INT, false>(ctx, blocks, r, f, par, fin);
  if (mode == MODE_DBL) return launch_reduce<AGG, MODE_DBL, false>(ctx, blocks, r, f, par, fin);
  return launch_reduce<AGG, MODE_DUAL, false>(ctx, blocks, r, f, par, fin);
}

static void dispatch_reduce(Slot* ctx, int agg, int mode, bool rate, unsigned blocks,
                            const ReduceArgs& r, const FinalArgs& f, bool par, bool fin) {
  switch (agg) {
    case 0: return dispatch_mode<0>(ctx, mode, rate, blocks, r, f, par, fin);
    case 1: return dispatch_mode<1>(ctx, mode, rate, blocks, r, f, par, fin);
    case 2: return dispatch_mode<2>(ctx, mode, rate, blocks, r, f, par, fin);
    case 3: return dispatch_mode<3>(ctx, mode, rate, blocks, r, f, par, fin);
    default: return dispatch_mode<4>(ctx, mode, rate, blocks, r, f, par, fin);
  }
}

template <int AGG, int MODE>
static void launch_combine(Slot* ctx, const ReduceArgs& src, const ReduceArgs& dst, uint64_t T,
                           uint32_t n_chunks) {
  if (n_chunks >= 64 && T >= 1024) {  // (large T: coalesced columns)
    FinalArgs nf = {};
    LAUNCH((k_chunks_cols<AGG, MODE, false, false>), dim3((unsigned)((T + 63) / 64)), dim3(64 * COLW), 0,
                       ctx->stream, src, dst, nf, T, n_chunks);
  } else if (n_chunks >= 64)  // (as the finalize: serial chunk loops are latency-bound)
    LAUNCH((k_combine_par<AGG, MODE>), dim3((unsigned)T), dim3(256), 0, ctx->stream, src, dst, T,
                       n_chunks);
  else
    LAUNCH((k_combine_chunks<AGG, MODE>), dim3(grid_for(T, 256)), dim3(256), 0, ctx->stream, src,
                       dst, T, n_chunks);
}
template <int AGG>
static void combine_mode(Slot* ctx, int mode, const ReduceArgs& s, const ReduceArgs& d, uint64_t T,
                         uint32_t n) {
  if (mode == MODE_INT) return launch_combine<AGG, MODE_INT>(ctx, s, d, T, n);
  if (mode == MODE_DBL) return launch_combine<AGG, MODE_DBL>(ctx, s, d, T, n);
  return launch_combine<AGG, MODE_DUAL>(ctx, s, d, T, n);
}
static void dispatch_combine(Slot* ctx, int agg, int mode, const ReduceArgs& s, const ReduceArgs& d,
                             uint64_t T, uint32_t n) {
  switch (agg) {
    case 0: return combine_mode<0>(ctx, mode, s, d, T, n);
    case 1: return combine_mode<1>(ctx, mode, s, d, T, n);
    case 2: return combine_mode<2>(ctx, mode, s, d, T, n);
    case 3: return combine_mode<3>(ctx, mode, s, d, T, n);
    default: return combine_mode<4>(ctx, mode, s, d, T, n);
  }
}

template <int AGG>
static void final_mode(Slot* ctx, int mode, bool rate, const ReduceArgs& r, const FinalArgs& f) {
  const dim3 g(grid_for(f.T, 256)), b(256);
  if (rate) LAUNCH((k_finalize_seq<AGG, MODE_DBL, true>), g, b, 0, ctx->stream, r, f);
  else if (mode == MODE_INT) LAUNCH((k_finalize_seq<AGG, MODE_INT, false>), g, b, 0, ctx->stream, r, f);
  else if (mode == MODE_DBL) LAUNCH((k_finalize_seq<AGG, MODE_DBL, false>), g, b, 0, ctx->stream, r, f);
  else LAUNCH((k_finalize_seq<AGG, MODE_DUAL, false>), g, b, 0, ctx->stream, r, f);
}
static void dispatch_final(Slot* ctx, int agg, int mode, bool rate, const ReduceArgs& r,
                           const FinalArgs& f) {
  switch (agg) {
    case 0: return final_mode<0>(ctx, mode, rate, r, f);
    case 1: return final_mode<1>(ctx, mode, rate, r, f);
    case 2: return final_mode<2>(ctx, mode, rate, r, f);
    case 3: return final_mode<3>(ctx, mode, rate, r, f);
    default: return final_mode<4>(ctx, mode, rate, r, f);
  }
}

// k_reduce launch geometry: (tile group, span chunk) per wave.
constexpr uint64_t RED_LDS_BLOCK = 40960;  // k_reduce span state: LDS bytes a block at most
struct ReduceGeom {
  uint32_t spc, n_chunks, tpw, ntg;
  uint64_t n_waves;
};
// target: waves in flight over 256 CUs (a group batch splits it over its
// groups); min_waves: floor for small groups
static ReduceGeom reduce_geom(uint64_t T, uint32_t n_kept, bool one_chunk, uint64_t target = 16384,
                              uint64_t min_waves = 2048, uint32_t spc_cap = 0) {
  ReduceGeom g;
  const uint64_t n_tiles = (T + 63) / 64;
  if (one_chunk || n_kept == 0) {
    g.n_chunks = 1;
    g.spc = std::max<uint32_t>(n_kept, 1);
  } else {
    // chunks of ~256 spans (fewer partials for the combine), but at
    // least ~2048 waves when the group is small
    uint64_t want = std::max<uint64_t>(1, target / n_tiles);
    const uint64_t by_size = std::max<uint64_t>((n_kept + 255) / 256, (min_waves + n_tiles - 1) / n_tiles);
    want = std::min<uint64_t>(want, by_size);
    want = std::min<uint64_t>(want, std::max<uint32_t>(1, n_kept / 16));
    // long grids: chunks small enough for the span state to stay in LDS
    // (read every tile; C4: 180k tiles)
    if (spc_cap && n_tiles >= 1024) want = std::max<uint64_t>(want, (n_kept + spc_cap - 1) / spc_cap);
    g.n_chunks = (uint32_t)std::max<uint64_t>(1, want);
    g.spc = (n_kept + g.n_chunks - 1) / g.n_chunks;
    g.n_chunks = (n_kept + g.spc - 1) / g.spc;
  }
  g.tpw = (uint32_t)std::max<uint64_t>(1, (n_tiles * g.n_chunks + target - 1) / target);
  g.ntg = (uint32_t)((n_tiles + g.tpw - 1) / g.tpw);
  g.n_waves = (uint64_t)g.ntg * g.n_chunks;
  return g;
}


// Device state of one spangroup_run call (err_raise keys, grid range, flags,
// counters); read back at the call's host round trips.
struct Small {
  unsigned long long err;  // first error (err_raise key), ERR_NONE: none
  uint32_t gflags[2];
  uint32_t reserved;
  unsigned long long range[2];
  unsigned long long fstar;
  unsigned long long n_input;
  unsigned long long nan_t;
  unsigned long long bad_at;
  uint64_t n_kept;
  uint64_t e_total;
  uint64_t T;
  unsigned long long bound[4];  // [min first ts, max last ts, max first ts, min last ts] of the kept spans
  uint32_t cnt[6];  // list counters, zero at the start of a call (no memsets):
                    // [0] assembly queue, [1] decode fallback, [2] direct list,
                    // [3] [4] k_ds_spans int / float leftovers, [5] lockstep
                    // proposal
  uint32_t seg[CK_NSEG];  // k_ds_spans integer leftovers, per segment
  uint32_t seg2[CK_NSEG];  // k_ds_reg leftovers, per segment
  // k_ds_reg's aligned-group reduction (FAP): the spans' class keys
  // (t0 << 32 | n, step) as [min, max, min, max], and a span outside it
  unsigned long long fap_key[4];
  uint32_t fap_broken, fap_done;  // (fap_done: the optimistic finish wrote the results)
  unsigned long long fap_valid;    // this rank's aligned-group partials stand (MIN over ranks when sharded)
  // sharded calls: two 64-bit hashes of the rank's grid bitmap (k_grid_popc /
  // k_grid_scan_blocks), and the agreed header words of the one collective
  // after the local grids (XH_*: MIN, or complemented MAX, over the ranks)
  unsigned long long ghash[2];
  // the lockstep proposal (k_direct_opt): class keys [min, max, min, max];
  // ls_broken: k_lockstep found a qualifier off the proposal (MAX over ranks)
  unsigned long long ls_key[4];
  uint32_t ls_broken, ls_pad;
  unsigned long long xh[14];  // (XH_N, + the aligned-group validity in an optimistic call)
  // the uniform-group proposal (assembly): the kept spans' class keys
  // (x0 << 32 | n, step << 32 | q0) as [min, max, min, max]; a span that
  // proposes none holds ~0 in the first word
  unsigned long long ukey[4];
  uint32_t ug_done;   // k_ug_ds_reg's blocks done (its last block runs the tail)
  uint32_t ug_tried;  // (speculative k_ug_ds_reg) the group was attempted
  uint32_t ug_go;     // (speculative) ug_spec_fits() of the kept spans, by the kept-list kernel
  uint32_t ug_pad2;
};
// Small.xh slots of the grid-agreement header. Every rank decides from these
// agreed words alone (never from its own lo / hi against them), so the ranks
// take the same branch: the grids agree iff min lo == max lo, min hi == max
// hi and both hashes are equal everywhere (the hashes are over word indices
// relative to each rank's own lo; equal lo makes them comparable)
enum { XH_ERR = 0, XH_GF0, XH_GF1, XH_FSTAR, XH_LO, XH_HI, XH_H1MIN, XH_H1MAX, XH_H2MIN, XH_H2MAX, XH_LOMAX, XH_HIMIN, XH_N };

// the agreement test on the agreed header (identical on every rank)
__host__ __device__ inline bool xh_grids_agree(const unsigned long long* xh) {
  return xh[XH_LO] == ~xh[XH_LOMAX] && ~xh[XH_HI] == xh[XH_HIMIN] && xh[XH_H1MIN] == ~xh[XH_H1MAX] &&
         xh[XH_H2MIN] == ~xh[XH_H2MAX];
}

static Small small_init() {
  Small init = {};
  init.err = ERR_NONE;
  init.range[0] = ~0ull;
  init.range[1] = 0;
  init.nan_t = ~0ull;
  init.bad_at = ~0ull;
  init.bound[0] = ~0ull;
  init.bound[1] = 0;
  init.bound[2] = 0;
  init.bound[3] = ~0ull;
  init.fap_key[0] = init.fap_key[2] = ~0ull;
  init.ls_key[0] = init.ls_key[2] = ~0ull;
  init.ukey[0] = init.ukey[2] = ~0ull;
  return init;
}
// the initial call state in device memory (a kernel argument by pointer: by
// value it made every call-end launch copy ~1 KB of kernel arguments)
static const Small* small_init_dev(Slot* ctx) {
  Buf& b = ctx->bufs["small_init"];
  if (!b.p) {
    const Small init = small_init();
    HIPCHK(hipMalloc(&b.p, sizeof init));
    b.n = sizeof init;
    HIPCHK(hipMemcpy(b.p, &init, sizeof init, hipMemcpyHostToDevice));
  }
  return (const Small*)b.p;
}
// Several MIN / MAX agreements on call-state fields as one MIN allreduce of a
// packed buffer (across GPUs each collective costs a latency of its own;
// one rank: the plain per-field calls)
// kind: 0 u64 MIN, 1 u64 MAX, 2 u32 MAX (written back to the field);
// 3 immediate MIN, 4 immediate MAX, 5 u64 field MIN, 6 u64 field MAX (left in
// the packed buffer only)
struct XField { void* p; uint8_t kind; uint64_t imm; };
constexpr uint32_t XM_MAX = 14;
struct XExtra { void* p; uint64_t count; XType t; XOp op; };
static void xchg_minmax(Slot* ctx, Xchg* X, const XField* f, uint32_t n, uint64_t* sum_u64 = nullptr,
                        uint64_t* buf = nullptr, const XExtra* extra = nullptr, uint32_t n_extra = 0);
// sharded double partials exchange rank-owned slices of G from this |G| on
// (below it, one allgather of every rank's partials is the cheaper collective)
constexpr uint64_t XSLICE_MIN_T = 65536;
static_assert(sizeof(Small) <= OUT_HDR - 8, "Small and the call's stamp must fit the output header");

// End of a call, after the finalize: the call state is snapshot ahead of the
// outputs (one D2H copy brings both back) and reset for the next call; the
// words of the grid points are cleared, which leaves the bitmap zero.
// Packing of small call-state fields for one MIN allreduce (a MAX field
// travels complemented): one thread moves up to 8 words in or out of a
// contiguous u64 buffer. kinds: 0 u64, 1 ~u64, 2 ~u32 (to u64); out: the same
// inverses.
struct XMove {
  uint32_t n;
  uint8_t kind[XM_MAX];
  uint64_t* buf;          // [n] the packed words
  void* field[XM_MAX];    // the call-state fields
  uint64_t imm[XM_MAX];   // kinds 3 / 4
  int32_t out;            // 0: fields -> buf, 1: buf -> fields
};
DEVI void xmove_one(const XMove& m, uint32_t i) {
  const uint8_t k = m.kind[i];
  const bool cpl = k == 1 || k == 2 || k == 4 || k == 6;  // MAX kinds travel complemented
  if (!m.out) {
    const uint64_t v = k == 2 ? (uint64_t)*(const uint32_t*)m.field[i]
                       : (k == 3 || k == 4) ? m.imm[i] : *(const uint64_t*)m.field[i];
    m.buf[i] = cpl ? ~v : v;
  } else if (k <= 2) {
    const uint64_t v = cpl ? ~m.buf[i] : m.buf[i];
    if (k == 2) *(uint32_t*)m.field[i] = (uint32_t)v;
    else *(uint64_t*)m.field[i] = v;
  }
}
DEVI void xmove_run(const XMove& m) {
  for (uint32_t i = 0; i < m.n; i++) xmove_one(m, i);
}
// a thread a field (one thread walking them paid a dependent round trip each:
// 6.7 us for the 12-field header)
__global__ void __launch_bounds__(64) k_xmove(XMove m) {
  if (threadIdx.x < m.n) xmove_one(m, threadIdx.x);
}

// (sum_u64: one more field, a u64 SUM, in the same collective group. The
// pack / unpack kernels stay outside the group: RCCL issues a group's
// collectives at its end.)
// the packing descriptor of xchg_minmax, for callers whose own kernels pack
// before (out = 0) and unpack after (out = 1) the group (xchg_group)
static XMove xchg_desc(Slot* ctx, const XField* f, uint32_t n, uint64_t* buf) {
  XMove m = {};
  m.n = n;
  m.buf = buf ? buf : scratch<uint64_t>(ctx, "x_pack", XM_MAX);
  for (uint32_t i = 0; i < n; i++) { m.kind[i] = f[i].kind; m.field[i] = f[i].p; m.imm[i] = f[i].imm; }
  return m;
}
static void xchg_group(Slot* ctx, Xchg* X, const XMove& m, uint64_t* sum_u64, const XExtra* extra, uint32_t n_extra) {
  X->group_start(ctx);
  X->allreduce(ctx, m.buf, m.n, X_U64, X_MIN);
  if (sum_u64) X->allreduce(ctx, sum_u64, 1, X_U64, X_SUM);
  for (uint32_t i = 0; i < n_extra; i++) X->allreduce(ctx, extra[i].p, extra[i].count, extra[i].t, extra[i].op);
  X->group_end(ctx);
}
static void xchg_minmax(Slot* ctx, Xchg* X, const XField* f, uint32_t n, uint64_t* sum_u64, uint64_t* buf,
                        const XExtra* extra, uint32_t n_extra) {
  XMove m = {};
  m.n = n;
  m.buf = buf ? buf : scratch<uint64_t>(ctx, "x_pack", XM_MAX);
  for (uint32_t i = 0; i < n; i++) { m.kind[i] = f[i].kind; m.field[i] = f[i].p; m.imm[i] = f[i].imm; }
  LAUNCH(k_xmove, dim3(1), dim3(64), 0, ctx->stream, m);
  X->group_start(ctx);
  X->allreduce(ctx, m.buf, n, X_U64, X_MIN);
  if (sum_u64) X->allreduce(ctx, sum_u64, 1, X_U64, X_SUM);
  for (uint32_t i = 0; i < n_extra; i++) X->allreduce(ctx, extra[i].p, extra[i].count, extra[i].t, extra[i].op);
  X->group_end(ctx);
  m.out = 1;
  LAUNCH(k_xmove, dim3(1), dim3(64), 0, ctx->stream, m);
}

// dst (global geometry [dst_lo, ...]) = src (a rank's bitmap over [src_lo,
// ...], src_lo >= dst_lo) shifted into place; bits outside src read as 0.
__global__ void __launch_bounds__(256) k_bitmap_remap(const uint32_t* src, uint64_t src_words, int64_t src_lo,
                                                      uint32_t* dst, uint64_t dst_words, int64_t dst_lo) {
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= dst_words) return;
  const int64_t sb = (int64_t)(32 * w) - (src_lo - dst_lo);  // src bit of dst bit 32 w
  const int64_t i0 = sb >= 0 ? sb / 32 : -((31 - sb) / 32);   // floor(sb / 32)
  const uint32_t sh = (uint32_t)(sb - 32 * i0);
  auto at = [&](int64_t i) { return i >= 0 && (uint64_t)i < src_words ? src[i] : 0u; };
  const uint32_t a = at(i0), b = at(i0 + 1);
  dst[w] = sh ? (a >> sh) | (b << (32 - sh)) : a;
}

// The call state to the host (host_publish) after a producer that could not
// publish it itself (a multi-block kernel, a collective).
__global__ void __launch_bounds__(64) k_publish(HostPub pub, const uint64_t* src) { host_publish(pub, src); }

// Groups of up to 1024 spans: the assembly (thread per span, then the
// deferred spans a wave each) and the kept-list compaction in one 1024-thread
// block, one launch instead of three.
__global__ void __launch_bounds__(1024) k_assemble_small(AssembleArgs a, KeptArgs K) {
  __shared__ uint32_t s_list[1024];
  __shared__ uint32_t s_n;
  const uint32_t t = threadIdx.x;
  if (t == 0) s_n = 0;
  __syncthreads();
  if (t < a.n_spans && assemble_fast_one(a, t)) s_list[atomicAdd(&s_n, 1u)] = t;
  __syncthreads();
  const uint32_t nd = s_n;
  for (uint32_t w = t / WAVE; w < nd; w += 1024 / WAVE) assemble_span_wave(a, s_list[w]);
  __syncthreads();  // (the block's global writes visible to the whole block)
  kept_compact_block(K);
}

// Groups of (nearly) single-row spans beyond one block (rows <= 2 x spans:
// C3's 1M series): a tile of 256 spans assembled (a thread a span, the
// block's waves walking the deferred ones, as k_assemble_small) and its kept
// sums in one launch, instead of k_assemble_fast, k_assemble and
// k_kept_tiles. The sums of the tile travel as one wave-reduced row per wave
// through LDS (one barrier).
__global__ void __launch_bounds__(256) k_assemble_tiles(AssembleArgs a, KeptTile* tile_sum, ulonglong2* tile_ke) {
  __shared__ uint32_t s_list[256];
  __shared__ uint32_t s_n;
  __shared__ uint64_t s_r[4][11];
  const uint32_t t = threadIdx.x, lane = lane_id(), w = t / WAVE;
  const uint32_t s = blockIdx.x * 256 + t;
  if (t == 0) s_n = 0;
  __syncthreads();
  if (s < a.n_spans && assemble_fast_one(a, s)) s_list[atomicAdd(&s_n, 1u)] = s;
  __syncthreads();
  const uint32_t nd = s_n;
  for (uint32_t i = w; i < nd; i += 256 / WAVE) assemble_span_wave(a, s_list[i]);
  if (nd) __syncthreads();  // (the block's global writes visible to the whole block)
  uint64_t sk = 0, se = 0, cnt = 0;
  int64_t f = INT64_MAX, l = INT64_MIN, fx = INT64_MIN, ln = INT64_MAX;
  UKeyAcc u;
  u.init();
  if (s < a.n_spans) {
    se = a.sp_cap[s];
    if (a.sp_kept[s]) {
      sk = 1;
      cnt = a.sp_ncells[s];
      f = fx = a.sp_first[s];
      l = ln = a.sp_last[s];
      if (a.u_key1) u.add(a.u_key1[s], a.u_key2[s]);
    }
  }
#pragma unroll
  for (int m = 1; m < WAVE; m <<= 1) {
    sk += shfl_xor_u64(sk, m);
    se += shfl_xor_u64(se, m);
    cnt += shfl_xor_u64(cnt, m);
    f = min(f, (int64_t)shfl_xor_u64((uint64_t)f, m));
    l = max(l, (int64_t)shfl_xor_u64((uint64_t)l, m));
    fx = max(fx, (int64_t)shfl_xor_u64((uint64_t)fx, m));
    ln = min(ln, (int64_t)shfl_xor_u64((uint64_t)ln, m));
  }
  if (a.u_key1) u.wave_reduce();
  if (lane == 0) {
    uint64_t* r = s_r[w];
    r[0] = sk; r[1] = se; r[2] = cnt; r[3] = (uint64_t)f; r[4] = (uint64_t)l; r[5] = (uint64_t)fx; r[6] = (uint64_t)ln;
    r[7] = u.a0; r[8] = u.a1; r[9] = u.b0; r[10] = u.b1;
  }
  __syncthreads();
  if (t == 0) {
    for (int i = 1; i < 4; i++) {
      const uint64_t* r = s_r[i];
      sk += r[0]; se += r[1]; cnt += r[2];
      f = min(f, (int64_t)r[3]); l = max(l, (int64_t)r[4]); fx = max(fx, (int64_t)r[5]); ln = min(ln, (int64_t)r[6]);
      u.a0 = min(u.a0, r[7]); u.a1 = max(u.a1, r[8]); u.b0 = min(u.b0, r[9]); u.b1 = max(u.b1, r[10]);
    }
    KeptTile o;
    o.k = sk; o.e = se; o.cnt = cnt; o.pad = 0;
    o.f = cnt ? f : INT64_MAX; o.l = cnt ? l : INT64_MIN; o.fx = cnt ? fx : INT64_MIN; o.ln = cnt ? ln : INT64_MAX;
    o.u = u;
    tile_sum[blockIdx.x] = o;
    tile_ke[blockIdx.x] = make_ulonglong2(sk, se);
  }
}

// Small unsharded calls also compute the lazy error index here (block 0,
// before the snapshot; bad.n_kept = 0: k_bad_index ran).
// (the optimistic aligned-group finish: `done` null, or the call is over only
// when *done; otherwise the state is snapshot for the host and left as it is)
// The call state's snapshot into mapped host memory and, with `init`, its
// reset: word by word over the block's threads, every thread of the block
// calling (one thread copying the ~1 KB across PCIe took most of a 10-12 us
// single-block launch)
static_assert(sizeof(Small) % 8 == 0, "Small is copied in 8-byte words");
// The call's stamp (the word after the snapshot, OUT_HDR - 8): the call's
// sequence number, stored last by thread 0 with a system-scope release once
// every thread's snapshot words are fenced. Every host-visible result of the
// call was written before it: the finalize's small results into the same
// mapped block and the reduce's long results into registered caller buffers
// by kernels that completed earlier in the stream, the aligned-group finish's
// results by this block before the fence. The host checks the stamp before it
// reads any of them (check_stamp).
DEVI void small_snap(Small* sm, Small* snap, const Small* init, uint64_t seq) {
  constexpr uint32_t NW = sizeof(Small) / 8;
  const volatile uint64_t* s = (const volatile uint64_t*)sm;
  uint64_t* d = (uint64_t*)snap;
  for (uint32_t i = threadIdx.x; i < NW; i += blockDim.x) d[i] = s[i];
  __threadfence_system();  // (the snapshot's host writes complete before this kernel does)
  __syncthreads();  // (every word read and fenced before any is reset, and before the stamp)
  if (threadIdx.x == 0)
    __hip_atomic_store((uint64_t*)((uint8_t*)snap + OUT_HDR - 8), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (!init) return;
  const uint64_t* in = (const uint64_t*)init;
  uint64_t* w = (uint64_t*)sm;
  for (uint32_t i = threadIdx.x; i < NW; i += blockDim.x) w[i] = in[i];
}
__global__ void __launch_bounds__(256) k_call_end(Small* sm, Small* snap, const Small* init, uint32_t* bitmap,
                                                  const uint32_t* grid, uint64_t T, int64_t lo, BadArgs bad,
                                                  uint64_t seq, const uint32_t* done = nullptr) {
  __shared__ unsigned long long s_min[4];
  if (done) {
    __shared__ uint64_t s_t;
    __shared__ uint32_t s_over;
    if (threadIdx.x == 0) {
      s_over = *(volatile const uint32_t*)done;
      s_t = sm->T;
    }
    __syncthreads();
    if (!s_over) {
      if (blockIdx.x == 0) small_snap(sm, snap, nullptr, seq);
      return;
    }
    T = s_t;
  }
  if (blockIdx.x == 0) {
    if (bad.n_kept) {
      unsigned long long m = ~0ull;
      for (uint32_t k = threadIdx.x; k < bad.n_kept; k += 256) m = min(m, (unsigned long long)bad_key(bad, k));
      for (int o = 1; o < WAVE; o <<= 1) m = min(m, (unsigned long long)shfl_xor_u64(m, o));
      if (lane_id() == 0) s_min[threadIdx.x / WAVE] = m;
      __syncthreads();
      if (threadIdx.x == 0) {
        m = min(min(s_min[0], s_min[1]), min(s_min[2], s_min[3]));
        if (m != ~0ull) atomicMin(&sm->bad_at, m);
        __threadfence();
      }
    }
    __syncthreads();  // (bad_at final)
    small_snap(sm, snap, init, seq);
    __syncthreads();  // (the ranks above read the bitmap cleared below)
  }
  if (bitmap)
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < T; i += (uint64_t)gridDim.x * 256)
      bitmap[(uint64_t)((int64_t)grid[i] - lo) >> 5] = 0u;
}

// ---- the optimistic aligned-group finish (no host round trip after the
// grid when the group turns out aligned; see spangroup_run) ----
// this rank's partials stand: every kept span in the one class, G its bucket
// sequence of at most 64 points, no float, no error
// (one thread; then, sharded, the agreement header packed for the group)
// (a whole wave: lane i packs field i; the validity is this wave's own value,
// not re-read from the call state)
DEVI void fap_valid_pack(Small* sm, uint32_t fap_ran, const XMove& pack, uint64_t T) {
  const bool v = fap_ran && sm->err == ERR_NONE && !sm->fap_broken && sm->fap_key[0] == sm->fap_key[1] &&
                 sm->fap_key[2] == sm->fap_key[3] && T > 0 && T <= WAVE && sm->gflags[0] == 0;
  const uint32_t lane = lane_id();
  if (lane == 0) sm->fap_valid = v ? 1ull : 0ull;
  if (lane < pack.n) {
    if (pack.field[lane] == (void*)&sm->fap_valid) pack.buf[lane] = v ? 1ull : 0ull;  // (kind 0: MIN, as is)
    else xmove_one(pack, lane);
  }
}
// this rank's 64-slot partials (k_fap_final64's reduce), its validity, the pack
template <int OP>
__global__ void __launch_bounds__(1024) k_fap_final64v(const int64_t* tmp, uint32_t n, uint32_t n_kept, int64_t* p_i,
                                                       uint32_t* p_cnt, Small* sm, XMove pack) {
  __shared__ int64_t s[16][WAVE];
  const int lane = lane_id();
  const uint32_t w = threadIdx.x / WAVE;
  int64_t acc = fap_rows_wave<OP>(tmp, w, 16, n);
  acc = fap_block_comb<OP>(acc, s);
  if (w == 0) {
    const uint64_t T = *(volatile const uint64_t*)&sm->T;
    const bool in = (uint64_t)lane < T;
    p_i[lane] = in ? acc : fap_neutral(OP);
    p_cnt[lane] = in ? n_kept : 0u;
    fap_valid_pack(sm, 1u, pack, T);
  }
}
// a rank without an aligned-group attempt: neutral partials for the exchange
__global__ void k_fap_neutral64(int64_t* p_i, uint32_t* p_cnt, int op, Small* sm, XMove pack) {
  p_i[threadIdx.x] = fap_neutral(op);
  p_cnt[threadIdx.x] = 0;
  fap_valid_pack(sm, 0u, pack, 0);
}
// The finalize of the (exchanged) 64-slot partials when the group stands
// everywhere (sharded: and every rank's grid is the global one; outputs at a
// fixed stride of 64: ts | bits | is_int), then k_call_end's `done` variant,
// in one block of 256 threads: the call state is snapshot, and reset with
// the bitmap cleared iff the group stood
template <int AGG>
__global__ void __launch_bounds__(256) k_fap_finish_end(Small* sm, const int64_t* p_i, const uint32_t* p_cnt,
                                                        FinalArgs f, int32_t sharded, XMove unpack, Small* snap,
                                                        const Small* init, uint32_t* bitmap, const uint32_t* grid, int64_t lo,
                                                        uint64_t seq) {
  __shared__ uint32_t s_ok, s_T;
  const uint32_t t = threadIdx.x;
  if (t < unpack.n) xmove_one(unpack, t);  // the agreed header back into the call state (sharded), a field a thread
  __syncthreads();
  if (t == 0) {
    bool ok = sm->fap_valid != 0 && sm->err == ERR_NONE && sm->gflags[0] == 0 && sm->T > 0 && sm->T <= WAVE;
    // (sharded: rank-independent: an empty grid anywhere makes lo's MIN / MAX
    // differ, ~0 vs a real lo; all empty fails T > 0 on every rank)
    if (sharded) ok = ok && xh_grids_agree(sm->xh);
    s_ok = ok ? 1u : 0u;
    s_T = (uint32_t)sm->T;
  }
  __syncthreads();
  if (!s_ok) {  // the group did not stand: the state stays for the usual path
    small_snap(sm, snap, nullptr, seq);
    return;
  }
  if (t < s_T) {
    Acc a;
    acc_init(a);
    a.cnt = p_cnt[t];
    a.ia = p_i[t];
    finalize_one<AGG, MODE_INT, false>(f, t, a);
  }
  __syncthreads();
  if (t == 0) sm->fap_done = 1;
  __syncthreads();
  small_snap(sm, snap, init, seq);
  __syncthreads();  // (the grid read below is this block's own)
  if (bitmap && t < s_T) bitmap[(uint64_t)((int64_t)grid[t] - lo) >> 5] = 0u;
}

// ---- the uniform path's aligned group in one launch (uniform_run) ----
// k_ds_reg's body with each block's 64 bucket partials combined by device
// atomics into one of `ncopy` copies (neutral on entry), then the tail in the
// launch's last block (the blocks count themselves done on Small.ug_done
// after their atomics are acknowledged): the copies combined (and reset), G
// from the class key (bucket b of every span: t0 + b kk step +
// floor(step (m_b - 1) / 2) over its m_b cells, Span.java:377-422), the
// group's validity; unsharded, also k_fap_finish_end's finish (the results
// into mapped host memory, the state snapshot + reset + stamp); sharded, the
// 64-slot partials and the agreement header for the exchange, the finish
// after it. One launch for k_ds_reg + k_fap_rows + k_fap_final64v
// (+ k_fap_finish_end).
constexpr uint32_t UG_NCOPY = 16;  // (4 a thread of the tail, loaded together)
__global__ void k_fill_u64(unsigned long long* p, uint32_t n, unsigned long long v) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}
struct UgTail {
  Small* sm;
  int op;        // the block combine (0 wrapping add, 1 min, 2 max)
  int agg;       // the cross-series aggregator (finalize)
  int32_t sharded;
  uint32_t n_kept, t0, step, kk, ncell, nb;
  uint32_t* grid;    // G (<= 64 points)
  int64_t* p_i;      // (sharded) the 64-slot partials for the exchange
  uint32_t* p_cnt;
  XMove pack;        // (sharded) the agreement header
  FinalArgs fo;      // (unsharded) the results into mapped host memory
  Small* snap;
  const Small* init;
  uint64_t seq;
  // (speculative, unsharded: the key, n_kept, kk and nb come from the call
  // state; a group that is not one leaves the state as the host would find it)
  uint32_t spec;
  int64_t interval;
};
template <typename T>
DEVI T coherent_load(const T* p) {  // (past any stale L2 line: the other blocks wrote by atomics)
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the tail of the launch the host sized (the key, n_kept, kk and nb in UgTail)
DEVI void ug_fap_tail(const FapArgs& fap, const UgTail& t) {
  __shared__ int64_t s_acc[4][WAVE];
  const uint32_t tid = threadIdx.x, lane = tid % WAVE, w = tid / WAVE;
  const int op = t.op;
  const int64_t neutral = fap_neutral(op);
  auto comb = [&](int64_t x, int64_t y) { return op == 0 ? ladd(x, y) : (op == 1 ? min(x, y) : max(x, y)); };
  int64_t acc = neutral;
  {  // (coherent loads, all in flight together; the copies reset to neutral after)
    int64_t v[UG_NCOPY / 4];
#pragma unroll
    for (uint32_t i = 0; i < UG_NCOPY / 4; i++)
      v[i] = (int64_t)coherent_load(fap.copies + (uint64_t)(w + 4 * i) * WAVE + lane);
#pragma unroll
    for (uint32_t i = 0; i < UG_NCOPY / 4; i++) {
      acc = comb(acc, v[i]);
      fap.copies[(uint64_t)(w + 4 * i) * WAVE + lane] = (unsigned long long)neutral;
    }
  }
  s_acc[w][lane] = acc;
  __syncthreads();
  Small* sm = t.sm;
  __shared__ uint32_t s_ok;
  if (w == 0) {
    acc = comb(comb(s_acc[0][lane], s_acc[1][lane]), comb(s_acc[2][lane], s_acc[3][lane]));
    const bool in = lane < t.nb;
    if (in) {
      const uint32_t sb = lane * t.kk, m = min(sb + t.kk, t.ncell) - sb;
      t.grid[lane] = t.t0 + sb * t.step + (uint32_t)((uint64_t)t.step * (m - 1) / 2);
    }
    const bool v = coherent_load(&sm->err) == ERR_NONE && !coherent_load(&sm->fap_broken) &&
                   coherent_load(&sm->fap_key[0]) == coherent_load(&sm->fap_key[1]) &&
                   coherent_load(&sm->fap_key[2]) == coherent_load(&sm->fap_key[3]) && t.nb > 0 && t.nb <= WAVE &&
                   coherent_load(&sm->gflags[0]) == 0;
    if (lane == 0) {
      sm->T = t.nb;
      sm->fap_valid = v ? 1ull : 0ull;
      s_ok = v ? 1u : 0u;
    }
    if (t.sharded) {
      t.p_i[lane] = in ? acc : neutral;
      t.p_cnt[lane] = in ? t.n_kept : 0u;
      if (lane < t.pack.n) {
        if (t.pack.field[lane] == (void*)&sm->fap_valid) t.pack.buf[lane] = v ? 1ull : 0ull;
        else xmove_one(t.pack, lane);
      }
    } else if (v && in) {
      Acc a;
      acc_init(a);
      a.cnt = t.n_kept;
      a.ia = acc;
      switch (t.agg) {
        case 1: finalize_one<1, MODE_INT, false>(t.fo, lane, a); break;
        case 2: finalize_one<2, MODE_INT, false>(t.fo, lane, a); break;
        case 3: finalize_one<3, MODE_INT, false>(t.fo, lane, a); break;
        default: finalize_one<0, MODE_INT, false>(t.fo, lane, a); break;
      }
    }
  }
  __syncthreads();
  if (t.sharded) return;
  // the finish: the results written, the state snapshot and, when the group
  // stood, reset (the host reads fap_done; else the general path runs)
  if (s_ok && tid == 0) sm->fap_done = 1;
  __syncthreads();
  small_snap(sm, t.snap, s_ok ? t.init : nullptr, t.seq);
}
// the speculative launch's tail (sharded): the verdict, key and counts from
// the call state
DEVI void ug_fap_tail_spec(const FapArgs& fap, const UgTail& t) {
  __shared__ int64_t s_acc[4][WAVE];
  const uint32_t tid = threadIdx.x, lane = tid % WAVE, w = tid / WAVE;
  // (the key's fields as locals: a copy of the UgTail, whose pack arrays are
  // indexed by lane, put the whole struct in scratch — 928 B a lane, the
  // launch 3x slower)
  uint32_t n_kept = t.n_kept, t0 = t.t0, step = t.step, kk0 = t.kk, ncell = t.ncell, nbk = t.nb;
  bool fits = true;
  if (t.spec) {
    Small* sm = t.sm;
    uint32_t nb = 0, kk = 0;
    fits = sm->ug_go != 0;
    ug_spec_fits(sm->ukey[0], sm->ukey[1], sm->ukey[2], sm->ukey[3], sm->n_kept, sm->err, t.interval, &nb, &kk);
    // (not one: this rank's partials neutral, its validity 0, as
    // k_fap_neutral64's; the exchange is every rank's)
    n_kept = fits ? (uint32_t)sm->n_kept : 0u;
    t0 = (uint32_t)(sm->ukey[0] >> 32);
    ncell = (uint32_t)sm->ukey[0];
    step = (uint32_t)(sm->ukey[2] >> 32);
    kk0 = fits ? kk : 1u;
    nbk = fits ? nb : 0u;
    if (tid == 0) sm->ug_tried = 1;
  }
  const int op = t.op;
  const int64_t neutral = fap_neutral(op);
  auto comb = [&](int64_t x, int64_t y) { return op == 0 ? ladd(x, y) : (op == 1 ? min(x, y) : max(x, y)); };
  int64_t acc = neutral;
  {  // (coherent loads, all in flight together; the copies reset to neutral after)
    int64_t v[UG_NCOPY / 4];
#pragma unroll
    for (uint32_t i = 0; i < UG_NCOPY / 4; i++)
      v[i] = (int64_t)coherent_load(fap.copies + (uint64_t)(w + 4 * i) * WAVE + lane);
#pragma unroll
    for (uint32_t i = 0; i < UG_NCOPY / 4; i++) {
      acc = comb(acc, v[i]);
      fap.copies[(uint64_t)(w + 4 * i) * WAVE + lane] = (unsigned long long)neutral;
    }
  }
  s_acc[w][lane] = acc;
  __syncthreads();
  Small* sm = t.sm;
  __shared__ uint32_t s_ok;
  if (w == 0) {
    acc = comb(comb(s_acc[0][lane], s_acc[1][lane]), comb(s_acc[2][lane], s_acc[3][lane]));
    const bool in = lane < nbk;
    if (in) {
      const uint32_t sb = lane * kk0, m = min(sb + kk0, ncell) - sb;
      t.grid[lane] = t0 + sb * step + (uint32_t)((uint64_t)step * (m - 1) / 2);
    }
    const bool v = coherent_load(&sm->err) == ERR_NONE && !coherent_load(&sm->fap_broken) &&
                   coherent_load(&sm->fap_key[0]) == coherent_load(&sm->fap_key[1]) &&
                   coherent_load(&sm->fap_key[2]) == coherent_load(&sm->fap_key[3]) && nbk > 0 && nbk <= WAVE &&
                   coherent_load(&sm->gflags[0]) == 0;
    if (lane == 0) {
      sm->T = nbk;
      sm->fap_valid = v ? 1ull : 0ull;
      s_ok = v ? 1u : 0u;
    }
    if (t.sharded) {
      t.p_i[lane] = in ? acc : neutral;
      t.p_cnt[lane] = in ? n_kept : 0u;
      if (lane < t.pack.n) {
        if (t.pack.field[lane] == (void*)&sm->fap_valid) {
          t.pack.buf[lane] = v ? 1ull : 0ull;
        } else if (t.spec && (lane == 4 || lane == 5 || lane == 10 || lane == 11)) {
          // (speculative: the class key's header words, uniform_run's fx[4, 5,
          // 10, 11], from the device key — ~0 / 0 for a rank without a group)
          const uint64_t a1 = fits ? sm->ukey[0] : ~0ull, a2 = fits ? sm->ukey[2] : 0ull;
          const uint64_t val = (lane == 4 || lane == 10) ? a1 : a2;
          t.pack.buf[lane] = t.pack.kind[lane] == 4 ? ~val : val;
        } else {
          xmove_one(t.pack, lane);
        }
      }
    } else if (v && in) {
      Acc a;
      acc_init(a);
      a.cnt = n_kept;
      a.ia = acc;
      switch (t.agg) {
        case 1: finalize_one<1, MODE_INT, false>(t.fo, lane, a); break;
        case 2: finalize_one<2, MODE_INT, false>(t.fo, lane, a); break;
        case 3: finalize_one<3, MODE_INT, false>(t.fo, lane, a); break;
        default: finalize_one<0, MODE_INT, false>(t.fo, lane, a); break;
      }
    }
  }
  __syncthreads();
  if (t.sharded) return;
  // the finish: the results written, the state snapshot and, when the group
  // stood, reset (the host reads fap_done; else the general path runs)
  if (s_ok && tid == 0) sm->fap_done = 1;
  __syncthreads();
  small_snap(sm, t.snap, s_ok ? t.init : nullptr, t.seq);
}
template <int AGG, bool SPEC>
#ifndef UG_LDS_CAP
#define UG_LDS_CAP 40960u  // (build knob) LDS a k_ug_ds_reg block claims: 40 KB = 4 blocks a CU
#endif
#ifndef UG_WPE
#define UG_WPE 0  // (build knob) waves per SIMD the register allocation aims at, 0: the compiler's choice
#endif
__global__ void __launch_bounds__(256)
#if UG_WPE
__attribute__((amdgpu_waves_per_eu(UG_WPE, UG_WPE)))
#endif
k_ug_ds_reg(DecodeArgs a, SpanDsArgs g, const uint32_t* ncells,
                                                   const uint32_t* vlen, FapArgs fap, UgTail t) {
  extern __shared__ uint8_t s_pad[];
  if (threadIdx.x == 0 && a.n_kept == 0xFFFFFFFFu) s_pad[0] = 1;
  if (SPEC && !sld(&t.sm->ug_go)) {
    // (speculative, no group: every block leaves at once — no counter; the
    // sharded tail, which packs this rank's neutral share, runs in block 0)
    if (t.sharded && blockIdx.x == 0) ug_fap_tail_spec(fap, t);
    return;
  }
  ds_reg_body<AGG, SPEC>(a, g, ncells, vlen, 0u, fap);
  __shared__ uint32_t s_last;
  __builtin_amdgcn_s_waitcnt(0);  // (this wave's atomics acknowledged)
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&t.sm->ug_done, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!s_last) return;
  // (two tails: the host-sized one is the code the unsharded C3* launch was
  // measured with — folding the speculative logic into it cost that launch
  // ~2.5 %, same box, through the whole kernel's code generation)
  if (SPEC) ug_fap_tail_spec(fap, t);
  else ug_fap_tail(fap, t);
}

// TSDBHIP_CHECK_CLEAN: counts non-zero words of a buffer (debug of the
// zero-on-entry invariants)
__global__ void k_count_nonzero(const uint32_t* p, uint64_t n, unsigned long long* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    if (p[i]) atomicAdd(out, 1ull);
}

// The device address of a host buffer registered mapped (tsdbhip_host_register)
// whose registration covers all `bytes` from h, or null (unregistered, or a
// registration shorter than the result: the caller copies D2H instead).
static void* mapped_dev_ptr(void* h, size_t bytes) {
  if (!h) return nullptr;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound((uintptr_t)h);
    if (it == g_reg.begin()) return nullptr;
    --it;
    if ((uintptr_t)h + bytes > it->first + it->second.n) return nullptr;
  }
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}

// grow-only scratch whose whole allocation is zero when `clean` (a new
// allocation, or a buffer the last call left dirty, is zeroed once, all of it)
template <typename T>
static T* scratch_zero_kept(Slot* ctx, const char* name, size_t count, bool clean) {
  T* p = scratch<T>(ctx, name, count);
  Buf& b = ctx->bufs[name];
  // (a grown buffer may come back at the same address: compare the size too)
  Buf& seen = ctx->zeroed[name];
  if (!clean || b.p != seen.p || b.n != seen.n) {
    HIPCHK(hipMemsetAsync(b.p, 0, b.n, ctx->stream));
    seen = b;
  }
  return p;
}

// per-t partial fields ([n][T] layout) under scratch names prefix + field
static void alloc_partials(Slot* ctx, ReduceArgs& r, const char* pre, uint64_t np, int agg) {
  auto nm = [&](const char* f) { return std::string(pre) + f; };
  r.p_cnt = scratch<uint32_t>(ctx, nm("cnt").c_str(), np);
  r.p_flag = scratch<uint8_t>(ctx, nm("flag").c_str(), np);
  r.p_i = scratch<int64_t>(ctx, nm("i").c_str(), np);
  r.p_d = scratch<double>(ctx, nm("d").c_str(), np);
  r.p_dhas = scratch<uint32_t>(ctx, nm("dhas").c_str(), np);
  r.p_wim = r.p_wiv = r.p_wdm = r.p_wdv = nullptr;
  if (agg == TSDBHIP_AGG_DEV) {
    r.p_wim = scratch<double>(ctx, nm("wim").c_str(), np);
    r.p_wiv = scratch<double>(ctx, nm("wiv").c_str(), np);
    r.p_wdm = scratch<double>(ctx, nm("wdm").c_str(), np);
    r.p_wdv = scratch<double>(ctx, nm("wdv").c_str(), np);
  }
}
// the fields acc_store writes for (agg, mode), at slot offset `off`, with the
// element type and the reduction an exchange applies to them
struct Fld { void* p; size_t esz; XType t; XOp op; };
static std::vector<Fld> partial_fields(const ReduceArgs& r, uint64_t off, int agg, int mode) {
  std::vector<Fld> v;
  v.push_back({r.p_cnt + off, 4, X_U32, X_SUM});
  if (mode == MODE_DUAL || agg == 1 || agg == 2) v.push_back({r.p_flag + off, 1, X_U8, X_MAX});
  if (mode != MODE_DBL && agg != 4)
    v.push_back({r.p_i + off, 8, agg == 1 ? X_I64 : agg == 2 ? X_I64 : X_U64,
                 agg == 1 ? X_MIN : agg == 2 ? X_MAX : X_SUM});
  if (mode != MODE_INT && agg != 4) v.push_back({r.p_d + off, 8, X_F64, X_SUM});
  if (mode != MODE_INT && (agg == 1 || agg == 2)) v.push_back({r.p_dhas + off, 4, X_U32, X_MAX});
  if (agg == 4) {
    if (mode != MODE_DBL) { v.push_back({r.p_wim + off, 8, X_F64, X_SUM}); v.push_back({r.p_wiv + off, 8, X_F64, X_SUM}); }
    if (mode != MODE_INT) { v.push_back({r.p_wdm + off, 8, X_F64, X_SUM}); v.push_back({r.p_wdv + off, 8, X_F64, X_SUM}); }
  }
  return v;
}

// ------------------------------------------------ the uniform path ----
// Every kept span one row on one cadence with one class key (x0, n, step,
// flags) proposed at assembly (ug_probe) — C3's and C3*'s series written in
// lockstep. The union grid is then that cadence (SpanGroup.java:510-608):
// no bitmap, no grid kernels, no second host round trip. Two variants:
//
//  * lockstep (no downsampling): k_lockstep streams every span's qualifiers
//    and values once, proving the cadence as it reduces; G is written by its
//    chunk-0 waves. Sharded, the ranks agreed on the key before the host's
//    round trip (one MIN allreduce of the packed key words, issued by every
//    rank for such a query), so every rank sizes G alike; the partials then
//    travel in one collective group with the broken flag and the input count.
//    Collectives: 2. A qualifier off the proposal: RC_REDO (the proven path).
//  * aligned group (downsampled integer sum / min / max / avg): k_ds_reg's
//    block partials, G from the key, and the optimistic finish of the
//    general path (k_fap_finish_end), the key agreed in the partials' group.
//    Collectives: 1. A group that does not stand anywhere: RC_UG_FALLBACK
//    (the call state reset; the general path runs the call).
//  * E (unsharded, other downsampled queries: doubles, dev, > 64 buckets,
//    spans of many rows — C2): k_ds_reg writes each span's bucket values on
//    the key's buckets and G; k_ug_reduce reads span k at g as E_k[g]. A span
//    off the cadence: RC_UG_FALLBACK after the call (results dropped).
constexpr int RC_REDO = 1000;  // a lockstep proposal did not hold: the proven path runs the call
constexpr int RC_UG_FALLBACK = 1001;
struct UgIn {
  const tsdbhip_sg_desc* d;
  Xchg* X;
  Small* sm;
  DecodeArgs da;  // (the aligned group: k_ds_reg's inputs, E of the call)
  const uint32_t* row_ncells;
  const uint32_t* row_val_len;
  const uint64_t* uk_vo;  // [n_kept] row offsets of the kept spans (k_lockstep)
  const uint64_t* uk_qo;
  uint32_t n_kept;
  uint64_t k1, k2;  // the class key (agreed, sharded lockstep)
  bool lockstep;     // else the aligned group
  bool mine;         // (aligned group) this rank's spans make the attempt
  bool dev;          // (lockstep, unsharded) integer dev: the chains of k_ug_dev
  bool e;            // (unsharded, downsampled) k_ds_reg's E + k_reduce's aligned spans
  bool spec;         // (aligned group, sharded) launched before the host read the call state:
                     // n_kept is the span count, the group's verdict and key come from the device
};

// The E variant's pieces a span (at most `want`): k_ds_reg's wave p takes
// rows [p rp, (p + 1) rp), rp = ceil(rows / pieces), and needs its first
// cell on a bucket head (cell index % kk == 0) — else the span is an
// outsider and the call falls back. The rows of a span on the key are its
// hourly rows (Const.MAX_TIMESPAN, RowKey base times: multiples of 3600 s)
// holding a cell of t0 + c step, c < n; the largest aligned count wins (1
// always is). A layout other than hourly rows only makes the device check
// refuse the pieces, as before (45-min or 3-h buckets over hourly
// 1-s rows).
#ifndef UG_DEV_GP
#define UG_DEV_GP 16u  // k_ug_dev: grid points (chains) a block
#endif
static uint32_t ug_e_pieces(uint32_t t0, uint32_t step, uint32_t n, uint32_t kk, uint32_t want) {
  if (want <= 1 || !step || !kk || n == 0) return 1;
  const uint64_t last = (uint64_t)t0 + (uint64_t)(n - 1) * step;
  const uint64_t b0 = t0 - t0 % 3600u, nb = (last - b0) / 3600 + 1;
  if (nb > (1u << 16)) return 1;
  std::vector<uint64_t> cell0;  // first cell of each non-empty row
  cell0.reserve(nb);
  for (uint64_t i = 0; i < nb; i++) {
    const uint64_t B = b0 + 3600 * i;
    const uint64_t c = B <= t0 ? 0 : (B - t0 + step - 1) / step;
    if (c < n && (cell0.empty() || cell0.back() != c)) cell0.push_back(c);
  }
  const uint64_t R = cell0.size();
  for (uint32_t P = (uint32_t)std::min<uint64_t>(want, R); P > 1; P--) {
    const uint64_t rp = (R + P - 1) / P;
    bool ok = true;
    for (uint64_t p = 1; p < P && p * rp < R && ok; p++) ok = cell0[p * rp] % kk == 0;
    if (ok) return P;
  }
  return 1;
}

// the aligned group (k_ug_ds_reg; sharded: one collective group and
// k_fap_finish_end); RC_UG_FALLBACK when the group did not stand
static int ug_aligned_group(Slot* ctx, const UgIn& u, tsdbhip_sg_out* out, tsdbhip_timing& tm) {
  const tsdbhip_sg_desc* d = u.d;
  Xchg* X = u.X;
  const bool sharded = X != nullptr;
  Small* sm = u.sm;
  hipStream_t st = ctx->stream;
  const int agg = d->agg;
  const uint32_t n = (uint32_t)u.k1, x0 = (uint32_t)(u.k1 >> 32);
  const uint32_t n_kept = u.n_kept;
  const uint32_t step = (uint32_t)(u.k2 >> 32);
  Small h;
  // ---- aligned group ----
  const int32_t I = d->ds_interval;
  // (a rank making no attempt may hold no key: step 0; speculative: the
  // device's key)
  const uint32_t kk = u.mine && !u.spec ? (uint32_t)(((int64_t)I + step - 1) / step) : 1u;
  const uint32_t nb = u.mine && !u.spec ? (n + kk - 1) / kk : 0u;
  const int fop = agg == TSDBHIP_AGG_MIN ? 1 : (agg == TSDBHIP_AGG_MAX ? 2 : 0);
  uint32_t* gridv = scratch<uint32_t>(ctx, "grid", WAVE);
  int64_t* o_pi = scratch<int64_t>(ctx, "fo_i", WAVE);
  uint32_t* o_pc = scratch<uint32_t>(ctx, "fo_cnt", WAVE);
  // the agreement header of the general path's optimistic finish, with the
  // class key in the grid-geometry words: xh_grids_agree() holds iff every
  // rank made the attempt on the same key
  const uint64_t a1 = u.mine ? u.k1 : ~0ull, a2 = u.mine ? u.k2 : 0ull;
  const XField fx[XH_N + 1] = {{&sm->err, 0, 0},  {&sm->gflags[0], 2, 0}, {&sm->gflags[1], 2, 0},
                               {&sm->fstar, 1, 0}, {nullptr, 3, a1},       {nullptr, 4, a2},
                               {nullptr, 3, 0},    {nullptr, 4, 0},        {nullptr, 3, 0},
                               {nullptr, 4, 0},    {nullptr, 4, a1},       {nullptr, 3, a2},
                               {&sm->fap_valid, 0, 0}};
  XMove pack = {};
  if (sharded) pack = xchg_desc(ctx, fx, XH_N + 1, (uint64_t*)sm->xh);
  XMove unpack = pack;
  unpack.out = 1;
  map_out_reserve(ctx, OUT_HDR + 17 * WAVE);
  const uint64_t end_seq = ++ctx->pub_seq;
  FinalArgs fo;
  std::memset(&fo, 0, sizeof fo);
  fo.T = WAVE;
  fo.n_chunks = 1;
  fo.grid = gridv;
  fo.out_ts = (int64_t*)(ctx->map_out_dev + OUT_HDR);
  fo.out_bits = fo.out_ts + WAVE;
  fo.out_isint = (uint8_t*)(fo.out_bits + WAVE);
  fo.nan_t = &sm->nan_t;
  Small* snap = (Small*)ctx->map_out_dev;
  const Small* ini = small_init_dev(ctx);
  if (!u.mine) {
    LAUNCH(k_fap_neutral64, dim3(1), dim3(WAVE), 0, st, o_pi, o_pc, fop, sm, pack);
  } else {
    // k_ds_reg, a wave a span, in the aligned group's mode, with the tail
    // in its last block (k_ug_ds_reg)
    const uint32_t rblocks = (n_kept + 3) / 4;
    SpanDsArgs gr = {};
    gr.nseg = CK_NSEG;
    gr.seg_cap = 4u * ((rblocks + CK_NSEG - 1) / CK_NSEG);
    gr.list = scratch<uint32_t>(ctx, "cr_list", (uint64_t)gr.seg_cap * CK_NSEG);
    gr.list_count = sm->seg2;
    gr.rate = 0;
    FapArgs fa = {};
    fa.op = fop;
    fa.key = sm->fap_key;
    fa.broken = &sm->fap_broken;
    fa.nrows = rblocks;
    fa.ncopy = UG_NCOPY;
    if (u.spec) {
      fa.spec_n_kept = &sm->n_kept;
      fa.spec_go = &sm->ug_go;
    }
    {  // the copies, neutral on entry (left neutral by every tail; a new allocation filled once)
      static const char* names[3] = {"ug_copies0", "ug_copies1", "ug_copies2"};
      fa.copies = scratch<unsigned long long>(ctx, names[fop], (uint64_t)UG_NCOPY * WAVE);
      Buf& b = ctx->bufs[names[fop]];
      Buf& seen = ctx->zeroed[names[fop]];
      if (b.p != seen.p || b.n != seen.n) {
        LAUNCH(k_fill_u64, dim3(UG_NCOPY), dim3(WAVE), 0, st, fa.copies, UG_NCOPY * WAVE,
               (unsigned long long)(fop == 1 ? INT64_MAX : (fop == 2 ? INT64_MIN : 0)));
        seen = b;
      }
    }
    UgTail t = {};
    t.sm = sm; t.op = fop; t.agg = agg; t.sharded = sharded ? 1 : 0;
    t.n_kept = n_kept; t.t0 = x0; t.step = step; t.kk = kk; t.ncell = n; t.nb = nb;
    t.grid = gridv; t.p_i = o_pi; t.p_cnt = o_pc; t.pack = pack; t.fo = fo; t.snap = snap; t.init = ini;
    t.seq = end_seq;
    t.spec = u.spec ? 1u : 0u;
    t.interval = I;
    auto reg = [&](auto aggc) {
      constexpr int A = decltype(aggc)::value;
      static const unsigned stat_lds = [] {
        hipFuncAttributes at = {};
        return hipFuncGetAttributes(&at, (const void*)k_ug_ds_reg<A, false>) == hipSuccess
                   ? (unsigned)at.sharedSizeBytes
                   : 21000u;
      }();
      const unsigned pad = stat_lds < UG_LDS_CAP ? UG_LDS_CAP - stat_lds : 0u;
      EV_START(ctx, 8);
      if (u.spec)
        LAUNCH_STOP(EV_STOP_K(ctx, 9), (k_ug_ds_reg<A, true>), dim3(rblocks), dim3(256), pad, st, u.da, gr,
                    u.row_ncells, u.row_val_len, fa, t);
      else
        LAUNCH_STOP(EV_STOP_K(ctx, 9), (k_ug_ds_reg<A, false>), dim3(rblocks), dim3(256), pad, st, u.da, gr,
                    u.row_ncells, u.row_val_len, fa, t);
      EV_STOP_M(ctx, 9);
    };
    switch (d->ds_agg) {
      case 0: reg(std::integral_constant<int, 0>()); break;
      case 1: reg(std::integral_constant<int, 1>()); break;
      case 2: reg(std::integral_constant<int, 2>()); break;
      default: reg(std::integral_constant<int, 3>()); break;
    }
    ctx->hot_kernel = TSDBHIP_HOT_UG_DS_REG;
  }
  if (sharded) {
    // the agreement, the validity (MIN) and the 64-slot partials: one
    // collective group; then the finish
    const XExtra ex[2] = {{o_pi, WAVE, fop ? X_I64 : X_U64, fop == 1 ? X_MIN : (fop == 2 ? X_MAX : X_SUM)},
                          {o_pc, WAVE, X_U32, X_SUM}};
    xchg_group(ctx, X, pack, (uint64_t*)&sm->n_input, ex, 2);
    auto fin = [&](auto aggc) {
      constexpr int A = decltype(aggc)::value;
      LAUNCH(k_fap_finish_end<A>, dim3(1), dim3(256), 0, st, sm, (const int64_t*)o_pi, (const uint32_t*)o_pc, fo,
             (int32_t)1, unpack, snap, ini, (uint32_t*)nullptr, (const uint32_t*)gridv, (int64_t)0, end_seq);
    };
    if (agg == TSDBHIP_AGG_MIN) fin(std::integral_constant<int, 1>());
    else if (agg == TSDBHIP_AGG_MAX) fin(std::integral_constant<int, 2>());
    else if (agg == TSDBHIP_AGG_AVG) fin(std::integral_constant<int, 3>());
    else fin(std::integral_constant<int, 0>());
  }
  EV_FINAL(ctx, 5);
  HIPCHK(hipStreamSynchronize(st));
  check_stamp(ctx, end_seq);
  tm.late_stamp = ctx->timing_late;
  std::memcpy(&h, ctx->map_out, sizeof h);
  if (!h.fap_done) {
    // the group did not stand (somewhere): the call state back to its
    // initial values, the general path runs the call
    const uint64_t seq2 = ++ctx->pub_seq;
    LAUNCH(k_call_end, dim3(1), dim3(256), 0, st, sm, (Small*)ctx->map_out_dev, ini, (uint32_t*)nullptr,
           (const uint32_t*)nullptr, (uint64_t)0, (int64_t)0, BadArgs{}, seq2, (const uint32_t*)nullptr);
    HIPCHK(hipStreamSynchronize(st));
    check_stamp(ctx, seq2);
    ctx->sm_ready = true;
    return RC_UG_FALLBACK;
  }
  ctx->sm_ready = true;
  const uint64_t T = h.T;
  out->n_input_points = h.n_input;
  tm.n_grid = T;
  tm.paths |= TSDBHIP_PATH_ALIGNED_GROUP;
  if (sharded) {
    tm.n_collectives = X->n_coll;
    tm.x_bytes = X->x_bytes;
  }
  if (ctx->hot_kernel) tm.hot_ms = ev_ms(ctx, 8, 9);
  tm.hot_kernel = ctx->hot_kernel;
  tm.total_ms = ev_ms(ctx, 0, 5);
  tm.n_emitted = T * h.n_kept;
  ctx->timing = tm;
  if (T > out->capacity && ctx->want_output) {
    out->err_code = TSDBHIP_E_CAPACITY;
    return TSDBHIP_E_CAPACITY;
  }
  if (ctx->want_output) {
    const uint8_t* hb = ctx->map_out;
    std::memcpy(out->ts, hb + OUT_HDR, T * 8);
    std::memcpy(out->bits, hb + OUT_HDR + 8 * WAVE, T * 8);
    std::memcpy(out->is_int, hb + OUT_HDR + 16 * WAVE, T);
  }
  out->n_out = T;
  out->err_code = TSDBHIP_OK;
  out->err_index = -1;
  return TSDBHIP_OK;
}

// the E variant's launches: k_ds_reg in E mode, then k_ug_reduce
static void ug_e_launch(Slot* ctx, const UgIn& u, uint64_t T, uint32_t e_kk, int mode, uint32_t* gridv,
                        const FinalArgs& fin) {
  const tsdbhip_sg_desc* d = u.d;
  Small* sm = u.sm;
  hipStream_t st = ctx->stream;
  const int agg = d->agg;
  const uint32_t n = (uint32_t)u.k1, x0 = (uint32_t)(u.k1 >> 32), step = (uint32_t)(u.k2 >> 32);
  const uint32_t n_kept = u.n_kept;
  // k_ds_reg in E mode (its block 0 writes G from the key, the spans their
  // bucket values; an outsider sets the broken flag), then k_ug_reduce:
  // every span's E is G itself (no bitmap, no grid ranks, no cursors)
  ctx->hot_kernel = TSDBHIP_HOT_DS_E;
  const uint64_t rps = d->n_rows / std::max<uint32_t>(n_kept, 1);
  const uint32_t wps_log2 = rps >= 12 ? 2 : (rps >= 6 ? 1 : 0);
  // (waves a span, its rows in contiguous pieces: C2's 24 rows a span, 0.266
  // ms a step with 3 pieces, 0.269 with 2, 0.281 with 4, 0.290 with 1,
  // 0.310 with 8, 0.489 with 24 — same box)
  uint32_t pieces = ug_e_pieces(x0, step, n, e_kk, (uint32_t)std::max<uint64_t>(1, rps / 8));
  if (const char* e = getenv("TSDBHIP_UG_P")) pieces = (uint32_t)std::max(1, atoi(e));  // (A/B runs)
  const uint32_t rblocks = (uint32_t)(((uint64_t)n_kept * pieces + 3) / 4);
  SpanDsArgs gr = {};
  gr.nseg = CK_NSEG;
  FapArgs fa = {};
  fa.op = -1;
  fa.broken = &sm->ls_broken;
  fa.ug_grid = gridv;
  fa.ug_t0 = x0; fa.ug_step = step; fa.ug_kk = e_kk; fa.ug_n = n; fa.ug_pieces = pieces;
  auto reg = [&](auto aggc) {
    constexpr int A = decltype(aggc)::value;
    static const unsigned stat_lds = [] {
      hipFuncAttributes at = {};
      return hipFuncGetAttributes(&at, (const void*)k_ds_reg<A>) == hipSuccess ? (unsigned)at.sharedSizeBytes
                                                                               : 18960u;
    }();
    const unsigned pad = pieces == 1 ? (stat_lds < 40960u ? 40960u - stat_lds : 0u) : 0u;
    EV_START(ctx, 8);
    LAUNCH_STOP(EV_STOP_K(ctx, 9), (k_ds_reg<A>), dim3(rblocks), dim3(256), pad, st, u.da, gr, u.row_ncells,
                u.row_val_len, wps_log2, fa);
    EV_STOP_M(ctx, 9);
  };
  switch (d->ds_agg) {
    case 0: reg(std::integral_constant<int, 0>()); break;
    case 1: reg(std::integral_constant<int, 1>()); break;
    case 2: reg(std::integral_constant<int, 2>()); break;
    default: reg(std::integral_constant<int, 3>()); break;
  }
  // (integer dev: one span-ordered chunk, Aggregators.java:196-217; else
  // chunks of 64 spans, merged in chunk order by the finalize)
  const bool seq = agg == TSDBHIP_AGG_DEV && mode != MODE_DBL;
  const uint32_t spc = seq ? std::max<uint32_t>(n_kept, 1) : 64u;
  ReduceArgs re;
  std::memset(&re, 0, sizeof re);
  re.e_off = u.da.e_off; re.e_val = u.da.e_val; re.n_kept = n_kept; re.grid = gridv; re.T = T;
  re.spans_per_chunk = spc;
  re.n_chunks = (n_kept + spc - 1) / spc;
  alloc_partials(ctx, re, "p_", (uint64_t)re.n_chunks * T, agg);
  FinalArgs fe = fin;
  fe.n_chunks = re.n_chunks;
  dispatch_ug_reduce(ctx, agg, mode, re, fe);
}

// the sharded lockstep group: this rank's lockstep partials combined, the
// exchange (exact integers: an allreduce a field; doubles: every rank's slot
// gathered and merged in rank order), then the finalize
static void ug_lockstep_sharded(Slot* ctx, const UgIn& u, uint64_t T, int mode, unsigned blocks, ReduceArgs& r,
                                const LsPlan& lsp, const FinalArgs& f, const FinalArgs& fin) {
  Xchg* X = u.X;
  Small* sm = u.sm;
  const int agg = u.d->agg;
  const bool rate = u.d->rate != 0;
  const uint32_t n_chunks = r.n_chunks;
  const int nr = X->nranks, rk = X->rank;
  dispatch_lockstep(ctx, agg, rate, blocks, r, lsp, f, false);
  ReduceArgs src;
  uint32_t n_src = 1;
  if (mode == MODE_INT) {  // exact integer partials: one allreduce a field
    ReduceArgs mine = r;
    alloc_partials(ctx, mine, "m_", T, agg);
    dispatch_combine(ctx, agg, mode, r, mine, T, n_chunks);
    X->group_start(ctx);
    for (const Fld& fl : partial_fields(mine, 0, agg, mode)) X->allreduce(ctx, fl.p, T, fl.t, fl.op);
    X->allreduce(ctx, &sm->ls_broken, 1, X_U32, X_MAX);
    X->allreduce(ctx, &sm->n_input, 1, X_U64, X_SUM);
    X->group_end(ctx);
    src = mine;
  } else {  // doubles: every rank's slot gathered, merged in rank order
    ReduceArgs all = r;
    alloc_partials(ctx, all, "x_", (uint64_t)nr * T, agg);
    ReduceArgs mine = all;
    const uint64_t off = (uint64_t)rk * T;
    mine.p_cnt += off; mine.p_flag += off; mine.p_i += off; mine.p_d += off; mine.p_dhas += off;
    if (agg == TSDBHIP_AGG_DEV) { mine.p_wim += off; mine.p_wiv += off; mine.p_wdm += off; mine.p_wdv += off; }
    dispatch_combine(ctx, agg, mode, r, mine, T, n_chunks);
    const std::vector<Fld> fm = partial_fields(mine, 0, agg, mode), fa = partial_fields(all, 0, agg, mode);
    X->group_start(ctx);
    for (size_t i = 0; i < fm.size(); i++) X->allgather(ctx, fm[i].p, fa[i].p, T * fm[i].esz);
    X->allreduce(ctx, &sm->ls_broken, 1, X_U32, X_MAX);
    X->allreduce(ctx, &sm->n_input, 1, X_U64, X_SUM);
    X->group_end(ctx);
    src = all;
    n_src = (uint32_t)nr;
  }
  FinalArgs ff = fin;
  ff.n_chunks = n_src;
  src.n_chunks = n_src;
  dispatch_final(ctx, agg, mode, rate, src, ff);
}

static int uniform_run(Slot* ctx, const UgIn& u, tsdbhip_sg_out* out, tsdbhip_timing& tm) {
  const tsdbhip_sg_desc* d = u.d;
  Xchg* X = u.X;
  const bool sharded = X != nullptr;
  Small* sm = u.sm;
  hipStream_t st = ctx->stream;
  const bool rate = d->rate != 0;
  const int agg = d->agg;
  const uint32_t n = (uint32_t)u.k1, x0 = (uint32_t)(u.k1 >> 32);
  const uint32_t q0 = (uint32_t)(u.k2 & 0xFFFFu), step = (uint32_t)(u.k2 >> 32);
  const uint32_t n_kept = u.n_kept;
  Small h;
  tm.paths |= TSDBHIP_PATH_UNIFORM;
  if (!u.lockstep && !u.e) return ug_aligned_group(ctx, u, out, tm);

  // ---- lockstep, E ----
  const uint32_t e_kk = u.e ? (uint32_t)(((int64_t)d->ds_interval + step - 1) / step) : 0u;
  const uint64_t T = u.e ? (n + e_kk - 1) / e_kk : (rate ? n - 1 : n);
  const bool flt = (q0 & 8u) != 0;
  const int mode = (rate || flt) ? MODE_DBL : MODE_INT;
  uint32_t* gridv = scratch<uint32_t>(ctx, "grid", T);
  const bool small_out = T * 17 <= (256u << 10) && ctx->want_output;
  map_out_reserve(ctx, OUT_HDR + (small_out ? 17 * T : 0));
  uint8_t* outblk = small_out ? ctx->map_out_dev : scratch<uint8_t>(ctx, "outblk", OUT_HDR + 17 * T);
  FinalArgs fin;
  std::memset(&fin, 0, sizeof fin);
  fin.T = T;
  fin.n_chunks = 1;
  fin.grid = gridv;
  fin.rate = rate;
  fin.out_ts = (int64_t*)(outblk + OUT_HDR);
  fin.out_bits = fin.out_ts + T;
  fin.out_isint = (uint8_t*)(fin.out_bits + T);
  fin.nan_t = &sm->nan_t;
  // tiles of LS_TILE grid points x chunks of spans (as the general path's ls_reduce)
  const uint32_t n_tiles = (uint32_t)((T + LS_TILE - 1) / LS_TILE);
  uint64_t want = std::max<uint64_t>(1, 16384 / n_tiles);
  want = std::min<uint64_t>(want, std::max<uint32_t>(1, n_kept / LS_MIN_SPC));
  const uint32_t spc = (uint32_t)((n_kept + want - 1) / want);
  const uint32_t n_chunks_s = (n_kept + spc - 1) / spc;
  const uint32_t n_chunks = (n_chunks_s + LS_GROUP - 1) / LS_GROUP;  // (a block's chunks merged in LDS)
  ReduceArgs r;
  std::memset(&r, 0, sizeof r);
  r.T = T;
  r.n_chunks = n_chunks;
  r.n_kept = n_kept;
  if (!u.e) alloc_partials(ctx, r, "p_", (uint64_t)n_chunks * T, agg);
  LsPlan lsp = {};
  lsp.a.d_voff = u.uk_vo;
  lsp.a.d_qoff = u.uk_qo;
  lsp.a.val = u.da.val;
  lsp.a.qual = u.da.qual;
  lsp.a.n = n;
  lsp.a.q0 = q0;
  lsp.a.step = step;
  lsp.a.broken = &sm->ls_broken;
  lsp.a.spc = spc;
  lsp.a.n_tiles = n_tiles;
  lsp.a.n_chunks = n_chunks_s;
  lsp.a.grid_out = gridv;
  lsp.a.x0 = x0;
  lsp.a.g_off = rate ? 1u : 0u;
  lsp.w8 = (q0 & 7u) == 7u;
  lsp.flt = flt;
  if (!u.dev && !u.e) tm.paths |= TSDBHIP_PATH_LOCKSTEP;
  ctx->hot_kernel = TSDBHIP_HOT_LOCKSTEP;
  const unsigned blocks = n_tiles * n_chunks;
  FinalArgs f = fin;
  f.n_chunks = n_chunks;
  if (u.e) {
    ug_e_launch(ctx, u, T, e_kk, mode, gridv, fin);
  } else if (u.dev) {  // integer dev: one sequential chain a grid point (k_ug_dev)
    ctx->hot_kernel = TSDBHIP_HOT_UG_DEV;
    EV_START(ctx, 8);
    constexpr uint32_t GP = UG_DEV_GP;  // (grid points a block)
    if (lsp.w8)
      LAUNCH_STOP(EV_STOP_K(ctx, 9), (k_ug_dev<8, GP>), dim3((unsigned)((T + GP - 1) / GP)), dim3(64 * (2 + UG_DEV_NP)), 0, st,
                  u.da.val, u.uk_vo, u.da.qual, u.uk_qo, q0, &sm->ls_broken, n_kept, T, gridv, x0, step, fin);
    else
      LAUNCH_STOP(EV_STOP_K(ctx, 9), (k_ug_dev<4, GP>), dim3((unsigned)((T + GP - 1) / GP)), dim3(64 * (2 + UG_DEV_NP)), 0, st,
                  u.da.val, u.uk_vo, u.da.qual, u.uk_qo, q0, &sm->ls_broken, n_kept, T, gridv, x0, step, fin);
    EV_STOP_M(ctx, 9);
  } else if (!sharded) {
    dispatch_lockstep(ctx, agg, rate, blocks, r, lsp, f, true);
  } else {
    ug_lockstep_sharded(ctx, u, T, mode, blocks, r, lsp, f, fin);
  }
  const uint64_t end_seq = ++ctx->pub_seq;
  LAUNCH(k_call_end, dim3(1), dim3(256), 0, st, sm, (Small*)ctx->map_out_dev, small_init_dev(ctx), (uint32_t*)nullptr,
         (const uint32_t*)nullptr, (uint64_t)0, (int64_t)0, BadArgs{}, end_seq, (const uint32_t*)nullptr);
  EV_FINAL(ctx, 5);
  HIPCHK(hipStreamSynchronize(st));
  check_stamp(ctx, end_seq);
  tm.late_stamp = ctx->timing_late;
  const uint8_t* hb = ctx->map_out;
  std::memcpy(&h, hb, sizeof h);
  ctx->sm_ready = true;
  if (h.ls_broken) {  // (agreed over the ranks) the proposal did not hold: the proven path runs the call
    ctx->timing = tm;
    return u.e ? RC_UG_FALLBACK : RC_REDO;
  }
  out->n_input_points = h.n_input;
  if (sharded) {
    tm.n_collectives = X->n_coll;
    tm.x_bytes = X->x_bytes;
  }
  tm.n_grid = T;
  if (ctx->hot_kernel) tm.hot_ms = ev_ms(ctx, 8, 9);
  tm.hot_kernel = ctx->hot_kernel;
  tm.total_ms = ev_ms(ctx, 0, 5);
  tm.n_emitted = u.e ? T * n_kept : 0;
  ctx->timing = tm;
  uint64_t n_ok = T;
  int code = TSDBHIP_OK;
  int64_t err_at = -1;
  if (h.nan_t != ~0ull) {
    err_at = (int64_t)h.nan_t;
    code = TSDBHIP_E_NAN_INF;
    n_ok = (uint64_t)err_at;
  }
  if (n_ok > out->capacity && ctx->want_output) {
    out->err_code = TSDBHIP_E_CAPACITY;
    return TSDBHIP_E_CAPACITY;
  }
  if (!ctx->want_output) {
  } else if (n_ok && small_out) {
    std::memcpy(out->ts, hb + OUT_HDR, n_ok * 8);
    std::memcpy(out->bits, hb + OUT_HDR + 8 * T, n_ok * 8);
    std::memcpy(out->is_int, hb + OUT_HDR + 16 * T, n_ok);
  } else if (n_ok) {
    HIPCHK(hipMemcpyAsync(out->ts, fin.out_ts, n_ok * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(out->is_int, fin.out_isint, n_ok, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(out->bits, fin.out_bits, n_ok * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  out->n_out = n_ok;
  out->err_code = code;
  out->err_index = err_at;
  return code;
}

// ------------------------------------------------------- the hot path ----
// One call of the general path (and the entry of the uniform path), as the
// stages the call runs in order, sharing the call's state as members:
//   begin           flags, the inputs in HBM, the call state
//   assemble        Span.addRow / RowSeq.addRow, the keep rule, the kept list
//                   (and the uniform path's class keys)
//   sync1           the first host round trip (the speculative sharded
//                   aligned group instead, which ends the call)
//   plan            the union grid's range, the aligned-group plan, E
//   uniform_try     the uniform path when every kept span proposed one key
//   decode          decode + downsampling (direct / lockstep proposals)
//   grid            the union-grid bitmap and its ranks
//   fap_finish      the optimistic aligned-group finish (ends the call if the
//                   group stood)
//   exchange_header the sharded agreement (sync 2), the global grid
//   plan_reduce     the reduce mode and variant, G emitted, the output block
//   reduce          the cross-span reduction, the exchange of the partials,
//                   the finalize
//   finish          the end of the call: the state snapshot, the outputs
// ls_allow: the lockstep proposal may be tried (k_direct_opt / k_lockstep);
// false for the rerun after k_lockstep found a qualifier off the proposal.
// ug_allow: the uniform path (uniform_run) may be taken; false for the rerun
// after it found the group not uniform (spangroup_run holds both edges).
constexpr int RC_CONTINUE = INT32_MIN;  // (a stage that did not end the call)
struct SgCall {
  Slot* ctx;
  const tsdbhip_sg_desc* d;
  tsdbhip_sg_out* out;
  bool ls_allow, ug_allow;
  // begin
  bool dev = false, exact = false, sharded = false, rate = false, check_clean = false, bm_clean = false;
  bool tgd_clean = false, tgd_used = false, detail = false;
  Xchg* X = nullptr;
  uint32_t S = 0;
  uint64_t R = 0;
  int agg = 0, ds_agg = 0;
  int32_t interval = 0;
  hipStream_t st = nullptr;
  tsdbhip_timing tm = {};
  const uint64_t* span_row_start = nullptr;
  const uint32_t* row_base = nullptr;
  const uint32_t* row_ncells = nullptr;
  const uint64_t* row_qual_off = nullptr;
  const uint64_t* row_val_off = nullptr;
  const uint32_t* row_val_len = nullptr;
  const uint8_t* qual = nullptr;
  const uint8_t* val = nullptr;
  Small* sm = nullptr;
  // assemble
  uint8_t* row_ok = nullptr;
  uint32_t* row_cell0 = nullptr;
  uint32_t* sp_ncells = nullptr;
  int64_t* sp_first = nullptr;
  int64_t* sp_last = nullptr;
  uint8_t* sp_kept = nullptr;
  uint64_t* sp_cap = nullptr;
  int64_t* sp_q1 = nullptr;
  int32_t* sp_q1s = nullptr;
  int64_t* sp_q1rs = nullptr;
  int64_t* sp_ovf = nullptr;
  uint32_t* kept = nullptr;
  uint64_t* eoff = nullptr;
  bool pub1 = false;
  HostPub p1 = {};
  bool auto_dec = false, ug_ls_q = false, ug_fap_q = false, ug_dev_q = false, ug_e_q = false, ug_q = false;
  bool ug_agree = false;
  uint64_t *u_key1 = nullptr, *u_key2 = nullptr, *u_vo = nullptr, *u_qo = nullptr, *uk_vo = nullptr, *uk_qo = nullptr;
  // sync1, plan
  Small h;
  bool poisoned = false;
  uint32_t n_kept = 0;
  uint64_t n_input_global = 0;
  int64_t lo = 0, hi = -1;
  bool empty_grid = true, used_bitmap_x = false;
  uint64_t nwords = 0;
  uint32_t* bitmap = nullptr;
  FapPlan fap;
  bool fap_off = false, fap_ran = false;
  uint64_t e_total = 0;
  uint32_t* e_ts = nullptr;
  int64_t* e_val = nullptr;
  uint8_t* e_flt = nullptr;
  uint32_t* e_len = nullptr;
  int64_t* e_bad = nullptr;
  DecodeArgs da;
  // decode, grid
  bool chunk_marked = false, direct = false, ls_try = false;
  uint64_t* d_qoff = nullptr;
  DirectArgs dg = {};
  const uint32_t* mark_list = nullptr;
  const uint32_t* mark_count = nullptr;
  bool fap_query = false, fap_opt = false;
  uint64_t T = 0;
  uint32_t* word_rank = nullptr;
  uint32_t* gridv = nullptr;
  GridArgs ga = {};
  // exchange_header, plan_reduce
  bool grids_agreed = true;
  int mode = 0;
  bool ls_use = false;
  LsPlan lsp = {};
  uint64_t fstar = 0;
  bool fap_use = false;
  BadArgs bad;
  bool bad_at_end = false, seq = false, int_parts = false, sliced = false, small_out = false, out_direct = false;
  uint64_t xs = 0, To = 0;
  uint8_t* outblk = nullptr;
  int64_t* o_ts = nullptr;
  int64_t* o_bits = nullptr;
  uint8_t* o_isint = nullptr;
  FinalArgs fin_map;

  SgCall(Slot* c, const tsdbhip_sg_desc* dd, tsdbhip_sg_out* o, bool ls, bool ug)
      : ctx(c), d(dd), out(o), ls_allow(ls), ug_allow(ug) {}
  int run() {
    begin();
    assemble();
    int rc = sync1();
    if (rc != RC_CONTINUE) return rc;
    plan();
    if ((rc = uniform_try()) != RC_CONTINUE) return rc;
    decode();
    grid();
    if ((rc = fap_finish()) != RC_CONTINUE) return rc;
    exchange_header();
    plan_reduce();
    reduce();
    return finish();
  }

  void begin() {
    dev = (d->flags & TSDBHIP_DESC_DEVICE) != 0;
    exact = (d->flags & TSDBHIP_EXACT_ORDER) != 0;
    // (a 1-rank communicator runs the same exchange code: tests use it)
    X = (d->flags & TSDBHIP_SHARDED) ? ctx->x : nullptr;
    sharded = X != nullptr;
    if (X) {
      X->n_coll = 0;
      X->x_bytes = 0;
    }
    S = d->n_spans;
    R = d->n_rows;
    rate = d->rate != 0;
    agg = d->agg;
    ds_agg = d->ds_agg;
    interval = d->ds_interval > 0 ? d->ds_interval : 0;
    st = ctx->stream;
    tm = {};
    ctx->timing_late = 0;
    ctx->hot_kernel = TSDBHIP_HOT_NONE;
    ctx->time_reduce = false;
    out->n_out = 0;
    out->n_input_points = 0;
    out->err_code = 0;
    out->err_index = -1;

    // ---- inputs in HBM ----
    span_row_start = stage(ctx, "in_srs", d->span_row_start, (size_t)S + 1, dev);
    row_base = stage(ctx, "in_base", d->row_base, R, dev);
    row_ncells = stage(ctx, "in_ncells", d->row_ncells, R, dev);
    row_qual_off = stage(ctx, "in_qoff", d->row_qual_off, R, dev);
    row_val_off = stage(ctx, "in_voff", d->row_val_off, R, dev);
    row_val_len = stage(ctx, "in_vlen", d->row_val_len, R, dev);
    qual = stage(ctx, "in_qual", d->qual_bytes, d->qual_nbytes, dev, 16);
    val = stage(ctx, "in_val", d->val_bytes, d->val_nbytes, dev, 16);

    sm = scratch<Small>(ctx, "small", 1);
    check_clean = ctx->opt.check_clean;
    if (check_clean && ctx->sm_ready) {  // (debug) the reset state must equal small_init()
      Small cur, ini = small_init();
      readback(ctx, &cur, sm, sizeof cur);
      if (std::memcmp(&cur, &ini, sizeof cur) != 0) {
        const uint8_t* a = (const uint8_t*)&cur; const uint8_t* b = (const uint8_t*)&ini;
        size_t i = 0;
        while (a[i] == b[i]) i++;
        fprintf(stderr, "TSDBHIP_CHECK_CLEAN: call state not reset (first differing byte %zu)\n", i);
      }
    }
    if (!ctx->sm_ready) {  // (a completed call leaves it reset: k_call_end)
      const Small init = small_init();
      std::memcpy(ctx->host_small, &init, sizeof init);
      HIPCHK(hipMemcpyAsync(sm, ctx->host_small, sizeof init, hipMemcpyHostToDevice, st));
    }
    ctx->sm_ready = false;
    bm_clean = ctx->bitmap_clean;
    ctx->bitmap_clean = false;
    tgd_clean = ctx->tgdone_clean;
    ctx->tgdone_clean = false;
    tgd_used = false;
    detail = ctx->opt.timing_detail;  // decode / grid event pairs
    g_ev_pend = nullptr;
    g_ev_pend_i = -1;
    std::memset(ctx->ev_alias, 0xff, sizeof ctx->ev_alias);
    EV_START(ctx, 0);
  }

  void assemble() {
    // ---- assemble ----
    row_ok = scratch<uint8_t>(ctx, "row_ok", R);
    row_cell0 = scratch<uint32_t>(ctx, "row_cell0", R);
    sp_ncells = scratch<uint32_t>(ctx, "sp_ncells", S);
    sp_first = scratch<int64_t>(ctx, "sp_first", S);
    sp_last = scratch<int64_t>(ctx, "sp_last", S);
    sp_kept = scratch<uint8_t>(ctx, "sp_kept", S);
    sp_cap = scratch<uint64_t>(ctx, "sp_cap", S);
    sp_q1 = scratch<int64_t>(ctx, "sp_q1", S);
    sp_q1s = scratch<int32_t>(ctx, "sp_q1s", S);
    sp_q1rs = scratch<int64_t>(ctx, "sp_q1rs", 2ull * S);
    sp_ovf = scratch<int64_t>(ctx, "sp_ovf", S);
    kept = nullptr;
    eoff = nullptr;
    pub1 = false;
    p1 = {};
    // the uniform path's queries (uniform_run): lockstep (no downsampling, the
    // conditions of the general path's lockstep try) or the aligned group
    // (downsampled exact integer aggregation); the spans' class keys are
    // proposed at assembly for them
    auto_dec = ctx->opt.decode == DEC_AUTO;
    // (unsharded, lockstep "on": the group needs >= 2048 lockstep waves, and
    // with C <= qual_nbytes / 2 cells in all and n in each of n_kept <= S
    // spans, ceil(n / LS_TILE) * max(1, n_kept / 64) <= max(ceil(C / LS_TILE),
    // C / (64 LS_TILE) + S / 64 + 1): a group under that bound cannot take it,
    // and its assembly skips the key probe — C1's 100 spans: 7 us)
    const uint64_t c_max = d->qual_nbytes / 2;
    const bool ls_size_ok = sharded || ctx->opt.lockstep == 2 ||
                            std::max<uint64_t>((c_max + LS_TILE - 1) / LS_TILE, c_max / (64 * LS_TILE) + S / 64 + 1) >= 2048;
    ug_ls_q = ug_allow && auto_dec && interval == 0 && ls_allow && ctx->opt.lockstep && !exact &&
                         (agg != TSDBHIP_AGG_DEV || rate) && ls_size_ok;
    ug_fap_q = ug_allow && auto_dec && interval > 0 && !rate && ds_agg <= 3 && agg <= 3 && !exact &&
                          ctx->opt.aligned_group && !ctx->opt.timing_detail;
    // (integer dev without rate, unsharded: the sequential chains of k_ug_dev)
    ug_dev_q = ug_allow && auto_dec && interval == 0 && !exact && agg == TSDBHIP_AGG_DEV && !rate &&
                          !sharded;
    // (other downsampled queries, unsharded: k_ds_reg's E on the key's buckets)
    ug_e_q = ug_allow && auto_dec && interval > 0 && !rate && ds_agg <= 3 && !exact && !sharded &&
                        !ctx->opt.timing_detail;
    ug_q = ug_ls_q || ug_fap_q || ug_dev_q || ug_e_q;
    // sharded lockstep: the ranks agree on the key before the host's round trip
    ug_agree = ug_ls_q && sharded;
    u_key1 = ug_q ? scratch<uint64_t>(ctx, "u_key1", S) : nullptr;
    u_key2 = ug_q ? scratch<uint64_t>(ctx, "u_key2", S) : nullptr;
    u_vo = ug_q ? scratch<uint64_t>(ctx, "u_vo", S) : nullptr;
    u_qo = ug_q ? scratch<uint64_t>(ctx, "u_qo", S) : nullptr;
    uk_vo = ug_q ? scratch<uint64_t>(ctx, "uk_vo", S) : nullptr;
    uk_qo = ug_q ? scratch<uint64_t>(ctx, "uk_qo", S) : nullptr;
    {
      AssembleArgs a;
      a.span_row_start = span_row_start; a.row_base = row_base; a.row_ncells = row_ncells;
      a.row_qual_off = row_qual_off; a.row_val_len = row_val_len; a.qual = qual;
      a.n_spans = S; a.start = d->start_time; a.end = d->end_time; a.interval = interval;
      a.row_ok = row_ok; a.row_cell0 = row_cell0; a.sp_ncells = sp_ncells; a.sp_first = sp_first;
      a.sp_last = sp_last; a.sp_kept = sp_kept; a.sp_cap = sp_cap; a.sp_q1 = sp_q1;
      a.sp_q1_shift = sp_q1s; a.sp_q1_rs = sp_q1rs; a.sp_ovf_cell = sp_ovf; a.err = &sm->err;
      a.span0 = sharded ? d->span0 : 0;
      a.row_val_off = row_val_off;
      a.u_key1 = u_key1; a.u_key2 = u_key2; a.u_vo = u_vo; a.u_qo = u_qo;
      // kept list, E offsets, counts and bounds (unsharded groups of up to
      // KC_MAX spans: the kernel hands the call state to the host itself)
      kept = scratch<uint32_t>(ctx, "kept", S);
      eoff = scratch<uint64_t>(ctx, "eoff", S);
      pub1 = S && S <= KC_MAX && !ug_agree;
      p1 = pub1 ? next_pub(ctx, sizeof(Small)) : HostPub{};
      KeptArgs K;
      K.kept = sp_kept; K.cap = sp_cap; K.ncells = sp_ncells; K.n = S; K.kept_list = kept; K.eoff_k = eoff;
      K.n_input = &sm->n_input; K.sp_first = sp_first; K.sp_last = sp_last; K.bound = sm->bound;
      K.n_kept_out = &sm->n_kept; K.e_total_out = &sm->e_total; K.pub = p1; K.pub_src = (const uint64_t*)sm;
      K.u_key1 = u_key1; K.u_key2 = u_key2; K.u_vo = u_vo; K.u_qo = u_qo; K.uk_vo = uk_vo; K.uk_qo = uk_qo;
      K.ukey = sm->ukey;
      // (the speculative aligned group's verdict: every fap query, see below)
      K.ug_go = ug_fap_q && sharded ? &sm->ug_go : nullptr;
      K.err = &sm->err;
      K.ug_interval = interval;
      // one block: assembly + kept list in one launch, for groups with few rows
      // (the block's 16 waves walk the deferred spans: a group of long spans of
      // many rows, C4's, needs the wave-per-span kernel's whole grid)
      if (S && S <= 1024 && R <= 8192) {
        LAUNCH(k_assemble_small, dim3(1), dim3(1024), 0, st, a, K);
      } else if (S > KC_MAX && R <= 2ull * S) {
        // (nearly) single-row spans: assembly + tile sums in one launch, then
        // the scatter (its last block publishes the call state)
        const uint32_t na = (S + 255) / 256, nt = (S + 1023) / 1024;  // (assembly tiles of 256, scatter tiles of 1024)
        KeptTile* ts = scratch<KeptTile>(ctx, "kept_tiles", na);
        ulonglong2* tke = scratch<ulonglong2>(ctx, "kept_tiles_ke", na);
        LAUNCH(k_assemble_tiles, dim3(na), dim3(256), 0, st, a, ts, tke);
        pub1 = !ug_agree;
        p1 = pub1 ? next_pub(ctx, sizeof(Small)) : HostPub{};
        LAUNCH(k_kept_scatter_tiles, dim3(nt), dim3(256), 0, st, sp_kept, sp_cap, S, (const KeptTile*)ts,
               (const ulonglong2*)tke, 4u, na, kept, eoff, &sm->n_input, sm->bound, &sm->n_kept, &sm->e_total, p1,
               (const uint64_t*)sm, K);
      } else if (S) {  // thread per span, then a wave per span for the ones it queued
        uint32_t* alist = scratch<uint32_t>(ctx, "asm_list", S);
        uint32_t* acount = &sm->cnt[0];
        LAUNCH(k_assemble_fast, dim3(grid_for(S, 256)), dim3(256), 0, st, a, alist, acount);
        LAUNCH(k_assemble, dim3(grid_for(S, 4, 4096)), dim3(256), 0, st, a, (const uint32_t*)alist,
                           (const uint32_t*)acount);
        if (S <= KC_MAX) {
          LAUNCH(k_kept_compact, dim3(1), dim3(1024), 0, st, K);
        } else {  // bigger groups: tile sums, then per-tile offsets + scatter
          const uint32_t nt = (S + 1023) / 1024;
          KeptTile* ts = scratch<KeptTile>(ctx, "kept_tiles", nt);
          ulonglong2* tke = scratch<ulonglong2>(ctx, "kept_tiles_ke", nt);
          LAUNCH(k_kept_tiles, dim3(nt), dim3(256), 0, st, sp_kept, sp_cap, sp_ncells, sp_first, sp_last, S, ts, tke,
                 (const uint64_t*)u_key1, (const uint64_t*)u_key2);
          // (its last block publishes the call state)
          pub1 = !ug_agree;
          p1 = pub1 ? next_pub(ctx, sizeof(Small)) : HostPub{};
          LAUNCH(k_kept_scatter_tiles, dim3(nt), dim3(256), 0, st, sp_kept, sp_cap, S, (const KeptTile*)ts,
                 (const ulonglong2*)tke, 1u, nt, kept, eoff, &sm->n_input, sm->bound, &sm->n_kept, &sm->e_total, p1,
                 (const uint64_t*)sm, K);
        }
      }
    }
  }

  int sync1() {
    // (sharded: no collective here. Each rank builds its grid on its own
    // bounds; one collective after the local grids tells whether they agree,
    // and only when they do not are the bitmaps remapped and exchanged.)
    if (ug_agree) {
      // the uniform path's key agreement (sharded lockstep queries, every rank):
      // the first error, the fewest kept spans and the keys' [min, max] over
      // the ranks, one MIN allreduce into Small.xh[0..5]
      const XField ag[6] = {{&sm->err, 5, 0},     {&sm->n_kept, 5, 0},  {&sm->ukey[0], 5, 0},
                            {&sm->ukey[1], 6, 0}, {&sm->ukey[2], 5, 0}, {&sm->ukey[3], 6, 0}};
      const XMove m = xchg_desc(ctx, ag, 6, (uint64_t*)sm->xh);
      LAUNCH(k_xmove, dim3(1), dim3(64), 0, st, m);
      X->group_start(ctx);
      X->allreduce(ctx, m.buf, 6, X_U64, X_MIN);
      X->group_end(ctx);
    }
    // the speculative aligned group (sharded downsampled integer sum / min /
    // max / avg): k_ug_ds_reg launched now, over every span slot, its blocks
    // reading the kept-list kernel's verdict (Small.ug_go) and the key from the
    // call state; the one collective group and the finish follow — no host
    // round trip before the call's end. Every rank, whatever its shard (the
    // collectives are everyone's). It saves ~35 us of a 0.94 ms C3* 8-way
    // shard step; unsharded, a launch that finds no group cost C2 ~10 us and
    // C3*'s own gained nothing measurable (same-box A/Bs, round 5), so the
    // unsharded aligned group waits for the round trip below.
    if (ug_fap_q && sharded) {
      DecodeArgs sa;
      std::memset(&sa, 0, sizeof sa);
      sa.span_row_start = span_row_start; sa.row_base = row_base; sa.row_qual_off = row_qual_off;
      sa.row_val_off = row_val_off; sa.qual = qual; sa.val = val; sa.row_ok = row_ok; sa.row_cell0 = row_cell0;
      sa.kept = kept; sa.n_kept = 0; sa.sp_ncells = sp_ncells; sa.sp_q1 = sp_q1; sa.sp_q1_shift = sp_q1s;
      sa.sp_q1_rs = sp_q1rs; sa.row_ncells = row_ncells; sa.row_val_len = row_val_len; sa.sp_ovf_cell = sp_ovf;
      sa.sp_cap = sp_cap; sa.e_off = eoff; sa.start = d->start_time; sa.end = d->end_time; sa.interval = interval;
      sa.ds_agg = ds_agg; sa.rate = rate; sa.err = &sm->err; sa.gflags = sm->gflags; sa.range = sm->range;
      sa.fstar = &sm->fstar; sa.span0 = d->span0; sa.sp_first = sp_first;
      UgIn u = {};
      u.d = d; u.X = X; u.sm = sm; u.da = sa; u.row_ncells = row_ncells; u.row_val_len = row_val_len;
      u.n_kept = S; u.lockstep = false; u.mine = S > 0; u.spec = true;
      const int rc = uniform_run(ctx, u, out, tm);
      ctx->bitmap_clean = bm_clean;  // (no bitmap touched)
      ctx->tgdone_clean = tgd_clean;
      return rc;
    }
    if (!pub1) {  // (the state's last writer cannot publish it: a one-wave kernel does)
      p1 = next_pub(ctx, sizeof(Small));
      LAUNCH(k_publish, dim3(1), dim3(64), 0, st, p1, (const uint64_t*)sm);
    }
    wait_pub(ctx, p1, &h, sizeof h);  // sync 1
    // a rank whose own scan failed still takes part in the agreement below (its
    // peers wait there for it), with nothing kept; every rank throws after it
    poisoned = h.err != ERR_NONE;
    if (poisoned && !sharded) throw Fail{err_code(h.err)};
    n_kept = poisoned ? 0u : (uint32_t)h.n_kept;
    out->n_input_points = h.n_input;
    n_input_global = h.n_input;
    return RC_CONTINUE;
  }

  void plan() {
    // ---- union-grid bitmap range: every E point lies in [first, last] of its
    // span and in [start, ...]; G keeps those <= end (SURVEY.md §8a closed form).
    // A kept span has first <= end and last >= start, so [lo, hi] is non-empty
    // whenever some span (of this rank) is kept.
    lo = std::max<int64_t>(d->start_time, h.bound[0] == ~0ull ? INT64_MAX : (int64_t)h.bound[0]);
    hi = std::min<int64_t>(d->end_time, (int64_t)h.bound[1]);
    if (h.bound[0] == ~0ull || poisoned) hi = -1;
    empty_grid = lo > hi;
    nwords = empty_grid ? 0 : (uint64_t)(hi - lo + 1 + 31) / 32;
    // (zero on entry without a memset: the last call's k_call_end cleared it)
    bitmap = empty_grid ? nullptr : scratch_zero_kept<uint32_t>(ctx, "gbitmap", nwords, bm_clean);
    used_bitmap_x = false;  // (sharded, grids not agreed: the global bitmap is "gbitmap_x")
    if (check_clean && bitmap) {  // (debug) the bitmap must be zero on entry
      unsigned long long* cnt = scratch<unsigned long long>(ctx, "chk_cnt", 1, true);
      const uint64_t nall = ctx->bufs["gbitmap"].n / 4;
      LAUNCH(k_count_nonzero, dim3(grid_for(nall, 256, 1024)), dim3(256), 0, st, bitmap, nall, cnt);
      unsigned long long nz = 0;
      readback(ctx, &nz, cnt, 8);
      if (nz) fprintf(stderr, "TSDBHIP_CHECK_CLEAN: %llu non-zero bitmap words on entry (clean=%d, nwords=%llu)\n", nz,
                      (int)bm_clean, (unsigned long long)nwords);
    }

    // ---- aligned-group reduction (k_ds_reg.hip FapArgs): tried when every
    // kept span has the same first and last timestamp (Small.bound), the group
    // downsamples, and the aggregation is exact integer (no rate, no dev) ----
    fap.a.op = -1;
    fap_off = !ctx->opt.aligned_group;
    if (!fap_off && interval > 0 && !rate && ds_agg <= 3 && agg <= 3 && !(sharded && exact) && n_kept > 0 &&
        h.bound[0] == h.bound[2] && h.bound[1] == h.bound[3] && h.bound[1] - h.bound[0] <= 62ull * (uint64_t)interval) {
      // (at most 64 buckets a span: a partial row holds them)
      fap.a.op = agg == TSDBHIP_AGG_MIN ? 1 : (agg == TSDBHIP_AGG_MAX ? 2 : 0);
      fap.a.key = sm->fap_key;
      fap.a.broken = &sm->fap_broken;
    }
    fap_ran = false;

    // ---- decode (+ downsample) ----
    e_total = h.e_total;
    e_ts = scratch<uint32_t>(ctx, "e_ts", e_total);
    e_val = scratch<int64_t>(ctx, "e_val", e_total);
    e_flt = scratch<uint8_t>(ctx, "e_flt", e_total);
    e_len = scratch<uint32_t>(ctx, "e_len", n_kept);
    e_bad = scratch<int64_t>(ctx, "e_bad", n_kept);
    da.span_row_start = span_row_start; da.row_base = row_base; da.row_qual_off = row_qual_off;
    da.row_val_off = row_val_off; da.qual = qual; da.val = val; da.row_ok = row_ok; da.row_cell0 = row_cell0;
    da.kept = kept; da.n_kept = n_kept; da.sp_ncells = sp_ncells; da.sp_q1 = sp_q1; da.sp_q1_shift = sp_q1s;
    da.sp_q1_rs = sp_q1rs; da.row_ncells = row_ncells; da.row_val_len = row_val_len;
    da.sp_ovf_cell = sp_ovf; da.sp_cap = sp_cap; da.e_off = eoff; da.e_ts = e_ts; da.e_val = e_val;
    da.e_flt = e_flt; da.e_len = e_len; da.e_bad = e_bad; da.start = d->start_time; da.end = d->end_time;
    da.interval = interval; da.ds_agg = ds_agg; da.rate = rate; da.err = &sm->err; da.gflags = sm->gflags;
    da.range = sm->range; da.fstar = &sm->fstar; da.span0 = sharded ? d->span0 : 0; da.sp_first = sp_first;
  }

  int uniform_try() {
    // ---- the uniform path (uniform_run): every kept span proposed one class key
    if (ug_q) {
      UgIn u = {};
      u.d = d; u.X = X; u.sm = sm; u.da = da; u.row_ncells = row_ncells; u.row_val_len = row_val_len;
      u.uk_vo = uk_vo; u.uk_qo = uk_qo; u.n_kept = n_kept;
      bool take = false;
      const bool local_ok = !poisoned && n_kept > 0 && h.ukey[0] != ~0ull && h.ukey[0] == h.ukey[1] &&
                            h.ukey[2] == h.ukey[3] && (uint32_t)h.ukey[0] >= 64;
      // (k_lockstep and k_ug_dev read one row a span: k2 bit 16 clear)
      const bool one_row = !(h.ukey[2] & 0x10000u);
      if (ug_dev_q) {
        u.lockstep = true;
        u.dev = true;
        u.k1 = h.ukey[0];
        u.k2 = h.ukey[2];
        take = local_ok && one_row && !(u.k2 & 8u);  // (integer cells)
      } else if (ug_ls_q) {
        u.lockstep = true;
        if (sharded) {  // (from the agreed words alone: every rank takes the same branch)
          const unsigned long long* x = h.xh;
          take = x[0] == ERR_NONE && x[1] > 0 && x[2] != ~0ull && x[2] == ~x[3] && x[4] == ~x[5] &&
                 (uint32_t)x[2] >= 64 && !(x[4] & 0x10000u);
          u.k1 = x[2];
          u.k2 = x[4];
        } else {
          const uint32_t n = (uint32_t)h.ukey[0];
          const uint64_t ls_waves = (n + LS_TILE - 1) / LS_TILE * std::max<uint64_t>(1, n_kept / 64);
          take = local_ok && one_row && (ctx->opt.lockstep == 2 || ls_waves >= 2048);
          u.k1 = h.ukey[0];
          u.k2 = h.ukey[2];
        }
      } else {
        u.lockstep = false;
        u.k1 = h.ukey[0];
        u.k2 = h.ukey[2];
        const uint32_t step = (uint32_t)(u.k2 >> 32), n = (uint32_t)u.k1;
        const uint64_t kk = step ? ((uint64_t)interval + step - 1) / step : 0;
        const bool fits = local_ok && !(u.k2 & 8u) && kk && (n + kk - 1) / kk <= WAVE;
        if (ug_fap_q && (sharded || fits)) {
          // (sharded: every rank makes the attempt, the key and the validity
          // agreed in its one collective group; unsharded: only a group that is one)
          u.mine = fits;
          take = true;
        } else if (ug_e_q && local_ok && kk) {
          u.e = true;
          take = true;
        }
      }
      if (take) {
        const int rc = uniform_run(ctx, u, out, tm);
        // (no bitmap was touched: it is as clean as scratch_zero_kept left it)
        ctx->bitmap_clean = bm_clean || bitmap != nullptr;
        ctx->tgdone_clean = tgd_clean;
        return rc;
      }
    }
    return RC_CONTINUE;
  }

  void decode() {
    if (detail) HIPCHK(hipEventRecord(ctx->ev[1], st));
    chunk_marked = false;     // k_ds_spans marked G for the spans it took
    direct = false;           // k_direct_scan took the no-downsampling path
    ls_try = false;           // k_direct_opt made the lockstep proposal
    d_qoff = nullptr;    // (its per-span qualifier offsets)
    dg = {};
    mark_list = nullptr;
    mark_count = nullptr;
    if (n_kept) {
      const unsigned blocks = grid_for(n_kept, 4, 65536);
      // wide rows (the reference's hourly compacted rows) take the streaming
      // kernels; rows of a few cells (sparse series) the general one. With
      // downsampling, regular-cadence integer spans go chunk-parallel first.
      const int force = ctx->opt.decode;
      bool fast = R > 0 && h.n_input / R >= 64;
      bool chunks = fast;
      direct = fast && interval == 0 && bitmap != nullptr;
      if (force == DEC_GENERAL) fast = chunks = direct = false;
      if (force == DEC_FAST) { fast = true; chunks = direct = false; }
      if (force == DEC_CHUNKS) { fast = chunks = true; direct = false; }
      // "spans": the chain-proved downsampler alone (k_ds_spans, no k_ds_reg first)
      const bool use_reg = force != DEC_SPANS;
      if (!use_reg) { fast = chunks = true; direct = false; }
      if (force == DEC_DIRECT) { fast = chunks = true; direct = interval == 0 && bitmap != nullptr; }
      da.fb_list = scratch<uint32_t>(ctx, "fb_list", n_kept);
      da.fb_count = &sm->cnt[1];
      da.use_fb = 0;
      da.span_list = nullptr;
      da.span_count = nullptr;
      DecodeArgs ga = da;  // spans the streaming kernels hand to the general ones
      ga.use_fb = 1;
      ctx->hot_kernel = fast ? TSDBHIP_HOT_DECODE_FAST : TSDBHIP_HOT_DECODE_GEN;
      if (!direct) EV_START(ctx, 8);
      if (!fast) {
        // (spans of many short rows, C4: a block per span decodes its rows in
        // parallel; else a wave per span walks them)
        if (interval == 0 && R >= 64ull * n_kept) LAUNCH(k_decode_rows, dim3(n_kept), dim3(DR_THREADS), 0, st, da);
        else if (interval == 0) LAUNCH(k_decode_nods, dim3(blocks), dim3(256), 0, st, da);
        else launch_agg<LaunchGeneralDs>(ds_agg, ctx, blocks, da);
        HIPCHK(hipEventRecord(ctx->ev[9], st));
      } else if (interval == 0) {
        DecodeArgs fa = da;
        if (direct) {
          // regular-cadence spans on consecutive grid ranks skip E (k_direct.hip)
          dg.info = scratch<uint32_t>(ctx, "d_info", n_kept);
          dg.n = scratch<uint32_t>(ctx, "d_n", n_kept);
          dg.x0 = scratch<uint32_t>(ctx, "d_x0", n_kept);
          dg.step = scratch<uint32_t>(ctx, "d_step", n_kept);
          dg.voff = scratch<uint64_t>(ctx, "d_voff", n_kept);
          dg.c0 = scratch<uint32_t>(ctx, "d_c0", n_kept);
          dg.r0 = scratch<uint64_t>(ctx, "d_r0", n_kept);
          dg.ga = scratch<uint32_t>(ctx, "d_ga", n_kept);
          dg.row_cpre = scratch<uint32_t>(ctx, "row_cpre", R);
          dg.list = scratch<uint32_t>(ctx, "d_list", n_kept);
          dg.list_count = &sm->cnt[2];
          dg.bitmap = bitmap;
          dg.lo = lo;
          dg.hi = hi;
          dg.rate = rate;
          ctx->hot_kernel = TSDBHIP_HOT_REDUCE_DIRECT;  // timed around k_reduce
          // (spans per wave: 32 for big groups; fewer below ~64k spans, so a
          // small group still spreads over ~2048 waves instead of a handful)
          dg.batch = std::max<uint32_t>(1, std::min<uint32_t>(DIRB, n_kept / 2048));
          // the lockstep proposal (k_lockstep.hip), where the reduce is not the
          // span-ordered pass (EXACT_ORDER, integer dev): three qualifiers a
          // span now, every other one proven by k_lockstep as it reduces
          // Unsharded, only when k_lockstep gets >= 2048 waves (LS_TILE grid
          // points x >= 64 spans each, the points per span estimated from the
          // input): C1's 100 spans made 8 waves (38 us) where k_reduce takes
          // 11 us. (Sharded: every rank alike, whatever its shard.)
          const uint64_t ls_waves = (h.n_input / n_kept + LS_TILE - 1) / LS_TILE * std::max<uint64_t>(1, n_kept / 64);
          ls_try = ls_allow && ctx->opt.lockstep && !exact && (agg != TSDBHIP_AGG_DEV || rate) &&
                   (ctx->opt.lockstep == 2 || sharded || ls_waves >= 2048);
          if (ls_try) {
            d_qoff = scratch<uint64_t>(ctx, "d_qoff", n_kept);
            dg.ls_key = sm->ls_key;
            dg.ls_other = &sm->cnt[5];
            LAUNCH(k_direct_opt, dim3(grid_for(n_kept, 256)), dim3(256), 0, st, da, dg, row_ncells,
                               row_val_len, d_qoff, sm->ls_key, &sm->cnt[5]);
          }
          LAUNCH(k_direct_scan, dim3(grid_for(n_kept, 4 * dg.batch, 1u << 20)), dim3(256), 0, st, da, dg,
                             row_ncells, row_val_len);
          fa.span_list = dg.list;
          fa.span_count = dg.list_count;
          mark_list = dg.list;
          mark_count = dg.list_count;
        }
        if (fa.span_list) {  // (the direct scan's leftovers: general code inline)
          LAUNCH((k_decode_fast<0, false, true>), dim3(std::min(blocks, 1024u)), dim3(256), 0, st, fa,
                             row_ncells, row_val_len);
        } else {
          LAUNCH((k_decode_fast<0, false>), dim3(blocks), dim3(256), 0, st, fa, row_ncells, row_val_len);
          HIPCHK(hipEventRecord(ctx->ev[9], st));
          LAUNCH(k_decode_nods, dim3(std::min(blocks, 1024u)), dim3(256), 0, st, ga);
        }
      } else {
        DecodeArgs fa = da;
        if (chunks && ds_agg != 4) {
          SpanDsArgs g = {};
          g.bitmap = bitmap;
          g.lo = lo;
          g.hi = hi;
          g.rate = rate;
          if (!bitmap) fap.a.op = -1;
          launch_agg<LaunchChunks>(ds_agg, ctx, da, fa, row_ncells, row_val_len, g, R, use_reg, &sm->cnt[3], sm->seg,
                                   sm->seg2, &fap);
          fap_ran = fap.a.op >= 0;
          chunk_marked = bitmap != nullptr && fa.span_list != nullptr;
        }
        if (chunk_marked) {
          mark_list = fa.span_list;
          mark_count = fa.span_count;
        }
        if (fa.span_list) {  // (grid-stride over the spans left by k_ds_spans: usually few; general inline)
          launch_agg<LaunchFastDsInl>(ds_agg, ctx, std::min(blocks, 1024u), fa, row_ncells, row_val_len);
        } else {
          launch_agg<LaunchFastDs>(ds_agg, ctx, blocks, fa, row_ncells, row_val_len);
          if (ctx->hot_kernel == TSDBHIP_HOT_DECODE_FAST) HIPCHK(hipEventRecord(ctx->ev[9], st));
          launch_agg<LaunchGeneralDs>(ds_agg, ctx, std::min(blocks, 1024u), ga);
        }
      }
    }
  }

  // (after sync 2: a scan / SpanGroup.add error throws; sharded, the agreed
  // input count)
  void after_sync2() {
    if (h.err != ERR_NONE) {
      // (a scan / SpanGroup.add error: no SpanGroup, aggregatedSize() never
      // reached; a sharded rank may have set its local count at sync 1)
      if ((h.err >> 62) < 2) out->n_input_points = 0;
      throw Fail{err_code(h.err)};
    }
    if (sharded) {
      n_input_global = h.n_input;
      out->n_input_points = n_input_global;
    }
  }

  // word ranks (block-local) and block sums of the bitmap (lo, nwords); the
  // single-block kernel that finishes T publishes the call state when `pub`
  void grid_ranks(bool pub, bool hash) {
    word_rank = scratch<uint32_t>(ctx, "word_rank", nwords);
    const uint64_t nb = (nwords + 1023) / 1024;
    ga.lo = lo; ga.hi = hi; ga.bitmap = bitmap; ga.nwords = nwords; ga.word_rank = word_rank;
    ga.block_sum = scratch<uint32_t>(ctx, "grid_bsum", nb);
    ga.hash = hash ? sm->ghash : nullptr;
    // (the optimistic aligned-group finish reads G right after: one block emits it)
    ga.emit1 = fap_opt && nb == 1 ? scratch<uint32_t>(ctx, "grid", nwords * 32) : nullptr;
    ga.block_hash = hash && nb > 1 ? scratch<unsigned long long>(ctx, "grid_bhash", 2 * nb) : nullptr;
    ga.pub = pub ? next_pub(ctx, sizeof(Small)) : HostPub{};
    LAUNCH(k_grid_popc, dim3((unsigned)nb), dim3(256), 0, st, ga);
    if (nb > 1) LAUNCH(k_grid_scan_blocks, dim3(1), dim3(256), 0, st, ga, (uint32_t)nb);
  }

  void grid() {
    if (detail) HIPCHK(hipEventRecord(ctx->ev[2], st));
    // (k_span_summary's work, empty spans and F*, is done by k_grid_mark below:
    // a kept span implies a non-empty grid range)
    // (no readback here: the flags, F*, errors and input count come back with
    // |G| below. A decode error leaves every e_len <= its capacity, so the grid
    // kernels stay inside E before the error is thrown.)


    // the optimistic aligned-group finish (below): unsharded, when this group
    // was tried as one; sharded, for every query that allows the attempt (all
    // ranks must issue the same collectives)
    fap_query = interval > 0 && !rate && ds_agg <= 3 && agg <= 3 && !exact && !fap_off;
    fap_opt = !detail && (sharded ? fap_query : (fap_ran && !empty_grid));
    // ---- union grid ----
    T = 0;
    word_rank = nullptr;
    gridv = nullptr;
    if (detail) HIPCHK(hipEventRecord(ctx->ev[3], st));
    ga = {};
    ga.e_off = eoff; ga.e_len = e_len; ga.e_ts = e_ts; ga.n_kept = n_kept; ga.rate = rate; ga.total = &sm->T;
    ga.e_flt = e_flt; ga.err = &sm->err; ga.fstar = &sm->fstar;
    ga.list = mark_list;  // spans k_ds_spans / the direct scan did not mark (null: all)
    ga.list_count = mark_count;
    // the direct path's verify appends to the direct / fallback lists again:
    // k_grid_popc zeroes their counters (cnt[1], cnt[2])
    ga.zero2 = direct && n_kept ? &sm->cnt[1] : nullptr;
    ga.pub_src = (const uint64_t*)sm;

    if (!empty_grid) {
      ga.lo = lo; ga.hi = hi; ga.bitmap = bitmap; ga.nwords = nwords;
      // (a bitmap of many slices marked by few spans each, C4: sliced through
      // LDS; else an atomic a point)
      const uint32_t n_sl = (uint32_t)((nwords + GM_WORDS - 1) >> GM_SHIFT);
      if (n_kept && n_sl >= 8 && (uint64_t)(n_sl + 1) * n_kept <= (64ull << 20)) {
        uint32_t* B = scratch<uint32_t>(ctx, "gm_bounds", (uint64_t)(n_sl + 1) * n_kept);
        LAUNCH(k_grid_bounds, dim3(mark_list ? std::min(grid_for(n_kept, 4, 65536), 1024u) : grid_for(n_kept, 4, 65536)),
                           dim3(256), 0, st, ga, B, n_sl);
        LAUNCH(k_grid_mark_slices, dim3(n_sl), dim3(256), 0, st, ga, (const uint32_t*)B, n_sl);
      } else if (n_kept) {
        LAUNCH(k_grid_mark, dim3(mark_list ? std::min(grid_for(n_kept, 4, 65536), 1024u) : grid_for(n_kept, 4, 65536)),
                           dim3(256), 0, st, ga);
      }
      grid_ranks(!sharded && !fap_opt, sharded);
    }
  }

  int fap_finish() {
    // ---- the optimistic aligned-group finish: when the group is tried as an
    // aligned group (sharded: every rank does this for a query that allows it,
    // so that all issue the same collectives), the rest of the call is enqueued
    // without the second host round trip: G emitted, the block partials reduced
    // to 64 slots (sharded: exchanged in the agreement's collective group), and
    // k_fap_finish writes the results iff the group stood (everywhere); the
    // host then waits once. If it did not stand, the state after the grid (and
    // the agreement) is intact and the usual path continues from it. ----
    if (fap_opt) {
      uint32_t* gridv_o = nullptr;
      if (!empty_grid) {
        gridv_o = scratch<uint32_t>(ctx, "grid", nwords * 32);  // (>= |G|)
        ga.grid = gridv_o;
        if (!ga.emit1) {  // (a single-block k_grid_popc emitted it)
          uint32_t* word_rank_f = scratch<uint32_t>(ctx, "word_rank_f", nwords);
          const uint32_t eb = grid_for(nwords, 256);
          LAUNCH(k_emit_verify, dim3(eb), dim3(256), 0, st, ga, word_rank_f, dg, 0u, eb);
        }
      }
      EV_START(ctx, 4);
      const int fop = agg == TSDBHIP_AGG_MIN ? 1 : (agg == TSDBHIP_AGG_MAX ? 2 : 0);
      int64_t* o_pi = scratch<int64_t>(ctx, "fo_i", WAVE);
      uint32_t* o_pc = scratch<uint32_t>(ctx, "fo_cnt", WAVE);
      const bool mine = fap_ran && !empty_grid;
      // (sharded: the agreement header packed by the partial kernel and unpacked
      // by the finish, no pack / unpack launches of their own)
      const uint64_t elo = empty_grid ? ~0ull : (uint64_t)lo, ehi = empty_grid ? 0ull : (uint64_t)hi;
      if (sharded && empty_grid) HIPCHK(hipMemsetAsync(sm->ghash, 0, sizeof sm->ghash, st));
      const XField fx[XH_N + 1] = {{&sm->err, 0, 0},      {&sm->gflags[0], 2, 0}, {&sm->gflags[1], 2, 0},
                                   {&sm->fstar, 1, 0},    {nullptr, 3, elo},      {nullptr, 4, ehi},
                                   {&sm->ghash[0], 5, 0}, {&sm->ghash[0], 6, 0},  {&sm->ghash[1], 5, 0},
                                   {&sm->ghash[1], 6, 0}, {nullptr, 4, elo},      {nullptr, 3, ehi},
                                   {&sm->fap_valid, 0, 0}};
      XMove pack = {};
      if (sharded) pack = xchg_desc(ctx, fx, XH_N + 1, (uint64_t*)sm->xh);
      XMove unpack = pack;
      unpack.out = 1;
      if (mine) {
        const uint32_t nrows = fap.a.nrows;
        const unsigned g1 = std::max(1u, std::min(256u, nrows / 128));
        int64_t* tmp = scratch<int64_t>(ctx, "fap_tmp", (uint64_t)g1 * WAVE);
        auto go = [&](auto opc) {
          constexpr int OP = decltype(opc)::value;
          // (two launches: a last-block-done fusion of the two measured slower,
          // 20.3 us against 4.6 + 9.3, its 244 blocks' counter atomics contended)
          LAUNCH((k_fap_rows<OP>), dim3(g1), dim3(1024), 0, st, (const int64_t*)fap.a.part, nrows, tmp);
          LAUNCH((k_fap_final64v<OP>), dim3(1), dim3(1024), 0, st, (const int64_t*)tmp, g1, n_kept, o_pi, o_pc, sm,
                 pack);
        };
        if (fop == 1) go(std::integral_constant<int, 1>());
        else if (fop == 2) go(std::integral_constant<int, 2>());
        else go(std::integral_constant<int, 0>());
      } else {
        LAUNCH(k_fap_neutral64, dim3(1), dim3(WAVE), 0, st, o_pi, o_pc, fop, sm, pack);
      }
      if (sharded) {  // the agreement, the validity (MIN) and the 64-slot partials: one collective group
        const XExtra ex[2] = {{o_pi, WAVE, fop ? X_I64 : X_U64, fop == 1 ? X_MIN : (fop == 2 ? X_MAX : X_SUM)},
                              {o_pc, WAVE, X_U32, X_SUM}};
        xchg_group(ctx, X, pack, (uint64_t*)&sm->n_input, ex, 2);
      }
      map_out_reserve(ctx, OUT_HDR + 17 * WAVE);
      const uint64_t end_seq = ++ctx->pub_seq;
      FinalArgs fo;
      std::memset(&fo, 0, sizeof fo);
      fo.T = WAVE;
      fo.n_chunks = 1;
      fo.grid = gridv_o;
      fo.out_ts = (int64_t*)(ctx->map_out_dev + OUT_HDR);
      fo.out_bits = fo.out_ts + WAVE;
      fo.out_isint = (uint8_t*)(fo.out_bits + WAVE);
      fo.nan_t = &sm->nan_t;
      {  // (an empty local grid: never valid; launched anyway, every rank alike)
        // the finish and the end of the call in one single-block launch
        const XMove um = sharded ? unpack : XMove{};
        Small* snap = (Small*)ctx->map_out_dev;
        const Small* ini = small_init_dev(ctx);
        const uint64_t seq = end_seq;
        if (agg == TSDBHIP_AGG_MIN)
          LAUNCH(k_fap_finish_end<1>, dim3(1), dim3(256), 0, st, sm, (const int64_t*)o_pi, (const uint32_t*)o_pc, fo, (int32_t)sharded, um, snap, ini, bitmap, (const uint32_t*)gridv_o, lo, seq);
        else if (agg == TSDBHIP_AGG_MAX)
          LAUNCH(k_fap_finish_end<2>, dim3(1), dim3(256), 0, st, sm, (const int64_t*)o_pi, (const uint32_t*)o_pc, fo, (int32_t)sharded, um, snap, ini, bitmap, (const uint32_t*)gridv_o, lo, seq);
        else if (agg == TSDBHIP_AGG_AVG)
          LAUNCH(k_fap_finish_end<3>, dim3(1), dim3(256), 0, st, sm, (const int64_t*)o_pi, (const uint32_t*)o_pc, fo, (int32_t)sharded, um, snap, ini, bitmap, (const uint32_t*)gridv_o, lo, seq);
        else
          LAUNCH(k_fap_finish_end<0>, dim3(1), dim3(256), 0, st, sm, (const int64_t*)o_pi, (const uint32_t*)o_pc, fo, (int32_t)sharded, um, snap, ini, bitmap, (const uint32_t*)gridv_o, lo, seq);
      }
      EV_FINAL(ctx, 5);
      HIPCHK(hipStreamSynchronize(st));
      check_stamp(ctx, end_seq);
      tm.late_stamp = ctx->timing_late;
      std::memcpy(&h, ctx->map_out, sizeof h);
      if (h.fap_done) {  // the call is over (state reset, bitmap clear)
        ctx->sm_ready = true;
        ctx->bitmap_clean = true;
        T = h.T;
        out->n_input_points = h.n_input;
        tm.n_grid = T;
        tm.paths |= TSDBHIP_PATH_ALIGNED_GROUP;
        if (sharded) {
          tm.n_collectives = X->n_coll;
          tm.x_bytes = X->x_bytes;
        }
        if (ctx->hot_kernel) tm.hot_ms = ev_ms(ctx, 8, 9);
        tm.hot_kernel = ctx->hot_kernel;
        tm.reduce_ms = ev_ms(ctx, 4, 5);
        tm.total_ms = ev_ms(ctx, 0, 5);
        tm.n_emitted = e_total;
        ctx->timing = tm;
        if (T > out->capacity && ctx->want_output) {
          out->err_code = TSDBHIP_E_CAPACITY;
          return TSDBHIP_E_CAPACITY;
        }
        if (ctx->want_output) {
          const uint8_t* hb = ctx->map_out;
          std::memcpy(out->ts, hb + OUT_HDR, T * 8);
          std::memcpy(out->bits, hb + OUT_HDR + 8 * WAVE, T * 8);
          std::memcpy(out->is_int, hb + OUT_HDR + 16 * WAVE, T);
        }
        out->n_out = T;
        out->err_code = TSDBHIP_OK;
        out->err_index = -1;
        return TSDBHIP_OK;
      }
    }
    return RC_CONTINUE;
  }

  void exchange_header() {
    grids_agreed = true;  // (sharded: every rank's local grid is the global one)
    if (sharded) {
      // One collective: the error, the int / float flags and F* (agreed in
      // place), the input count (sum), and each rank's grid geometry and bitmap
      // hashes as MIN / MAX pairs. Equal geometry and hashes on every rank: the
      // local grid is the global one (aligned series, C3 / C3*), nothing else is
      // exchanged before the partials. Otherwise the bitmaps are remapped onto
      // the global [lo, hi] and OR-ed over the ranks (allgather) below.
      // (an empty local grid: hashes 0, never a non-empty grid's, so the ranks
      // agree only when every grid is empty)
      const uint64_t elo = empty_grid ? ~0ull : (uint64_t)lo, ehi = empty_grid ? 0ull : (uint64_t)hi;
      if (empty_grid) HIPCHK(hipMemsetAsync(sm->ghash, 0, sizeof sm->ghash, st));
      const XField fx[XH_N] = {{&sm->err, 0, 0}, {&sm->gflags[0], 2, 0}, {&sm->gflags[1], 2, 0}, {&sm->fstar, 1, 0},
                               {nullptr, 3, elo}, {nullptr, 4, ehi}, {&sm->ghash[0], 5, 0}, {&sm->ghash[0], 6, 0},
                               {&sm->ghash[1], 5, 0}, {&sm->ghash[1], 6, 0}, {nullptr, 4, elo}, {nullptr, 3, ehi}};
      if (!fap_opt) {  // (an optimistic call ran the agreement already; h holds it)
        xchg_minmax(ctx, X, fx, XH_N, (uint64_t*)&sm->n_input, (uint64_t*)sm->xh);
        const HostPub p2 = next_pub(ctx, sizeof(Small));
        LAUNCH(k_publish, dim3(1), dim3(64), 0, st, p2, (const uint64_t*)sm);
        wait_pub(ctx, p2, &h, sizeof h);  // sync 2: agreed error / flags / count, the grids' geometry and hashes
      }
      after_sync2();
      const int64_t glo = (int64_t)h.xh[XH_LO], ghi = (int64_t)~h.xh[XH_HI];
      const bool all_empty = h.xh[XH_LO] == ~0ull;
      // (from the agreed words only: every rank takes the same branch)
      const bool agreed = all_empty || xh_grids_agree(h.xh);
      grids_agreed = agreed;
      if (!agreed) {
        // the global geometry: this rank's bitmap shifted onto [glo, ghi] (a
        // separate buffer; the local one is cleared), then OR-ed over the ranks
        const uint64_t gw = (uint64_t)(ghi - glo + 1 + 31) / 32;
        const bool clean_x = ctx->bitmapx_clean;
        ctx->bitmapx_clean = false;
        uint32_t* gbm = scratch_zero_kept<uint32_t>(ctx, "gbitmap_x", gw, clean_x);
        if (!empty_grid) {
          LAUNCH(k_bitmap_remap, dim3(grid_for(gw, 256)), dim3(256), 0, st, (const uint32_t*)bitmap, nwords,
                             lo, gbm, gw, glo);
          HIPCHK(hipMemsetAsync(bitmap, 0, nwords * 4, st));
        }
        bitmap = gbm;
        lo = glo;
        hi = ghi;
        nwords = gw;
        empty_grid = false;
        used_bitmap_x = true;
        uint32_t* all = scratch<uint32_t>(ctx, "bitmap_all", nwords * X->nranks);
        X->allgather(ctx, bitmap, all, nwords * 4);
        LAUNCH(k_bitmap_or, dim3(grid_for(nwords, 256)), dim3(256), 0, st, all, (uint32_t)X->nranks,
                           nwords, bitmap);
        grid_ranks(true, false);
        wait_pub(ctx, ga.pub, &h, sizeof h);  // sync 3: |G| of the global grid
      }
      dg.lo = lo;
      dg.hi = hi;
    } else if (!empty_grid) {
      if (!fap_opt) wait_pub(ctx, ga.pub, &h, sizeof h);  // sync 2: |G|, flags, F*, errors
      after_sync2();
    } else {
      readback(ctx, &h, sm, sizeof h);  // sync 2 (no grid)
      after_sync2();
    }
  }

  void plan_reduce() {
    // lockstep: every kept span proposed the one class key, and the grid is
    // its pattern (sharded: no other rank put a point elsewhere). A rank whose
    // proposal stood but whose grid is wider cannot use it: the call is marked
    // broken and runs again on the proven path (every rank, after the exchange)
    // The reduce mode is the agreed one (sharded: every rank's flags); a rank
    // whose lockstep proposal would reduce in another mode (an int shard next
    // to a float shard on one cadence: MODE_INT where the group is MODE_DUAL,
    // so the double partials would go unwritten) cannot use it either
    const bool anyf = h.gflags[0] != 0, anyi = h.gflags[1] != 0;
    mode = rate ? MODE_DBL : (!anyf ? MODE_INT : (!anyi ? MODE_DBL : MODE_DUAL));
    ls_use = false;
    lsp = {};
    if (ls_try && h.cnt[5] == 0 && h.ls_key[0] != ~0ull && h.ls_key[0] == h.ls_key[1] && h.ls_key[2] == h.ls_key[3]) {
      const uint32_t ln = (uint32_t)h.ls_key[0];
      const bool ls_flt = (h.ls_key[2] & 8u) != 0;
      const int ls_mode = (rate || ls_flt) ? MODE_DBL : MODE_INT;
      if (h.T == (uint64_t)(rate ? ln - 1 : ln) && ls_mode == mode) {
        ls_use = true;
        lsp.a.d_voff = dg.voff;
        lsp.a.d_qoff = d_qoff;
        lsp.a.val = val;
        lsp.a.qual = qual;
        lsp.a.n = ln;
        lsp.a.q0 = (uint32_t)(h.ls_key[2] & 0xFFFFu);
        lsp.a.step = (uint32_t)(h.ls_key[2] >> 32);
        lsp.a.broken = &sm->ls_broken;
        lsp.w8 = ((lsp.a.q0 & 7u) == 7u);
        lsp.flt = (lsp.a.q0 & 8u) != 0;
        tm.paths |= TSDBHIP_PATH_LOCKSTEP;
      } else {
        HIPCHK(hipMemsetD32Async((hipDeviceptr_t)&sm->ls_broken, 1, 1, st));
      }
    }
    if (!empty_grid) {
      T = h.T;
      gridv = scratch<uint32_t>(ctx, "grid", T);
      ga.grid = gridv;
      // G emitted with the final word ranks (word_rank_f); in the same launch
      // the direct candidates whose points are not consecutive grid ranks go
      // to the E path (their grid points are already marked; types, F* and
      // errors already counted)
      uint32_t* word_rank_f = scratch<uint32_t>(ctx, "word_rank_f", nwords);
      const bool verify = direct && n_kept && !ls_use;  // (lockstep: every span's points are G itself)
      dg.word_rank = word_rank;  // (block-local ranks + ga.block_sum)
      dg.bitmap = bitmap;
      const uint32_t eb = grid_for(nwords, 256);
      LAUNCH(k_emit_verify, dim3(eb + (verify ? grid_for(n_kept, 256) : 0)), dim3(256), 0, st, ga,
                         word_rank_f, dg, verify ? n_kept : 0u, eb);
      word_rank = word_rank_f;
      dg.word_rank = word_rank_f;
      if (verify) {
        DecodeArgs fa = da;
        fa.span_list = dg.list;
        fa.span_count = dg.list_count;
        LAUNCH((k_decode_fast<0, false, true>), dim3(std::min(grid_for(n_kept, 4, 65536), 1024u)), dim3(256),
                           0, st, fa, row_ncells, row_val_len);
      }
    }
    fstar = h.fstar;
    // the aligned-group partials stand for the reduce iff every kept span was in
    // the one class (no span outside it, one key) and G is the class's bucket
    // sequence (sharded: the local grid is the global one); else the members'
    // E is written now by a rerun of k_ds_reg
    fap_use = fap_ran && !h.fap_broken && h.fap_key[0] == h.fap_key[1] && h.fap_key[2] == h.fap_key[3] &&
                         !anyf && T > 0 && T <= WAVE && grids_agreed;
    if (fap_ran && !fap_use) launch_agg<LaunchRegRerun>(ds_agg, ctx, da, fap, row_ncells, row_val_len);
    tm.paths |= fap_use ? TSDBHIP_PATH_ALIGNED_GROUP : (fap_ran ? TSDBHIP_PATH_ALIGNED_RERUN : 0u);
    EV_START(ctx, 4);
    tm.n_grid = T;
    // lazy error index for illegal cells (every span's E and e_bad are final
    // here; sharded: a rank of the global grid, reduced with the exchange)
    bad.e_bad = e_bad; bad.e_off = eoff; bad.e_ts = e_ts; bad.n_kept = n_kept; bad.rate = (int32_t)rate; bad.hi = hi;
    bad.lo = lo; bad.bitmap = bitmap; bad.word_rank = word_rank; bad.T = T;
    // (small unsharded calls: computed by k_call_end instead, one launch fewer)
    // (k_call_end then runs as one block: its bitmap clearing must follow the
    // error index's grid ranks)
    bad_at_end = !sharded && n_kept <= 4096 && T <= 65536;
    // (an aligned group holds no E span, hence no bad cell)
    // (an aligned or lockstep group holds no E span, hence no bad cell)
    if (ls_use) bad.n_kept = 0;
    if (n_kept && !bad_at_end && !fap_use && !ls_use)
      LAUNCH(k_bad_index, dim3(grid_for(n_kept, 256)), dim3(256), 0, st, bad, &sm->bad_at);

    // ---- the reduce's shape: the span-ordered pass (integer dev before the
    // (long) truncation, Aggregators.java:196-217, or EXACT_ORDER), exact
    // integer partials, or order-dependent doubles; sharded doubles over a long
    // grid exchange rank-owned slices of G (below) ----
    seq = exact || (agg == TSDBHIP_AGG_DEV && mode != MODE_DBL);
    int_parts = mode == MODE_INT && agg != TSDBHIP_AGG_DEV;
    // (per rank (N-1)/N (esz + 17) B a point against (N-1) esz: a gain from 3
    // ranks on; at 2 it is even, and the slices cost a second collective)
    sliced = sharded && T > 0 && !seq && !int_parts && X->nranks >= 3 && T >= XSLICE_MIN_T;
    xs = sliced ? (T + X->nranks - 1) / X->nranks : 0;  // slice length (the last one shorter)
    // ---- output block: [Small snapshot | ts T | bits T | is_int T], written
    // by the kernels straight into mapped pinned host memory when small (a
    // sliced exchange gathers the results in device memory: T padded to whole
    // slices) ----
    To = sliced ? xs * X->nranks : T;
    small_out = To * 17 <= (256u << 10) && ctx->want_output && !sliced;
    map_out_reserve(ctx, OUT_HDR + (small_out ? 17 * To : 0));
    outblk = small_out ? ctx->map_out_dev : scratch<uint8_t>(ctx, "outblk", OUT_HDR + 17 * To);
    o_ts = (int64_t*)(outblk + OUT_HDR);
    o_bits = o_ts + To;
    o_isint = (uint8_t*)(o_bits + To);
    // a long unsharded result into registered (mapped) caller buffers: the
    // reduce finalizes each tile group into them as soon as its last chunk is
    // done, so the results cross PCIe while the reduce still runs (no D2H copy
    // after it; C4: 178 MB)
    std::memset(&fin_map, 0, sizeof fin_map);
    if (!sharded && !small_out && ctx->want_output && T >= 65536 && out->capacity >= T) {
      fin_map.out_ts = (int64_t*)mapped_dev_ptr(out->ts, T * 8);
      fin_map.out_bits = (int64_t*)mapped_dev_ptr(out->bits, T * 8);
      fin_map.out_isint = (uint8_t*)mapped_dev_ptr(out->is_int, T);
      if (!fin_map.out_ts || !fin_map.out_bits || !fin_map.out_isint) fin_map.out_ts = nullptr;
    }
    out_direct = false;  // the results are already in the caller's buffers
  }

  void partials(ReduceArgs& r, const char* pre, uint64_t np) { alloc_partials(ctx, r, pre, np, agg); }
  std::vector<Fld> fields(const ReduceArgs& r, uint64_t off) { return partial_fields(r, off, agg, mode); }

  // one reduce launch over this rank's kept spans; `init`: the per-t state
  // to continue from (one chunk)
  ReduceArgs run_reduce(bool one_chunk, bool finalize, const ReduceArgs* init, const FinalArgs& fin) {
    // span state in LDS while 4 waves' regions fit 40 KB (4 blocks a CU)
    const uint32_t spc_cap = (uint32_t)(RED_LDS_BLOCK / 4 / red_lds_span_bytes(rate));
    const ReduceGeom rg = reduce_geom(T, n_kept, one_chunk || init, 16384, 2048, spc_cap);
    const uint32_t spc = rg.spc, n_chunks = rg.n_chunks, tpw = rg.tpw, ntg = rg.ntg;
    const uint64_t n_waves = rg.n_waves;
    ReduceArgs r;
    std::memset(&r, 0, sizeof r);
    r.e_off = eoff; r.e_len = e_len; r.e_ts = e_ts; r.e_val = e_val; r.e_flt = e_flt; r.n_kept = n_kept;
    r.grid = gridv; r.T = T; r.bitmap = bitmap; r.word_rank = word_rank; r.lo = lo;
    r.spans_per_chunk = spc; r.n_chunks = n_chunks; r.tiles_per_wave = tpw; r.n_tile_groups = ntg;
    r.d_info = direct ? dg.info : nullptr;
    r.d_n = dg.n; r.d_ga = dg.ga; r.d_voff = dg.voff; r.d_x0 = dg.x0; r.d_step = dg.step; r.d_c0 = dg.c0;
    r.d_r0 = dg.r0; r.span_row_start = span_row_start; r.kept = kept; r.row_cpre = dg.row_cpre;
    r.row_ncells = row_ncells; r.row_val_off = row_val_off; r.val = val;
    r.chunk_e = nullptr;
    r.fstar = fstar;
    r.exact = exact ? 1 : 0;
    r.lds_state = 4 * red_lds_stride(spc, rate) <= RED_LDS_BLOCK ? 1u : 0u;
    if (init) {
      r.i_cnt = init->p_cnt; r.i_flag = init->p_flag; r.i_i = init->p_i; r.i_d = init->p_d;
      r.i_dhas = init->p_dhas; r.i_wim = init->p_wim; r.i_wiv = init->p_wiv; r.i_wdm = init->p_wdm;
      r.i_wdv = init->p_wdv;
    }
    // (small reductions: the general instantiation takes every chunk, direct
    // spans included; no flags, one launch)
    if (direct && n_waves > 4096) {
      uint32_t* ce = scratch<uint32_t>(ctx, "chunk_e", n_chunks);
      LAUNCH(k_chunk_flags_w, dim3(grid_for(n_chunks, 4)), dim3(256), 0, st, dg.info, n_kept, spc,
                         n_chunks, ce);
      r.chunk_e = ce;
    }
    // the in-kernel finalize into the mapped result (unsharded, one pass,
    // no direct spans, few chunks: the last chunk-wave merges them)
    if (finalize && !init && !one_chunk && !direct && fin_map.out_ts && n_chunks > 1 && n_chunks < 64) {
      r.tg_done = scratch_zero_kept<uint32_t>(ctx, "tg_done", ntg, tgd_clean);
      tgd_used = true;
      r.fin = fin;
      r.fin.n_chunks = n_chunks;
      r.fin.out_ts = fin_map.out_ts;
      r.fin.out_bits = fin_map.out_bits;
      r.fin.out_isint = fin_map.out_isint;
      out_direct = true;
      finalize = false;
    }
    r.ptr = scratch<uint32_t>(ctx, "cursor", n_waves * spc);
    r.st_x = scratch<uint2>(ctx, "st_x", n_waves * spc);
    r.st_y = scratch<longlong2>(ctx, "st_y", n_waves * spc);
    r.st_rv = scratch<double>(ctx, "st_rv", n_waves * spc);
    r.st_f = scratch<uint32_t>(ctx, "st_f", n_waves * spc);
    partials(r, "p_", (uint64_t)n_chunks * T);
    FinalArgs f = fin;
    f.n_chunks = n_chunks;
    const unsigned blocks = (unsigned)((n_waves + 3) / 4);
    dispatch_reduce(ctx, agg, mode, rate, blocks, r, f, n_chunks >= 64, finalize);
    return r;
  }

  // the lockstep group: tiles of LS_TILE grid points x chunks of spans
  ReduceArgs ls_reduce(bool finalize, const FinalArgs& fin) {
    const uint32_t n_tiles = (uint32_t)((T + LS_TILE - 1) / LS_TILE);
    uint64_t want = std::max<uint64_t>(1, 16384 / n_tiles);
    want = std::min<uint64_t>(want, std::max<uint32_t>(1, n_kept / LS_MIN_SPC));
    const uint32_t spc = (uint32_t)((n_kept + want - 1) / want);
    const uint32_t n_chunks = (n_kept + spc - 1) / spc;
    const uint32_t n_cg = (n_chunks + LS_GROUP - 1) / LS_GROUP;  // (a block's chunks merged in LDS)
    ReduceArgs r;
    std::memset(&r, 0, sizeof r);
    r.T = T;
    r.n_chunks = n_cg;
    r.n_kept = n_kept;
    partials(r, "p_", (uint64_t)n_cg * T);
    LsPlan p = lsp;
    p.a.spc = spc;
    p.a.n_tiles = n_tiles;
    p.a.n_chunks = n_chunks;
    FinalArgs f = fin;
    f.n_chunks = n_cg;
    ctx->hot_kernel = TSDBHIP_HOT_LOCKSTEP;
    dispatch_lockstep(ctx, agg, rate, n_tiles * n_cg, r, p, f, finalize);
    return r;
  }

  // the aligned group: its block partials reduced into the 1-chunk layout
  ReduceArgs fap_reduce(bool finalize, const FinalArgs& fin) {
    ReduceArgs r;
    std::memset(&r, 0, sizeof r);
    r.T = T;
    r.n_chunks = 1;
    r.n_kept = n_kept;
    partials(r, "p_", T);
    const uint32_t nrows = fap.a.nrows;
    // (16-wave blocks, >= 128 rows each, at most 256 of them)
    const unsigned g1 = std::max(1u, std::min(256u, nrows / 128));
    int64_t* tmp = scratch<int64_t>(ctx, "fap_tmp", (uint64_t)g1 * WAVE);
    FinalArgs f = fin;
    f.n_chunks = 1;
    auto go = [&](auto opc) {
      constexpr int OP = decltype(opc)::value;
      LAUNCH((k_fap_rows<OP>), dim3(g1), dim3(1024), 0, st, (const int64_t*)fap.a.part, nrows, tmp);
      if (!finalize) {
        LAUNCH((k_fap_final<OP>), dim3(1), dim3(1024), 0, st, (const int64_t*)tmp, g1, T, n_kept, r.p_i,
                           r.p_cnt, r.p_flag);
        return;
      }
      // (the cross-series aggregator: OP 0 is sum or avg)
      if (OP == 1) LAUNCH((k_fap_final_out<OP, 1>), dim3(1), dim3(1024), 0, st, (const int64_t*)tmp, g1, n_kept, f);
      else if (OP == 2) LAUNCH((k_fap_final_out<OP, 2>), dim3(1), dim3(1024), 0, st, (const int64_t*)tmp, g1, n_kept, f);
      else if (agg == TSDBHIP_AGG_AVG) LAUNCH((k_fap_final_out<0, 3>), dim3(1), dim3(1024), 0, st, (const int64_t*)tmp, g1, n_kept, f);
      else LAUNCH((k_fap_final_out<0, 0>), dim3(1), dim3(1024), 0, st, (const int64_t*)tmp, g1, n_kept, f);
    };
    if (fap.a.op == 1) go(std::integral_constant<int, 1>());
    else if (fap.a.op == 2) go(std::integral_constant<int, 2>());
    else go(std::integral_constant<int, 0>());
    return r;
  }

  void reduce() {
    // ---- reduce ----
    if (T > 0) {
      ctx->time_reduce = direct;
      // (integer dev is reduced in one span-ordered pass, and, sharded, in rank
      // order: the reference's sequential Welford before the (long)
      // truncation admits no merge of partial states; EXACT_ORDER does the
      // same for every aggregator)
      FinalArgs fin;
      std::memset(&fin, 0, sizeof fin);
      fin.T = T; fin.n_chunks = 1; fin.grid = gridv; fin.fstar = fstar; fin.rate = rate;
      fin.out_ts = o_ts;
      fin.out_isint = o_isint;
      fin.out_bits = o_bits;
      fin.nan_t = &sm->nan_t;
      if (!sharded) {
        if (fap_use) fap_reduce(true, fin);
        else if (ls_use) ls_reduce(true, fin);
        else run_reduce(seq, true, nullptr, fin);
      } else {
        const int nr = X->nranks, rk = X->rank;
        ReduceArgs src;  // per-t partials the finalize merges ([n_src][T])
        uint32_t n_src = 1;
        if (seq) {
          // span order across ranks: rank 0 reduces its spans in one chunk;
          // rank r continues from rank r-1's per-t state, which reaches it by
          // broadcast; the last broadcast gives every rank the final state
          ReduceArgs S;
          std::memset(&S, 0, sizeof S);
          partials(S, "s_", T);
          if (detail) HIPCHK(hipEventRecord(ctx->ev[6], st));
          for (int step = 0; step < nr; step++) {
            ReduceArgs P = S;  // (non-roots: the send side of the broadcast is unused)
            if (rk == step) P = run_reduce(true, false, step ? &S : nullptr, fin);
            const std::vector<Fld> fp = fields(P, 0), fs = fields(S, 0);
            X->group_start(ctx);
            for (size_t i = 0; i < fp.size(); i++) X->broadcast(ctx, fp[i].p, fs[i].p, T * fp[i].esz, step);
            if (step == 0) {
              X->allreduce(ctx, &sm->bad_at, 1, X_U64, X_MIN);
              X->allreduce(ctx, &sm->ls_broken, 1, X_U32, X_MAX);
            }
            X->group_end(ctx);
          }
          if (detail) HIPCHK(hipEventRecord(ctx->ev[7], st));
          src = S;
        } else {
          // this rank's chunks combined in order into one slot per t
          ReduceArgs loc = fap_use ? fap_reduce(false, fin) : ls_use ? ls_reduce(false, fin) : run_reduce(false, false, nullptr, fin);
          if (int_parts) {
            // exact integer partials: one allreduce per field (wrapping u64
            // sum, i64 min / max, count sum), no ordering needed
            ReduceArgs mine = loc;
            if (!fap_use) {  // (the aligned group's partials are one slot per t already, every count > 0)
              partials(mine, "m_", T);
              dispatch_combine(ctx, agg, mode, loc, mine, T, loc.n_chunks);
              if (agg == TSDBHIP_AGG_MIN || agg == TSDBHIP_AGG_MAX)
                LAUNCH(k_neutral_minmax, dim3(grid_for(T, 256)), dim3(256), 0, st, mine.p_cnt, mine.p_i, T,
                                   agg == TSDBHIP_AGG_MIN ? INT64_MAX : INT64_MIN);
            }
            if (detail) HIPCHK(hipEventRecord(ctx->ev[6], st));
            X->group_start(ctx);
            for (const Fld& f : fields(mine, 0)) X->allreduce(ctx, f.p, T, f.t, f.op);
            X->allreduce(ctx, &sm->bad_at, 1, X_U64, X_MIN);
            X->allreduce(ctx, &sm->ls_broken, 1, X_U32, X_MAX);
            X->group_end(ctx);
            if (detail) HIPCHK(hipEventRecord(ctx->ev[7], st));
            src = mine;
          } else if (sliced) {
            // doubles over a long grid (C4): rank q owns slice q of G (xs
            // points). Each rank's combined partials of slice q reach rank q
            // (alltoall), which merges them in rank order (chunk-then-rank, as
            // unsharded; SpanGroup.java:647-667) and finalizes its slice; the
            // slices' results are then gathered. Per rank (N-1)/N of the
            // partials plus the results, instead of N-1 times the partials.
            ReduceArgs mine = loc, recv = loc;
            partials(mine, "m_", xs * nr);  // [T] used
            partials(recv, "x_", xs * nr);  // [rank q][xs]: rank q's partials of this rank's slice
            dispatch_combine(ctx, agg, mode, loc, mine, T, loc.n_chunks);
            if (detail) HIPCHK(hipEventRecord(ctx->ev[6], st));
            const std::vector<Fld> fm = fields(mine, 0), fr = fields(recv, 0);
            X->group_start(ctx);
            for (size_t i = 0; i < fm.size(); i++) X->alltoall(ctx, fm[i].p, fr[i].p, xs * fm[i].esz);
            X->allreduce(ctx, &sm->bad_at, 1, X_U64, X_MIN);
            X->allreduce(ctx, &sm->ls_broken, 1, X_U32, X_MAX);
            X->group_end(ctx);
            const uint64_t g0 = (uint64_t)rk * xs, ns = g0 < T ? std::min<uint64_t>(xs, T - g0) : 0;
            FinalArgs f = fin;
            f.T = ns;
            f.stride = xs;
            f.n_chunks = (uint32_t)nr;
            f.g_base = g0;
            f.grid = gridv + g0;
            f.out_ts = o_ts + g0;
            f.out_bits = o_bits + g0;
            f.out_isint = o_isint + g0;
            recv.n_chunks = (uint32_t)nr;
            if (ns) dispatch_final(ctx, agg, mode, rate, recv, f);
            X->group_start(ctx);
            X->allgather(ctx, o_ts + g0, o_ts, xs * 8);
            X->allgather(ctx, o_bits + g0, o_bits, xs * 8);
            X->allgather(ctx, o_isint + g0, o_isint, xs);
            X->allreduce(ctx, &sm->nan_t, 1, X_U64, X_MIN);
            X->group_end(ctx);
            if (detail) HIPCHK(hipEventRecord(ctx->ev[7], st));
          } else {
            // doubles (sums / Welford states depend on the order): every
            // rank's slot gathered, merged in rank order on every rank
            ReduceArgs all = loc;
            partials(all, "x_", (uint64_t)nr * T);
            ReduceArgs mine = all;
            const uint64_t off = (uint64_t)rk * T;
            mine.p_cnt += off; mine.p_flag += off; mine.p_i += off; mine.p_d += off; mine.p_dhas += off;
            if (agg == TSDBHIP_AGG_DEV) { mine.p_wim += off; mine.p_wiv += off; mine.p_wdm += off; mine.p_wdv += off; }
            dispatch_combine(ctx, agg, mode, loc, mine, T, loc.n_chunks);
            if (detail) HIPCHK(hipEventRecord(ctx->ev[6], st));
            const std::vector<Fld> fm = fields(mine, 0), fa = fields(all, 0);
            X->group_start(ctx);
            for (size_t i = 0; i < fm.size(); i++) X->allgather(ctx, fm[i].p, fa[i].p, T * fm[i].esz);
            X->allreduce(ctx, &sm->bad_at, 1, X_U64, X_MIN);
            X->allreduce(ctx, &sm->ls_broken, 1, X_U32, X_MAX);
            X->group_end(ctx);
            if (detail) HIPCHK(hipEventRecord(ctx->ev[7], st));
            src = all;
            n_src = (uint32_t)nr;
          }
        }
        if (!sliced) {
          FinalArgs f = fin;
          f.n_chunks = n_src;
          src.n_chunks = n_src;
          dispatch_final(ctx, agg, mode, rate, src, f);
        }
      }
    } else if (sharded) {
      X->group_start(ctx);
      X->allreduce(ctx, &sm->bad_at, 1, X_U64, X_MIN);
      X->allreduce(ctx, &sm->ls_broken, 1, X_U32, X_MAX);
      X->group_end(ctx);
    }
  }

  int finish() {
    // ---- end of call: snapshot + reset of the call state, bitmap cleared ----
    const uint64_t end_seq = ++ctx->pub_seq;
    LAUNCH(k_call_end, dim3(bad_at_end ? 1u : grid_for(T, 256, 1024)), dim3(256), 0, st, sm,
                (Small*)ctx->map_out_dev, small_init_dev(ctx), bitmap, (const uint32_t*)gridv, T, lo, bad_at_end ? bad : BadArgs{},
                end_seq, (const uint32_t*)nullptr);
    EV_FINAL(ctx, 5);
    HIPCHK(hipStreamSynchronize(st));  // (the header and small results are already in host memory)
    check_stamp(ctx, end_seq);
    tm.late_stamp = ctx->timing_late;
    const uint8_t* hb = ctx->map_out;
    std::memcpy(&h, hb, sizeof h);
    ctx->sm_ready = true;
    ctx->bitmap_clean = true;
    if (used_bitmap_x) ctx->bitmapx_clean = true;
    if (tgd_used) ctx->tgdone_clean = true;  // (every counter reset by its group's last wave)
    // the proposal did not hold: discard, run again. Sharded, from the agreed
    // flag alone (MAX over the ranks): whether a rank tried depends on its own
    // shard (empty, short rows), and every rank must issue the rerun's
    // collectives. Unsharded the flag is only ever set by a try.
    if (h.ls_broken) {
      ctx->timing = tm;
      return RC_REDO;
    }
    if (sharded) {
      tm.exchange_ms = T > 0 && detail ? ev_ms(ctx, 6, 7) : 0.f;  // (timing_detail only)
      tm.n_collectives = X->n_coll;
      tm.x_bytes = X->x_bytes;
    }
    if (detail) {
      tm.decode_ms = ev_ms(ctx, 1, 2);
      tm.grid_ms = ev_ms(ctx, 3, 4);
    }
    if (ctx->hot_kernel) tm.hot_ms = ev_ms(ctx, 8, 9);
    tm.hot_kernel = ctx->hot_kernel;
    tm.reduce_ms = ev_ms(ctx, 4, 5);
    tm.total_ms = ev_ms(ctx, 0, 5);
    tm.n_emitted = e_total;
    ctx->timing = tm;

    // ---- outputs ----
    uint64_t n_ok = T;
    int code = TSDBHIP_OK;
    int64_t err_at = -1;
    if (h.bad_at != ~0ull) {
      err_at = (int64_t)(h.bad_at >> 4);
      code = (h.bad_at & 15) == BAD_OOB ? TSDBHIP_E_OUT_OF_BOUNDS : TSDBHIP_E_ILLEGAL_DATA;
    }
    if (h.nan_t != ~0ull && (err_at < 0 || (int64_t)h.nan_t < err_at)) {
      err_at = (int64_t)h.nan_t;
      code = TSDBHIP_E_NAN_INF;
    }
    if (err_at >= 0) n_ok = (uint64_t)err_at;
    if (n_ok > out->capacity && ctx->want_output) {
      out->err_code = TSDBHIP_E_CAPACITY;
      return TSDBHIP_E_CAPACITY;
    }
    if (!ctx->want_output || out_direct) {
      // (a non-zero rank of an in-process sharded call: rank 0 returns the
      // output; or the reduce wrote it into the mapped caller buffers)
    } else if (n_ok && small_out) {  // (already in the pinned staging with the header)
      std::memcpy(out->ts, hb + OUT_HDR, n_ok * 8);
      std::memcpy(out->bits, hb + OUT_HDR + 8 * To, n_ok * 8);
      std::memcpy(out->is_int, hb + OUT_HDR + 16 * To, n_ok);
    } else if (n_ok) {
      HIPCHK(hipMemcpyAsync(out->ts, o_ts, n_ok * 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(out->is_int, o_isint, n_ok, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(out->bits, o_bits, n_ok * 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    out->n_out = n_ok;
    out->err_code = code;
    out->err_index = err_at;
    // algorithmic bytes: reference row bytes + T x 17 B
    tm.alg_bytes = 0;
    ctx->timing = tm;
    return code;
  }
};

static int spangroup_run_once(Slot* ctx, const tsdbhip_sg_desc* d, tsdbhip_sg_out* out, bool ls_allow,
                              bool ug_allow) {
  SgCall c(ctx, d, out, ls_allow, ug_allow);
  return c.run();
}


// The call's attempts and their rerun edges, in one place. An attempt is
// spangroup_run_once with the proposals it may try; an attempt that returns
// a rerun code hands the call to the attempt its edge names (every rank of a
// sharded call returns the same code: the verdicts are agreed):
//   FULL     --RC_UG_FALLBACK--> NO_UNIFORM  the aligned group / E did not stand
//                                            (test_uniform.py: *_fallback*)
//   FULL     --RC_REDO---------> PROVEN      the uniform lockstep's proposal did
//                                            not hold (test_uniform.py:67)
//   NO_UNIFORM --RC_REDO-------> PROVEN      the general path's lockstep proposal
//                                            did not hold (test_lockstep.py)
// PROVEN tries no proposal and so ends the call. A rerun stages nothing
// again: the host-resident inputs the first attempt copied are still in HBM
// (ADVICE r5).
enum SgAttempt { SG_FULL, SG_NO_UNIFORM, SG_PROVEN, SG_DONE };
struct SgEdge {
  SgAttempt from;
  int rc;
  SgAttempt to;
  uint32_t path;  // (tsdbhip_timing.paths)
};
static const SgEdge kSgEdges[] = {
    {SG_FULL, RC_UG_FALLBACK, SG_NO_UNIFORM, TSDBHIP_PATH_UNIFORM_FALLBACK},
    {SG_FULL, RC_REDO, SG_PROVEN, TSDBHIP_PATH_DIRECT_REDO},
    {SG_NO_UNIFORM, RC_REDO, SG_PROVEN, TSDBHIP_PATH_DIRECT_REDO},
};
static int spangroup_run(Slot* ctx, const tsdbhip_sg_desc* d, tsdbhip_sg_out* out) {
  struct Reuse {  // (reset on every exit, exceptions included)
    Slot* c;
    ~Reuse() { c->reuse_inputs = false; }
  } reuse{ctx};
  ctx->h2d_bytes = 0;
  ctx->reuse_inputs = false;
  uint32_t paths = 0;
  int rc = 0;
  for (SgAttempt a = SG_FULL; a != SG_DONE;) {
    rc = spangroup_run_once(ctx, d, out, a != SG_PROVEN, a == SG_FULL);
    SgAttempt next = SG_DONE;
    for (const SgEdge& e : kSgEdges)
      if (e.from == a && e.rc == rc) {
        next = e.to;
        paths |= e.path;
      }
    if (next == SG_DONE && (rc == RC_REDO || rc == RC_UG_FALLBACK)) {  // (an attempt that may not rerun)
      set_error(ctx, "spangroup_run: rerun code %d with no edge from attempt %d", rc, (int)a);
      throw Fail{TSDBHIP_E_HIP};
    }
    ctx->reuse_inputs = true;
    a = next;
  }
  ctx->timing.paths |= paths;
  ctx->timing.h2d_bytes = ctx->h2d_bytes;
  return rc;
}

// One call on a plain context: a slot of its pool; x = the exchange of a
// sharded call (null: unsharded).
static int run_plain(tsdbhip_ctx* c, const tsdbhip_sg_desc* desc, tsdbhip_sg_out* out, Xchg* x, bool want_output) {
  try {
    Lease L(c);
    Slot* ctx = L.s;
    ctx->x = x;
    ctx->want_output = want_output;
    try {
      int rc = spangroup_run(ctx, desc, out);
      if (rc) set_error(ctx, "spangroup_run: error %d at output %lld", rc, (long long)out->err_index);
      return rc;
    } catch (Fail& f) {
      out->err_code = f.code;
      if (f.code != TSDBHIP_E_HIP && f.code != TSDBHIP_E_RCCL) {
        out->err_index = 0;
        set_error(ctx, "spangroup_run: error %d", f.code);
      }
      hipStreamSynchronize(ctx->stream);
      return f.code;
    }
  } catch (Fail& f) {  // (no slot)
    out->err_code = f.code;
    return f.code;
  }
}

// ---- in-process sharding (tsdbhip_open_devices) ----
// Rank r of a multi-device context takes the contiguous span range
// [b[r], b[r+1]) of the group (span order kept), balanced by
// cell count for host descs and by span count for device descs, as a desc of
// its own (rows and bytes rebased to the shard).
struct ShardDesc {
  tsdbhip_sg_desc d;
  std::vector<uint64_t> srs, qoff, voff;  // host descs: the rebased arrays
};

static void plan_shards(tsdbhip_ctx* mc, const tsdbhip_sg_desc* desc, std::vector<ShardDesc>& sh) {
  Multi* m = mc->multi;
  Slot* ctx = nullptr;  // (for set_error in the checks)
  const int n = m->n;
  const uint32_t S = desc->n_spans;
  sh.assign(n, ShardDesc());
  std::vector<uint32_t> b(n + 1);
  const bool dev = (desc->flags & TSDBHIP_DESC_DEVICE) != 0;
  std::vector<uint64_t> srs_h;
  const uint64_t* srs = desc->span_row_start;
  if (dev) {  // the span -> row index, read once
    srs_h.resize((size_t)S + 1);
    HIPCHK(hipMemcpy(srs_h.data(), desc->span_row_start, 8ull * (S + 1), hipMemcpyDeviceToHost));
    srs = srs_h.data();
    for (int r = 0; r <= n; r++) b[r] = (uint32_t)((uint64_t)S * r / n);
  } else {  // balanced by points
    std::vector<uint64_t> pre((size_t)S + 1, 0);
    for (uint32_t s = 0; s < S; s++) {
      uint64_t c = 0;
      for (uint64_t r = srs[s]; r < srs[s + 1]; r++) c += desc->row_ncells[r];
      pre[s + 1] = pre[s] + c;
    }
    b[0] = 0;
    b[n] = S;
    for (int r = 1; r < n; r++) {
      const uint64_t want = pre[S] * r / n;
      b[r] = (uint32_t)(std::lower_bound(pre.begin(), pre.end(), want) - pre.begin());
      b[r] = std::max(b[r - 1], std::min(b[r], S));
    }
  }
  for (int r = 0; r < n; r++) {
    ShardDesc& x = sh[r];
    const uint32_t s0 = b[r], s1 = b[r + 1];
    const uint64_t r0 = srs[s0], r1 = srs[s1];
    x.d = *desc;
    x.d.span0 = desc->span0 + s0;  // (global span order of the shard's errors)
    x.d.n_spans = s1 - s0;
    x.d.n_rows = r1 - r0;
    x.srs.resize((size_t)(s1 - s0) + 1);
    for (uint32_t s = s0; s <= s1; s++) x.srs[s - s0] = srs[s] - r0;
    x.d.row_base = desc->row_base + r0;
    x.d.row_ncells = desc->row_ncells + r0;
    x.d.row_val_len = desc->row_val_len + r0;
    if (dev) {
      // (row offsets stay absolute into the shared byte arrays; only the
      // span -> row index moves, uploaded to rank r's device)
      std::string key = "shard_srs";
      tsdbhip_ctx* c = m->members[r];
      Buf& bb = c->owned[key];
      const size_t bytes = 8 * x.srs.size() + 64;
      if (bb.n < bytes) {
        HIPCHK(hipSetDevice(c->device));
        if (bb.p) HIPCHK(hipFree(bb.p));
        bb.p = nullptr;
        HIPCHK(hipMalloc(&bb.p, bytes));
        bb.n = bytes;
      }
      HIPCHK(hipMemcpy(bb.p, x.srs.data(), 8 * x.srs.size(), hipMemcpyHostToDevice));
      x.d.span_row_start = (const uint64_t*)bb.p;
      x.d.row_qual_off = desc->row_qual_off + r0;
      x.d.row_val_off = desc->row_val_off + r0;
      continue;
    }
    // host desc: the shard's byte ranges only (16-B aligned starts keep the
    // packer's row alignment), offsets rebased
    uint64_t qmin = ~0ull, qmax = 0, vmin = ~0ull, vmax = 0;
    for (uint64_t rr = r0; rr < r1; rr++) {
      qmin = std::min<uint64_t>(qmin, desc->row_qual_off[rr]);
      qmax = std::max<uint64_t>(qmax, desc->row_qual_off[rr] + 2ull * desc->row_ncells[rr]);
      vmin = std::min<uint64_t>(vmin, desc->row_val_off[rr]);
      vmax = std::max<uint64_t>(vmax, desc->row_val_off[rr] + desc->row_val_len[rr]);
    }
    if (r1 == r0) qmin = qmax = vmin = vmax = 0;
    qmin &= ~15ull;
    vmin &= ~15ull;
    x.qoff.resize(r1 - r0);
    x.voff.resize(r1 - r0);
    for (uint64_t rr = r0; rr < r1; rr++) {
      x.qoff[rr - r0] = desc->row_qual_off[rr] - qmin;
      x.voff[rr - r0] = desc->row_val_off[rr] - vmin;
    }
    x.d.span_row_start = x.srs.data();
    x.d.row_qual_off = x.qoff.data();
    x.d.row_val_off = x.voff.data();
    x.d.qual_bytes = desc->qual_bytes + qmin;
    x.d.qual_nbytes = std::min<uint64_t>(desc->qual_nbytes, std::max<uint64_t>(qmax, qmin + 16)) - qmin;
    x.d.val_bytes = desc->val_bytes + vmin;
    x.d.val_nbytes = std::min<uint64_t>(desc->val_nbytes, std::max<uint64_t>(vmax, vmin + 16)) - vmin;
  }
}

static int multi_run(tsdbhip_ctx* mc, const tsdbhip_sg_desc* desc, tsdbhip_sg_out* out) {
  Multi* m = mc->multi;
  std::lock_guard<std::mutex> lk(m->call_mu);
  const int n = m->n;
  std::vector<ShardDesc> sh;
  try {
    plan_shards(mc, desc, sh);
  } catch (Fail& f) {
    out->err_code = f.code;
    return f.code;
  }
  std::vector<tsdbhip_sg_out> outs(n);
  std::vector<int> rcs(n, 0);
  std::vector<std::string> errs(n);
  for (int r = 0; r < n; r++) {
    sh[r].d.flags |= TSDBHIP_SHARDED;
    outs[r] = tsdbhip_sg_out();
  }
  outs[0] = *out;
  auto rank_main = [&](int r) {
    rcs[r] = run_plain(m->members[r], &sh[r].d, &outs[r], m->xs[r].get(), r == 0);
    if (rcs[r]) {
      errs[r] = g_thread_err;
      if (!m->rccl) m->local.abort();  // peers waiting at a barrier give up
    }
  };
  std::vector<std::thread> th;
  for (int r = 1; r < n; r++) th.emplace_back(rank_main, r);
  rank_main(0);
  for (auto& t : th) t.join();
  if (!m->rccl) m->local.reset();
  *out = outs[0];
  g_last_ctx = mc;
  g_last_timing = mc->multi->members[0]->last;
  {
    std::lock_guard<std::mutex> l2(mc->mu);
    mc->last = g_last_timing;
    timing_add(mc, g_last_timing);
  }
  int rc = rcs[0];
  int first = -1;
  for (int r = 0; r < n; r++)
    if (rcs[r] && first < 0) first = r;
  if (!rc && first >= 0) rc = rcs[first];
  if (first >= 0) {
    g_thread_err = "rank " + std::to_string(first) + ": " + errs[first];
    if (rc != rcs[0]) out->err_code = rc;
  }
  return rc;
}

extern "C" int tsdbhip_spangroup_run(tsdbhip_ctx* ctx, const tsdbhip_sg_desc* desc, tsdbhip_sg_out* out) {
  if (!ctx || !desc || !out) return TSDBHIP_E_INVALID_ARG;
  if (desc->agg > 4 || (desc->ds_interval > 0 && desc->ds_agg > 4) || desc->ds_interval < 0 ||
      desc->start_time < 0 || desc->end_time < 0) {
    set_error(ctx, "invalid SpanGroup arguments");
    out->err_code = TSDBHIP_E_INVALID_ARG;
    return TSDBHIP_E_INVALID_ARG;
  }
  if (ctx->multi) return multi_run(ctx, desc, out);
  if ((desc->flags & TSDBHIP_SHARDED) && ctx->rccl) {
    std::lock_guard<std::mutex> lk(ctx->comm_mu);  // collectives in the same order on every rank
    return run_plain(ctx, desc, out, ctx->rccl, true);
  }
  return run_plain(ctx, desc, out, nullptr, true);
}

#include "batch.hip"
#include "fmt.hip"

// ------------------------------------------------- synthetic inputs ------
// Device buffers of a generated desc are owned by ctx under keys derived from
// the desc address, so several datasets can coexist.
static std::string synth_key(const tsdbhip_sg_desc* d, const char* f) {
  char b[64];
  snprintf(b, sizeof b, "syn%p_%s", (const void*)d, f);
  return b;
}


extern "C" int tsdbhip_synth_generate(tsdbhip_ctx* c, const tsdbhip_synth_params* p, tsdbhip_sg_desc* d) {
  if (!c || !p || !d || p->n_spans == 0 || p->n_points == 0 || p->step == 0 || 3600 % p->step ||
      p->t0 % 3600 || p->kind > 2)
    return TSDBHIP_E_INVALID_ARG;
  c = plain_of(c);
  try {
    Lease L(c);
    Slot* ctx = L.s;
    SynthArgs a;
    a.seed = p->seed; a.n_spans = p->n_spans; a.n_points = p->n_points; a.t0 = p->t0; a.step = p->step;
    a.kind = p->kind;
    a.span0 = p->span0;
    a.k = 3600 / p->step;
    a.rps = (p->n_points + a.k - 1) / a.k;
    a.w = p->kind == TSDBHIP_SYN_FLOAT32 ? 4 : 8;
    a.flags = p->kind == TSDBHIP_SYN_INT64_COUNTER ? 0x7 : (p->kind == TSDBHIP_SYN_FLOAT32 ? 0xB : 0xF);
    a.qstride = ((2ull * a.k) + 15) / 16 * 16;
    a.vstride = ((uint64_t)a.k * a.w + 1 + 15) / 16 * 16;
    const uint64_t n_rows = (uint64_t)p->n_spans * a.rps;
    auto al = [&](const char* f, size_t bytes) -> void* {
      std::string k = synth_key(d, f);
      void* q = nullptr;
      {
        std::lock_guard<std::mutex> lk(c->mu);
        auto it = c->owned.find(k);
        if (it != c->owned.end()) {
          q = it->second.p;
          c->owned.erase(it);
        }
      }
      if (q) HIPCHK(hipFree(q));
      q = nullptr;
      HIPCHK(hipMalloc(&q, bytes + 64));
      {
        std::lock_guard<std::mutex> lk(c->mu);
        c->owned[k] = Buf{q, bytes + 64};
      }
      HIPCHK(hipMemsetAsync(q, 0, bytes + 64, ctx->stream));
      return q;
    };
    a.span_row_start = (uint64_t*)al("srs", 8ull * (p->n_spans + 1));
    a.row_base = (uint32_t*)al("base", 4ull * n_rows);
    a.row_ncells = (uint32_t*)al("ncells", 4ull * n_rows);
    a.row_qual_off = (uint64_t*)al("qoff", 8ull * n_rows);
    a.row_val_off = (uint64_t*)al("voff", 8ull * n_rows);
    a.row_val_len = (uint32_t*)al("vlen", 4ull * n_rows);
    a.qual = (uint8_t*)al("qual", n_rows * a.qstride);
    a.val = (uint8_t*)al("val", n_rows * a.vstride);
    LAUNCH(k_synth_rows, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx->stream, a);
    const uint64_t cells = (uint64_t)p->n_spans * p->n_points;
    LAUNCH(k_synth_cells, dim3(grid_for(cells, 256, 0x7fffffff)), dim3(256), 0, ctx->stream, a);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    d->flags |= TSDBHIP_DESC_DEVICE;
    d->n_spans = p->n_spans;
    d->n_rows = n_rows;
    d->span_row_start = a.span_row_start;
    d->row_base = a.row_base;
    d->row_ncells = a.row_ncells;
    d->row_qual_off = a.row_qual_off;
    d->row_val_off = a.row_val_off;
    d->row_val_len = a.row_val_len;
    d->qual_bytes = a.qual;
    d->qual_nbytes = n_rows * a.qstride;
    d->val_bytes = a.val;
    d->val_nbytes = n_rows * a.vstride;
  } catch (Fail& f) {
    return f.code;
  }
  return TSDBHIP_OK;
}

extern "C" int tsdbhip_synth_free(tsdbhip_ctx* c, tsdbhip_sg_desc* d) {
  if (!c || !d) return TSDBHIP_E_INVALID_ARG;
  c = plain_of(c);
  hipSetDevice(c->device);
  hipDeviceSynchronize();  // (no call may still read the dataset)
  std::lock_guard<std::mutex> lock(c->mu);
  for (const char* f : {"srs", "base", "ncells", "qoff", "voff", "vlen", "qual", "val"}) {
    auto it = c->owned.find(synth_key(d, f));
    if (it != c->owned.end()) {
      if (it->second.p) hipFree(it->second.p);
      c->owned.erase(it);
    }
  }
  return TSDBHIP_OK;
}

extern "C" int tsdbhip_desc_download(tsdbhip_ctx* c, const tsdbhip_sg_desc* d, uint64_t* srs, uint32_t* base,
                                     uint32_t* ncells, uint64_t* qoff, uint64_t* voff, uint32_t* vlen,
                                     uint8_t* qual, uint8_t* val) {
  if (!c || !d || !(d->flags & TSDBHIP_DESC_DEVICE)) return TSDBHIP_E_INVALID_ARG;
  c = plain_of(c);
  try {
    Lease L(c);
    Slot* ctx = L.s;
    const uint64_t R = d->n_rows;
    HIPCHK(hipMemcpy(srs, d->span_row_start, 8ull * (d->n_spans + 1), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(base, d->row_base, 4 * R, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(ncells, d->row_ncells, 4 * R, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(qoff, d->row_qual_off, 8 * R, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(voff, d->row_val_off, 8 * R, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(vlen, d->row_val_len, 4 * R, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(qual, d->qual_bytes, d->qual_nbytes, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(val, d->val_bytes, d->val_nbytes, hipMemcpyDeviceToHost));
  } catch (Fail& f) {
    return f.code;
  }
  return TSDBHIP_OK;
}

// ------------------------------------------------------- compaction ------
// CompactionQueue.compact (CompactionQueue.java:243-743) for a batch of rows:
// k_compact_wave (a wave per run of rows), k_compact_rows for the rows it leaves, k_compact_complex
// for the biggest complex rows, k_compact_dups for the pending rows' write/delete decisions.
static int compact_rows(Slot* ctx, const tsdbhip_rows_desc* d, tsdbhip_rows_out* out);
extern "C" int tsdbhip_compact_rows(tsdbhip_ctx* c, const tsdbhip_rows_desc* d, tsdbhip_rows_out* out) {
  if (!c || !d || !out) return TSDBHIP_E_INVALID_ARG;
  try {
    Lease L(plain_of(c));
    return compact_rows(L.s, d, out);
  } catch (Fail& f) {
    return f.code;
  }
}

static int compact_rows(Slot* ctx, const tsdbhip_rows_desc* d, tsdbhip_rows_out* out) {
  out->qual_used = out->val_used = out->n_complex = 0;
  const uint64_t R = d->n_rows;
  if (R == 0) return TSDBHIP_OK;
  if (!d->row_kv_start || !d->row_qual_off || !d->row_val_off || (d->n_kvs && (!d->kv_qual_len || !d->kv_val_len)) ||
      !d->qual_bytes || !d->val_bytes || !out->row_status || !out->row_qual_off || !out->row_qual_len ||
      !out->row_val_off || !out->row_val_len || !out->qual_bytes || !out->val_bytes || R >= (1ull << 32) ||
      (!out->row_write != !out->row_keep_kv)) {
    set_error(ctx, "tsdbhip_compact_rows: null array, row_write without row_keep_kv, or too many rows");
    return TSDBHIP_E_INVALID_ARG;
  }
  try {
    const bool dev = (d->flags & TSDBHIP_DESC_DEVICE) != 0;
    ctx->h2d_bytes = 0;
    ctx->reuse_inputs = false;
    // the batch's extents row_qual_off[0], [R], row_val_off[0], [R]: read on
    // the host for a host descriptor; for a device descriptor the kernels
    // read them (k_compact_wave's first lane) and the call checks them with
    // the counters at its end — no round trip before the first launch (every
    // kernel keeps each row inside the buffers and capacities on its own)
    uint64_t ext[4] = {0, 0, 0, 0};
    auto check_ext = [&]() -> int {
      if (ext[1] < ext[0] || ext[3] < ext[2] || ext[1] > d->qual_nbytes || ext[3] > d->val_nbytes) {
        set_error(ctx, "tsdbhip_compact_rows: row offsets out of range");
        return TSDBHIP_E_INVALID_ARG;
      }
      const uint64_t qx = ext[1] - ext[0], vx = ext[3] - ext[2];
      if (out->qual_capacity < qx || out->val_capacity < vx + R) {
        set_error(ctx, "tsdbhip_compact_rows: output needs %llu qualifier / %llu value bytes", (unsigned long long)qx,
                  (unsigned long long)(vx + R));
        return TSDBHIP_E_CAPACITY;
      }
      return TSDBHIP_OK;
    };
    if (!dev) {
      ext[0] = d->row_qual_off[0];
      ext[1] = d->row_qual_off[R];
      ext[2] = d->row_val_off[0];
      ext[3] = d->row_val_off[R];
      if (const int rc = check_ext()) return rc;
    }
    // (device descriptor: bounds for the scratch sizes until the extents are known)
    const uint64_t qext = dev ? d->qual_nbytes : ext[1] - ext[0], vext = dev ? d->val_nbytes : ext[3] - ext[2];
    CompactArgs a = {};
    a.n_rows = R;
    a.n_kvs = d->n_kvs;
    a.row_kv_start = stage(ctx, "c_rks", d->row_kv_start, R + 1, dev);
    a.row_qual_off = stage(ctx, "c_rqo", d->row_qual_off, R + 1, dev);
    a.row_val_off = stage(ctx, "c_rvo", d->row_val_off, R + 1, dev);
    a.kv_qual_len = stage(ctx, "c_kql", d->kv_qual_len, d->n_kvs, dev);
    a.kv_val_len = stage(ctx, "c_kvl", d->kv_val_len, d->n_kvs, dev);
    a.qual = stage(ctx, "c_qual", d->qual_bytes, d->qual_nbytes, dev, 64);
    a.val = stage(ctx, "c_val", d->val_bytes, d->val_nbytes, dev, 64);
    a.qual_nbytes = d->qual_nbytes;
    a.val_nbytes = d->val_nbytes;
    a.qcap = out->qual_capacity;
    a.vcap = out->val_capacity;
    a.out_write = nullptr;
    a.out_keep = nullptr;
    if (dev) {
      a.out_write = out->row_write;
      a.out_keep = out->row_keep_kv;
      a.status = out->row_status;
      a.out_qoff = out->row_qual_off;
      a.out_qlen = out->row_qual_len;
      a.out_voff = out->row_val_off;
      a.out_vlen = out->row_val_len;
      a.oq = out->qual_bytes;
      a.ov = out->val_bytes;
    } else {
      a.status = scratch<uint8_t>(ctx, "c_st", R);
      a.out_qoff = scratch<uint64_t>(ctx, "c_oqo", R);
      a.out_qlen = scratch<uint32_t>(ctx, "c_oql", R);
      a.out_voff = scratch<uint64_t>(ctx, "c_ovo", R);
      a.out_vlen = scratch<uint32_t>(ctx, "c_ovl", R);
      a.oq = scratch<uint8_t>(ctx, "c_oq", qext);
      a.ov = scratch<uint8_t>(ctx, "c_ov", vext + R);
      a.qcap = qext;
      a.vcap = vext + R;
      if (out->row_write || out->row_keep_kv) {  // both, or neither
        a.out_write = scratch<uint8_t>(ctx, "c_ow", R);
        a.out_keep = scratch<int32_t>(ctx, "c_ok", R);
      }
    }
    a.counters = scratch<uint32_t>(ctx, "c_cnt", 16, true);
    a.ext_out = dev ? (uint64_t*)(a.counters + 8) : nullptr;
    a.list_lds = scratch<uint32_t>(ctx, "c_llds", R);
    a.list_big = scratch<uint32_t>(ctx, "c_lbig", R);
    a.big_cells = scratch<uint64_t>(ctx, "c_cells", qext / 2 + R + 1);
    hipStream_t st = ctx->stream;
    g_ev_pend = nullptr;
    g_ev_pend_i = -1;
    std::memset(ctx->ev_alias, 0xff, sizeof ctx->ev_alias);
    const bool det = ctx->opt.timing_detail;
    // the plain rows through k_compact_wave (a wave per run of rows,
    // LDS-staged), the others (CQ_PENDING) through k_compact_rows (a wave per
    // row), the biggest complex rows through k_compact_complex and their
    // write/delete decisions. k_compact_wave's time reads as hot_ms,
    // k_compact_rows' as grid_ms, the rest as reduce_ms (under
    // "timing_detail": each boundary an event; else only the call's first and
    // last events, and hot_ms is the whole call)
    if (!det) ctx->ev_alias[4] = ctx->ev_alias[2] = ctx->ev_alias[9] = ctx->ev_alias[3] = 1;
    else ctx->ev_alias[4] = ctx->ev_alias[2] = 8;
    EV_START(ctx, 8);
    LAUNCH_STOP(det ? EV_STOP_K(ctx, 9) : nullptr, k_compact_wave, dim3(grid_for(R, CW_ROWS * CW_WAVES, 1u << 30)),
                dim3(WAVE * CW_WAVES), 0, st, a);
    if (det) EV_STOP_M(ctx, 9);
    LAUNCH_STOP(det ? EV_STOP_K(ctx, 3) : nullptr, k_compact_rows, dim3(grid_for(R, CR_RANGE, 1u << 14)),
                dim3(WAVE * CR_WAVES), 0, st, a);
    if (det) EV_STOP_M(ctx, 3);
    HIPCHK(hipGetLastError());
    LAUNCH(k_compact_complex<true>, dim3(1024), dim3(256), 0, ctx->stream, a);
    LAUNCH(k_compact_complex<false>, dim3(256), dim3(256), 0, ctx->stream, a);
    if (a.out_write) LAUNCH(k_compact_dups, dim3(256), dim3(256), 0, ctx->stream, a);
    HIPCHK(hipGetLastError());
    EV_FINAL(ctx, 1);
    uint32_t cnt[16];
    readback(ctx, cnt, a.counters, sizeof cnt);
    if (dev) {
      std::memcpy(ext, cnt + 8, sizeof ext);
      if (const int rc = check_ext()) return rc;
    }
    if (cnt[2]) {
      set_error(ctx, "tsdbhip_compact_rows: a row's KV lengths do not match its offsets");
      return TSDBHIP_E_INVALID_ARG;
    }
    const uint64_t n_cx = (uint64_t)cnt[0] + cnt[1] + cnt[3];
    if (!dev) {
      HIPCHK(hipMemcpyAsync(out->row_status, a.status, R, hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipMemcpyAsync(out->row_qual_off, a.out_qoff, 8 * R, hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipMemcpyAsync(out->row_qual_len, a.out_qlen, 4 * R, hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipMemcpyAsync(out->row_val_off, a.out_voff, 8 * R, hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipMemcpyAsync(out->row_val_len, a.out_vlen, 4 * R, hipMemcpyDeviceToHost, ctx->stream));
      if (qext) HIPCHK(hipMemcpyAsync(out->qual_bytes, a.oq, qext, hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipMemcpyAsync(out->val_bytes, a.ov, vext + R, hipMemcpyDeviceToHost, ctx->stream));
      if (a.out_write) {
        HIPCHK(hipMemcpyAsync(out->row_write, a.out_write, R, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(out->row_keep_kv, a.out_keep, 4 * R, hipMemcpyDeviceToHost, ctx->stream));
      }
      HIPCHK(hipStreamSynchronize(ctx->stream));
    }
    tsdbhip_timing t = {};
    t.total_ms = ev_ms(ctx, 8, 1);
    t.hot_ms = ev_ms(ctx, 8, 4) + ev_ms(ctx, 2, 9);  // k_compact_wave
    t.hot_kernel = TSDBHIP_HOT_COMPACT;
    t.decode_ms = ev_ms(ctx, 4, 2);  // (0)
    t.grid_ms = ev_ms(ctx, 9, 3);    // k_compact_rows
    t.reduce_ms = ev_ms(ctx, 3, 1);  // k_compact_complex + k_compact_dups
    t.h2d_bytes = ctx->h2d_bytes;
    ctx->timing = t;
    out->qual_used = ext[1] - ext[0];
    out->val_used = ext[3] - ext[2] + R;
    out->n_complex = n_cx;
  } catch (Fail& f) {
    return f.code;
  }
  return TSDBHIP_OK;
}

// ------------------------------------------------------ bandwidth probe ---
// mode 0: streaming read of a device desc's row bytes with k_ds_spans'
// geometry; mode 1: device-to-device copy of its value bytes. Returns the
// kernel time (HIP events) and the bytes it moved.
extern "C" int tsdbhip_bw_probe(tsdbhip_ctx* c, const tsdbhip_sg_desc* d, int32_t mode, uint32_t width,
                                float* ms, uint64_t* bytes) {
  if (!c || !d || !ms || !bytes || !(d->flags & TSDBHIP_DESC_DEVICE) || (width != 4 && width != 8))
    return TSDBHIP_E_INVALID_ARG;
  try {
    Lease L(plain_of(c));
    Slot* ctx = L.s;
    hipStream_t st = ctx->stream;
    uint32_t* sink = scratch<uint32_t>(ctx, "probe_sink", 1);
    HIPCHK(hipEventRecord(ctx->ev[0], st));
    if (mode == 0) {
      LAUNCH(k_probe_read, dim3(grid_for(d->n_spans, 4, 1u << 20)), dim3(256), 0, st, d->span_row_start,
                         d->row_ncells, d->row_qual_off, d->row_val_off, d->qual_bytes, d->val_bytes, d->n_spans,
                         width, sink);
      *bytes = d->qual_nbytes + d->val_nbytes;
    } else if (mode == 2) {
      const uint64_t n16 = d->val_nbytes / 16;
      LAUNCH(k_probe_flat, dim3(grid_for(n16, 1024, 1u << 16)), dim3(256), 0, st,
                         (const uint4*)d->val_bytes, n16, sink);
      *bytes = n16 * 16;
    } else if (mode == 3) {
      LAUNCH(k_probe_read2, dim3(grid_for(d->n_spans, 4, 1u << 20)), dim3(256), 0, st,
                         d->span_row_start, d->row_ncells, d->row_qual_off, d->row_val_off, d->qual_bytes,
                         d->val_bytes, d->n_spans, sink);
      *bytes = d->qual_nbytes + d->val_nbytes;
    } else {
      const uint64_t n16 = d->val_nbytes / 16;
      uint4* dst = scratch<uint4>(ctx, "probe_dst", n16);
      LAUNCH(k_probe_copy, dim3(grid_for(n16, 256, 1u << 16)), dim3(256), 0, st,
                         (const uint4*)d->val_bytes, dst, n16);
      *bytes = 2 * n16 * 16;
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ctx->ev[1], st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipEventElapsedTime(ms, ctx->ev[0], ctx->ev[1]));  // (markers whatever the "events" option)
  } catch (Fail& f) {
    return f.code;
  }
  return TSDBHIP_OK;
}

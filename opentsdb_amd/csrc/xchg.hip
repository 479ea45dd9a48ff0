// xchg.hip — the exchange step of a series-sharded SpanGroup:
// the few collectives spangroup_run issues between the ranks that each hold
// a contiguous range of the group's spans.
//
//   RcclXchg   one RCCL communicator (ncclAllReduce / AllGather / Broadcast
//              over xGMI): one process per GPU (tsdbhip_comm_init), or one
//              process driving several distinct GPUs (tsdbhip_open_devices,
//              ncclCommInitAll).
//   LocalXchg  the ranks are host threads of this process whose devices may
//              repeat (several shards on one GPU): the same collectives as
//              device-to-device / peer copies ordered by HIP events, the
//              threads meeting at a host barrier. This is what runs an N-rank
//              exchange on a single GPU (tests, oversubscription).
// Every rank issues the same collectives in the same order; buffers are
// device memory, operations are stream-ordered on the caller's stream.
#pragma once
#include <condition_variable>
#include <mutex>
#include <vector>

enum XType { X_U8 = 0, X_I32, X_U32, X_I64, X_U64, X_F64 };
enum XOp { X_SUM = 0, X_MIN, X_MAX };

static size_t xsize(XType t) {
  switch (t) {
    case X_U8: return 1;
    case X_I32:
    case X_U32: return 4;
    default: return 8;
  }
}

struct Xchg {
  int nranks = 1, rank = 0;
  // collective launches of the current call: one per group (RCCL issues a
  // group's operations as one launch at its end) or ungrouped operation
  uint32_t n_coll = 0;
  // bytes this rank receives in the current call's collectives (algorithmic:
  // a ring allreduce 2(N-1)/N of the buffer, an allgather (N-1) blocks, a
  // broadcast one buffer off the root, an alltoall (N-1) blocks)
  uint64_t x_bytes = 0;
  int depth = 0;
  virtual ~Xchg() {}
  void group_start(Slot* ctx) {
    if (depth++ == 0) do_group_start(ctx);
  }
  void group_end(Slot* ctx) {
    if (--depth == 0) {
      do_group_end(ctx);
      n_coll++;
    }
  }
  void allreduce(Slot* ctx, void* buf, size_t count, XType t, XOp op) {
    if (!depth) n_coll++;
    x_bytes += 2 * (uint64_t)(nranks - 1) * count * xsize(t) / nranks;
    do_allreduce(ctx, buf, count, t, op);
  }
  void allgather(Slot* ctx, const void* send, void* recv, size_t bytes) {
    if (!depth) n_coll++;
    x_bytes += (uint64_t)(nranks - 1) * bytes;
    do_allgather(ctx, send, recv, bytes);
  }
  void broadcast(Slot* ctx, const void* send, void* recv, size_t bytes, int root) {
    if (!depth) n_coll++;
    if (rank != root) x_bytes += bytes;
    do_broadcast(ctx, send, recv, bytes, root);
  }
  // recv[q * bytes, (q+1) * bytes) = rank q's send[rank * bytes, (rank+1) * bytes)
  void alltoall(Slot* ctx, const void* send, void* recv, size_t bytes) {
    if (!depth) n_coll++;
    x_bytes += (uint64_t)(nranks - 1) * bytes;
    do_alltoall(ctx, send, recv, bytes);
  }

 protected:
  virtual void do_group_start(Slot* ctx) {}
  virtual void do_group_end(Slot* ctx) {}
  // in place, element-wise over the ranks
  virtual void do_allreduce(Slot* ctx, void* buf, size_t count, XType t, XOp op) = 0;
  // recv[r * bytes, (r+1) * bytes) = rank r's send
  virtual void do_allgather(Slot* ctx, const void* send, void* recv, size_t bytes) = 0;
  // every rank's recv = root's send (the root's recv too)
  virtual void do_broadcast(Slot* ctx, const void* send, void* recv, size_t bytes, int root) = 0;
  virtual void do_alltoall(Slot* ctx, const void* send, void* recv, size_t bytes) = 0;
};

// ---------------------------------------------------------------- RCCL ----
static ncclDataType_t nccl_type(XType t) {
  switch (t) {
    case X_U8: return ncclUint8;
    case X_I32: return ncclInt32;
    case X_U32: return ncclUint32;
    case X_I64: return ncclInt64;
    case X_U64: return ncclUint64;
    default: return ncclFloat64;
  }
}

struct RcclXchg : Xchg {
  ncclComm_t comm = nullptr;
  void do_group_start(Slot* ctx) override { NCCLCHK(ncclGroupStart()); }
  void do_group_end(Slot* ctx) override { NCCLCHK(ncclGroupEnd()); }
  void do_allreduce(Slot* ctx, void* buf, size_t count, XType t, XOp op) override {
    const ncclRedOp_t o = op == X_SUM ? ncclSum : op == X_MIN ? ncclMin : ncclMax;
    NCCLCHK(ncclAllReduce(buf, buf, count, nccl_type(t), o, comm, ctx->stream));
  }
  void do_allgather(Slot* ctx, const void* send, void* recv, size_t bytes) override {
    NCCLCHK(ncclAllGather(send, recv, bytes, ncclUint8, comm, ctx->stream));
  }
  void do_broadcast(Slot* ctx, const void* send, void* recv, size_t bytes, int root) override {
    NCCLCHK(ncclBroadcast(send, recv, bytes, ncclUint8, root, comm, ctx->stream));
  }
  // point-to-point pairs in one group (a nested group inside a caller's)
  void do_alltoall(Slot* ctx, const void* send, void* recv, size_t bytes) override {
    NCCLCHK(ncclGroupStart());
    for (int q = 0; q < nranks; q++) {
      NCCLCHK(ncclSend((const char*)send + (size_t)q * bytes, bytes, ncclUint8, q, comm, ctx->stream));
      NCCLCHK(ncclRecv((char*)recv + (size_t)q * bytes, bytes, ncclUint8, q, comm, ctx->stream));
    }
    NCCLCHK(ncclGroupEnd());
  }
};

// ------------------------------------------------------------ in-process ----
namespace tsdb {
// out[i] = op over ranks r (in rank order) of all[r * count + i]
template <typename T, int OP>
__global__ void k_xreduce(const T* all, uint32_t n, uint64_t count, T* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  T x = all[i];
  for (uint32_t r = 1; r < n; r++) {
    const T y = all[(uint64_t)r * count + i];
    if (OP == X_SUM) x = (T)(x + y);  // (unsigned types: wrapping)
    else if (OP == X_MIN) x = y < x ? y : x;
    else x = y > x ? y : x;
  }
  out[i] = x;
}
}  // namespace tsdb

struct LocalGroup {
  int n = 0;
  std::vector<int> dev;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  std::vector<const void*> ptr;       // each rank's source buffer of the current op
  std::vector<hipEvent_t> ready, done;

  // Host barrier of the n rank threads; throws once a rank has failed (its
  // peers would otherwise wait for it forever).
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (broken) throw Fail{TSDBHIP_E_RCCL};
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      gen++;
      cv.notify_all();
      return;
    }
    cv.wait(lk, [&] { return gen != g || broken; });
    if (gen == g) throw Fail{TSDBHIP_E_RCCL};  // (woken by abort(), not by the last arrival)
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    broken = true;
    cv.notify_all();
  }
  void reset() {
    std::lock_guard<std::mutex> lk(m);
    broken = false;
    arrived = 0;
  }
};

struct LocalXchg : Xchg {
  LocalGroup* G = nullptr;

  void copy_from(Slot* ctx, void* dst, int q, const void* src, size_t bytes) {
    if (!bytes) return;
    if (G->dev[q] == G->dev[rank])
      HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    else
      HIPCHK(hipMemcpyPeerAsync(dst, G->dev[rank], src, G->dev[q], bytes, ctx->stream));
  }
  // publish `src` (ready once this stream reaches here), wait for every rank
  void publish(Slot* ctx, const void* src) {
    G->ptr[rank] = src;
    HIPCHK(hipEventRecord(G->ready[rank], ctx->stream));
    G->barrier();
  }
  // this rank has finished reading the others' buffers; nobody overwrites
  // its source before every reader is done
  void retire(Slot* ctx) {
    HIPCHK(hipEventRecord(G->done[rank], ctx->stream));
    G->barrier();
    for (int q = 0; q < nranks; q++)
      if (q != rank) HIPCHK(hipStreamWaitEvent(ctx->stream, G->done[q], 0));
  }
  void do_allgather(Slot* ctx, const void* send, void* recv, size_t bytes) override {
    publish(ctx, send);
    for (int q = 0; q < nranks; q++) {
      if (q != rank) HIPCHK(hipStreamWaitEvent(ctx->stream, G->ready[q], 0));
      char* dst = (char*)recv + (size_t)q * bytes;
      if (q == rank && dst == (const char*)send) continue;  // (in place)
      copy_from(ctx, dst, q, G->ptr[q], bytes);
    }
    retire(ctx);
  }
  void do_alltoall(Slot* ctx, const void* send, void* recv, size_t bytes) override {
    publish(ctx, send);
    for (int q = 0; q < nranks; q++) {
      if (q != rank) HIPCHK(hipStreamWaitEvent(ctx->stream, G->ready[q], 0));
      copy_from(ctx, (char*)recv + (size_t)q * bytes, q, (const char*)G->ptr[q] + (size_t)rank * bytes, bytes);
    }
    retire(ctx);
  }
  void do_broadcast(Slot* ctx, const void* send, void* recv, size_t bytes, int root) override {
    publish(ctx, send);
    if (rank != root) HIPCHK(hipStreamWaitEvent(ctx->stream, G->ready[root], 0));
    if (rank != root || send != recv) copy_from(ctx, recv, root, G->ptr[root], bytes);
    retire(ctx);
  }
  void do_allreduce(Slot* ctx, void* buf, size_t count, XType t, XOp op) override {
    const size_t bytes = count * xsize(t);
    uint8_t* all = scratch<uint8_t>(ctx, "x_allreduce", bytes * nranks);
    do_allgather(ctx, buf, all, bytes);
    if (!count) return;
    const dim3 g(grid_for(count, 256)), b(256);
    const uint32_t n = (uint32_t)nranks;
#define XR(T, O) hipLaunchKernelGGL((k_xreduce<T, O>), g, b, 0, ctx->stream, (const T*)all, n, (uint64_t)count, (T*)buf)
#define XR3(TS, TM)              \
  if (op == X_SUM) XR(TS, X_SUM); \
  else if (op == X_MIN) XR(TM, X_MIN); \
  else XR(TM, X_MAX)
    switch (t) {
      case X_U8: XR3(uint8_t, uint8_t); break;
      case X_I32: XR3(uint32_t, int32_t); break;
      case X_U32: XR3(uint32_t, uint32_t); break;
      case X_I64: XR3(uint64_t, int64_t); break;
      case X_U64: XR3(uint64_t, uint64_t); break;
      default: XR3(double, double); break;
    }
#undef XR3
#undef XR
  }
};

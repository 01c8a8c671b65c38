// Data-parallel gradient exchange over RCCL (xGMI between the GPUs of a node).
//
// The reference has no distributed code. Data parallelism here shards the users
// over the ranks, so the user table and its Adam moments never move; the one exchange per step is
// the mean of the replicated dense gradient: 393,276 floats (1.57 MB) at d = H = 128. The library
// calls RCCL itself, so a data-parallel step stays a single host call (dcue_plan_step): RCCL's
// launch cost is a few microseconds, where a Python all-reduce per bucket plus the stream waits
// and a separate divide cost tens of microseconds of host time on a step that is host-issue bound.
//
// A process loads torch (which links RCCL) before this library, so its librccl.so.1 is the one
// resolved here: one RCCL per process.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>

#include "dcue_internal.h"

struct dcue_comm {
  ncclComm_t nc = nullptr;         // RCCL transport (dcue_comm_create)
  dcue_host_allreduce_fn host_fn = nullptr;  // host transport (dcue_comm_create_host)
  void* host_ctx = nullptr;
  void* hbuf = nullptr;            // pinned staging of the host transport
  size_t hbuf_bytes = 0;
  int world = 1, rank = 0;
  hipStream_t stream = nullptr;  // the exchange's own stream (beside the step's side streams)
  hipEvent_t ev_tail = nullptr;  // the caller's stream at the step's end
  hipEvent_t ev_done = nullptr;  // the exchange complete
};

namespace dcue {

namespace {
int nccl_status(ncclResult_t r, const char* what, int line) {
  if (r == ncclSuccess) return DCUE_OK;
  char msg[160];
  snprintf(msg, sizeof msg, "%s: %s", what, ncclGetErrorString(r));
  set_last_error(msg, hipErrorUnknown, __FILE__, line);
  return DCUE_ERR_HIP;
}
}  // namespace

#define DCUE_NCCL_CHECK(call)                                         \
  do {                                                                \
    const int st_ = nccl_status((call), #call, __LINE__);             \
    if (st_) return st_;                                              \
  } while (0)

__global__ __launch_bounds__(256) void k_div_world(float* __restrict__ buf, long n, float w) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    buf[i] = __fdiv_rn(buf[i], w);  // grad.div_(world)
}

// Host transport: the comm's stream is drained (it has waited for whatever produced `buf`), the
// buffer is staged through pinned host memory, the caller's function sums it over the ranks, and
// the result goes back, all before this returns. The plan's exchange keeps its stream/event order,
// so the same library code runs over either transport.
static int host_allreduce(dcue_comm* c, void* buf, long n, int dtype) {
  const size_t bytes = (size_t)n * (dtype == DCUE_COMM_U64 ? 8 : 4);
  if (bytes > c->hbuf_bytes) {
    if (c->hbuf) DCUE_HIP_CHECK(hipHostFree(c->hbuf));
    c->hbuf = nullptr;
    c->hbuf_bytes = 0;
    DCUE_HIP_CHECK(hipHostMalloc(&c->hbuf, bytes, hipHostMallocDefault));
    c->hbuf_bytes = bytes;
  }
  DCUE_HIP_CHECK(hipMemcpyAsync(c->hbuf, buf, bytes, hipMemcpyDeviceToHost, c->stream));
  DCUE_HIP_CHECK(hipStreamSynchronize(c->stream));
  if (c->host_fn(c->host_ctx, c->hbuf, (int64_t)n, dtype) != 0) {
    set_last_error("dcue_comm host transport: the all-reduce callback failed", hipSuccess, __FILE__, __LINE__);
    return DCUE_ERR_HIP;
  }
  DCUE_HIP_CHECK(hipMemcpyAsync(buf, c->hbuf, bytes, hipMemcpyHostToDevice, c->stream));
  DCUE_HIP_CHECK(hipStreamSynchronize(c->stream));
  return DCUE_OK;
}

// Sum all-reduce of n floats in place on the comm's stream; timed as DCUE_TIMED_ALLREDUCE.
int comm_allreduce_sum(dcue_comm* c, float* buf, long n) {
  if (n <= 0) return DCUE_OK;
  if (c->host_fn) return host_allreduce(c, buf, n, DCUE_COMM_F32);
  hipEvent_t a = nullptr, b = nullptr;
  if (timer_take_turn(DCUE_TIMED_ALLREDUCE)) {
    a = timer_event();
    b = timer_event();
    if (!a || !b) return DCUE_ERR_HIP;
    DCUE_HIP_CHECK(hipEventRecord(a, c->stream));
  }
  DCUE_NCCL_CHECK(ncclAllReduce(buf, buf, (size_t)n, ncclFloat, ncclSum, c->nc, c->stream));
  if (a) {
    DCUE_HIP_CHECK(hipEventRecord(b, c->stream));
    timer_add_recorded(DCUE_TIMED_ALLREDUCE, a, b);
  }
  return DCUE_OK;
}

int comm_world(const dcue_comm* c) { return c->world; }

int comm_allreduce_u64(dcue_comm* c, unsigned long long* buf, long n, hipStream_t s) {
  if (n <= 0) return DCUE_OK;
  DCUE_HIP_CHECK(hipEventRecord(c->ev_tail, s));
  DCUE_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_tail, 0));
  if (c->host_fn) {
    TRY(host_allreduce(c, buf, n, DCUE_COMM_U64));
  } else {
    DCUE_NCCL_CHECK(ncclAllReduce(buf, buf, (size_t)n, ncclUint64, ncclSum, c->nc, c->stream));
  }
  DCUE_HIP_CHECK(hipEventRecord(c->ev_done, c->stream));
  DCUE_HIP_CHECK(hipStreamWaitEvent(s, c->ev_done, 0));
  return DCUE_OK;
}

// The plan's exchange (dcue_plan_set_comm): `side_done` marks the side streams' join (the flat
// gradient is final past `late` floats), the caller's stream `s` is at the step's end. Returns with
// `s` waiting for both buckets.
int comm_exchange_step(dcue_comm* c, float* grad, long late, long n, hipEvent_t side_done, hipStream_t s) {
  DCUE_HIP_CHECK(hipStreamWaitEvent(c->stream, side_done, 0));
  TRY(comm_allreduce_sum(c, grad + late, n - late));
  DCUE_HIP_CHECK(hipEventRecord(c->ev_tail, s));
  DCUE_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_tail, 0));
  TRY(comm_allreduce_sum(c, grad, late));
  DCUE_HIP_CHECK(hipEventRecord(c->ev_done, c->stream));
  DCUE_HIP_CHECK(hipStreamWaitEvent(s, c->ev_done, 0));
  return DCUE_OK;
}

int comm_exchange_split(dcue_comm* c, const dcue_model* m, const dcue_adam_args* dense, const int64_t* poff,
                        long late, long n, const hipEvent_t* side, int nside, hipEvent_t late_done, hipStream_t s) {
  for (int i = 0; i < nside; ++i)
    if (side[i]) DCUE_HIP_CHECK(hipStreamWaitEvent(c->stream, side[i], 0));
  TRY(comm_allreduce_sum(c, m->grads + late, n - late));
  // The caller's stream may still run its last input gradient, the dgrad of conv 2, which reads conv
  // 2's packed weights: the late Adam leaves those to the next forward of conv 2 (launch_adam
  // defer_dgrad2), so it waits for nothing on `s` and overlaps the conv-1 weight gradient
  // (DCUE_LEGACY_ORDERS=1: the round-4 order, the repack here)
  TRY(debug_delay(DCUE_SITE_LATE_ADAM, c->stream));
  TRY(launch_adam(m, dense, poff, c->stream, true, late, n, !legacy_orders()));  // the late segments' Adam, divide fused
  DCUE_HIP_CHECK(hipEventRecord(late_done, c->stream));
  DCUE_HIP_CHECK(hipEventRecord(c->ev_tail, s));
  DCUE_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_tail, 0));
  TRY(comm_allreduce_sum(c, m->grads, late));
  DCUE_HIP_CHECK(hipEventRecord(c->ev_done, c->stream));
  DCUE_HIP_CHECK(hipStreamWaitEvent(s, c->ev_done, 0));
  return DCUE_OK;
}

// grad[0:n) /= world on `s` (DDP's grad.div_(world)), for steps whose optimizer does not fold the
// divide into its sweep (plan launches followed by a separate optimizer call)
int comm_divide(const dcue_comm* c, float* grad, long n, hipStream_t s) {
  if (c->world <= 1 || n <= 0) return DCUE_OK;
  const long blocks = std::min<long>((n + 255) / 256, 2048);
  DCUE_LAUNCH(k_div_world, dim3((unsigned)blocks), dim3(256), 0, s, grad, n, (float)c->world);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue

using namespace dcue;

extern "C" int dcue_comm_unique_id(void* id_host) {
  static_assert(sizeof(ncclUniqueId) == DCUE_COMM_ID_BYTES, "RCCL unique id size");
  if (!id_host) return DCUE_ERR_INVALID;
  ncclUniqueId id;
  DCUE_NCCL_CHECK(ncclGetUniqueId(&id));
  memcpy(id_host, &id, sizeof id);
  return DCUE_OK;
}

extern "C" int dcue_comm_create(const void* id_host, int32_t world, int32_t rank, dcue_comm** comm_host) {
  if (!id_host || !comm_host || world < 1 || rank < 0 || rank >= world) return DCUE_ERR_INVALID;
  *comm_host = nullptr;
  ncclUniqueId id;
  memcpy(&id, id_host, sizeof id);
  dcue_comm* c = new dcue_comm;
  c->world = world;
  c->rank = rank;
  int st = nccl_status(ncclCommInitRank(&c->nc, world, id, rank), "ncclCommInitRank", __LINE__);
  if (!st && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) st = DCUE_ERR_HIP;
  if (!st && hipEventCreateWithFlags(&c->ev_tail, sync_event_flags()) != hipSuccess) st = DCUE_ERR_HIP;
  if (!st && hipEventCreateWithFlags(&c->ev_done, sync_event_flags()) != hipSuccess) st = DCUE_ERR_HIP;
  if (st) {
    dcue_comm_destroy(c);
    return st;
  }
  *comm_host = c;
  return DCUE_OK;
}

extern "C" int dcue_comm_create_host(int32_t world, int32_t rank, dcue_host_allreduce_fn fn, void* ctx,
                                     dcue_comm** comm_host) {
  if (!fn || !comm_host || world < 1 || rank < 0 || rank >= world) return DCUE_ERR_INVALID;
  *comm_host = nullptr;
  dcue_comm* c = new dcue_comm;
  c->world = world;
  c->rank = rank;
  c->host_fn = fn;
  c->host_ctx = ctx;
  int st = DCUE_OK;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) st = DCUE_ERR_HIP;
  if (!st && hipEventCreateWithFlags(&c->ev_tail, sync_event_flags()) != hipSuccess) st = DCUE_ERR_HIP;
  if (!st && hipEventCreateWithFlags(&c->ev_done, sync_event_flags()) != hipSuccess) st = DCUE_ERR_HIP;
  if (st) {
    dcue_comm_destroy(c);
    return st;
  }
  *comm_host = c;
  return DCUE_OK;
}

extern "C" int dcue_comm_destroy(dcue_comm* c) {
  if (!c) return DCUE_OK;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->nc) (void)ncclCommDestroy(c->nc);
  if (c->hbuf) (void)hipHostFree(c->hbuf);
  if (c->ev_tail) (void)hipEventDestroy(c->ev_tail);
  if (c->ev_done) (void)hipEventDestroy(c->ev_done);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return DCUE_OK;
}

extern "C" int dcue_comm_allgather(dcue_comm* c, float* buf, int64_t count, void* stream) {
  if (!c || (!buf && count > 0) || count < 0) return DCUE_ERR_INVALID;
  if (count == 0 || c->world == 1) return DCUE_OK;
  hipStream_t s = (hipStream_t)stream;
  DCUE_HIP_CHECK(hipEventRecord(c->ev_tail, s));
  DCUE_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_tail, 0));
  const size_t part = sizeof(float) * (size_t)count;
  if (c->host_fn) {  // exact: every part is its owner's values plus zeros
    if (c->rank > 0) DCUE_HIP_CHECK(hipMemsetAsync(buf, 0, part * c->rank, c->stream));
    if (c->rank + 1 < c->world)
      DCUE_HIP_CHECK(hipMemsetAsync(buf + (size_t)count * (c->rank + 1), 0, part * (c->world - c->rank - 1), c->stream));
    TRY(host_allreduce(c, buf, count * c->world, DCUE_COMM_F32));
  } else {
    DCUE_NCCL_CHECK(ncclAllGather(buf + (size_t)count * c->rank, buf, (size_t)count, ncclFloat, c->nc, c->stream));
  }
  DCUE_HIP_CHECK(hipEventRecord(c->ev_done, c->stream));
  DCUE_HIP_CHECK(hipStreamWaitEvent(s, c->ev_done, 0));
  return DCUE_OK;
}

extern "C" int dcue_comm_allreduce_mean(dcue_comm* c, float* buf, int64_t n, void* stream) {
  if (!c || (!buf && n > 0) || n < 0) return DCUE_ERR_INVALID;
  if (n == 0) return DCUE_OK;
  hipStream_t s = (hipStream_t)stream;
  DCUE_HIP_CHECK(hipEventRecord(c->ev_tail, s));
  DCUE_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_tail, 0));
  TRY(comm_allreduce_sum(c, buf, n));
  DCUE_HIP_CHECK(hipEventRecord(c->ev_done, c->stream));
  DCUE_HIP_CHECK(hipStreamWaitEvent(s, c->ev_done, 0));
  return comm_divide(c, buf, (long)n, s);
}

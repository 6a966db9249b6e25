// Collectives for the landmark-sharded local BA (include/rspl.h, rspl_ba_set_shard):
//  * rspl_comm  -- RCCL over xGMI, one process per GPU.  librccl is dlopen'ed at first use, so
//                  the product library carries no load-time RCCL dependency.
//  * rspl_group -- nranks handles on ONE device in one process, one host thread each: two host
//                  barriers per all-reduce around stream-ordered work (inputs ready -> every rank
//                  sums all inputs in rank order into its own staging -> everyone has read ->
//                  copy back), so no stream is ever synchronised by the host.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "shard.hpp"

using namespace rspl;

// ---------------------------------------------------------------------------
// RCCL
// ---------------------------------------------------------------------------
namespace {

struct Rccl {
  bool ok = false;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) =
      nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.all_reduce && r.comm_destroy && r.error_string;
  });
  return &r;
}

}  // namespace

struct rspl_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1, device = 0;
};

extern "C" int rspl_comm_unique_id(uint8_t* id) {
  RSPL_CHECK_ARG(id, "rspl_comm_unique_id: NULL id");
  const Rccl* r = rccl();
  if (!r->ok) {
    set_error("librccl could not be loaded");
    return RSPL_E_DEVICE;
  }
  ncclUniqueId u;
  const ncclResult_t e = r->get_unique_id(&u);
  if (e != ncclSuccess) {
    set_error("ncclGetUniqueId: %s", r->error_string(e));
    return RSPL_E_DEVICE;
  }
  static_assert(sizeof(u.internal) == RSPL_COMM_ID_BYTES, "unique id size");
  memcpy(id, u.internal, RSPL_COMM_ID_BYTES);
  return RSPL_OK;
}

extern "C" int rspl_comm_create(const uint8_t* id, int rank, int nranks, int device, rspl_comm** out) {
  RSPL_CHECK_ARG(id && out && nranks >= 1 && rank >= 0 && rank < nranks, "rspl_comm_create: bad arguments");
  *out = nullptr;
  const Rccl* r = rccl();
  if (!r->ok) {
    set_error("librccl could not be loaded");
    return RSPL_E_DEVICE;
  }
  RSPL_HIP(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(u.internal, id, RSPL_COMM_ID_BYTES);
  auto* c = new rspl_comm();
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  const ncclResult_t e = r->comm_init_rank(&c->comm, nranks, u, rank);
  if (e != ncclSuccess) {
    set_error("ncclCommInitRank(rank %d of %d): %s", rank, nranks, r->error_string(e));
    delete c;
    return RSPL_E_DEVICE;
  }
  *out = c;
  return RSPL_OK;
}

extern "C" int rspl_comm_allreduce_sum(void* comm, double* d, size_t count, void* stream) {
  auto* c = static_cast<rspl_comm*>(comm);
  RSPL_CHECK_ARG(c && (d || !count), "rspl_comm_allreduce_sum: bad arguments");
  if (!count) return RSPL_OK;
  const Rccl* r = rccl();
  const ncclResult_t e = r->all_reduce(d, d, count, ncclDouble, ncclSum, c->comm, static_cast<hipStream_t>(stream));
  if (e != ncclSuccess) {
    set_error("ncclAllReduce: %s", r->error_string(e));
    return RSPL_E_DEVICE;
  }
  return RSPL_OK;
}

extern "C" void rspl_comm_destroy(rspl_comm* c) {
  if (!c) return;
  if (c->comm) (void)rccl()->comm_destroy(c->comm);
  delete c;
}

extern "C" int rspl_ba_set_comm(rspl_ba* ba, rspl_comm* c) {
  RSPL_CHECK_ARG(ba && c, "rspl_ba_set_comm: NULL argument");
  return rspl_ba_set_shard(ba, c->rank, c->nranks, rspl_comm_allreduce_sum, c);
}

// ---------------------------------------------------------------------------
// in-process group
// ---------------------------------------------------------------------------
struct rspl_group {
  struct RankCtx {
    rspl_group* g;
    int rank;
  };
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  unsigned long long gen = 0;
  bool broken = false;
  std::vector<double*> bufs;
  std::vector<size_t> counts;
  std::vector<hipEvent_t> ev_in, ev_sum;
  std::vector<double*> stage;
  std::vector<size_t> stage_cap;
  std::vector<RankCtx> ctx;

  // generation barrier, bounded: a rank that never arrives (it failed before the collective)
  // breaks the group instead of hanging the others
  bool barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (broken) return false;
    const unsigned long long g0 = gen;
    if (++arrived == n) {
      arrived = 0;
      gen++;
      cv.notify_all();
      return true;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return gen != g0 || broken; }) || broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

namespace {

int group_allreduce(void* vctx, double* d, size_t count, void* vstream) {
  auto* rc = static_cast<rspl_group::RankCtx*>(vctx);
  rspl_group* g = rc->g;
  const int r = rc->rank;
  auto st = static_cast<hipStream_t>(vstream);
  if (count > g->stage_cap[r]) {  // staging grows once (the stream is drained first)
    RSPL_HIP(hipStreamSynchronize(st));
    if (g->stage[r]) (void)hipFree(g->stage[r]);
    g->stage[r] = nullptr;
    g->stage_cap[r] = 0;
    RSPL_HIP(hipMalloc((void**)&g->stage[r], sizeof(double) * count));
    g->stage_cap[r] = count;
  }
  g->bufs[r] = d;
  g->counts[r] = count;
  RSPL_HIP(hipEventRecord(g->ev_in[r], st));
  if (!g->barrier()) {
    set_error("rspl_group: rank %d timed out waiting for the other ranks", r);
    return RSPL_E_DEVICE;
  }
  for (int q = 0; q < g->n; q++)
    if (g->counts[q] != count) {
      set_error("rspl_group: ranks disagree on the all-reduce length (%zu vs %zu)", g->counts[q], count);
      g->broken = true;
      return RSPL_E_ARG;
    }
  shard::SumArgs a{};
  for (int q = 0; q < g->n; q++) {
    RSPL_HIP(hipStreamWaitEvent(st, g->ev_in[q], 0));
    a.src[q] = g->bufs[q];
  }
  a.dst = g->stage[r];
  a.count = count;
  a.n = g->n;
  RSPL_HIP(shard::group_sum(a, st));
  RSPL_HIP(hipEventRecord(g->ev_sum[r], st));
  if (!g->barrier()) {
    set_error("rspl_group: rank %d timed out waiting for the other ranks", r);
    return RSPL_E_DEVICE;
  }
  for (int q = 0; q < g->n; q++) RSPL_HIP(hipStreamWaitEvent(st, g->ev_sum[q], 0));  // all inputs read
  if (count) RSPL_HIP(hipMemcpyAsync(d, g->stage[r], sizeof(double) * count, hipMemcpyDeviceToDevice, st));
  return RSPL_OK;
}

}  // namespace

extern "C" int rspl_group_create(int nranks, rspl_group** out) {
  RSPL_CHECK_ARG(out && nranks >= 1 && nranks <= shard::kMaxGroup, "rspl_group_create: 1..%d ranks",
                 shard::kMaxGroup);
  auto* g = new rspl_group();
  g->n = nranks;
  g->bufs.assign(nranks, nullptr);
  g->counts.assign(nranks, 0);
  g->ev_in.assign(nranks, nullptr);
  g->ev_sum.assign(nranks, nullptr);
  g->stage.assign(nranks, nullptr);
  g->stage_cap.assign(nranks, 0);
  g->ctx.resize(nranks);
  for (int r = 0; r < nranks; r++) {
    g->ctx[r] = {g, r};
    if (hipEventCreateWithFlags(&g->ev_in[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_sum[r], hipEventDisableTiming) != hipSuccess) {
      set_error("rspl_group_create: event creation failed");
      rspl_group_destroy(g);
      return RSPL_E_DEVICE;
    }
  }
  *out = g;
  return RSPL_OK;
}

extern "C" void rspl_group_destroy(rspl_group* g) {
  if (!g) return;
  (void)hipDeviceSynchronize();
  for (int r = 0; r < g->n; r++) {
    if (g->ev_in[r]) (void)hipEventDestroy(g->ev_in[r]);
    if (g->ev_sum[r]) (void)hipEventDestroy(g->ev_sum[r]);
    if (g->stage[r]) (void)hipFree(g->stage[r]);
  }
  delete g;
}

extern "C" int rspl_ba_set_group(rspl_ba* ba, rspl_group* g, int rank) {
  RSPL_CHECK_ARG(ba && g && rank >= 0 && rank < g->n, "rspl_ba_set_group: bad arguments");
  return rspl_ba_set_shard(ba, rank, g->n, group_allreduce, &g->ctx[rank]);
}

// Communicators of the row-partitioned handles: RCCL (one rank per GPU) and the in-process
// thread group (W ranks on one device), and their C-ABI constructors.
#include "engine.h"

#include <atomic>
#include <shared_mutex>

using namespace n2v2r_int;

namespace n2v2r_int {
// abort() may come from the multi handle's coordinator thread while rank threads enqueue
// collectives on the same communicator.  `aborted` is atomic and every operation checks it
// under a shared lock held only while it enqueues (the host call returns once the collective is
// queued; a rank stuck later waits in its stream synchronisation, which the abort unblocks), so
// no operation is enqueued on a communicator ncclCommAbort has freed: it throws NcclFail
// (ncclInvalidUsage) instead.  The abort takes the lock exclusively, waiting at most 2 s for
// enqueues in progress (an enqueue that never returns must not keep the peers hanging).
struct RcclComm : Comm {
  ncclComm_t c = nullptr;
  std::atomic<bool> aborted{false};
  std::shared_timed_mutex mu;
  ~RcclComm() override {
    if (c && !aborted.load()) (void)ncclCommDestroy(c);
  }
  void abort() override {
    const bool locked = mu.try_lock_for(std::chrono::seconds(2));
    if (c && !aborted.exchange(true)) (void)ncclCommAbort(c);
    if (locked) mu.unlock();
  }
  template <class F>
  void op(const char* what, F&& f) {
    std::shared_lock<std::shared_timed_mutex> lk(mu);
    if (aborted.load()) throw NcclFail{ncclInvalidUsage, std::string(what) + " (communicator aborted)"};
    const ncclResult_t r = f();
    if (r != ncclSuccess) throw NcclFail{r, what};
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t st) override {
    op("ncclAllGather", [&] { return ncclAllGather(send, recv, bytes, ncclChar, c, st); });
  }
  void allreduce_sum_f64(double* buf, size_t count, hipStream_t st) override {
    op("ncclAllReduce(f64 sum)",
       [&] { return ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, c, st); });
  }
  void allreduce_max_u64(unsigned long long* buf, size_t count, hipStream_t st) override {
    op("ncclAllReduce(u64 max)",
       [&] { return ncclAllReduce(buf, buf, count, ncclUint64, ncclMax, c, st); });
  }
  void allreduce_sum_f32(float* buf, size_t count, hipStream_t st) override {
    op("ncclAllReduce(f32 sum)",
       [&] { return ncclAllReduce(buf, buf, count, ncclFloat, ncclSum, c, st); });
  }
  void reduce_scatter_sum_f32(const float* send, float* recv, size_t count,
                              hipStream_t st) override {
    op("ncclReduceScatter",
       [&] { return ncclReduceScatter(send, recv, count, ncclFloat, ncclSum, c, st); });
  }
  const char* kind() const override { return "rccl"; }
};

std::unique_ptr<Comm> make_rccl_comm(ncclComm_t c, int rank, int world) {
  auto r = std::make_unique<RcclComm>();
  r->c = c;
  r->rank = rank;
  r->world = world;
  return r;
}


struct ThreadComm : Comm {
  n2v2r_simgroup* g = nullptr;
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t st) override {
    HIPCHK(hipStreamSynchronize(st));
    g->ptrs[rank] = send;
    g->barrier();
    for (int r = 0; r < world; ++r)
      HIPCHK(hipMemcpyAsync(static_cast<char*>(recv) + (size_t)r * bytes, g->ptrs[r], bytes,
                            hipMemcpyDeviceToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    g->barrier();
  }
  template <class T, class Op>
  void allreduce(T* buf, size_t count, hipStream_t st, Op op) {
    auto& mine = g->host[rank];
    mine.resize(sizeof(T) * count);
    HIPCHK(hipMemcpyAsync(mine.data(), buf, sizeof(T) * count, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    g->barrier();
    std::vector<T> acc(count);
    std::memcpy(acc.data(), g->host[0].data(), sizeof(T) * count);
    for (int r = 1; r < world; ++r) {
      const T* o = reinterpret_cast<const T*>(g->host[r].data());
      for (size_t i = 0; i < count; ++i) acc[i] = op(acc[i], o[i]);
    }
    g->barrier();
    HIPCHK(hipMemcpyAsync(buf, acc.data(), sizeof(T) * count, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  void allreduce_sum_f64(double* buf, size_t count, hipStream_t st) override {
    allreduce(buf, count, st, [](double a, double b) { return a + b; });
  }
  void allreduce_max_u64(unsigned long long* buf, size_t count, hipStream_t st) override {
    allreduce(buf, count, st,
              [](unsigned long long a, unsigned long long b) { return a > b ? a : b; });
  }
  void allreduce_sum_f32(float* buf, size_t count, hipStream_t st) override {
    allreduce(buf, count, st, [](float a, float b) { return a + b; });
  }
  // fixed rank order, on the device (every rank's send buffer is on this one device)
  void reduce_scatter_sum_f32(const float* send, float* recv, size_t count,
                              hipStream_t st) override {
    HIPCHK(hipStreamSynchronize(st));
    g->ptrs[rank] = send;
    g->barrier();
    const int64_t rows8 = (int64_t)(count / 8);  // count is a multiple of 8 (b = 8..64 panels)
    int r = 0;
    bool first = true;
    while (r < world) {  // 8 ranks, then the running sum + 7 more at a time
      const float* parts[8];
      int np = 0;
      if (!first) parts[np++] = recv;
      while (r < world && np < 8)
        parts[np++] = static_cast<const float*>(g->ptrs[r++]) + (size_t)rank * count;
      HIPCHK(n2v2r_launch_zsum(parts, np, recv, rows8, st));
      first = false;
    }
    HIPCHK(hipStreamSynchronize(st));
    g->barrier();  // no rank rewrites its send buffer while another still reads it
  }
  const char* kind() const override { return "thread"; }
  bool shares_device() const override {
    std::lock_guard<std::mutex> lk(g->m);
    for (int r = 0; r < world; ++r)
      if (r != rank && g->dev[r] == g->dev[rank]) return true;
    return false;
  }
  void abort() override { g->abort(); }
};

std::unique_ptr<Comm> make_thread_comm(n2v2r_simgroup* g, int rank, int device) {
  auto t = std::make_unique<ThreadComm>();
  t->g = g;
  t->rank = rank;
  t->world = g->world;
  {
    std::lock_guard<std::mutex> lk(g->m);
    if (g->dev.size() != (size_t)g->world) g->dev.assign(g->world, -1);
    g->dev[rank] = device;
  }
  return t;
}
}  // namespace n2v2r_int

extern "C" {

int n2v2r_comm_unique_id(char* out, size_t len) {
  if (!out || len < sizeof(ncclUniqueId)) return N2V2R_ERR_BAD_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return N2V2R_ERR_RCCL;
  std::memcpy(out, &id, sizeof(id));
  return N2V2R_OK;
}

int n2v2r_create_rccl(int device, int rank, int world, const char* unique_id,
                      n2v2r_handle** out) {
  if (!out || !unique_id || world < 1 || rank < 0 || rank >= world) return N2V2R_ERR_BAD_ARG;
  *out = nullptr;
  n2v2r_handle* h = new_handle(device);
  if (!h) return N2V2R_ERR_HIP;
  auto c = std::make_unique<RcclComm>();
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  c->rank = rank;
  c->world = world;
  if (ncclCommInitRank(&c->c, world, id, rank) != ncclSuccess) {
    n2v2r_destroy(h);
    return N2V2R_ERR_RCCL;
  }
  h->rank = rank;
  h->world = world;
  h->comm = std::move(c);
  *out = h;
  return N2V2R_OK;
}

int n2v2r_simgroup_create(int world, n2v2r_simgroup** out) {
  if (!out || world < 1) return N2V2R_ERR_BAD_ARG;
  auto* g = new (std::nothrow) n2v2r_simgroup();
  if (!g) return N2V2R_ERR_OUT_OF_MEMORY;
  g->world = world;
  g->ptrs.assign(world, nullptr);
  g->host.resize(world);
  g->dev.assign(world, -1);
  *out = g;
  return N2V2R_OK;
}

void n2v2r_simgroup_destroy(n2v2r_simgroup* g) { delete g; }

int n2v2r_create_sim(int device, n2v2r_simgroup* g, int rank, n2v2r_handle** out) {
  if (!out || !g || rank < 0 || rank >= g->world) return N2V2R_ERR_BAD_ARG;
  *out = nullptr;
  n2v2r_handle* h = new_handle(device);
  if (!h) return N2V2R_ERR_HIP;
  h->rank = rank;
  h->world = g->world;
  h->comm = make_thread_comm(g, rank, device);
  *out = h;
  return N2V2R_OK;
}

int n2v2r_dist_info(const n2v2r_handle* h, int* rank, int* world, int64_t* row0,
                    int64_t* n_local) {
  if (!h) return N2V2R_ERR_BAD_ARG;
  if (rank) *rank = h->rank;
  if (world) *world = h->world;
  if (row0) *row0 = h->row0;
  if (n_local) *n_local = h->nloc;
  return N2V2R_OK;
}

}  // extern "C"

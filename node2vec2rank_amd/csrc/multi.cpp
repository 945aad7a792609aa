// One process, N GPUs: the drop-in API's multi-GPU handle (n2v2r_create_multi, include/n2v2r.h).
//
// "one host thread drives all GPUs ... or one thread per GPU internal to the
// library".  A multi handle owns one row-partitioned rank handle per device (the same ranks the
// one-process-per-GPU RCCL path builds, SURVEY 8(e): rank g owns rows [g R, (g + 1) R) of every
// layer, Krylov block and embedding) and a communicator over all of them: RCCL over the
// process's devices (ncclCommInitAll) when they are distinct, the in-process thread group when a
// device repeats (W ranks on one GPU: how the tests run it on a one-GPU box).  Every C-ABI call
// on the multi handle runs the same call on every rank, one host thread per rank (collective
// semantics), and the results come back as from a single-GPU handle: global embeddings, global
// distance / Borda tables, rank 0's solver statistics (every rank takes identical decisions).
//
// Failure: arguments are validated identically on every rank, so a bad argument fails every
// rank alike.  A rank that fails alone (e.g. out of memory on its device) would leave the others
// waiting in a collective: the coordinator then aborts the communicator (the thread group's
// barriers throw; ncclCommAbort on RCCL), every rank's call returns, and the handle is marked
// broken -- later calls fail until it is destroyed.
#include "engine.h"

#include <functional>

using namespace n2v2r_int;

// One persistent host thread per rank of a multi handle (round 5 started W new threads per C-ABI
// call): fanout() posts fn(rank_handle, rank) as a new job generation, every worker runs it once
// and reports its status.  The ranks start together (a rank running alone would wait in its first
// collective for ever), or not at all.
struct n2v2r_int_rank_pool {
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv_job, cv_done;
  uint64_t gen = 0;  // job generation: a worker runs each generation once
  bool stop = false;
  std::function<int(n2v2r_handle*, int)> job;
  std::vector<int> st;
  int done = 0, failed = 0;
};

namespace n2v2r_int {
namespace {

void pool_worker(n2v2r_handle* h, n2v2r_int_rank_pool* p, int i) {
  uint64_t seen = 0;
  for (;;) {
    std::function<int(n2v2r_handle*, int)> fn;
    {
      std::unique_lock<std::mutex> lk(p->m);
      p->cv_job.wait(lk, [&] { return p->stop || p->gen != seen; });
      if (p->stop) return;
      seen = p->gen;
      fn = p->job;
    }
    int s;
    try {
      s = fn(h->ranks[i], i);
    } catch (...) {  // (the C-ABI entry points are guarded; this keeps the pool alive regardless)
      s = N2V2R_ERR_INTERNAL;
    }
    std::lock_guard<std::mutex> lk(p->m);
    p->st[i] = s;
    ++p->done;
    if (s != N2V2R_OK) ++p->failed;
    p->cv_done.notify_all();
  }
}

// start the pool (once per handle); false when the threads cannot be created
bool pool_start(n2v2r_handle* h) {
  if (h->pool) return true;
  auto* p = new (std::nothrow) n2v2r_int_rank_pool();
  if (!p) return false;
  const int W = (int)h->ranks.size();
  p->st.assign(W, N2V2R_OK);
  try {
    for (int i = 0; i < W; ++i) p->th.emplace_back(pool_worker, h, p, i);
  } catch (const std::system_error&) {
    {
      std::lock_guard<std::mutex> lk(p->m);
      p->stop = true;
    }
    p->cv_job.notify_all();
    for (auto& t : p->th) t.join();
    delete p;
    return false;
  }
  h->pool = p;
  return true;
}

void pool_stop(n2v2r_handle* h) {
  n2v2r_int_rank_pool* p = h->pool;
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(p->m);
    p->stop = true;
  }
  p->cv_job.notify_all();
  for (auto& t : p->th) t.join();
  delete p;
  h->pool = nullptr;
}

template <class F>
int fanout(n2v2r_handle* h, F&& fn) {
  if (h->broken) {
    h->err = "a rank of this multi-GPU handle failed alone earlier and its communicator was "
             "aborted: destroy the handle";
    return N2V2R_ERR_INTERNAL;
  }
  if (!pool_start(h)) {
    h->err = "could not start one host thread per GPU";
    return N2V2R_ERR_INTERNAL;
  }
  n2v2r_int_rank_pool* p = h->pool;
  const int W = (int)h->ranks.size();
  {
    std::lock_guard<std::mutex> lk(p->m);
    p->job = [&fn](n2v2r_handle* r, int i) { return fn(r, i); };
    std::fill(p->st.begin(), p->st.end(), N2V2R_OK);
    p->done = p->failed = 0;
    ++p->gen;
  }
  p->cv_job.notify_all();
  {
    // a failure on some ranks while others are still running: give them 10 s to fail alike
    // (the symmetric case: a bad argument, a non-converged fit), then abort the communicator
    std::unique_lock<std::mutex> lk(p->m);
    p->cv_done.wait(lk, [&] { return p->done == W || p->failed > 0; });
    if (p->done < W &&
        !p->cv_done.wait_for(lk, std::chrono::seconds(10), [&] { return p->done == W; })) {
      lk.unlock();
      if (h->own_group) h->own_group->abort();
      for (n2v2r_handle* r : h->ranks)
        if (r->comm) r->comm->abort();
      h->broken = true;
      lk.lock();
    }
    // every rank's call has returned before fn (this frame's) goes out of scope
    p->cv_done.wait(lk, [&] { return p->done == W; });
    p->job = nullptr;
  }
  for (int i = 0; i < W; ++i)
    if (p->st[i] != N2V2R_OK) {
      h->err = "rank " + std::to_string(i) + " (device " + std::to_string(h->ranks[i]->device) +
               "): " + h->ranks[i]->err;
      return p->st[i];
    }
  return N2V2R_OK;
}

}  // namespace

int multi_destroy(n2v2r_handle* h) {
  pool_stop(h);
  // every rank at once: tearing down an RCCL communicator finalises it with its peers
  std::vector<std::thread> th;
  for (n2v2r_handle* r : h->ranks) {
    try {
      th.emplace_back([r] { n2v2r_destroy(r); });
    } catch (const std::system_error&) {
      n2v2r_destroy(r);
    }
  }
  for (auto& t : th) t.join();
  h->ranks.clear();
  h->own_group.reset();
  delete h;
  return N2V2R_OK;
}

int multi_synchronize(n2v2r_handle* h) {
  return fanout(h, [](n2v2r_handle* r, int) { return n2v2r_synchronize(r); });
}

int multi_set_num_layers(n2v2r_handle* h, int num_layers, int64_t n) {
  const int st = fanout(h, [&](n2v2r_handle* r, int) { return n2v2r_set_num_layers(r, num_layers, n); });
  if (st == N2V2R_OK) {
    // the multi handle's own view: every row (n2v2r_dist_info reports rank 0 of W, N rows)
    h->K = num_layers;
    h->n = h->nloc = h->npad = n;
    h->row0 = 0;
  }
  return st;
}

// Layers are sliced on the host: no rank ever holds (or receives over PCIe) the whole layer
// (a GPU owns a contiguous row range).  Symmetry (N2V2R_SYM_DETECT) is decided once,
// on the host, by hash sums over the entries and the transposed entries (host_csr_symmetric);
// a symmetric layer: every rank uploads its own rows (n2v2r_set_layer_csr_rows); a directed one:
// every rank thread also builds its rows of A^T from the host CSR (host_transpose_rows) and
// uploads both.  Arguments the slicing cannot take go to every rank's whole-layer ingest, which
// fails them alike.
int multi_set_layer_csr(n2v2r_handle* h, int k, int64_t n, int64_t nnz, const int64_t* indptr,
                        const int32_t* indices, const float* data, int symmetric) {
  if ((symmetric != N2V2R_SYM_YES && symmetric != N2V2R_SYM_NO &&
       symmetric != N2V2R_SYM_DETECT) ||
      !indptr || n != h->n || nnz < 0 || k < 0 || k >= h->K ||
      (nnz > 0 && (!indices || !data)) || indptr[0] != 0 || indptr[n] != nnz)
    return fanout(h, [&](n2v2r_handle* r, int) {
      return n2v2r_set_layer_csr(r, k, n, nnz, indptr, indices, data, symmetric);
    });
  for (int64_t i = 0; i < n; ++i)
    if (indptr[i + 1] < indptr[i]) {
      h->set_err("layer %d: indptr not monotone", k);
      return N2V2R_ERR_BAD_ARG;
    }
  if (!host_indices_in_range(nnz, indices, n)) {
    h->set_err("layer %d: column index out of range", k);
    return N2V2R_ERR_BAD_ARG;
  }
  const bool sym = symmetric == N2V2R_SYM_YES ||
                   (symmetric == N2V2R_SYM_DETECT && host_csr_symmetric(n, indptr, indices, data));
  if (!sym)
    return fanout(h, [&](n2v2r_handle* r, int) {
      const int64_t r0 = r->row0, nr = r->nloc;
      const int64_t p0 = indptr[r0];
      std::vector<int64_t> lip((size_t)nr + 1), tip;
      for (int64_t i = 0; i <= nr; ++i) lip[i] = indptr[r0 + i] - p0;
      std::vector<int32_t> tix;
      std::vector<float> tdv;
      host_transpose_rows(n, indptr, indices, data, r0, nr, tip, tix, tdv);
      static const int32_t zi = 0;
      static const float zf = 0.f;
      const bool e = indptr[r0 + nr] == p0;
      return set_layer_rows_directed(r, k, lip.data(), e ? &zi : indices + p0, e ? &zf : data + p0,
                                     tip.data(), tix.data(), tdv.data());
    });
  return fanout(h, [&](n2v2r_handle* r, int) {
    const int64_t r0 = r->row0, nr = r->nloc;
    const int64_t p0 = indptr[r0], p1 = indptr[r0 + nr];
    std::vector<int64_t> lip((size_t)nr + 1);
    for (int64_t i = 0; i <= nr; ++i) lip[i] = indptr[r0 + i] - p0;
    return n2v2r_set_layer_csr_rows(r, k, n, r0, nr, p1 - p0, lip.data(),
                                    p1 > p0 ? indices + p0 : indices, p1 > p0 ? data + p0 : data);
  });
}

int multi_set_layer_dense(n2v2r_handle* h, int k, int64_t n, const float* A, int symmetric) {
  return fanout(h, [&](n2v2r_handle* r, int) { return n2v2r_set_layer_dense(r, k, n, A, symmetric); });
}

int multi_column_sums(n2v2r_handle* h, int k, float* out) {
  // validated here, alike for every rank (rank 0 alone would see a null `out`, and the others
  // would wait for it in the all-gather)
  if (!out) {
    h->err = "column sums: null output buffer";
    return N2V2R_ERR_BAD_ARG;
  }
  if (k < 0 || k >= h->K) {
    h->set_err("column sums: layer %d out of range [0, %d)", k, h->K);
    return N2V2R_ERR_BAD_ARG;
  }
  // every rank returns the global sums (an all-gather inside); rank 0 writes the caller's buffer
  std::vector<std::vector<float>> tmp(h->ranks.size());
  return fanout(h, [&](n2v2r_handle* r, int i) {
    float* dst = out;
    if (i > 0) {
      tmp[i].resize((size_t)std::max<int64_t>(r->n, 1));
      dst = tmp[i].data();
    }
    return n2v2r_column_sums(r, k, dst);
  });
}

int multi_uase(n2v2r_handle* h, int d, const n2v2r_eig_opts* opts, n2v2r_eig_stats* stats) {
  std::vector<n2v2r_eig_stats> rs(h->ranks.size());
  const int st = fanout(h, [&](n2v2r_handle* r, int i) {
    return n2v2r_uase(r, d, opts, stats ? &rs[i] : nullptr);
  });
  if (stats) *stats = rs[0];  // identical solver decisions on every rank
  if (st == N2V2R_OK || st == N2V2R_ERR_NO_CONVERGENCE) h->d = d;  // (an embedding either way)
  return st;
}

int multi_get_embedding(n2v2r_handle* h, float* Y) {
  if (!Y) return N2V2R_ERR_BAD_ARG;
  // rank r's rows land at row0 of every layer block of the global [K][N][d] array
  return fanout(h, [&](n2v2r_handle* r, int) {
    return guarded(r, [&]() -> int {
      if (!r->have_embedding) {
        r->err = "No n2v2r embeddings found";
        return N2V2R_ERR_NOT_READY;
      }
      copy_embedding(r, Y + (size_t)r->row0 * r->d, (int64_t)r->n * r->d);
      return N2V2R_OK;
    });
  });
}

int multi_get_left_embedding(n2v2r_handle* h, float* X) {
  if (!X) return N2V2R_ERR_BAD_ARG;
  return fanout(h, [&](n2v2r_handle* r, int) {
    return n2v2r_get_left_embedding(r, X + (size_t)r->row0 * r->d);
  });
}

int multi_rank(n2v2r_handle* h, int strategy, const int* dims, int n_dims, const int* metrics,
               int n_metrics, int method, int* n_comparisons, int* n_cols) {
  std::vector<int> nc(h->ranks.size()), cc(h->ranks.size());
  const int st = fanout(h, [&](n2v2r_handle* r, int i) {
    return n2v2r_rank(r, strategy, dims, n_dims, metrics, n_metrics, method, &nc[i], &cc[i]);
  });
  if (st == N2V2R_OK) {
    if (n_comparisons) *n_comparisons = nc[0];
    if (n_cols) *n_cols = cc[0];
  }
  return st;
}

}  // namespace n2v2r_int

extern "C" {

int n2v2r_create_multi(const int* devices, int n_gpus, n2v2r_handle** out) {
  if (!out || !devices || n_gpus < 1) return N2V2R_ERR_BAD_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return N2V2R_ERR_HIP;
  bool distinct = true;
  for (int i = 0; i < n_gpus; ++i) {
    if (devices[i] < 0 || devices[i] >= count) return N2V2R_ERR_BAD_ARG;
    for (int j = 0; j < i; ++j) distinct &= devices[j] != devices[i];
  }
  auto* h = new (std::nothrow) n2v2r_handle();
  if (!h) return N2V2R_ERR_OUT_OF_MEMORY;
  h->device = devices[0];
  h->world = n_gpus;
  std::vector<ncclComm_t> comms;
  if (distinct) {
    comms.assign(n_gpus, nullptr);
    if (ncclCommInitAll(comms.data(), n_gpus, devices) != ncclSuccess) {
      delete h;
      return N2V2R_ERR_RCCL;
    }
  } else {
    h->own_group = std::make_unique<n2v2r_simgroup>();
    h->own_group->world = n_gpus;
    h->own_group->ptrs.assign(n_gpus, nullptr);
    h->own_group->host.resize(n_gpus);
  }
  for (int i = 0; i < n_gpus; ++i) {
    n2v2r_handle* r = new_handle(devices[i]);
    if (!r) {
      for (int j = i; j < n_gpus && distinct; ++j) (void)ncclCommDestroy(comms[j]);
      (void)multi_destroy(h);
      return N2V2R_ERR_HIP;
    }
    r->rank = i;
    r->world = n_gpus;
    r->comm = distinct ? make_rccl_comm(comms[i], i, n_gpus)
                       : make_thread_comm(h->own_group.get(), i, devices[i]);
    h->ranks.push_back(r);
  }
  *out = h;
  return N2V2R_OK;
}

int n2v2r_h2d_layer_bytes(const n2v2r_handle* h, int64_t* per_rank, int cap) {
  if (!h) return N2V2R_ERR_BAD_ARG;
  if (!h->multi()) {
    if (per_rank && cap >= 1) per_rank[0] = h->h2d_layer_bytes;
    return 1;
  }
  const int w = (int)h->ranks.size();
  for (int i = 0; per_rank && i < std::min(w, cap); ++i) per_rank[i] = h->ranks[i]->h2d_layer_bytes;
  return w;
}

int n2v2r_multi_devices(const n2v2r_handle* h, int* devices, int cap) {
  if (!h) return N2V2R_ERR_BAD_ARG;
  if (!h->multi()) {
    if (devices && cap >= 1) devices[0] = h->device;
    return 1;
  }
  const int w = (int)h->ranks.size();
  for (int i = 0; devices && i < std::min(w, cap); ++i) devices[i] = h->ranks[i]->device;
  return w;
}

}  // extern "C"

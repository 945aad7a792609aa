// Ranking: per-node distances for every (comparison, dim, metric) column, Borda by GPU radix
// sort (the reference's tie order on flagged columns), and the host-array seams.
#include "engine.h"

using namespace n2v2r_int;

extern "C" {

// Borda of nseg descending-sorted columns, ncols per output group.  tied_dev (optional): the
// per-column exact-tie flags (n2v2r_launch_tie_flags).  given (optional): columns whose order the
// caller supplies (device int32 permutations, best first) in place of the stable radix order.
struct GivenOrder {
  int col;
  const int32_t* order_dev;
};
static void run_borda(n2v2r_handle* h, const double* Ddev, int64_t n, int nseg, int ncols,
                      int64_t* borda_dev, int32_t* tied_dev = nullptr,
                      const std::vector<GivenOrder>* given = nullptr) {
  hipStream_t st = h->stream;
  const size_t tot = (size_t)nseg * n;
  for (int i = 0; i < 2; ++i) {
    h->rs_keys[i].ensure(sizeof(uint64_t) * tot);
    h->rs_idx[i].ensure(sizeof(int32_t) * tot);
  }
  h->rs_pos.ensure(sizeof(int32_t) * tot);
  h->rs_hist.ensure(sizeof(uint32_t) * n2v2r_radix_hist_elems(n, nseg));
  h->rs_or.ensure(sizeof(unsigned long long) * nseg);
  h->rs_and.ensure(sizeof(unsigned long long) * nseg);
  HIPCHK(n2v2r_launch_borda_init(Ddev, n, nseg, h->rs_keys[0].as<uint64_t>(),
                                 h->rs_idx[0].as<int32_t>(), h->rs_or.as<unsigned long long>(),
                                 h->rs_and.as<unsigned long long>(), st));
  std::vector<unsigned long long> kor(nseg), kand(nseg);
  HIPCHK(hipMemcpyAsync(kor.data(), h->rs_or.p, sizeof(unsigned long long) * nseg,
                        hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(kand.data(), h->rs_and.p, sizeof(unsigned long long) * nseg,
                        hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  unsigned long long varying = 0;
  for (int s = 0; s < nseg; ++s) varying |= kor[s] ^ kand[s];
  int cur = 0;
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = pass * 8;
    if (((varying >> shift) & 0xFFull) == 0) continue;  // stable pass on a constant digit = identity
    HIPCHK(n2v2r_launch_radix_pass(h->rs_keys[cur].as<uint64_t>(), h->rs_idx[cur].as<int32_t>(),
                                   h->rs_keys[cur ^ 1].as<uint64_t>(),
                                   h->rs_idx[cur ^ 1].as<int32_t>(), n, nseg, shift,
                                   h->rs_hist.as<uint32_t>(), st));
    cur ^= 1;
  }
  if (tied_dev) HIPCHK(n2v2r_launch_tie_flags(h->rs_keys[cur].as<uint64_t>(), n, nseg, tied_dev, st));
  if (given)
    for (const GivenOrder& g : *given)
      HIPCHK(hipMemcpyAsync(h->rs_idx[cur].as<int32_t>() + (size_t)g.col * n, g.order_dev,
                            sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st));
  HIPCHK(n2v2r_launch_borda_finish(h->rs_idx[cur].as<int32_t>(), n, nseg, ncols,
                                   h->rs_pos.as<int32_t>(), borda_dev, st));
}

int n2v2r_rank(n2v2r_handle* h, int strategy, const int* dims, int n_dims, const int* metrics,
               int n_metrics, int method, int* n_comparisons, int* n_cols) {
  if (h && h->multi())
    return multi_rank(h, strategy, dims, n_dims, metrics, n_metrics, method, n_comparisons, n_cols);
  return guarded(h, [&]() -> int {
    if (method != N2V2R_AGG_BORDA && method != N2V2R_AGG_NONE) {
      h->err = "Aggregation method not found. Available methods: Borda";
      return N2V2R_ERR_UNSUPPORTED_AGG;
    }
    if (!h->have_embedding) {
      h->err = "No n2v2r embeddings found";
      return N2V2R_ERR_NOT_READY;
    }
    if (strategy < 0 || strategy > 2 || n_dims < 1 || n_metrics < 1 || !dims || !metrics) {
      h->err = "bad rank arguments";
      return N2V2R_ERR_BAD_ARG;
    }
    for (int m = 0; m < n_metrics; ++m)
      if (metrics[m] < 0 || metrics[m] > 2) {
        h->err = "Unsupported metric";
        return N2V2R_ERR_UNSUPPORTED_METRIC;
      }
    // columns: dims outer, metrics inner, cosine skipped at dim 1 (model.py:73,87-90)
    std::vector<std::pair<int, int>> cols;
    for (int i = 0; i < n_dims; ++i) {
      if (dims[i] < 1 || dims[i] > h->d) {
        h->set_err("dimension %d outside [1, %d]", dims[i], h->d);
        return N2V2R_ERR_BAD_ARG;
      }
      for (int m = 0; m < n_metrics; ++m) {
        if (metrics[m] == N2V2R_COSINE && dims[i] == 1) continue;
        cols.emplace_back(dims[i], metrics[m]);
      }
    }
    if (cols.empty() || (int)cols.size() > DIST_MAX_COLS) {
      h->err = "no ranking columns (or too many)";
      return N2V2R_ERR_BAD_ARG;
    }
    DistPlan plan{};
    plan.n_cols = (int)cols.size();
    std::vector<int> order(cols.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return cols[a].first < cols[b].first; });
    plan.dmax = 0;
    for (int e = 0; e < plan.n_cols; ++e) {
      plan.col_dim[e] = cols[order[e]].first;
      plan.col_metric[e] = cols[order[e]].second;
      plan.col_out[e] = order[e];
      plan.dmax = std::max(plan.dmax, plan.col_dim[e]);
    }
    // comparisons (model.py:59-66)
    std::vector<int> layer_i;
    for (int i = 0; i < h->K; ++i) {
      if (i == 0 && strategy != N2V2R_ONE_VS_REST) continue;
      layer_i.push_back(i);
    }
    if (layer_i.empty()) {
      h->err = "need at least two layers to compare";
      return N2V2R_ERR_BAD_ARG;
    }
    const int ncmp = (int)layer_i.size();
    const int C = plan.n_cols;
    const int64_t n = h->n;
    h->D.ensure(sizeof(double) * (size_t)ncmp * C * n);
    h->borda.ensure(sizeof(int64_t) * (size_t)ncmp * n);
    const double t0 = now_ms();
    if (!h->comm) {
      for (int c = 0; c < ncmp; ++c)
        HIPCHK(n2v2r_launch_distances(h->Y.as<float>(), h->K, n, h->ldy, h->npad, strategy,
                                      layer_i[c], plan, h->D.as<double>() + (size_t)c * C * n, n,
                                      h->stream));
    } else {
      // local rows -> [ncmp][C][npad], then every column gathered into the global table
      h->Dloc.ensure(sizeof(double) * (size_t)ncmp * C * h->npad);
      h->Dgat.ensure(sizeof(double) * (size_t)h->world * h->npad);
      for (int c = 0; c < ncmp; ++c)
        HIPCHK(n2v2r_launch_distances(h->Y.as<float>(), h->K, h->nloc, h->ldy, h->npad, strategy,
                                      layer_i[c], plan,
                                      h->Dloc.as<double>() + (size_t)c * C * h->npad, h->npad,
                                      h->stream));
      for (int s = 0; s < ncmp * C; ++s) {
        h->comm->allgather(h->Dloc.as<double>() + (size_t)s * h->npad, h->Dgat.p,
                           sizeof(double) * h->npad, h->stream);
        HIPCHK(hipMemcpyAsync(h->D.as<double>() + (size_t)s * n, h->Dgat.p, sizeof(double) * n,
                              hipMemcpyDeviceToDevice, h->stream));
      }
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    const double t1 = now_ms();
    h->have_borda = method == N2V2R_AGG_BORDA;
    if (h->have_borda) run_borda(h, h->D.as<double>(), n, ncmp * C, C, h->borda.as<int64_t>());
    HIPCHK(hipStreamSynchronize(h->stream));
    h->ms_dist = t1 - t0;
    h->ms_borda = now_ms() - t1;
    h->ncmp = ncmp;
    h->ncols = C;
    if (n_comparisons) *n_comparisons = ncmp;
    if (n_cols) *n_cols = C;
    return N2V2R_OK;
  });
}

int n2v2r_get_distances(n2v2r_handle* h, int comparison, double* D) {
  if (h && h->multi()) h = h->ranks[0];  // the global table is on every rank
  return guarded(h, [&]() -> int {
    if (comparison < 0 || comparison >= h->ncmp || !D) return N2V2R_ERR_BAD_ARG;
    HIPCHK(hipMemcpyAsync(D, h->D.as<double>() + (size_t)comparison * h->ncols * h->n,
                          sizeof(double) * h->ncols * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_get_borda(n2v2r_handle* h, int comparison, int64_t* borda) {
  if (h && h->multi()) h = h->ranks[0];
  return guarded(h, [&]() -> int {
    if (comparison < 0 || comparison >= h->ncmp || !borda) return N2V2R_ERR_BAD_ARG;
    if (!h->have_borda) {
      h->err = "n2v2r_rank ran without aggregation (N2V2R_AGG_NONE)";
      return N2V2R_ERR_NOT_READY;
    }
    HIPCHK(hipMemcpyAsync(borda, h->borda.as<int64_t>() + (size_t)comparison * h->n,
                          sizeof(int64_t) * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_rank_timing(n2v2r_handle* h, double* ms_distances, double* ms_borda) {
  if (!h) return N2V2R_ERR_BAD_ARG;
  if (h->multi()) h = h->ranks[0];
  if (ms_distances) *ms_distances = h->ms_dist;
  if (ms_borda) *ms_borda = h->ms_borda;
  return N2V2R_OK;
}

int n2v2r_pairwise_distances(n2v2r_handle* h, const double* m1, const double* m2, int64_t n,
                             int dim, int metric, double* out) {
  if (h && h->multi()) h = h->ranks[0];  // host-array seams: no collective, rank 0's GPU
  return guarded(h, [&]() -> int {
    if (metric < 0 || metric > 2) {
      h->err = "Unsupported metric";
      return N2V2R_ERR_UNSUPPORTED_METRIC;
    }
    if (n < 1 || dim < 1 || !m1 || !m2 || !out) return N2V2R_ERR_BAD_ARG;
    DevBuf a, b, o;
    a.ensure(sizeof(double) * n * dim);
    b.ensure(sizeof(double) * n * dim);
    o.ensure(sizeof(double) * n);
    HIPCHK(hipMemcpyAsync(a.p, m1, sizeof(double) * n * dim, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(b.p, m2, sizeof(double) * n * dim, hipMemcpyHostToDevice, h->stream));
    HIPCHK(n2v2r_launch_pairwise(a.as<double>(), b.as<double>(), n, dim, metric, o.as<double>(),
                                 h->stream));
    HIPCHK(hipMemcpyAsync(out, o.p, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_borda_columns(n2v2r_handle* h, const double* D, int64_t n, int n_cols, int64_t* borda) {
  if (h && h->multi()) h = h->ranks[0];
  return guarded(h, [&]() -> int {
    if (n < 1 || n_cols < 1 || !D || !borda) return N2V2R_ERR_BAD_ARG;
    DevBuf dd, bo;
    dd.ensure(sizeof(double) * n * n_cols);
    bo.ensure(sizeof(int64_t) * n);
    HIPCHK(hipMemcpyAsync(dd.p, D, sizeof(double) * n * n_cols, hipMemcpyHostToDevice, h->stream));
    run_borda(h, dd.as<double>(), n, n_cols, n_cols, bo.as<int64_t>());
    HIPCHK(hipMemcpyAsync(borda, bo.p, sizeof(int64_t) * n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_borda_columns_ex(n2v2r_handle* h, const double* D, int64_t n, int n_cols,
                           const int32_t* given_cols, int n_given, const int32_t* given_orders,
                           int64_t* borda, int32_t* tied) {
  if (h && h->multi()) h = h->ranks[0];
  return guarded(h, [&]() -> int {
    if (n < 1 || n_cols < 1 || !D || !borda || n_given < 0 || n_given > n_cols ||
        (n_given > 0 && (!given_cols || !given_orders)) || n > INT32_MAX)
      return N2V2R_ERR_BAD_ARG;
    // the caller's orders must be permutations of 0..n-1 of distinct columns (checked here: the
    // GPU's inverse permutation scatters by them)
    std::vector<char> seen_col(n_cols, 0), seen((size_t)n);
    for (int g = 0; g < n_given; ++g) {
      const int c = given_cols[g];
      if (c < 0 || c >= n_cols || seen_col[c]) {
        h->set_err("given column %d out of range or repeated", c);
        return N2V2R_ERR_BAD_ARG;
      }
      seen_col[c] = 1;
      std::fill(seen.begin(), seen.end(), 0);
      const int32_t* o = given_orders + (size_t)g * n;
      for (int64_t i = 0; i < n; ++i) {
        if (o[i] < 0 || o[i] >= n || seen[o[i]]) {
          h->set_err("given order of column %d is not a permutation of 0..n-1", c);
          return N2V2R_ERR_BAD_ARG;
        }
        seen[o[i]] = 1;
      }
    }
    DevBuf dd, bo, tf, go;
    dd.ensure(sizeof(double) * n * n_cols);
    bo.ensure(sizeof(int64_t) * n);
    tf.ensure(sizeof(int32_t) * n_cols);
    HIPCHK(hipMemcpyAsync(dd.p, D, sizeof(double) * n * n_cols, hipMemcpyHostToDevice, h->stream));
    std::vector<GivenOrder> given;
    if (n_given > 0) {
      go.ensure(sizeof(int32_t) * (size_t)n_given * n);
      HIPCHK(hipMemcpyAsync(go.p, given_orders, sizeof(int32_t) * (size_t)n_given * n,
                            hipMemcpyHostToDevice, h->stream));
      for (int g = 0; g < n_given; ++g)
        given.push_back({given_cols[g], go.as<int32_t>() + (size_t)g * n});
    }
    run_borda(h, dd.as<double>(), n, n_cols, n_cols, bo.as<int64_t>(), tf.as<int32_t>(),
              n_given > 0 ? &given : nullptr);
    HIPCHK(hipMemcpyAsync(borda, bo.p, sizeof(int64_t) * n, hipMemcpyDeviceToHost, h->stream));
    if (tied)
      HIPCHK(hipMemcpyAsync(tied, tf.p, sizeof(int32_t) * n_cols, hipMemcpyDeviceToHost,
                            h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

}  // extern "C"

// n2v2r engine: handle lifecycle and the diagnostic entry points (include/n2v2r_diag.h).
// The rest of the C-ABI: layers.cpp (ingest), solver.cpp (UASE), ranking.cpp (distances,
// Borda), comm.cpp (row-partitioned communicators), multi.cpp (one process, N GPUs).
#include "engine.h"

using namespace n2v2r_int;

namespace n2v2r_int {
n2v2r_handle* new_handle(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return nullptr;
  if (device < 0 || device >= count) return nullptr;
  auto* h = new (std::nothrow) n2v2r_handle();
  if (!h) return nullptr;
  h->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return nullptr;
  }
  return h;
}

}  // namespace n2v2r_int

extern "C" {

const char* n2v2r_version(void) { return "n2v2r-mi355x 0.2.0 (gfx950)"; }

int n2v2r_create(int device, n2v2r_handle** out) {
  if (!out) return N2V2R_ERR_BAD_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return N2V2R_ERR_HIP;
  if (device < 0 || device >= count) return N2V2R_ERR_BAD_ARG;
  n2v2r_handle* h = new_handle(device);
  if (!h) return N2V2R_ERR_HIP;
  *out = h;
  return N2V2R_OK;
}

void n2v2r_destroy(n2v2r_handle* h) {
  if (!h) return;
  if (h->multi()) {
    (void)multi_destroy(h);
    return;
  }
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  h->layers.clear();
  h->comm.reset();
  for (hipEvent_t& e : h->cb_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->side) (void)hipStreamDestroy(h->side);
  if (h->pin) (void)hipHostFree(h->pin);
  for (hipEvent_t e : h->tev) (void)hipEventDestroy(e);
  if (h->cstream) (void)hipStreamSynchronize(h->cstream);
  for (hipEvent_t& e : h->cev)
    if (e) (void)hipEventDestroy(e);
  if (h->cstream) (void)hipStreamDestroy(h->cstream);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int n2v2r_last_error(const n2v2r_handle* h, char* buf, size_t len) {
  if (!h || !buf || len == 0) return N2V2R_ERR_BAD_ARG;
  snprintf(buf, len, "%s", h->err.c_str());
  return N2V2R_OK;
}

int n2v2r_synchronize(n2v2r_handle* h) {
  if (h && h->multi()) return multi_synchronize(h);
  return guarded(h, [&]() -> int {
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

// Rayleigh-Ritz stage alone (tests): top-p eigenpairs of a host symmetric c x c matrix through
// the same GPU tridiagonalisation + host tridiagonal solve + GPU back-transform as UASE.
int n2v2r_rr_top(n2v2r_handle* h, int c, const double* H, int p, double* w, float* S) {
  if (h && h->multi()) h = h->ranks[0];  // (diagnostics: rank 0)
  return guarded(h, [&]() -> int {
    if (c < 3 || c > 768 || p < 1 || p > c || !H || !w || !S) return N2V2R_ERR_BAD_ARG;
    DevBuf a, tri, refl, y, s;
    a.ensure(sizeof(double) * c * c);
    tri.ensure(sizeof(double) * 3 * c);
    refl.ensure(sizeof(double) * c * c);
    y.ensure(sizeof(double) * c * p);
    s.ensure(sizeof(float) * c * p);
    HIPCHK(hipMemcpyAsync(a.p, H, sizeof(double) * c * c, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));  // pageable source: complete before the kernel
    double* t = tri.as<double>();
    DevBuf trs;
    trs.ensure(n2v2r_rr_tridiag_scratch_bytes(c));
    HIPCHK(n2v2r_launch_rr_tridiag(a.as<double>(), c, t, t + c, t + 2 * c, refl.as<double>(),
                                   trs.p, h->stream));
    DevBuf wd, scr;
    wd.ensure(sizeof(double) * p);
    scr.ensure(sizeof(double) * 6 * (size_t)((p + 63) / 64 * 64) * c);
    HIPCHK(n2v2r_launch_rr_tri_eig(t, t + c, c, p, wd.as<double>(), y.as<double>(),
                                   scr.as<double>(), h->stream));
    HIPCHK(hipMemcpyAsync(w, wd.p, sizeof(double) * p, hipMemcpyDeviceToHost, h->stream));
    DevBuf btf;
    btf.ensure(n2v2r_rr_bt_scratch_bytes(c));
    HIPCHK(n2v2r_launch_rr_backtransform(refl.as<double>(), t + 2 * c, c, y.as<double>(), p,
                                         s.as<float>(), p, btf.as<double>(), h->stream));
    HIPCHK(hipMemcpyAsync(S, s.p, sizeof(float) * c * p, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_rr_band_top(n2v2r_handle* h, int c, int kp, const double* hband, int64_t hband_len,
                      const double* theta_prev, int p, double* w, float* S) {
  if (h && h->multi()) h = h->ranks[0];  // (diagnostics: rank 0)
  return guarded(h, [&]() -> int {
    const int b = 8;
    if (c < 3 || c > 512 || c % b || kp % b || kp + b > 192 || kp >= c || p < 1 || p > c ||
        !hband || !w || !S || (kp > 0 && !theta_prev))
      return N2V2R_ERR_BAD_ARG;
    const int64_t need = (int64_t)(kp + b) * b + (int64_t)(c / b - kp / b - 1) * 2 * b * b;
    if (hband_len < need) return N2V2R_ERR_BAD_ARG;
    DevBuf hb, th, ab, va, ta, tri, y, s, er, rf;
    rf.ensure(sizeof(double) * c * n2v2r_rr_band_jm(c) * 9);
    hb.ensure(sizeof(double) * hband_len);
    th.ensure(sizeof(double) * c);
    ab.ensure(sizeof(double) * c * (b + 1));
    va.ensure(sizeof(double) * (kp + b) * (kp + b));
    ta.ensure(sizeof(double) * (kp + b));
    tri.ensure(sizeof(double) * 2 * c);
    y.ensure(sizeof(double) * c * p);
    s.ensure(sizeof(float) * c * p);
    er.ensure(4 * sizeof(int));
    HIPCHK(hipMemsetAsync(er.p, 0, 4 * sizeof(int), h->stream));  // the chase only sets it on failure
    HIPCHK(hipMemcpyAsync(hb.p, hband, sizeof(double) * hband_len, hipMemcpyHostToDevice,
                          h->stream));
    if (kp > 0)
      HIPCHK(hipMemcpyAsync(th.p, theta_prev, sizeof(double) * kp, hipMemcpyHostToDevice,
                            h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));  // pageable sources: complete before the kernels
    if (rr_sturm_enabled()) {  // the solver's default form (N2V2R_RR=band: the reducing one)
      DevBuf scr;
      scr.ensure(sizeof(double) * n2v2r_rr_sturm_scratch(c, p));
      HIPCHK(n2v2r_launch_rr_sturm(hb.as<double>(), c, kp, th.as<double>(), scr.as<double>(),
                                   scr.bytes / sizeof(double), y.as<double>(), s.as<float>(), p,
                                   p, er.as<int>(), h->stream));
      int e = 0;
      HIPCHK(hipMemcpyAsync(&e, er.p, sizeof(int), hipMemcpyDeviceToHost, h->stream));
      HIPCHK(hipMemcpyAsync(w, th.p, sizeof(double) * p, hipMemcpyDeviceToHost, h->stream));
      HIPCHK(hipMemcpyAsync(S, s.p, sizeof(float) * c * p, hipMemcpyDeviceToHost, h->stream));
      HIPCHK(hipStreamSynchronize(h->stream));
      if (!e) return N2V2R_OK;
      // a vector failed its residual check: the reducing path, as the solver falls back
      HIPCHK(hipMemsetAsync(er.p, 0, 4 * sizeof(int), h->stream));
      if (kp > 0)
        HIPCHK(hipMemcpyAsync(th.p, theta_prev, sizeof(double) * kp, hipMemcpyHostToDevice,
                              h->stream));
      HIPCHK(hipStreamSynchronize(h->stream));
    }
    HIPCHK(n2v2r_launch_rr_band(hb.as<double>(), c, kp, th.as<double>(), ab.as<double>(),
                                va.as<double>(), ta.as<double>(), tri.as<double>(),
                                tri.as<double>() + c, rf.as<double>(), y.as<double>(),
                                s.as<float>(), p, p, er.as<int>(), h->stream));
    int e = 0;
    HIPCHK(hipMemcpyAsync(&e, er.p, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(w, th.p, sizeof(double) * p, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(S, s.p, sizeof(float) * c * p, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    if (e) throw StatusFail{N2V2R_ERR_NO_CONVERGENCE, "banded Rayleigh-Ritz: bulge chase aborted"};
    return N2V2R_OK;
  });
}

int n2v2r_spmm_col_blocks(const n2v2r_handle* h, int b) {
  if (h && h->multi()) h = h->ranks[0];  // (diagnostics: rank 0)
  if (!h) return N2V2R_ERR_BAD_ARG;
  return col_blocks_wanted(h, b) ? 1 : 0;
}

// The flat-window tiled SpMM of layer k (A_k X, or A_k^T X) with `nb` column blocks (0: the fit's
// rule, panel blocks of <= 2 MB, at most 64) from device panels, timed with HIP events over `reps`
// launches after a warm-up.  N2V2R_ERR_BAD_ARG when the layer cannot take packed blocks.
static int time_tiled(n2v2r_handle* h, int k, int transpose, int nb, const float* xd, float* yd,
                      int reps, double* avg_ms, int b = 8) {
  if (nb <= 0) {
    nb = 4;
    while (nb < 64 && (double)h->n * 32.0 / nb > 2.0 * 1024 * 1024) nb *= 2;
  }
  if (nb != 4 && nb != 8 && nb != 16 && nb != 32 && nb != 64 && nb != 128) return N2V2R_ERR_BAD_ARG;
  LayerDev& L = *h->layers[k];
  const int wb = tile_wbits(h->layers, nb);
  if (!ensure_col_blocks(L, h->n, h->stream, nb, wb)) return N2V2R_ERR_BAD_ARG;
  const LayerDev::ColBlocks& cbs = (transpose && !L.symmetric) ? L.cb_t : L.cb;
  DevBuf tb;
  tb.ensure(sizeof(CsrBlk) * nb);
  HIPCHK(hipMemcpyAsync(tb.p, cbs.blk, sizeof(CsrBlk) * nb, hipMemcpyHostToDevice, h->stream));
  int ncu = 0;
  HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->device));
  SpmmTileArgs a{};
  a.blk = tb.as<CsrBlk>();
  a.X[0] = xd;
  a.Y[0] = yd;
  a.ldx = b;
  a.ldy = b;
  a.n = h->nloc;
  a.K = 1;
  a.nb = nb;
  a.sum = 0;
  a.tile_rows = n2v2r_spmm_tile_rows_b(h->nloc, ncu, b == 16 ? N2V2R_SPMM16_WPC : 2, wb, b);
  a.wbits = wb;
  a.width = b;
  HIPCHK(n2v2r_launch_spmm_tile(a, h->stream));  // warm-up
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipEventRecord(e0, h->stream));
  for (int r = 0; r < reps; ++r) HIPCHK(n2v2r_launch_spmm_tile(a, h->stream));
  HIPCHK(hipEventRecord(e1, h->stream));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (avg_ms) *avg_ms = (double)ms / reps;
  HIPCHK(hipStreamSynchronize(h->stream));  // tb dies here
  return N2V2R_OK;
}

int n2v2r_bench_spmm(n2v2r_handle* h, int k, int transpose, int b, int reps, const float* X,
                     float* Y, double* avg_ms, double* algo_bytes) {
  if (h && h->multi()) h = h->ranks[0];  // (diagnostics: rank 0)
  return guarded(h, [&]() -> int {
    if (k < 0 || k >= h->K || !h->layers[k]->loaded || (b != 8 && b != 16 && b != 32 && b != 64) ||
        reps < 1 || !X)
      return N2V2R_ERR_BAD_ARG;
    const LayerDev& L = *h->layers[k];
    DevBuf xd, yd;
    xd.ensure(sizeof(float) * h->n * b);
    yd.ensure(sizeof(float) * std::max<int64_t>(h->nloc, 1) * b);
    HIPCHK(hipMemcpyAsync(xd.p, X, sizeof(float) * h->n * b, hipMemcpyHostToDevice, h->stream));
    if (L.dense) {
      // dense layer: the GEMM Y = A_k X (or A_k^T X) over this rank's rows
      const float* am = transpose ? L.dense_at() : L.dense_a();
      const float* bt = h->comm ? nullptr : (transpose ? L.dense_a() : L.dense_at());
      h->dense_apply(am, L.lda, xd.as<float>(), b, b, yd.as<float>(), b, 0.f, nullptr, bt);
      hipEvent_t e0, e1;
      HIPCHK(hipEventCreate(&e0));
      HIPCHK(hipEventCreate(&e1));
      HIPCHK(hipEventRecord(e0, h->stream));
      for (int r = 0; r < reps; ++r)
        h->dense_apply(am, L.lda, xd.as<float>(), b, b, yd.as<float>(), b, 0.f, nullptr, bt);
      HIPCHK(hipEventRecord(e1, h->stream));
      HIPCHK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, e0, e1));
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      if (avg_ms) *avg_ms = (double)ms / reps;
      if (algo_bytes)
        *algo_bytes = 4.0 * (double)h->nloc * (double)h->n + 4.0 * (double)(h->n + h->nloc) * b;
      if (Y)
        HIPCHK(hipMemcpyAsync(Y, yd.p, sizeof(float) * h->nloc * b, hipMemcpyDeviceToHost,
                              h->stream));
      HIPCHK(hipStreamSynchronize(h->stream));
      return N2V2R_OK;
    }
    if (col_blocks_wanted(h, b)) {
      // the flat-window tiled SpMM of one layer (the fit's form at this panel size)
      double ms = 0.0;
      const int st_ = time_tiled(h, k, transpose, 0, xd.as<float>(), yd.as<float>(), reps, &ms);
      if (st_ == N2V2R_OK) {
        const CsrDev c0 = transpose ? L.csr_t() : L.csr();
        if (avg_ms) *avg_ms = ms;
        if (algo_bytes) *algo_bytes = spmm_algo_bytes(c0.nnz, c0.unit != 0, h->nloc, h->n, b);
        if (Y)
          HIPCHK(hipMemcpyAsync(Y, yd.p, sizeof(float) * h->nloc * b, hipMemcpyDeviceToHost,
                                h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        return N2V2R_OK;
      }
    }
    SpmmArgs a{};
    a.K = 1;
    a.sum = 0;
    a.ldx = b;
    a.ldy = b;
    a.colscale = nullptr;
    a.A[0] = transpose ? L.csr_t() : L.csr();
    a.X[0] = xd.as<float>();
    a.Y[0] = yd.as<float>();
    HIPCHK(n2v2r_launch_spmm(a, b, h->stream));  // warm-up
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, h->stream));
    for (int r = 0; r < reps; ++r) HIPCHK(n2v2r_launch_spmm(a, b, h->stream));
    HIPCHK(hipEventRecord(e1, h->stream));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (avg_ms) *avg_ms = (double)ms / reps;
    if (algo_bytes)
      *algo_bytes = spmm_algo_bytes(a.A[0].nnz, a.A[0].unit != 0, h->nloc, h->n, b);
    if (Y)
      HIPCHK(hipMemcpyAsync(Y, yd.p, sizeof(float) * h->nloc * b, hipMemcpyDeviceToHost,
                            h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}


int n2v2r_bench_spmm_tiled(n2v2r_handle* h, int k, int transpose, int b, int nb, int reps,
                           const float* X, float* Y, double* avg_ms) {
  if (h && h->multi()) h = h->ranks[0];  // (diagnostics: rank 0)
  return guarded(h, [&]() -> int {
    if (k < 0 || k >= h->K || !h->layers[k]->loaded || h->layers[k]->dense ||
        (b != 8 && b != 16) || reps < 1 || !X || h->comm)
      return N2V2R_ERR_BAD_ARG;
    DevBuf xd, yd;
    xd.ensure(sizeof(float) * h->n * b);
    yd.ensure(sizeof(float) * std::max<int64_t>(h->nloc, 1) * b);
    HIPCHK(hipMemcpyAsync(xd.p, X, sizeof(float) * h->n * b, hipMemcpyHostToDevice, h->stream));
    const int st_ =
        time_tiled(h, k, transpose, nb, xd.as<float>(), yd.as<float>(), reps, avg_ms, b);
    if (st_ != N2V2R_OK) return st_;
    if (Y)
      HIPCHK(hipMemcpyAsync(Y, yd.p, sizeof(float) * h->nloc * b, hipMemcpyDeviceToHost,
                            h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

}  // extern "C"

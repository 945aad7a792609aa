// n2v2r engine: handle, CSR ingest, block Krylov-Schur UASE driver, ranking orchestration
// and the extern "C" boundary declared in include/n2v2r.h.
//
// UASE (replaces se.UASE -> scipy svds/ARPACK, model.py:51-55): top-d eigenpairs of
// M = sum_k A_k A_k^T (N x N, = A A^T for the unfolded A = [A_1 | ... | A_K]) by a block
// Krylov-Schur iteration with explicit Rayleigh-Ritz:
//   basis Q = [Q_0 .. Q_{m-1}] (b-wide fp32 blocks in HBM), W_j = M Q_j kept beside it;
//   expand: Z = W_last, CGS2 against Q, CholeskyQR2 (+random refill of deficient columns),
//           Q_m = Z, W_m = M Q_m (2 SpMM launches: Z_k = A_k^T Q ; W = sum_k A_k Z_k);
//   cycle:  H = Q^T W (fp64) -> host top-p eigenpairs -> Ritz X = Q S, MX = W S,
//           residuals ||MX_j - theta_j X_j||; converged when all d <= tol * theta_1;
//   restart: next block = orth(W_last) against the old Q, keep [X_p | next] (thick restart).
// Embedding: Y_k = A_k^T U diag(sigma)^(-1/2) (= V diag(sigma)^(1/2) split per layer),
// sigma = sqrt(theta), columns in descending sigma order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/n2v2r.h"
#include "common.h"

// ---- kernel launchers (spmm.hip, dense.hip, rank.hip) ------------------------------------
#define SPMM_MAX_LAYERS 8
struct SpmmArgs {
  CsrDev A[SPMM_MAX_LAYERS];
  const float* X[SPMM_MAX_LAYERS];
  float* Y[SPMM_MAX_LAYERS];
  int64_t ldx;
  int64_t ldy;
  int K;
  int sum;
  const float* colscale;
};
#define DIST_MAX_COLS 256
struct DistPlan {
  int n_cols;
  int col_dim[DIST_MAX_COLS];
  int col_metric[DIST_MAX_COLS];
  int col_out[DIST_MAX_COLS];
  int dmax;
};
extern "C" {
hipError_t n2v2r_launch_spmm(const SpmmArgs& args, int B, hipStream_t stream);
hipError_t n2v2r_launch_row_sums(const CsrDev& A, float* out, hipStream_t stream);
hipError_t n2v2r_launch_ts_tn(const BlockList& A, const BlockList& B, int64_t n, double* partial,
                              size_t partial_elems, double* out, const int* cond,
                              hipStream_t stream);
hipError_t n2v2r_launch_ts_nn(const BlockList& A, const float* G, int ldg, int cb,
                              const OutBlockList& O, const BlockList& C, float alpha, float beta,
                              int64_t n, const int* cond, hipStream_t stream);
hipError_t n2v2r_launch_f64_to_f32(const double* in, float* out, int64_t elems, float scale,
                                   const int* cond, hipStream_t stream);
hipError_t n2v2r_launch_chol_inv(const double* G, int b, float* Rinv, int* flags, int* any_flag,
                                 hipStream_t stream);
hipError_t n2v2r_launch_pip_chol(const double* G, int c, int b, float* F, int* flags,
                                 int* any_flag, const int* cond, hipStream_t stream);
hipError_t n2v2r_launch_fill_normal(float* blk, int w, int64_t n, uint64_t seed, const int* flags,
                                    const int* cond, hipStream_t stream);
hipError_t n2v2r_launch_resid(const BlockList& X, const BlockList& MX, const double* theta,
                              int64_t n, double* partial, size_t partial_elems, double* out,
                              hipStream_t stream);
hipError_t n2v2r_launch_scale_cols(float* blk, int w, int64_t n, const float* s,
                                   hipStream_t stream);
hipError_t n2v2r_launch_sign_convention(float* U, int64_t ldu, int64_t n, int d,
                                        unsigned long long* keys, size_t key_elems, float* sign,
                                        hipStream_t stream);
hipError_t n2v2r_launch_distances(const float* Y, int K, int64_t n, int64_t ldy, int strategy,
                                  int layer_i, const DistPlan& plan, double* out,
                                  hipStream_t stream);
hipError_t n2v2r_launch_pairwise(const double* a, const double* b, int64_t n, int dim, int metric,
                                 double* out, hipStream_t stream);
hipError_t n2v2r_launch_borda_init(const double* vals, int64_t n, int nseg, uint64_t* keys,
                                   int32_t* idx, unsigned long long* seg_or,
                                   unsigned long long* seg_and, hipStream_t stream);
int n2v2r_radix_tiles(int64_t n);
hipError_t n2v2r_launch_radix_pass(const uint64_t* kin, const int32_t* pin, uint64_t* kout,
                                   int32_t* pout, int64_t n, int nseg, int shift, uint32_t* hist,
                                   hipStream_t stream);
hipError_t n2v2r_launch_borda_finish(const int32_t* sorted_idx, int64_t n, int nseg, int ncols,
                                     int32_t* pos, int64_t* borda, hipStream_t stream);
int n2v2r_host_sym_eig_top(int n, double* A, int p, double* w, double* Z);
}

namespace {

struct HipFail {
  hipError_t e;
  std::string where;
};
struct StatusFail {
  int code;
  std::string msg;
};

#define HIPCHK(expr)                                                  \
  do {                                                                \
    hipError_t _e = (expr);                                           \
    if (_e != hipSuccess) throw HipFail{_e, #expr};                   \
  } while (0)

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// Device allocation owned by the handle.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void ensure(size_t b) {
    if (bytes >= b && p) return;
    release();
    if (b == 0) b = 16;
    hipError_t e = hipMalloc(&p, b);
    if (e != hipSuccess) {
      p = nullptr;
      throw StatusFail{N2V2R_ERR_OUT_OF_MEMORY,
                       "hipMalloc of " + std::to_string(b) + " bytes failed"};
    }
    bytes = b;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct LayerDev {
  DevBuf indptr, indices, data;        // A (CSR)
  DevBuf t_indptr, t_indices, t_data;  // A^T (CSR) when not symmetric
  int64_t nnz = 0;
  bool symmetric = true;
  bool loaded = false;
  CsrDev csr() const {
    return CsrDev{indptr.as<int64_t>(), indices.as<int32_t>(), data.as<float>(), n_rows, nnz};
  }
  CsrDev csr_t() const {
    if (symmetric) return csr();
    return CsrDev{t_indptr.as<int64_t>(), t_indices.as<int32_t>(), t_data.as<float>(), n_rows,
                  nnz};
  }
  int64_t n_rows = 0;
};

}  // namespace

struct n2v2r_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  int K = 0;
  int64_t n = 0;
  std::vector<std::unique_ptr<LayerDev>> layers;

  // UASE results
  int d = 0;
  int ldy = 0;              // row stride of the per-layer embedding
  DevBuf Y;                 // [K][n][ldy] fp32
  DevBuf U;                 // [n][ldu] fp32 left singular vectors (ldu = ldy)
  std::vector<double> sigma;
  bool have_embedding = false;

  // rank results
  int ncmp = 0, ncols = 0;
  DevBuf D;                 // [ncmp][ncols][n] fp64
  DevBuf borda;             // [ncmp][n] int64
  double ms_dist = 0, ms_borda = 0;

  // scratch
  DevBuf partial;           // chunk partials of the tall-skinny reductions
  size_t partial_elems = 0;
  DevBuf small64;           // c x c fp64 (H, G, ...)
  DevBuf small32;           // c x c fp32 (coefficients)
  DevBuf flags;             // int flags
  DevBuf theta;             // fp64 Ritz values
  DevBuf resid;             // fp64 residuals
  DevBuf colscale;          // fp32
  DevBuf rs_keys[2], rs_idx[2], rs_pos, rs_hist, rs_or, rs_and;

  void set_err(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    err = buf;
  }
};

namespace {

template <class F>
int guarded(n2v2r_handle* h, F&& f) {
  if (!h) return N2V2R_ERR_BAD_ARG;
  try {
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) throw HipFail{e, "hipSetDevice"};
    return f();
  } catch (const HipFail& hf) {
    h->set_err("HIP error %d (%s) at %s", (int)hf.e, hipGetErrorString(hf.e), hf.where.c_str());
    return N2V2R_ERR_HIP;
  } catch (const StatusFail& sf) {
    h->err = sf.msg;
    return sf.code;
  } catch (const std::bad_alloc&) {
    h->err = "host allocation failed";
    return N2V2R_ERR_OUT_OF_MEMORY;
  }
}

// ---- host CSR helpers -------------------------------------------------------------------
void host_transpose(int64_t n, int64_t nnz, const int64_t* ip, const int32_t* ix, const float* dv,
                    std::vector<int64_t>& tp, std::vector<int32_t>& tx, std::vector<float>& td) {
  tp.assign(n + 1, 0);
  for (int64_t p = 0; p < nnz; ++p) tp[ix[p] + 1]++;
  for (int64_t i = 0; i < n; ++i) tp[i + 1] += tp[i];
  tx.resize(nnz);
  td.resize(nnz);
  std::vector<int64_t> cur(tp.begin(), tp.end() - 1);
  for (int64_t r = 0; r < n; ++r)
    for (int64_t p = ip[r]; p < ip[r + 1]; ++p) {
      const int64_t q = cur[ix[p]]++;
      tx[q] = (int32_t)r;
      td[q] = dv[p];
    }
}

bool host_is_symmetric(int64_t n, int64_t nnz, const int64_t* ip, const int32_t* ix,
                       const float* dv, const std::vector<int64_t>& tp,
                       const std::vector<int32_t>& tx, const std::vector<float>& td) {
  // A == A^T iff row r of A equals row r of A^T as (sorted col, value) multisets.
  for (int64_t r = 0; r < n; ++r) {
    const int64_t a0 = ip[r], a1 = ip[r + 1], b0 = tp[r], b1 = tp[r + 1];
    if (a1 - a0 != b1 - b0) return false;
    std::vector<std::pair<int32_t, float>> ra, rb;
    ra.reserve(a1 - a0);
    rb.reserve(b1 - b0);
    for (int64_t p = a0; p < a1; ++p) ra.emplace_back(ix[p], dv[p]);
    for (int64_t p = b0; p < b1; ++p) rb.emplace_back(tx[p], td[p]);
    bool sorted_a = true;
    for (size_t i = 1; i < ra.size(); ++i)
      if (ra[i].first < ra[i - 1].first) sorted_a = false;
    if (!sorted_a) std::sort(ra.begin(), ra.end());
    if (ra != rb) return false;  // transpose rows come out column-sorted already
  }
  return true;
}

// ---- the eigensolver ----------------------------------------------------------------------
struct Eig {
  n2v2r_handle* h;
  hipStream_t st;
  int64_t n;
  int K;
  int b;            // block width
  int nb_max;       // max basis blocks
  int pb;           // kept blocks at restart
  int d;
  uint64_t seed;
  std::vector<std::unique_ptr<DevBuf>> pool;  // all N x b blocks
  std::vector<float*> freelist;
  std::vector<float*> Q, W;                   // current basis / images
  std::vector<std::unique_ptr<DevBuf>> zk;    // K stage-1 panels
  DevBuf rinv, flg, anyflag, gsmall, csmall;
  n2v2r_eig_stats* stats;
  double t_spmm = 0, t_ortho = 0;
  int64_t launches = 0;
  double algo_bytes = 0;
  uint64_t fill_counter = 0;

  float* take() {
    if (freelist.empty()) {
      pool.emplace_back(new DevBuf());
      pool.back()->ensure(sizeof(float) * n * b);
      return pool.back()->as<float>();
    }
    float* p = freelist.back();
    freelist.pop_back();
    return p;
  }
  void give(float* p) { freelist.push_back(p); }

  BlockList blocks(const std::vector<float*>& v, int from, int count) const {
    BlockList L{};
    L.count = count;
    L.width = b;
    for (int i = 0; i < count; ++i) L.blk[i] = v[from + i];
    return L;
  }
  BlockList one(const float* p) const {
    BlockList L{};
    L.count = 1;
    L.width = b;
    L.blk[0] = p;
    return L;
  }
  OutBlockList out_one(float* p) const {
    OutBlockList L{};
    L.count = 1;
    L.width = b;
    L.blk[0] = p;
    return L;
  }

  // W = M X = sum_k A_k (A_k^T X)
  void apply_M(const float* X, float* Wout) {
    const double t0 = now_ms();
    for (int k0 = 0; k0 < K; k0 += SPMM_MAX_LAYERS) {
      const int kc = std::min(SPMM_MAX_LAYERS, K - k0);
      SpmmArgs a{};
      a.K = kc;
      a.sum = 0;
      a.ldx = b;
      a.ldy = b;
      a.colscale = nullptr;
      for (int k = 0; k < kc; ++k) {
        a.A[k] = h->layers[k0 + k]->csr_t();
        a.X[k] = X;
        a.Y[k] = zk[k]->as<float>();
      }
      HIPCHK(n2v2r_launch_spmm(a, b, st));
      SpmmArgs s{};
      s.K = kc;
      s.sum = 1;
      s.ldx = b;
      s.ldy = b;
      s.colscale = nullptr;
      for (int k = 0; k < kc; ++k) {
        s.A[k] = h->layers[k0 + k]->csr();
        s.X[k] = zk[k]->as<float>();
      }
      s.Y[0] = Wout;
      if (k0 > 0) throw StatusFail{N2V2R_ERR_BAD_ARG, "more than 8 layers not supported yet"};
      HIPCHK(n2v2r_launch_spmm(s, b, st));
      for (int k = 0; k < kc; ++k) {
        const double nnz = (double)h->layers[k0 + k]->nnz;
        algo_bytes += 2.0 * (8.0 * nnz + 4.0 * (n + 1) + 8.0 * n * b);
      }
      launches += 2;
    }
    t_spmm += now_ms() - t0;
  }

  // One fused BCGS + CholQR pass: G = [Q Z]^T Z -> F -> Z <- [Q Z] F, refill deficient columns.
  // `cond` (device int, nullptr = always) skips the whole pass when zero.
  void pip_pass(float* Z, const std::vector<float*>& basis, const int* cond, int* flags_out,
                int* any_out) {
    const int nq = (int)basis.size();
    std::vector<float*> qz(basis);
    qz.push_back(Z);
    const BlockList L = blocks(qz, 0, nq + 1);
    HIPCHK(n2v2r_launch_ts_tn(L, one(Z), n, h->partial.as<double>(), h->partial_elems,
                              gsmall.as<double>(), cond, st));
    HIPCHK(n2v2r_launch_pip_chol(gsmall.as<double>(), nq * b, b, csmall.as<float>(), flags_out,
                                 any_out, cond, st));
    HIPCHK(n2v2r_launch_ts_nn(L, csmall.as<float>(), b, b, out_one(Z), one(nullptr), 1.f, 0.f, n,
                              cond, st));
    HIPCHK(n2v2r_launch_fill_normal(Z, b, n, seed ^ (0xABCDull + ++fill_counter), flags_out,
                                    any_out, st));
  }

  // orthonormalise Z against Q[0..nq) and within itself: two fused passes (BCGS-PIP2), a third
  // only when the second one had to refill a rank-deficient column.
  void orthonormalize(float* Z, const std::vector<float*>& basis) {
    const double t0 = now_ms();
    pip_pass(Z, basis, nullptr, flg.as<int>(), anyflag.as<int>());
    pip_pass(Z, basis, nullptr, flg.as<int>() + 64, anyflag.as<int>() + 1);
    pip_pass(Z, basis, anyflag.as<int>() + 1, flg.as<int>() + 128, anyflag.as<int>() + 2);
    t_ortho += now_ms() - t0;
  }

  // z = orth(W_from) against `basis`, w = M z; appended to (qs, ws)
  void expand_one(const float* w_from, const std::vector<float*>& basis, std::vector<float*>& qs,
                  std::vector<float*>& ws) {
    float* z = take();
    HIPCHK(hipMemcpyAsync(z, w_from, sizeof(float) * n * b, hipMemcpyDeviceToDevice, st));
    orthonormalize(z, basis);
    float* w = take();
    apply_M(z, w);
    qs.push_back(z);
    ws.push_back(w);
  }

  int run(int d_, const n2v2r_eig_opts& o, std::vector<double>& theta_out, float* Uout,
          int ldu) {
    d = d_;
    seed = o.seed ? o.seed : 0x5EEDull;
    const double tol = o.tol > 0 ? o.tol : 1e-6;
    const int max_restarts = o.max_restarts > 0 ? o.max_restarts : 2000;
    b = o.block ? o.block : 8;
    if (b != 8 && b != 16 && b != 32 && b != 64)
      throw StatusFail{N2V2R_ERR_BAD_ARG, "block must be 8, 16, 32 or 64"};
    // small graphs: shrink the block until the Krylov space fits well inside R^n
    int keep = 0, maxc = 0;
    for (;; b /= 2) {
      keep = o.keep ? o.keep : std::max(d + 16, (d * 5) / 4);
      keep = ((keep + b - 1) / b) * b;
      maxc = o.max_basis ? o.max_basis : std::max(keep + 3 * b, (16 * keep) / 5);
      maxc = ((maxc + b - 1) / b) * b;
      const int cap =
          (int)std::min<int64_t>((n / 2) / b * b, (int64_t)(N2V2R_MAX_BLOCKS - 1) * b);
      if (maxc > cap) maxc = cap;
      if (maxc >= keep + b) break;
      if (b == 8)
        throw StatusFail{N2V2R_ERR_BAD_ARG,
                         "graph too small for the requested dimension: need n >= 2*(keep+8)"};
    }
    pb = keep / b;
    nb_max = maxc / b;
    const int c_max = maxc;
    // scratch
    zk.clear();
    for (int k = 0; k < std::min(K, SPMM_MAX_LAYERS); ++k) {
      zk.emplace_back(new DevBuf());
      zk.back()->ensure(sizeof(float) * n * b);
    }
    h->partial_elems = std::max<size_t>(4096ull * 1024ull, (size_t)c_max * c_max * 8);
    h->partial.ensure(sizeof(double) * h->partial_elems);
    gsmall.ensure(sizeof(double) * (size_t)c_max * c_max);
    csmall.ensure(sizeof(float) * (size_t)c_max * c_max);
    rinv.ensure(sizeof(float) * 64 * 64);
    flg.ensure(sizeof(int) * 256);
    anyflag.ensure(sizeof(int) * 4);
    h->theta.ensure(sizeof(double) * c_max);
    h->resid.ensure(sizeof(double) * c_max);

    std::vector<double> Sh((size_t)c_max * keep), wh(keep);
    std::vector<double> res2(keep);

    // start block
    float* q0 = take();
    HIPCHK(n2v2r_launch_fill_normal(q0, b, n, seed, nullptr, nullptr, st));
    Q.assign(1, q0);
    orthonormalize(q0, {});
    W.assign(1, take());
    apply_M(Q[0], W[0]);
    int apps = 1;
    int cycle = 0;
    double maxres = 0;
    int conv = 0;
    std::vector<float*> X(pb), MX(pb);
    std::vector<double> hist_res;
    int stagnated = 0;
    const double t_start = now_ms();
    double t_rr = 0;
    // pinned host staging for the projected matrix and the Ritz coefficients
    double* Hh = nullptr;
    float* Sf = nullptr;
    HIPCHK(hipHostMalloc((void**)&Hh, sizeof(double) * (size_t)c_max * c_max, 0));
    HIPCHK(hipHostMalloc((void**)&Sf, sizeof(float) * (size_t)c_max * keep, 0));
    struct PinnedFree {
      double* h;
      float* s;
      ~PinnedFree() {
        if (h) (void)hipHostFree(h);
        if (s) (void)hipHostFree(s);
      }
    } pinned_guard{Hh, Sf};
    hipEvent_t ev_h, ev_e0, ev_e1;
    HIPCHK(hipEventCreateWithFlags(&ev_h, hipEventDisableTiming));
    HIPCHK(hipEventCreate(&ev_e0));
    HIPCHK(hipEventCreate(&ev_e1));
    struct EvFree {
      hipEvent_t a, b, c;
      ~EvFree() {
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        (void)hipEventDestroy(c);
      }
    } ev_guard{ev_h, ev_e0, ev_e1};
    // extra blocks expanded (against the old basis) while the host solves the projected
    // problem; adapted so that their GPU time covers the host Rayleigh-Ritz time
    int extras = 0;
    if (o.overlap == -2) extras = std::max(1, std::min(nb_max - pb - 1, (nb_max - pb) / 2));
    if (o.overlap > 0) extras = std::min(o.overlap, nb_max - pb - 1);
    const bool adaptive = o.overlap == -2;
    double t_blk_est = 0.0;
    for (;; ++cycle) {
      const double tcy0 = now_ms();
      int nexp = 0;
      while ((int)Q.size() < nb_max) {
        expand_one(W.back(), Q, Q, W);
        ++apps;
        ++nexp;
      }
      const int nq = (int)Q.size();
      const int c = nq * b;
      // H = Q^T W -> pinned host, then the host solves it on a worker thread
      HIPCHK(n2v2r_launch_ts_tn(blocks(Q, 0, nq), blocks(W, 0, nq), n, h->partial.as<double>(),
                                h->partial_elems, gsmall.as<double>(), nullptr, st));
      HIPCHK(hipMemcpyAsync(Hh, gsmall.as<double>(), sizeof(double) * c * c,
                            hipMemcpyDeviceToHost, st));
      HIPCHK(hipEventRecord(ev_h, st));
      double rr_ms = 0.0;
      int rr_status = 0;
      std::thread rr([&]() {
        if (hipEventSynchronize(ev_h) != hipSuccess) {
          rr_status = -1;
          return;
        }
        const double tr0 = now_ms();
        for (int i = 0; i < c; ++i)
          for (int j = 0; j < i; ++j) {
            const double sv = 0.5 * (Hh[(size_t)i * c + j] + Hh[(size_t)j * c + i]);
            Hh[(size_t)i * c + j] = sv;
            Hh[(size_t)j * c + i] = sv;
          }
        rr_status = n2v2r_host_sym_eig_top(c, Hh, keep, wh.data(), Sh.data());
        for (size_t i = 0; i < (size_t)c * keep; ++i) Sf[i] = (float)Sh[i];
        rr_ms = now_ms() - tr0;
      });
      // meanwhile: continue the Krylov sequence against the un-restarted basis
      std::vector<float*> E, EW, basis_e(Q);
      HIPCHK(hipEventRecord(ev_e0, st));
      for (int i = 0; i < extras; ++i) {
        expand_one(i == 0 ? W.back() : EW.back(), basis_e, E, EW);
        basis_e.push_back(E.back());
        ++apps;
      }
      HIPCHK(hipEventRecord(ev_e1, st));
      rr.join();
      if (rr_status != 0)
        throw StatusFail{N2V2R_ERR_NO_CONVERGENCE, "Rayleigh-Ritz eigensolve failed"};
      t_rr += rr_ms;
      HIPCHK(hipMemcpyAsync(csmall.as<float>(), Sf, sizeof(float) * c * keep,
                            hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(h->theta.as<double>(), wh.data(), sizeof(double) * keep,
                            hipMemcpyHostToDevice, st));
      // Ritz vectors X = Q S, MX = W S (keep columns, pb blocks)
      for (int q = 0; q < pb; ++q) {
        X[q] = take();
        MX[q] = take();
      }
      const double to0 = now_ms();
      const int per_launch = std::max(1, 128 / b);  // output blocks per ts_nn launch (<= 128 cols)
      for (int q0b = 0; q0b < pb; q0b += per_launch) {
        const int nt = std::min(per_launch, pb - q0b);
        OutBlockList ox{}, omx{};
        ox.width = omx.width = b;
        ox.count = omx.count = nt;
        for (int t = 0; t < nt; ++t) {
          ox.blk[t] = X[q0b + t];
          omx.blk[t] = MX[q0b + t];
        }
        // G slice: columns [q0b*b, q0b*b + nt*b) of S (ld = keep)
        const float* g = csmall.as<float>() + q0b * b;
        HIPCHK(n2v2r_launch_ts_nn(blocks(Q, 0, nq), g, keep, nt * b, ox, one(nullptr), 1.f, 0.f, n,
                                  nullptr, st));
        HIPCHK(n2v2r_launch_ts_nn(blocks(W, 0, nq), g, keep, nt * b, omx, one(nullptr), 1.f, 0.f,
                                  n, nullptr, st));
      }
      HIPCHK(n2v2r_launch_resid(blocks(X, 0, pb), blocks(MX, 0, pb), h->theta.as<double>(), n,
                                h->partial.as<double>(), h->partial_elems, h->resid.as<double>(),
                                st));
      HIPCHK(hipMemcpyAsync(res2.data(), h->resid.as<double>(), sizeof(double) * keep,
                            hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      t_ortho += now_ms() - to0;
      // adapt the overlap: enough extra blocks that their GPU time covers the host solve
      if (extras > 0 && adaptive) {
        float ems = 0.f;
        HIPCHK(hipEventElapsedTime(&ems, ev_e0, ev_e1));
        const double per_blk = std::max(1e-3, (double)ems / extras);
        t_blk_est = t_blk_est > 0 ? 0.5 * (t_blk_est + per_blk) : per_blk;
        const int want = (int)std::ceil(1.1 * rr_ms / t_blk_est);
        extras = std::max(1, std::min(nb_max - pb - 1, want));
      }
      (void)tcy0;
      (void)nexp;
      maxres = 0;
      conv = 0;
      const double th1 = std::max(wh[0], 1e-300);
      for (int j = 0; j < d; ++j) {
        const double r = std::sqrt(std::max(res2[j], 0.0)) / th1;
        maxres = std::max(maxres, r);
        if (r <= tol) ++conv;
      }
      bool done = (conv == d || cycle + 1 >= max_restarts);
      if (!done) {
        // fp32 noise floor: the true residual of W = M Q cannot fall below ~eps32 *
        // sqrt(nnz/row) * theta_1.  Stop when the worst residual has not improved by 2% over
        // 8 cycles and is within 100x of tol.
        hist_res.push_back(maxres);
        if (hist_res.size() >= 9) {
          const double prev = *std::min_element(hist_res.end() - 9, hist_res.end() - 1);
          if (maxres > 0.98 * prev && maxres <= 100.0 * tol) {
            stagnated = 1;
            done = true;
          }
        }
      }
      if (done) {
        for (float* p : E) give(p);
        for (float* p : EW) give(p);
        break;
      }
      // restart: [X | extras]; the extras are orthogonal to the old basis, hence to X.
      // Without overlap, the classic Krylov-Schur next block (W_last against the old basis).
      if (E.empty()) {
        expand_one(W.back(), Q, E, EW);
        ++apps;
      }
      for (float* p : Q) give(p);
      for (float* p : W) give(p);
      Q.assign(X.begin(), X.end());
      W.assign(MX.begin(), MX.end());
      Q.insert(Q.end(), E.begin(), E.end());
      W.insert(W.end(), EW.begin(), EW.end());
    }
    // U = first d columns of X (row stride ldu); theta
    theta_out.assign(wh.begin(), wh.begin() + d);
    for (int q = 0; q * b < d; ++q) {
      const int cols = std::min(b, d - q * b);
      HIPCHK(hipMemcpy2DAsync(Uout + q * b, sizeof(float) * ldu, X[q], sizeof(float) * b,
                              sizeof(float) * cols, n, hipMemcpyDeviceToDevice, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    if (stats) {
      stats->restarts = cycle + 1;
      stats->block_applications = apps;
      stats->converged = conv;
      stats->basis = c_max;
      stats->max_residual = maxres;
      stats->ms_total = now_ms() - t_start;
      stats->ms_spmm = t_spmm;
      stats->ms_ortho = t_ortho;
      stats->ms_rr_host = t_rr;
      stats->spmm_launches = launches;
      stats->spmm_algo_bytes = algo_bytes;
      stats->stagnated = stagnated;
    }
    return (conv == d || stagnated) ? N2V2R_OK : N2V2R_ERR_NO_CONVERGENCE;
  }
};

}  // namespace

// ======================================================================================
extern "C" {

const char* n2v2r_version(void) { return "n2v2r-mi355x 0.1.0 (gfx950)"; }

int n2v2r_create(int device, n2v2r_handle** out) {
  if (!out) return N2V2R_ERR_BAD_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return N2V2R_ERR_HIP;
  if (device < 0 || device >= count) return N2V2R_ERR_BAD_ARG;
  auto* h = new (std::nothrow) n2v2r_handle();
  if (!h) return N2V2R_ERR_OUT_OF_MEMORY;
  h->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return N2V2R_ERR_HIP;
  }
  *out = h;
  return N2V2R_OK;
}

void n2v2r_destroy(n2v2r_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  h->layers.clear();
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int n2v2r_last_error(const n2v2r_handle* h, char* buf, size_t len) {
  if (!h || !buf || len == 0) return N2V2R_ERR_BAD_ARG;
  snprintf(buf, len, "%s", h->err.c_str());
  return N2V2R_OK;
}

int n2v2r_synchronize(n2v2r_handle* h) {
  return guarded(h, [&]() -> int {
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_set_num_layers(n2v2r_handle* h, int num_layers, int64_t n) {
  return guarded(h, [&]() -> int {
    if (num_layers < 1 || n < 1 || n > (int64_t)INT32_MAX) {
      h->set_err("bad layer count %d or node count %lld", num_layers, (long long)n);
      return N2V2R_ERR_BAD_ARG;
    }
    if (num_layers > SPMM_MAX_LAYERS) {
      h->set_err("at most %d layers are supported", SPMM_MAX_LAYERS);
      return N2V2R_ERR_BAD_ARG;
    }
    h->K = num_layers;
    h->n = n;
    h->layers.clear();
    for (int k = 0; k < num_layers; ++k) h->layers.emplace_back(new LayerDev());
    h->have_embedding = false;
    h->ncmp = h->ncols = 0;
    return N2V2R_OK;
  });
}

int n2v2r_set_layer_csr(n2v2r_handle* h, int k, int64_t n, int64_t nnz, const int64_t* indptr,
                        const int32_t* indices, const float* data, int symmetric) {
  return guarded(h, [&]() -> int {
    if (k < 0 || k >= h->K || n != h->n || nnz < 0 || !indptr || (nnz > 0 && (!indices || !data))) {
      h->set_err("bad CSR arguments for layer %d", k);
      return N2V2R_ERR_BAD_ARG;
    }
    if (indptr[0] != 0 || indptr[n] != nnz) {
      h->set_err("layer %d: indptr must start at 0 and end at nnz", k);
      return N2V2R_ERR_BAD_ARG;
    }
    for (int64_t r = 0; r < n; ++r)
      if (indptr[r + 1] < indptr[r]) {
        h->set_err("layer %d: indptr not monotone", k);
        return N2V2R_ERR_BAD_ARG;
      }
    for (int64_t p = 0; p < nnz; ++p)
      if (indices[p] < 0 || indices[p] >= n) {
        h->set_err("layer %d: column index out of range", k);
        return N2V2R_ERR_BAD_ARG;
      }
    LayerDev& L = *h->layers[k];
    L.n_rows = n;
    L.nnz = nnz;
    L.indptr.ensure(sizeof(int64_t) * (n + 1));
    L.indices.ensure(sizeof(int32_t) * std::max<int64_t>(nnz, 1));
    L.data.ensure(sizeof(float) * std::max<int64_t>(nnz, 1));
    HIPCHK(hipMemcpyAsync(L.indptr.p, indptr, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice,
                          h->stream));
    if (nnz) {
      HIPCHK(hipMemcpyAsync(L.indices.p, indices, sizeof(int32_t) * nnz, hipMemcpyHostToDevice,
                            h->stream));
      HIPCHK(hipMemcpyAsync(L.data.p, data, sizeof(float) * nnz, hipMemcpyHostToDevice,
                            h->stream));
    }
    bool sym = symmetric == N2V2R_SYM_YES;
    std::vector<int64_t> tp;
    std::vector<int32_t> tx;
    std::vector<float> td;
    if (symmetric != N2V2R_SYM_YES) {
      host_transpose(n, nnz, indptr, indices, data, tp, tx, td);
      if (symmetric == N2V2R_SYM_DETECT)
        sym = host_is_symmetric(n, nnz, indptr, indices, data, tp, tx, td);
    }
    L.symmetric = sym;
    if (!sym) {
      L.t_indptr.ensure(sizeof(int64_t) * (n + 1));
      L.t_indices.ensure(sizeof(int32_t) * std::max<int64_t>(nnz, 1));
      L.t_data.ensure(sizeof(float) * std::max<int64_t>(nnz, 1));
      HIPCHK(hipMemcpyAsync(L.t_indptr.p, tp.data(), sizeof(int64_t) * (n + 1),
                            hipMemcpyHostToDevice, h->stream));
      if (nnz) {
        HIPCHK(hipMemcpyAsync(L.t_indices.p, tx.data(), sizeof(int32_t) * nnz,
                              hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(L.t_data.p, td.data(), sizeof(float) * nnz, hipMemcpyHostToDevice,
                              h->stream));
      }
    }
    HIPCHK(hipStreamSynchronize(h->stream));  // host vectors die here
    L.loaded = true;
    h->have_embedding = false;
    return N2V2R_OK;
  });
}

int n2v2r_uase(n2v2r_handle* h, int d, const n2v2r_eig_opts* opts, n2v2r_eig_stats* stats) {
  return guarded(h, [&]() -> int {
    if (h->K < 1) {
      h->err = "no layers set";
      return N2V2R_ERR_BAD_ARG;
    }
    for (auto& L : h->layers)
      if (!L->loaded) {
        h->err = "a layer was not loaded";
        return N2V2R_ERR_BAD_ARG;
      }
    if (d < 1 || d > 256 || d >= h->n) {
      h->set_err("embedding dimension %d out of range [1, min(256, n-1)]", d);
      return N2V2R_ERR_BAD_ARG;
    }
    n2v2r_eig_opts o{};
    if (opts) o = *opts;
    if (stats) memset(stats, 0, sizeof(*stats));
    Eig eig{};
    eig.h = h;
    eig.st = h->stream;
    eig.n = h->n;
    eig.K = h->K;
    eig.stats = stats;
    const int ldu = ((d + 63) / 64) * 64;  // a multiple of every block width
    h->U.ensure(sizeof(float) * h->n * ldu);
    HIPCHK(hipMemsetAsync(h->U.p, 0, sizeof(float) * h->n * ldu, h->stream));
    std::vector<double> theta;
    const int st = eig.run(d, o, theta, h->U.as<float>(), ldu);
    const int b = eig.b;
    // deterministic signs: largest-magnitude entry of every column of U positive
    h->partial.ensure(sizeof(double) * 1024 * (size_t)ldu);
    h->colscale.ensure(sizeof(float) * ldu);
    HIPCHK(n2v2r_launch_sign_convention(h->U.as<float>(), ldu, h->n, d,
                                        h->partial.as<unsigned long long>(),
                                        h->partial.bytes / sizeof(unsigned long long),
                                        h->colscale.as<float>(), h->stream));
    // Y_k = A_k^T U diag(theta)^(-1/4)  (sigma = sqrt(theta); V sqrt(sigma) = A^T U sigma^-1/2)
    h->d = d;
    h->ldy = ldu;
    h->sigma.assign(d, 0.0);
    std::vector<float> sc(ldu, 0.f);
    for (int j = 0; j < d; ++j) {
      h->sigma[j] = std::sqrt(std::max(theta[j], 0.0));
      sc[j] = h->sigma[j] > 0 ? (float)(1.0 / std::sqrt(h->sigma[j])) : 0.f;
    }
    h->colscale.ensure(sizeof(float) * ldu);
    HIPCHK(hipMemcpyAsync(h->colscale.p, sc.data(), sizeof(float) * ldu, hipMemcpyHostToDevice,
                          h->stream));
    h->Y.ensure(sizeof(float) * (size_t)h->K * h->n * ldu);
    for (int q = 0; q * b < ldu; ++q) {
      SpmmArgs a{};
      a.K = h->K;
      a.sum = 0;
      a.ldx = ldu;
      a.ldy = ldu;
      a.colscale = h->colscale.as<float>() + q * b;
      for (int k = 0; k < h->K; ++k) {
        a.A[k] = h->layers[k]->csr_t();
        a.X[k] = h->U.as<float>() + q * b;
        a.Y[k] = h->Y.as<float>() + (size_t)k * h->n * ldu + q * b;
      }
      HIPCHK(n2v2r_launch_spmm(a, b, h->stream));
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    h->have_embedding = true;
    h->ncmp = h->ncols = 0;
    if (st != N2V2R_OK)
      h->set_err("UASE did not converge: max residual %.3e (tol %.1e)",
                 stats ? stats->max_residual : -1.0, o.tol > 0 ? o.tol : 1e-6);
    return st;
  });
}

int n2v2r_get_embedding(n2v2r_handle* h, float* Y) {
  return guarded(h, [&]() -> int {
    if (!h->have_embedding) {
      h->err = "No n2v2r embeddings found";
      return N2V2R_ERR_NOT_READY;
    }
    for (int k = 0; k < h->K; ++k)
      HIPCHK(hipMemcpy2DAsync(Y + (size_t)k * h->n * h->d, sizeof(float) * h->d,
                              h->Y.as<float>() + (size_t)k * h->n * h->ldy,
                              sizeof(float) * h->ldy, sizeof(float) * h->d, h->n,
                              hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_get_left_embedding(n2v2r_handle* h, float* X) {
  return guarded(h, [&]() -> int {
    if (!h->have_embedding || h->U.p == nullptr) {
      h->err = "No n2v2r embeddings found";
      return N2V2R_ERR_NOT_READY;
    }
    HIPCHK(hipMemcpy2DAsync(X, sizeof(float) * h->d, h->U.as<float>(), sizeof(float) * h->ldy,
                            sizeof(float) * h->d, h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    for (int64_t i = 0; i < h->n; ++i)
      for (int j = 0; j < h->d; ++j) X[i * h->d + j] *= (float)std::sqrt(h->sigma[j]);
    return N2V2R_OK;
  });
}

int n2v2r_get_singular_values(n2v2r_handle* h, double* s) {
  return guarded(h, [&]() -> int {
    if (!h->have_embedding) {
      h->err = "No n2v2r embeddings found";
      return N2V2R_ERR_NOT_READY;
    }
    std::copy(h->sigma.begin(), h->sigma.end(), s);
    return N2V2R_OK;
  });
}

int n2v2r_set_embedding(n2v2r_handle* h, int num_layers, int64_t n, int d, const float* Y) {
  return guarded(h, [&]() -> int {
    if (num_layers < 1 || n < 1 || d < 1 || !Y) return N2V2R_ERR_BAD_ARG;
    h->K = num_layers;
    h->n = n;
    h->d = d;
    h->ldy = d;
    h->Y.ensure(sizeof(float) * (size_t)num_layers * n * d);
    HIPCHK(hipMemcpyAsync(h->Y.p, Y, sizeof(float) * (size_t)num_layers * n * d,
                          hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    h->sigma.assign(d, 0.0);
    h->have_embedding = true;
    h->ncmp = h->ncols = 0;
    return N2V2R_OK;
  });
}

static void run_borda(n2v2r_handle* h, const double* Ddev, int64_t n, int nseg, int ncols,
                      int64_t* borda_dev) {
  hipStream_t st = h->stream;
  const size_t tot = (size_t)nseg * n;
  for (int i = 0; i < 2; ++i) {
    h->rs_keys[i].ensure(sizeof(uint64_t) * tot);
    h->rs_idx[i].ensure(sizeof(int32_t) * tot);
  }
  h->rs_pos.ensure(sizeof(int32_t) * tot);
  const int ntiles = n2v2r_radix_tiles(n);
  h->rs_hist.ensure(sizeof(uint32_t) * (size_t)nseg * 256 * ntiles);
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
  HIPCHK(n2v2r_launch_borda_finish(h->rs_idx[cur].as<int32_t>(), n, nseg, ncols,
                                   h->rs_pos.as<int32_t>(), borda_dev, st));
}

int n2v2r_rank(n2v2r_handle* h, int strategy, const int* dims, int n_dims, const int* metrics,
               int n_metrics, int method, int* n_comparisons, int* n_cols) {
  return guarded(h, [&]() -> int {
    if (method != 0) {
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
    h->D.ensure(sizeof(double) * (size_t)ncmp * C * h->n);
    h->borda.ensure(sizeof(int64_t) * (size_t)ncmp * h->n);
    const double t0 = now_ms();
    for (int c = 0; c < ncmp; ++c)
      HIPCHK(n2v2r_launch_distances(h->Y.as<float>(), h->K, h->n, h->ldy, strategy, layer_i[c],
                                    plan, h->D.as<double>() + (size_t)c * C * h->n, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    const double t1 = now_ms();
    run_borda(h, h->D.as<double>(), h->n, ncmp * C, C, h->borda.as<int64_t>());
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
  return guarded(h, [&]() -> int {
    if (comparison < 0 || comparison >= h->ncmp || !D) return N2V2R_ERR_BAD_ARG;
    HIPCHK(hipMemcpyAsync(D, h->D.as<double>() + (size_t)comparison * h->ncols * h->n,
                          sizeof(double) * h->ncols * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_get_borda(n2v2r_handle* h, int comparison, int64_t* borda) {
  return guarded(h, [&]() -> int {
    if (comparison < 0 || comparison >= h->ncmp || !borda) return N2V2R_ERR_BAD_ARG;
    HIPCHK(hipMemcpyAsync(borda, h->borda.as<int64_t>() + (size_t)comparison * h->n,
                          sizeof(int64_t) * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_rank_timing(n2v2r_handle* h, double* ms_distances, double* ms_borda) {
  if (!h) return N2V2R_ERR_BAD_ARG;
  if (ms_distances) *ms_distances = h->ms_dist;
  if (ms_borda) *ms_borda = h->ms_borda;
  return N2V2R_OK;
}

int n2v2r_pairwise_distances(n2v2r_handle* h, const double* m1, const double* m2, int64_t n,
                             int dim, int metric, double* out) {
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

int n2v2r_column_sums(n2v2r_handle* h, int k, float* out) {
  return guarded(h, [&]() -> int {
    if (k < 0 || k >= h->K || !out || !h->layers[k]->loaded) return N2V2R_ERR_BAD_ARG;
    DevBuf o;
    o.ensure(sizeof(float) * h->n);
    HIPCHK(n2v2r_launch_row_sums(h->layers[k]->csr_t(), o.as<float>(), h->stream));
    HIPCHK(hipMemcpyAsync(out, o.p, sizeof(float) * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

int n2v2r_bench_spmm(n2v2r_handle* h, int k, int transpose, int b, int reps, const float* X,
                     float* Y, double* avg_ms, double* algo_bytes) {
  return guarded(h, [&]() -> int {
    if (k < 0 || k >= h->K || !h->layers[k]->loaded || (b != 8 && b != 16 && b != 32 && b != 64) ||
        reps < 1 || !X)
      return N2V2R_ERR_BAD_ARG;
    const LayerDev& L = *h->layers[k];
    DevBuf xd, yd;
    xd.ensure(sizeof(float) * h->n * b);
    yd.ensure(sizeof(float) * h->n * b);
    HIPCHK(hipMemcpyAsync(xd.p, X, sizeof(float) * h->n * b, hipMemcpyHostToDevice, h->stream));
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
      *algo_bytes = 8.0 * (double)L.nnz + 4.0 * (double)(h->n + 1) + 8.0 * (double)h->n * b;
    if (Y)
      HIPCHK(hipMemcpyAsync(Y, yd.p, sizeof(float) * h->n * b, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

}  // extern "C"

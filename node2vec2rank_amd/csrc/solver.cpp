// UASE solver (n2v2r_uase and the embedding getters of include/n2v2r.h): the block
// Krylov-Schur driver, on one GPU or on one rank of a row-partitioned handle.
//
// UASE (replaces se.UASE -> scipy svds/ARPACK, model.py:51-55): top-d eigenpairs of
// M = sum_k A_k A_k^T (N x N, = A A^T for the unfolded A = [A_1 | ... | A_K]) by a block
// Krylov-Schur iteration with explicit Rayleigh-Ritz:
//   basis Q = [Q_0 .. Q_{m-1}] (b-wide fp32 blocks in HBM), W_j = M Q_j kept beside it;
//   expand: Z = W_last, two fused BCGS + CholeskyQR passes (+random refill of deficient
//           columns, third pass only then), Q_m = Z, W_m = M Q_m
//           (2 SpMM launches: Z_k = A_k^T Q ; W = sum_k A_k Z_k);
//   cycle:  H = Q^T W (fp64) -> host top-p eigenpairs -> Ritz X = Q S, MX = W S,
//           residuals ||MX_j - theta_j X_j||; converged when all d <= tol * theta_1;
//   restart: next block = orth(W_last) against the old Q, keep [X_p | next] (thick restart).
// Embedding: Y_k = A_k^T U diag(sigma)^(-1/2) (= V diag(sigma)^(1/2) split per layer),
// sigma = sqrt(theta), columns in descending sigma order.
//
// Multi-GPU: rank g of W owns rows [g R, min(N, (g+1) R)), R = ceil(N / W), of
// every layer (and of A_k^T), of every basis block and of the embedding.  Column indices stay
// global: a panel gathered from all ranks (W x R rows, rank-major) is indexed by them directly.
// Per application of M: all-gather X, local SpMM, all-gather each Z_k, local SpMM.  Every
// reduction over rows (Gram blocks, H, residuals, sign keys) is a local fixed-order partial
// + an all-reduce, so every rank holds identical small matrices and runs the identical host
// Rayleigh-Ritz.  Communicators: RCCL (one process per GPU) or an in-process thread group
// (W ranks on one GPU, for testing the partitioned algorithm without W devices).
#include "engine.h"

using namespace n2v2r_int;

namespace n2v2r_int {
// The column-block SpMM (the flat-window tiled form): b = 8 CSR panels beyond 8 MB (beyond one
// XCD's L2); N2V2R_SPMM_CB=1 / 0 forces it on / off (tests, A/B runs).
// Read on every call, so a test can switch it between fits.
bool col_blocks_wanted(const n2v2r_handle* h, int b);

// Partitioned handles: the stage-1 panel Z_k of each layer all-gathered on a stream of its own
// while the next layer's stage 1 runs, unless N2V2R_GATHER_OVERLAP=0.  Read per call.
bool gather_overlap() {
  const char* e = std::getenv("N2V2R_GATHER_OVERLAP");
  return !(e && e[0] == '0');
}

// XCD-split second SpMM stage: b = 8 CSR layers on one GPU whose K stage-2 panels together
// exceed an XCD's 4 MB L2 (cfg2: 33.5 -> 24 us per stage; at N = 30k, where both panels fit,
// 4 % slower).  N2V2R_SPMM_SPLIT=1 / 0 forces it on / off.
bool split2_wanted(const n2v2r_handle* h, int b) {
  const char* e = std::getenv("N2V2R_SPMM_SPLIT");  // read per fit (tests flip it)
  const int force = e ? (e[0] == '0' ? 0 : 1) : -1;
  if (b != 8 || h->comm || h->dense_layers() || h->K < 2 || h->K > 8) return false;
  if (force >= 0) return force == 1;
  return (double)h->K * (double)h->n * 32.0 > 4.0 * 1024 * 1024;
}

// Paired-panel mode by default (no N2V2R_EIG_PANEL16 / PANEL8 flag): not yet (measured first).
bool pair_default(const n2v2r_handle* h, int d) {
  (void)h;
  (void)d;
  return false;
}

// The default basis cap of the b = 8 banded fits: 640 columns, N2V2R_BAND_MAXC = 768 for graphs
// from 4M nodes (round 6: the fused PIP pass past 64 KB of LDS; at cfg4's 1M nodes 768 columns
// are no better -- 771 block applications against 788 on one graph, 846 against 788 on the
// bench's --, at cfg5's 10M they are, see the kept-set rule below; profiles/r06_keep_basis.jsonl).
// The paired-panel mode keeps 640 (its measured configuration), and so does the reducing banded
// Rayleigh-Ritz (its arrow, chase and back-transform were never run past 640 columns: the Sturm
// form's fallback beyond is the dense one on H expanded from the band).
constexpr int kAutoMaxc = 640;
constexpr int kPairMaxc = 640;
constexpr int kReduceMaxc = 640;

// ---- the eigensolver ----------------------------------------------------------------------
struct Eig {
  n2v2r_handle* h;
  hipStream_t st;
  int64_t n;        // local rows
  int64_t npad;     // local rows incl. padding (panel allocation)
  int64_t row0;     // global index of local row 0
  int K;
  int b;            // block width
  int nb_max;       // max basis blocks
  int pb;           // kept blocks at restart
  int d;
  uint64_t seed;
  std::vector<float*> freelist;
  std::vector<float*> Q, W;                   // current basis / images
  n2v2r_eig_stats* stats;
  double t_spmm = 0, t_ortho = 0;
  int64_t launches = 0;
  double algo_bytes = 0;
  uint64_t fill_counter = 0;
  int kry0 = 0;             // index of the first Krylov block of the current cycle
  bool full_first = false;  // N2V2R_EIG_FULL_FIRST_PASS
  bool band_rr = false;     // banded Rayleigh-Ritz (b = 8, c <= 640), else dense
  bool band_reduce = false; // the reducing banded path takes the cycle (keep + 8 <= 192, c <= 640)
  // the flat-window tiled column-block SpMM (b = 8, panels beyond 8 MB): row tiles with LDS
  // accumulators walking tile_nb column-block phases, one launch per stage
  bool col_blocks = false;
  // the final lean check's stage-1 products Z_k = A_k^T X[q] of the d wanted Ritz vectors, kept
  // in the embedding buffer (h->Y, unscaled): they ARE the embedding's A_k^T U before the sign
  // and sigma^-1/2 column scaling -- the same tiled launch, the same summation order -- so the
  // embedding step skips its d/8 SpMM launches (cfg4: 16 x 0.74 ms)
  bool y_captured = false;
  int tile_rows = 0, tile_nb = CB_NB, tile_wb = CB_WIN_BITS_MIN;
  // Paired-panel mode (pair.hip): 8-wide basis blocks, every application of M multiplies the
  // last TWO as one N x 16 panel (spmm16_flat_kernel, tile_rows16 rows per tile); the projected
  // matrix (half-bandwidth 16) is assembled from the local passes' saved Gram rows -- hcol slot
  // s - kry0 holds column block s's rows hc_lo[s] .. + hc_nr[s] / 8 blocks -- and solved densely.
  bool pair = false;
  int tile_rows16 = 0;
  std::vector<int> hc_lo, hc_nr;
  int64_t hc_ld = 0;  // doubles per hcol slot
  int pcab_blk = 0;   // the block of E_b's saved first-pass Gram rows that holds E_a's
  // partitioned CSR handles: stage 2 as a reduce-scatter of this rank's column share (default
  // at W > 1) instead of all-gathers of every layer's stage-1 panel (N2V2R_DIST_STAGE2=gather)
  bool rs_form = false;
  // reduce-scatter form: stage 2 in rs_chunks row chunks of rs_rc local rows, each chunk's
  // reduce-scatter overlapped with the next chunk's product (N2V2R_RS_CHUNKS, default 4; 1: one
  // launch and one reduce-scatter)
  int rs_chunks = 1;
  int64_t rs_rc = 0;
  // XCD-split second SpMM stage (b = 8, one GPU): A_k Z_k lands in per-layer partials on the
  // XCDs of layer k; the image W = sum_k of them is stored by the next Gram pass that reads it
  // (the local first pass of the next expansion), or by materialize() before any other use
  bool split2 = false;
  float* pending = nullptr;  // the W block whose value still sits in the partials
  int stats_rr_fallbacks = 0;  // Sturm Rayleigh-Ritz cycles redone by the reducing path
  // dense Rayleigh-Ritz: the multi-workgroup tridiagonalisation's error word of the current
  // cycle (nullptr: the one-workgroup kernel ran), and whether a timeout switched the fit to the
  // one-workgroup kernel
  int* tri_err = nullptr;
  bool tri_single = false;
  int tri_fallbacks = 0;
  // Lean images: only the images a later step reads are kept (the cycle's input and the newest
  // one), so the basis alone (<= 154 MB at cfg2) stays in the 256 MB Infinity Cache between its
  // Gram and apply passes.  Residuals are the Krylov-Schur estimates ||R_E s_j|| (R_E: the
  // triangular factor of the restart block's projection), and a fit is finished only after the
  // true residuals of its d vectors (their images by SpMM) pass.
  bool lean_off = false;  // set by the caller to rerun a fit without lean images
  // selective reorthogonalisation: a full pass after the local one is skipped (in the fused
  // launch, by every workgroup alike) when max |Q^T z_j| <= reorth_tol ||z_j||
  float reorth_tol = 0.f;
  // deferred full passes (lean images, lazy two-pass mode; N2V2R_REORTH_DEFER=0: off): every other Krylov
  // block goes to its SpMM after the local pass alone and gets its full pass together with the
  // next block's (a pair shares one read of the old basis once a two-block Gram exists); its
  // image keeps the uncorrected block, whose components along older blocks are removed from
  // the next block by that block's full pass.  `deferred`: the block awaiting its full pass.
  bool defer = false, pair_gram = true;
  float* deferred = nullptr;
  struct LeanRetry {};
  // Gram scratch of the orthogonalisation passes (the workspace's)
  double* part_p = nullptr;
  size_t part_n = 0;
  double* gsm_p = nullptr;
  int* flg_p = nullptr;
  int* any_p = nullptr;

  // N2V2R_EIG_TIME_SPMM: an event pair around every SpMM stage launch (h->tev, reused), its
  // stage (0: A_k^T X, 1: A_k Z_k) and algorithmic bytes; summed after the fit's last sync
  bool time_spmm = false;
  std::vector<int> tkind;
  std::vector<double> tbytes;
  int tbeg() {
    if (!time_spmm) return -1;
    const size_t i = tkind.size();
    while (h->tev.size() < 2 * (i + 1)) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      h->tev.push_back(e);
    }
    HIPCHK(hipEventRecord(h->tev[2 * i], st));
    tkind.push_back(-1);
    tbytes.push_back(0.0);
    return (int)i;
  }
  void tend(int i, int kind, double bytes) {
    if (i < 0) return;
    HIPCHK(hipEventRecord(h->tev[2 * (size_t)i + 1], st));
    tkind[i] = kind;
    tbytes[i] = bytes;
  }
  void tsum(n2v2r_eig_stats* out) {
    if (!time_spmm || !out) return;
    HIPCHK(hipStreamSynchronize(st));
    for (size_t i = 0; i < tkind.size(); ++i) {
      if (tkind[i] < 0) continue;
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, h->tev[2 * i], h->tev[2 * i + 1]));
      out->gpu_ms_spmm[tkind[i]] += ms;
      out->spmm_timed_launches[tkind[i]] += 1;
      out->spmm_stage_bytes[tkind[i]] += tbytes[i];
    }
  }
  double layer_bytes(int k, bool transposed, int width = 0) const {
    const LayerDev& L = *h->layers[k];
    const bool t = transposed && !L.symmetric;
    return spmm_algo_bytes(t ? L.t_nnz : L.nnz, t ? L.t_unit : L.unit, n,
                           (int64_t)h->world * npad, width ? width : b);
  }

  // N2V2R_DEBUG_FINITE: stop at the first stage whose output holds a non-finite value
  int dbg_cycle = 0, dbg_apps = 0;
  void dbg(const void* p, int64_t count, bool f64, const char* what) {
    if (!debug_finite() || !p || count <= 0) return;
    int* flag = h->ews.dbgflag.as<int>();
    HIPCHK(hipMemsetAsync(flag, 0, sizeof(int), st));
    HIPCHK(n2v2r_launch_nonfinite(p, count, f64 ? 1 : 0, flag, st));
    int bad = 0;
    HIPCHK(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (bad) {
      const std::string msg = std::string("non-finite values first seen in ") + what +
                              " (cycle " + std::to_string(dbg_cycle) + ", block application " +
                              std::to_string(dbg_apps) + ", b " + std::to_string(b) + ")";
      fprintf(stderr, "[n2v2r] %s\n", msg.c_str());
      throw StatusFail{N2V2R_ERR_INTERNAL, msg};
    }
  }
  // N2V2R_DEBUG_ORTHO=1 (diagnostics): the Gram of a new block against the basis and itself,
  // reported on stderr when it is off the identity by more than 1e-3 (the block may still be
  // waiting for its deferred full pass: then its coupling to the old blocks is expected)
  void dbg_ortho(float* z, const std::vector<float*>& basis, const char* what,
                 const int* flags = nullptr) {
    if (!debug_ortho()) return;
    std::vector<float*> all(basis);
    all.push_back(z);
    const int nq = (int)all.size();
    DevBuf g;
    g.ensure(sizeof(double) * (size_t)nq * b * b);
    tn(blocks(all, 0, nq), one(z), g.as<double>(), nullptr);
    std::vector<double> hg((size_t)nq * b * b);
    HIPCHK(hipMemcpyAsync(hg.data(), g.p, sizeof(double) * hg.size(), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    double off = 0.0, self = 0.0, nrm = 0.0;
    for (int r = 0; r < nq * b; ++r)
      for (int j = 0; j < b; ++j) {
        const double v = hg[(size_t)r * b + j];
        if (r >= (nq - 1) * b) {
          const int i = r - (nq - 1) * b;
          self = std::max(self, std::fabs(v - (i == j ? 1.0 : 0.0)));
          if (i == j) nrm = std::max(nrm, v);
        } else {
          off = std::max(off, std::fabs(v));
        }
      }
    int fl[8] = {};
    if (flags) {
      HIPCHK(hipMemcpyAsync(fl, flags, sizeof(fl), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    if (off > 1e-3 || self > 1e-3)
      fprintf(stderr, "[n2v2r] %s: cycle %d, application %d, basis %d blocks: |Q^T z| %.3e, "
              "|z^T z - I| %.3e, max z_j^T z_j %.3e%s flags %d%d%d%d%d%d%d%d\n", what,
              dbg_cycle, dbg_apps, nq - 1, off, self, nrm, deferred == z ? " (deferred)" : "",
              fl[0], fl[1], fl[2], fl[3], fl[4], fl[5], fl[6], fl[7]);
  }

  // N2V2R_POISON: NaN-fill the scratch a fit must write before it reads it
  void poison_scratch() {
    if (!debug_poison()) return;
    EigWorkspace& w = h->ews;
    for (DevBuf* d : {&w.rinv, &w.flg, &w.anyflag, &w.gsmall, &w.csmall, &w.tri, &w.refl,
                      &w.ytri, &w.tscr, &w.hband, &w.band, &w.varr, &w.taua, &w.rrerr, &w.fcoef,
                      &h->partial, &h->theta, &h->resid})
      if (d->p) HIPCHK(hipMemsetAsync(d->p, 0xFF, d->bytes, st));
    for (auto& d : w.pool) HIPCHK(hipMemsetAsync(d->p, 0xFF, d->bytes, st));
    for (auto& d : w.zk) HIPCHK(hipMemsetAsync(d->p, 0xFF, d->bytes, st));
  }

  // N2V2R_POISON: NaN bytes into every CU's LDS before the next launch
  void lds_poison() {
    if (debug_poison()) HIPCHK(n2v2r_launch_lds_poison(st));
  }

  float* take() {
    if (freelist.empty()) {
      h->ews.pool.emplace_back(new DevBuf());
      h->ews.pool.back()->ensure(sizeof(float) * npad * b, st);
      return h->ews.pool.back()->as<float>();
    }
    float* p = freelist.back();
    freelist.pop_back();
    return p;
  }
  void give(float* p) {
    if (p) freelist.push_back(p);
  }

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

  float* s2part(int k) const { return h->ews.s2part.as<float>() + (size_t)k * npad * 8; }
  // store the pending image W = sum_k partial_k (fixed layer order)
  void materialize() {
    if (!pending) return;
    const float* parts[8];
    for (int k = 0; k < K; ++k) parts[k] = s2part(k);
    HIPCHK(n2v2r_launch_zsum(parts, K, pending, n, st));
    pending = nullptr;
  }

  // TN over local rows, summed over ranks
  void tn(const BlockList& A, const BlockList& B, double* out, const int* cond) {
    HIPCHK(n2v2r_launch_ts_tn(A, B, n, part_p, part_n, out, cond, st));
    if (h->comm)
      h->allreduce_f64(out, (size_t)A.count * A.width * B.count * B.width);
  }

  // Partitioned CSR handles, reduce-scatter form (the default at W > 1):
  // stage 1 as the gather form on the all-gathered X, then this rank's column share of stage 2,
  // P = sum_k A_k[:, own rows] Z_k[own rows] over all (padded) global rows -- gathered from the
  // rank's own Z rows only -- and ONE reduce-scatter of P into W's own rows: one all-gather + one
  // reduce-scatter per application instead of K + 1 all-gathers.
  void apply_M_rs(const float* xg, float* Wout) {
    const int64_t ng = (int64_t)h->world * npad;
    float* P = h->ews.zg.as<float>();  // the gather form's Z panels' buffer (>= ng x b)
    double b0 = 0.0, b1 = 0.0;
    for (int k = 0; k < K; ++k) b0 += layer_bytes(k, true);
    int te;
    if (col_blocks) {
      SpmmTileArgs a{};
      a.blk = h->ews.tblk.as<CsrBlk>();
      a.ldx = a.ldy = 8;
      a.n = n;
      a.K = K;
      a.nb = tile_nb;
      a.sum = 0;
      a.tile_rows = tile_rows;
      a.wbits = tile_wb;
      for (int k = 0; k < K; ++k) {
        a.X[k] = xg;
        a.Y[k] = h->ews.zk[k]->as<float>();
      }
      te = tbeg();
      HIPCHK(n2v2r_launch_spmm_tile(a, st));
    } else {
      SpmmArgs a{};
      a.K = K;
      a.ldx = a.ldy = b;
      for (int k = 0; k < K; ++k) {
        a.A[k] = h->layers[k]->csr_t();
        a.X[k] = xg;
        a.Y[k] = h->ews.zk[k]->as<float>();
      }
      te = tbeg();
      HIPCHK(n2v2r_launch_spmm(a, b, st));
    }
    tend(te, 0, b0);
    SpmmArgs s2{};
    s2.K = K;
    s2.sum = 1;
    s2.ldx = s2.ldy = b;
    for (int k = 0; k < K; ++k) {
      const LayerDev& L = *h->layers[k];
      s2.A[k] = L.csr_c();
      s2.X[k] = h->ews.zk[k]->as<float>();
      b1 += spmm_algo_bytes(L.c_nnz, s2.A[k].unit != 0, ng, npad, b);
    }
    s2.Y[0] = P;
    te = tbeg();
    if (rs_chunks <= 1) {
      HIPCHK(n2v2r_launch_spmm(s2, b, st));
      tend(te, 1, b1);
      h->comm->reduce_scatter_sum_f32(P, Wout, (size_t)npad * b, st);
    } else {
      // pipelined: the column share's rows are chunk-major (ensure_colcsr), so chunk c's product
      // -- rows [c rs_rc, ...) of every rank's block -- is one contiguous range of P, reduce-
      // scattered on the collective stream while chunk c + 1's product runs.  Every row is
      // summed as in the one-launch form (same rows per wave), and every element of W sums the
      // same ranks' values: the same result, with one chunk's reduce-scatter exposed.
      s2.rpw = n2v2r_spmm_rpw(s2, b);
      const int W = h->world;
      for (int c = 0; c < rs_chunks; ++c) {
        const int64_t r0 = (int64_t)c * rs_rc;
        const int64_t rows_c = std::min<int64_t>(rs_rc, npad - r0);
        if (rows_c <= 0) break;
        SpmmArgs sc = s2;
        for (int k = 0; k < K; ++k) {
          sc.A[k].indptr = s2.A[k].indptr + (size_t)r0 * W;
          sc.A[k].n_rows = (int64_t)W * rows_c;
        }
        float* pc = P + (size_t)r0 * W * b;
        sc.Y[0] = pc;
        HIPCHK(n2v2r_launch_spmm(sc, b, st));
        h->reduce_scatter_async(pc, Wout + (size_t)r0 * b, (size_t)rows_c * b);
      }
      tend(te, 1, b1);
      h->rs_wait_all();
    }
    algo_bytes += b0 + b1;
    launches += 2;
  }

  // W = M X = sum_k A_k (A_k^T X); X, W local, gathered panels for the column side
  void apply_M(const float* X, float* Wout) {
    const double t0 = now_ms();
    lds_poison();
    const int64_t ng = (int64_t)h->world * npad;  // rows of a gathered panel
    const float* xg = X;
    if (h->comm) {
      float* xgb = h->gath.as<float>();
      h->gather_panel(X, xgb, b);
      xg = xgb;
    }
    if (h->dense_layers()) {
      // Z_k = A_k^T X, W = sum_k A_k Z_k (fixed layer order), dense GEMMs on the local rows
      // per GEMM launch: the layer rows read once (4 n N) + the panel read and the output rows
      const double gb = 4.0 * (double)n * (double)h->n + 4.0 * (double)(ng + n) * b;
      for (int k = 0; k < K; ++k) {
        const LayerDev& L = *h->layers[k];
        const int te = tbeg();
        h->dense_apply(L.dense_at(), L.lda, xg, b, b, h->ews.zk[k]->as<float>(), b, 0.f, nullptr,
                       h->comm ? nullptr : L.dense_a());
        tend(te, 0, gb);
      }
      for (int k = 0; k < K; ++k) {
        const LayerDev& L = *h->layers[k];
        const float* zin = h->ews.zk[k]->as<float>();
        if (h->comm) {
          float* zgk = h->ews.zg.as<float>() + (size_t)k * ng * b;
          h->gather_panel(h->ews.zk[k]->as<float>(), zgk, b);
          zin = zgk;
        }
        const int te = tbeg();
        h->dense_apply(L.dense_a(), L.lda, zin, b, b, Wout, b, k == 0 ? 0.f : 1.f, nullptr,
                       h->comm ? nullptr : L.dense_at());
        tend(te, 1, gb);
        algo_bytes += 2.0 * gb;
      }
      launches += 2 * K;
      t_spmm += now_ms() - t0;
      return;
    }
    if (rs_form) {
      apply_M_rs(xg, Wout);
      t_spmm += now_ms() - t0;
      return;
    }
    if (col_blocks) {
      apply_M_tiled(xg, Wout, ng);
      t_spmm += now_ms() - t0;
      return;
    }
    SpmmArgs a{};
    a.K = K;
    a.sum = 0;
    a.ldx = b;
    a.ldy = b;
    a.colscale = nullptr;
    a.split = split2 ? 1 : 0;  // first stage split over the XCDs too (24.2 -> 23.4 us at cfg2)
    for (int k = 0; k < K; ++k) {
      a.A[k] = h->layers[k]->csr_t();
      a.X[k] = xg;
      a.Y[k] = h->ews.zk[k]->as<float>();
    }
    double sb0 = 0.0, sb1 = 0.0;
    for (int k = 0; k < K; ++k) {
      sb0 += layer_bytes(k, true);
      sb1 += layer_bytes(k, false);
    }
    // partitioned: stage 1 one layer per launch, each layer's Z_k all-gathered on the
    // collective stream while the next layer's stage 1 runs (N2V2R_GATHER_OVERLAP=0: in line)
    const bool ovl = h->comm && K > 1 && gather_overlap() && st == h->stream;
    int te = -1;
    if (ovl) {
      for (int k = 0; k < K; ++k) {
        SpmmArgs a1 = a;
        a1.K = 1;
        a1.split = 0;
        a1.A[0] = a.A[k];
        a1.X[0] = xg;
        a1.Y[0] = a.Y[k];
        te = tbeg();
        HIPCHK(n2v2r_launch_spmm(a1, b, st));
        tend(te, 0, layer_bytes(k, true));
        h->gather_panel_async(h->ews.zk[k]->as<float>(),
                              h->ews.zg.as<float>() + (size_t)k * ng * b, b, k);
      }
      for (int k = 0; k < K; ++k) h->gather_wait(k);
    } else {
      te = tbeg();
      HIPCHK(n2v2r_launch_spmm(a, b, st));
      tend(te, 0, sb0);
    }
    SpmmArgs s{};
    s.K = K;
    s.sum = 1;
    s.ldx = b;
    s.ldy = b;
    s.colscale = nullptr;
    for (int k = 0; k < K; ++k) {
      s.A[k] = h->layers[k]->csr();
      if (h->comm) {
        float* zgk = h->ews.zg.as<float>() + (size_t)k * ng * b;
        if (!ovl) h->gather_panel(h->ews.zk[k]->as<float>(), zgk, b);
        s.X[k] = zgk;
      } else {
        s.X[k] = h->ews.zk[k]->as<float>();
      }
    }
    s.Y[0] = Wout;
    if (split2) {
      materialize();  // (a previous image is always consumed by now; kept for safety)
      s.sum = 0;
      s.split = 1;
      for (int k = 0; k < K; ++k) s.Y[k] = s2part(k);
      pending = Wout;
    }
    te = tbeg();
    HIPCHK(n2v2r_launch_spmm(s, b, st));
    tend(te, 1, sb1);
    for (int k = 0; k < K; ++k) {
      const LayerDev& L = *h->layers[k];
      algo_bytes += spmm_algo_bytes(L.nnz, L.unit, n, n, b) +
                    spmm_algo_bytes(L.symmetric ? L.nnz : L.t_nnz,
                                    L.symmetric ? L.unit : L.t_unit, n, n, b);
    }
    launches += 2;
    t_spmm += now_ms() - t0;
  }

  // apply_M with the tiled column-block SpMM: one launch per stage over all layers
  void apply_M_tiled(const float* xg, float* Wout, int64_t ng) {
    const CsrBlk* tb = h->ews.tblk.as<CsrBlk>();
    SpmmTileArgs a{};
    a.blk = tb;
    a.ldx = a.ldy = 8;
    a.n = n;
    a.K = K;
    a.nb = tile_nb;
    a.sum = 0;
    a.tile_rows = tile_rows;
    a.wbits = tile_wb;
    double b0 = 0.0, b1 = 0.0;
    for (int k = 0; k < K; ++k) {
      a.X[k] = xg;
      a.Y[k] = h->ews.zk[k]->as<float>();
      b0 += layer_bytes(k, true);
      b1 += layer_bytes(k, false);
    }
    // partitioned: one launch per layer, Z_k gathered while layer k + 1 runs (as apply_M)
    const bool ovl = h->comm && K > 1 && gather_overlap() && st == h->stream;
    int te = -1;
    if (ovl) {
      for (int k = 0; k < K; ++k) {
        SpmmTileArgs a1 = a;
        a1.K = 1;
        a1.blk = tb + (size_t)k * tile_nb;
        a1.X[0] = xg;
        a1.Y[0] = a.Y[k];
        te = tbeg();
        HIPCHK(n2v2r_launch_spmm_tile(a1, st));
        tend(te, 0, layer_bytes(k, true));
        h->gather_panel_async(h->ews.zk[k]->as<float>(),
                              h->ews.zg.as<float>() + (size_t)k * ng * b, b, k);
      }
      for (int k = 0; k < K; ++k) h->gather_wait(k);
    } else {
      te = tbeg();
      HIPCHK(n2v2r_launch_spmm_tile(a, st));
      tend(te, 0, b0);
    }
    SpmmTileArgs s2 = a;
    s2.blk = tb + (size_t)K * tile_nb;
    s2.sum = 1;
    for (int k = 0; k < K; ++k) {
      s2.X[k] = h->ews.zk[k]->as<float>();
      if (h->comm) {
        float* zgk = h->ews.zg.as<float>() + (size_t)k * ng * b;
        if (!ovl) h->gather_panel(h->ews.zk[k]->as<float>(), zgk, b);
        s2.X[k] = zgk;
      }
      s2.Y[k] = nullptr;
    }
    s2.Y[0] = Wout;
    te = tbeg();
    HIPCHK(n2v2r_launch_spmm_tile(s2, st));
    tend(te, 1, b1);
    algo_bytes += b0 + b1;
    launches += 2;
  }

  // One fused BCGS + CholQR pass: G = [Q Z]^T Z -> R^{-1} -> Z <- [Q Z] [-C R^{-1}; R^{-1}],
  // refill deficient columns.  `cond` (device int, nullptr = always) skips the pass when zero.
  void pip_pass(float* Z, const std::vector<float*>& basis, const int* cond, int* flags_out,
                int* any_out, const float* Zin = nullptr, double* save = nullptr,
                int save_row0 = 0, int save_rows = 0, int* sticky = nullptr,
                double* rsave = nullptr, float skip_tol = 0.f, bool first = false) {
    // first: the block's first pass (a pivot the Pythagorean Gram cannot resolve is clamped and
    // the column kept); later passes refill such columns (dense.hip, PIP_CANCEL)
    // Zin (default Z): the block to orthogonalise; the result is written to Z
    const float* zin = Zin ? Zin : Z;
    const int nq = (int)basis.size();
    std::vector<float*> qz(basis);
    qz.push_back(const_cast<float*>(zin));
    const BlockList L = blocks(qz, 0, nq + 1);
    bool done = false;
    if (pending && zin == pending && !cond && !h->comm) {
      // the Gram pass that first reads the pending image also stores it
      const float* parts[8];
      for (int k = 0; k < K; ++k) parts[k] = s2part(k);
      const hipError_t e = n2v2r_launch_ts_tn_zsum(L, n, parts, K, pending, part_p, part_n, gsm_p,
                                                   st);
      if (e == hipSuccess) {
        pending = nullptr;
        done = true;
      } else if (e != hipErrorNotSupported) {
        throw HipFail{e, "n2v2r_launch_ts_tn_zsum"};
      }
    }
    if (!done) {
      if (zin == pending) materialize();
      tn(L, one(zin), gsm_p, cond);
    }
    if (b == 8 && nq * b <= N2V2R_BAND_MAXC && pip_fused()) {
      // b = 8: the Cholesky step runs inside the apply launch (every workgroup factors G)
      HIPCHK(n2v2r_launch_pip_fused(blocks(qz, 0, nq), zin, Z, gsm_p, nq * b,
                                    n, cond, flags_out, any_out, save, save_row0, save_rows,
                                    sticky, seed ^ (0xABCDull + ++fill_counter), row0, rsave,
                                    skip_tol, skip_tol != 0.f ? h->ews.skipc.as<int>() : nullptr,
                                    first ? 1 : 0, st));
      return;
    }
    if (rsave && b != 8) throw StatusFail{N2V2R_ERR_INTERNAL, "R output needs b = 8"};
    // (skip_tol: the unfused pass always applies)
    HIPCHK(n2v2r_launch_pip_chol(gsm_p, nq * b, b, h->ews.rinv.as<double>(),
                                 flags_out, any_out, cond, save, save_row0, save_rows,
                                 h->ews.fcoef.as<float>(), sticky, rsave, first ? 1 : 0, st));
    // rank-deficient columns (flags_out) are refilled with random values by the same launch
    HIPCHK(n2v2r_launch_pip_apply(L, h->ews.fcoef.as<float>(), nq * b, b, out_one(Z), n, cond,
                                  flags_out, seed ^ (0xABCDull + ++fill_counter), row0, st));
  }

  // orthonormalise Zin (default: Z in place) against `basis` and within itself into Z.
  // Default: a first fused pass against `local` only (the blocks W_from = M Q_last couples to in
  // exact arithmetic: the block three-term recurrence), then one full pass (block CGS2 with a
  // local first pass: the full pass removes the fp32 loss-of-orthogonality components); a third
  // full pass only when the second one had to refill a rank-deficient column.  `local` empty or
  // full_first: the first pass is a full one too (BCGS-PIP2).
  // save (band Rayleigh-Ritz): the first pass's Gram rows of the `local` blocks,
  // Q_loc^T W_from, are kept as band column j of the projected matrix.
  // lazy: no third pass; a refill in the second pass sets the cycle's sticky flag instead and
  // the cycle is expanded again with the third pass (rank deficiency after a local + full pass
  // is rare: it saves four launches per block).
  // rsave_first: R of the first pass (lean images: its column norms are the residual estimates)
  void orthonormalize(float* Z, const std::vector<float*>& basis, const float* Zin = nullptr,
                      const std::vector<float*>* local = nullptr, double* save = nullptr,
                      bool lazy = false, double* rsave_first = nullptr) {
    const double t0 = now_ms();
    lds_poison();
    int* flg = flg_p;
    int* any = any_p;
    const bool loc = local && !full_first && local->size() < basis.size();
    const std::vector<float*>& first = loc ? *local : basis;
    const int nsave = (save && local) ? (int)local->size() : 0;
    // (no sticky flag here: a column the first pass cancelled -- scaled, not normalised -- is
    // normalised by the full pass that always follows; a refill there (a later pass) sets it.
    // BASELINE cfg3's first images cancel: with the flag each fit expanded cycle 0 twice)
    pip_pass(Z, first, nullptr, flg, any, Zin, nsave ? save : nullptr,
             ((int)first.size() - nsave) * b, nsave * b, nullptr, rsave_first, 0.f, true);
    if (debug_ortho()) {  // pass 1's Gram [Q Z]^T Z (still in gsm_p)
      const int c1 = (int)first.size() * b;
      std::vector<double> g((size_t)(c1 + b) * b);
      HIPCHK(hipMemcpyAsync(g.data(), gsm_p, sizeof(double) * g.size(), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      fprintf(stderr, "[n2v2r] pass 1 Gram (c %d): Z^T Z diag", c1);
      for (int j = 0; j < b; ++j) fprintf(stderr, " %.4e", g[(size_t)(c1 + j) * b + j]);
      fprintf(stderr, "; C^T C diag");
      for (int j = 0; j < b; ++j) {
        double a = 0.0;
        for (int r = 0; r < c1; ++r) a += g[(size_t)r * b + j] * g[(size_t)r * b + j];
        fprintf(stderr, " %.4e", a);
      }
      fprintf(stderr, "\n");
    }
    dbg_ortho(Z, first, "after pass 1 (local)", flg);
    // (rsave_first: the second pass's R too, folded into the first's: R2 R1)
    pip_pass(Z, basis, nullptr, flg + 64, any + 1, nullptr, nullptr, 0, 0,
             lazy ? any + 3 : nullptr, rsave_first ? rsave_first + 64 : nullptr, reorth_tol);
    if (rsave_first) HIPCHK(n2v2r_launch_rmul8(rsave_first + 64, rsave_first, st));
    dbg_ortho(Z, basis, "after pass 2 (full, selective)", flg + 64);
    if (!lazy) pip_pass(Z, basis, any + 1, flg + 128, any + 2);
    if (!lazy) dbg_ortho(Z, basis, "after pass 3", flg + 128);
    t_ortho += now_ms() - t0;
  }

  // the deferred block's full pass against the blocks before it (its place in `basis`)
  void flush_deferred(const std::vector<float*>& basis) {
    if (!deferred) return;
    const auto it = std::find(basis.begin(), basis.end(), deferred);
    if (it == basis.end()) throw StatusFail{N2V2R_ERR_INTERNAL, "deferred block left the basis"};
    const std::vector<float*> pre(basis.begin(), it);
    const double t0 = now_ms();
    if (!pre.empty())
      pip_pass(deferred, pre, nullptr, flg_p + 64, any_p + 1, nullptr, nullptr, 0, 0, any_p + 3,
               nullptr, reorth_tol);
    t_ortho += now_ms() - t0;
    deferred = nullptr;
  }

  // The full passes of the deferred block Za (the last block of `basis`) and of the new block
  // Zb in one read of the old basis Q: G = [Q Za Zb]^T [Za Zb] (ts_tn_stream2), Za's selective
  // pass against Q (its R kept), Zb's Gram against the corrected Za (pair_fixup), Zb's selective
  // pass against [Q Za].  false when the two-block Gram does not apply (then the caller runs the
  // two passes one after the other).
  bool pair_pass(float* zb, const std::vector<float*>& basis) {
    if (!deferred || basis.empty() || basis.back() != deferred) return false;
    const int nq_old = (int)basis.size() - 1;
    if (nq_old + 2 > N2V2R_MAX_BLOCKS || (nq_old + 1) * 8 > N2V2R_BAND_MAXC) return false;
    std::vector<float*> all(basis);
    all.push_back(zb);
    // sized for the largest basis when the fit starts (a growing buffer reallocated here cost a
    // device-wide synchronisation per pair in a fit's first cycle: cfg2 +1.5 ms per fit)
    if (h->ews.g2.bytes < sizeof(double) * 2 * (size_t)(nq_old + 2) * 64) return false;
    double* g2 = h->ews.g2.as<double>();
    const double t0 = now_ms();
    lds_poison();
    const hipError_t e = n2v2r_launch_ts_tn2(blocks(all, 0, nq_old + 2), deferred, zb, n, part_p,
                                             part_n, g2, st);
    if (e == hipErrorNotSupported) return false;
    if (e != hipSuccess) throw HipFail{e, "n2v2r_launch_ts_tn2"};
    if (h->comm) h->allreduce_f64(g2, 2 * (size_t)(nq_old + 2) * 64);
    double* ra = h->ews.pair_ra.as<double>();
    int* skc = reorth_tol != 0.f ? h->ews.skipc.as<int>() : nullptr;
    HIPCHK(n2v2r_launch_pip_fused(blocks(basis, 0, nq_old), deferred, deferred, g2, nq_old * b, n,
                                  nullptr, flg_p + 64, any_p + 1, nullptr, 0, 0, any_p + 3,
                                  seed ^ (0xABCDull + ++fill_counter), row0, ra, reorth_tol, skc,
                                  0, st));
    HIPCHK(n2v2r_launch_pair_fixup(g2, nq_old + 2, nq_old, ra, st));
    HIPCHK(n2v2r_launch_pip_fused(blocks(basis, 0, nq_old + 1), zb, zb,
                                  g2 + (size_t)(nq_old + 2) * 64, (nq_old + 1) * b, n, nullptr,
                                  flg_p + 64, any_p + 1, nullptr, 0, 0, any_p + 3,
                                  seed ^ (0xABCDull + ++fill_counter), row0, nullptr, reorth_tol,
                                  skc, 0, st));
    t_ortho += now_ms() - t0;
    deferred = nullptr;
    return true;
  }

  // blocks M Q[last] couples to: Q[last-1], Q[last]; for the first Krylov block of a cycle
  // (kry0: the start block, or the block E appended at a thick restart) every block before it
  // (the kept Ritz vectors X, whose residuals M X - X Theta lie in span(E))
  std::vector<float*> local_of(const std::vector<float*>& basis) const {
    const int last = (int)basis.size() - 1;
    const int lo = last <= kry0 ? 0 : last - 1;
    return std::vector<float*>(basis.begin() + lo, basis.end());
  }

  // offset of band column j (the local Gram of W_j) in the band store: column kry0 holds
  // [X E]^T W_E ((kry0 + 1) b x b), later ones [Q_{j-1} Q_j]^T W_j (2b x b)
  size_t band_off(int j) const {
    if (j == kry0) return 0;
    return (size_t)(kry0 * b + b) * b + (size_t)(j - kry0 - 1) * 2 * b * b;
  }

  // z = orth(W_from) against `basis`, w = M z; appended to (qs, ws).  save_band: W_from is the
  // image of the last basis block; keep its local Gram as a band column.
  void expand_one(const float* w_from, const std::vector<float*>& basis, std::vector<float*>& qs,
                  std::vector<float*>& ws, bool save_band = false, bool lazy = false) {
    float* z = take();
    const std::vector<float*> loc = local_of(basis);
    double* save = (save_band && band_rr)
                       ? h->ews.hband.as<double>() + band_off((int)basis.size() - 1)
                       : nullptr;
    if (defer && lazy && !full_first) {
      // local pass; then either this block waits (its full pass with the next one) or the
      // waiting block and this one get their full passes
      const double t0 = now_ms();
      lds_poison();
      const bool lp = loc.size() < basis.size();
      const std::vector<float*>& first = lp ? loc : basis;
      const int nsave = save ? (int)loc.size() : 0;
      // a refill or heavy cancellation here sets the sticky flag: the block may not go to its
      // SpMM before its full pass, so the cycle is expanded again without deferral
      pip_pass(z, first, nullptr, flg_p, any_p, w_from, nsave ? save : nullptr,
               ((int)first.size() - nsave) * b, nsave * b, any_p + 3, nullptr, 0.f, true);
      t_ortho += now_ms() - t0;
      if (deferred && pair_gram && pair_pass(z, basis)) {
        // (both full passes done)
      } else if (deferred) {
        flush_deferred(basis);
        const double t1 = now_ms();
        pip_pass(z, basis, nullptr, flg_p + 64, any_p + 1, nullptr, nullptr, 0, 0, any_p + 3,
                 nullptr, reorth_tol);
        t_ortho += now_ms() - t1;
      } else {
        deferred = z;
      }
    } else {
      orthonormalize(z, basis, w_from, &loc, save, lazy);  // reads W_from, writes z: no copy
    }
    dbg(z, n * b, false, "orthonormalised Krylov block");
    dbg_ortho(z, basis, "Krylov block before its SpMM");
    float* w = take();
    apply_M(z, w);
    if (debug_finite()) materialize();
    dbg(w, n * b, false, "SpMM image M q");
    ++dbg_apps;
    qs.push_back(z);
    ws.push_back(w);
  }

  // Paired mode: [Wa | Wb] = M [za | zb] with the tiled SpMM at 64-B panel rows: the two blocks
  // interleaved into one N x 16 panel, stage 1 Z_k = A_k^T X (N x 16 per layer), stage 2 summed
  // over the layers in LDS and written straight into the two 8-wide image blocks
  void apply_M_pair(const float* za, const float* zb, float* wa, float* wb) {
    const double t0 = now_ms();
    lds_poison();
    float* x16 = h->ews.x16.as<float>();
    HIPCHK(n2v2r_launch_interleave16(za, zb, x16, n, st));
    const CsrBlk* tb = h->ews.tblk.as<CsrBlk>();
    SpmmTileArgs a{};
    a.blk = tb;
    a.ldx = a.ldy = 16;
    a.n = n;
    a.K = K;
    a.nb = tile_nb;
    a.sum = 0;
    a.tile_rows = tile_rows16;
    a.wbits = tile_wb;
    a.width = 16;
    double b0 = 0.0, b1 = 0.0;
    for (int k = 0; k < K; ++k) {
      a.X[k] = x16;
      a.Y[k] = h->ews.zk[k]->as<float>();
      b0 += layer_bytes(k, true, 16);
      b1 += layer_bytes(k, false, 16);
    }
    int te = tbeg();
    HIPCHK(n2v2r_launch_spmm_tile(a, st));
    tend(te, 0, b0);
    SpmmTileArgs s2 = a;
    s2.blk = tb + (size_t)K * tile_nb;
    s2.sum = 1;
    for (int k = 0; k < K; ++k) {
      s2.X[k] = h->ews.zk[k]->as<float>();
      s2.Y[k] = nullptr;
    }
    s2.Y[0] = wa;
    s2.Y2 = wb;
    te = tbeg();
    HIPCHK(n2v2r_launch_spmm_tile(s2, st));
    tend(te, 1, b1);
    algo_bytes += b0 + b1;
    launches += 2;
    t_spmm += now_ms() - t0;
  }

  // hcol slot of basis column block s (its saved band rows)
  double* hcol_at(int s) const { return h->ews.hcol.as<double>() + (size_t)(s - kry0) * hc_ld; }

  // the blocks the images of the pair at basis indices p, p + 1 couple to in exact arithmetic:
  // the previous pair and this one (p - 2 .. p + 1), or every block for the first Krylov pair of
  // a cycle (the kept Ritz vectors' residuals lie in span(E))
  int pair_lo(int p) const { return p <= kry0 ? 0 : p - 2; }

  // Paired mode: the next pair (za, zb) from the images (wa, wb) of the last pair of `Q`, and its
  // images.  za: local pass against the pair's coupling blocks L (band column p saved), zb: local
  // pass against L + [za] (band column p + 1); then both full passes from one read of the old
  // basis (pair_pass: za's selective pass, zb's Gram against the corrected za, zb's selective
  // pass) -- or, not lazy (after a refill), three passes each; then one SpMM application.
  void expand_pair(const float* wa, const float* wb, std::vector<float*>& qs,
                   std::vector<float*>& ws, bool lazy) {
    const int p = (int)Q.size() - 2;
    const int lo = pair_lo(p);
    const std::vector<float*> La(Q.begin() + lo, Q.end());
    float* za = take();
    float* zb = take();
    std::vector<float*> Lb(La);
    Lb.push_back(za);
    std::vector<float*> qa(Q);
    qa.push_back(za);
    hc_lo[p] = lo;
    hc_nr[p] = (int)La.size() * 8;
    hc_lo[p + 1] = lo;
    hc_nr[p + 1] = (int)Lb.size() * 8;
    if (lazy && defer && !full_first) {
      const double t0 = now_ms();
      lds_poison();
      pip_pass(za, La, nullptr, flg_p, any_p, wa, hcol_at(p), 0, (int)La.size() * 8, nullptr,
               nullptr, 0.f, true);
      pip_pass(zb, Lb, nullptr, flg_p, any_p, wb, hcol_at(p + 1), 0, (int)Lb.size() * 8, nullptr,
               nullptr, 0.f, true);
      t_ortho += now_ms() - t0;
      deferred = za;
      if (!(pair_gram && pair_pass(zb, qa))) {
        flush_deferred(qa);
        const double t1 = now_ms();
        pip_pass(zb, qa, nullptr, flg_p + 64, any_p + 1, nullptr, nullptr, 0, 0, any_p + 3,
                 nullptr, reorth_tol);
        t_ortho += now_ms() - t1;
      }
    } else {
      orthonormalize(za, Q, wa, &La, hcol_at(p), lazy);
      orthonormalize(zb, qa, wb, &Lb, hcol_at(p + 1), lazy);
    }
    dbg(za, n * 8, false, "orthonormalised Krylov block (pair a)");
    dbg(zb, n * 8, false, "orthonormalised Krylov block (pair b)");
    dbg_ortho(zb, qa, "Krylov pair before its SpMM");
    float* w0 = take();
    float* w1 = take();
    apply_M_pair(za, zb, w0, w1);
    dbg(w0, n * 8, false, "SpMM image M q (pair a)");
    dbg(w1, n * 8, false, "SpMM image M q (pair b)");
    dbg_apps += 2;
    qs.push_back(za);
    qs.push_back(zb);
    ws.push_back(w0);
    ws.push_back(w1);
  }

  int run(int d_, const n2v2r_eig_opts& o, std::vector<double>& theta_out, float* Uout,
          int ldu) {
    d = d_;
    seed = o.seed ? o.seed : 0x5EEDull;
    full_first = (o.solver_flags & N2V2R_EIG_FULL_FIRST_PASS) != 0;
    time_spmm = (o.solver_flags & N2V2R_EIG_TIME_SPMM) != 0;
    tkind.clear();
    tbytes.clear();
    kry0 = 0;
    bool lazy = true;
    const bool test_redo = (o.solver_flags & N2V2R_EIG_TEST_REDO_CYCLE) != 0;
    const bool test_band_fail = (o.solver_flags & N2V2R_EIG_TEST_BAND_FAIL) != 0;
    const bool test_sturm_fail = (o.solver_flags & N2V2R_EIG_TEST_STURM_FAIL) != 0;
    const double tol = o.tol > 0 ? o.tol : 1e-6;
    const int max_restarts = o.max_restarts > 0 ? o.max_restarts : 2000;
    const bool no_stagnation = (o.solver_flags & N2V2R_EIG_TEST_NO_STAGNATION) != 0;
    // default panel width: 8 for CSR layers (vector-applications grow with b); 32 for dense
    // layers, where one application streams all of A whatever b is (HBM-bound up to b = 32)
    b = o.block ? o.block : (h->dense_layers() ? 32 : 8);
    if (b != 8 && b != 16 && b != 32 && b != 64)
      throw StatusFail{N2V2R_ERR_BAD_ARG, "block must be 8, 16, 32 or 64"};
    const int64_t nglob = h->n;
    // small graphs: shrink the block until the Krylov space fits well inside R^n
    int keep = 0, maxc = 0;
    // CSR layers: keep 21d/16 (rounded up to b) -- round 4, on two graphs each: cfg4 795-838
    // block applications against 812-856 at the former 5d/4 (1.51-1.59 vs 1.53-1.63 s), cfg2
    // (84 -> 88) 270 against 276-314, and 11d/8 mixed (profiles/r04_keep_sweep.jsonl); round 5
    // at basis 640, cfg4: keep 152 / 168 / 184 / 200 / 224 / 256 -> 812 / 788 / 821 / 795 / 808
    // / 800 block applications (profiles/r05_keep_b8.jsonl)
    // dense layers (b = 32): keep d + b, basis <= 704 -- on three cfg3-family graphs 61 block
    // applications and 215-218 ms per fit against 66 and 236-240 ms with the general rule's
    // keep 5d/4 = 320 and basis 768 (profiles/r04_cfg3_sweep*.jsonl)
    const bool dense_rule = h->dense_layers() && !o.block;
    // graphs from 4M nodes (d <= 160, CSR layers): keep 7d/4 and bases up to 768 columns (round
    // 6, d = 128: cfg5's N = 10M 1,728 block applications and 41.9 s per fit against 1,909 and
    // 44.7 s at keep 168 / basis 640; at N = 3M keep 224 and 168 tie, at cfg4's 1M keep 168 and
    // basis 640 win; profiles/r06_keep_basis.jsonl)
    const bool big_graph = !dense_rule && nglob >= ((int64_t)1 << 22) && d <= 160;
    for (;; b /= 2) {
      keep = o.keep ? o.keep : (dense_rule ? d + b : std::max(d + 16, (d * 21) / 16));
      keep = ((keep + b - 1) / b) * b;
      // (not past the banded Rayleigh-Ritz's 184 kept vectors where the former rule fit them)
      if (!o.keep && !dense_rule && b == 8 && keep > 184 && std::max(d + 16, (d * 5) / 4) <= 184)
        keep = 184;
      if (!o.keep && big_graph && b == 8) keep = std::max(keep, ((d * 7) / 4 + 7) / 8 * 8);
      // default basis: 3.2 keep for the dense Rayleigh-Ritz (its cost grows as c^3); 4.8 keep
      // (<= 512) for the banded one (b = 8), where fewer, longer cycles win (cfg2: 14 cycles
      // at c = 256, 7 at c = 384, 13 % fewer block applications)
      // (a keep that does not fit the banded form's 512-column basis takes the dense one's)
      // (the banded form's basis follows the former keep rule, 5d/4: cfg2 keeps c = 384 -- 270
      // block applications against 305 at 4.8 x 88 = 424)
      const int keep_basis = (o.keep || dense_rule)
                                 ? keep
                                 : ((std::max(d + 16, (d * 5) / 4) + b - 1) / b) * b;
      const bool band_ok = b == 8 && !(o.solver_flags & N2V2R_EIG_DENSE_RR) && keep + b <= 512;
      // (round 5: up to N2V2R_BAND_MAXC = 640 columns -- cfg4 786-791 block applications and
      // 1.41-1.42 s per fit at c = 576-640 against 838 and 1.51 s at 512,
      // profiles/r05_basis_b8.jsonl)
      maxc = o.max_basis ? o.max_basis
                         : (band_ok ? std::min(big_graph ? N2V2R_BAND_MAXC : kAutoMaxc,
                                               std::max(keep + 3 * b, (24 * keep_basis) / 5))
                                    : std::max(keep + 3 * b, (16 * keep_basis) / 5));
      maxc = ((maxc + b - 1) / b) * b;
      const int cap =
          (int)std::min<int64_t>((nglob / 2) / b * b, (int64_t)(N2V2R_MAX_BLOCKS - 1) * b);
      if (maxc > cap) maxc = cap;
      if (maxc > 768) maxc = 768 / b * b;  // Rayleigh-Ritz kernels: c <= 768
      if (dense_rule && !o.max_basis && maxc > 704) maxc = 704 / b * b;
      if (maxc >= keep + b) break;
      // the auto keep 21d/16 does not fit the basis (d near the 600 limit, small graphs): the
      // former 5d/4
      const int keep_old = ((std::max(d + 16, (d * 5) / 4) + b - 1) / b) * b;
      if (!o.keep && !dense_rule && keep > keep_old && maxc >= keep_old + b) {
        keep = keep_old;
        break;
      }
      if (b == 8)
        throw StatusFail{N2V2R_ERR_BAD_ARG,
                         "graph too small for the requested dimension: need n >= 2*(keep+8)"};
    }
    // paired-panel mode: N2V2R_EIG_PANEL16 / N2V2R_EIG_PANEL8 force it on / off; by default on
    // for one-GPU CSR fits that take the tiled SpMM (pair_default).  It needs lean images (the
    // projected matrix comes from the saved band, not from kept images), keeps and bases in
    // whole pairs, and a basis the fused passes take (<= N2V2R_BAND_MAXC columns).
    pair = false;
    if (b == 8 && !h->comm && !h->dense_layers() && !lean_off && lean_enabled() &&
        !full_first && !(o.solver_flags & N2V2R_EIG_PANEL8) && !(o.solver_flags & N2V2R_EIG_DENSE_RR) &&
        col_blocks_wanted(h, 8) &&
        ((o.solver_flags & N2V2R_EIG_PANEL16) || pair_default(h, d))) {
      int pk = (keep + 15) / 16 * 16;
      int pc = o.max_basis ? o.max_basis / 16 * 16
                           : std::min(kPairMaxc,
                                      std::max(pk + 48, (24 * ((std::max(d + 16, (d * 5) / 4) + 7) / 8 * 8)) / 5));
      pc = pc / 16 * 16;
      const int cap16 = (int)std::min<int64_t>((nglob / 2) / 16 * 16, (int64_t)kPairMaxc);
      if (pc > cap16) pc = cap16;
      if (pk + 32 <= pc && pc <= kPairMaxc) {
        pair = true;
        keep = pk;
        maxc = pc;
      }
    }
    pb = keep / b;
    nb_max = maxc / b;
    const int c_max = maxc;
    // A fit that stops because its residuals went flat (the fp32 floor) is a success only within
    // stag_cap.  The floor: a Ritz vector X = Q S is assembled in fp32 from c basis columns, so
    // its entries carry ~sqrt(c) 2^-24 relative rounding, and ||M x - theta x|| / theta_1 cannot
    // fall much below that (1.35e-6 at c = 512; the cfg4-grid fixture's last column stops at
    // 1.28e-6, its host fp64 residual agrees, and 12 more cycles do not lower it:
    // tests/test_gpu_configs.py::test_cfg4_grid_vs_reference).  Past the cap the fit returns
    // N2V2R_ERR_NO_CONVERGENCE.
    const double stag_cap = 2.0 * std::max(tol, std::sqrt((double)c_max) * 0x1p-24);
    // scratch
    // reuse the workspace of the previous fit: every pool block is free again
    const size_t bb = sizeof(float) * npad * b;
    if (h->ews.block_bytes != bb) {
      h->ews.pool.clear();
      h->ews.block_bytes = bb;
    }
    freelist.clear();
    for (auto& blk : h->ews.pool) freelist.push_back(blk->as<float>());
    while ((int)h->ews.zk.size() < K) h->ews.zk.emplace_back(new DevBuf());
    for (int k = 0; k < K; ++k) h->ews.zk[k]->ensure(pair ? 2 * bb : bb);  // (pair: N x 16)
    if (h->comm) {
      h->gath.ensure(sizeof(float) * h->world * npad * b);
      h->ews.zg.ensure(sizeof(float) * (size_t)K * h->world * npad * b);
    }
    col_blocks = col_blocks_wanted(h, b);
    if (col_blocks) {
      // the flat-window tiled SpMM: column blocks (phases) per layer of <= 2 MB of panel, so a
      // phase's block stays in the XCD's 4 MB L2 beside the index stream (cfg4: 16 blocks,
      // 0.748 ms per stage launch; 8 blocks 0.896, 32 blocks 0.817: 4 MB blocks left 31 % of
      // the gathers missing L2), at most 64 (cfg5's 320 MB panel, one layer launch: 4.36 ms at
      // 64 blocks of 5 MB, 4.62 at 32 of 10 MB, 5.14 at 16 -- round 5, window offsets,
      // profiles/r05_tile_cfg5.jsonl; with round 4's per-row block pointers 64 blocks lost).
      // N2V2R_SPMM_TILE_NB = 4..64 overrides (read per fit).
      int nb_auto = 4;
      while (nb_auto < 64 && (double)nglob * 32.0 / nb_auto > 2.0 * 1024 * 1024) nb_auto *= 2;
      if (pair) {
        // 64-B panel rows (round 6, spmm16_flat_kernel per layer launch): blocks of <= 2 MB while
        // the N x 16 panel stays well inside the Infinity Cache (cfg4, 64 MB: 32 blocks 0.526 ms
        // against 0.559 at 16); beyond it longer runs per window win over L2 residency (cfg5,
        // 640 MB: 16 blocks 5.45 ms, 32 5.45-5.82, 64 5.85-7.37; profiles/r06_spmm16_*.jsonl)
        nb_auto = 4;
        if ((double)nglob * 64.0 > 128.0 * 1024 * 1024)
          nb_auto = 16;
        else
          while (nb_auto < 64 && (double)nglob * 64.0 / nb_auto > 2.0 * 1024 * 1024) nb_auto *= 2;
      }
      const char* tn_ = std::getenv("N2V2R_SPMM_TILE_NB");
      tile_nb = tn_ ? std::atoi(tn_) : nb_auto;
      if (tile_nb != 4 && tile_nb != 8 && tile_nb != 16 && tile_nb != 32 && tile_nb != 64 &&
          tile_nb != 128)
        tile_nb = nb_auto;
      // packed entries need the in-block column bits to fit beside the row-in-window bits
      // (always, for N < 2^26 per block); otherwise the row kernel runs
      tile_wb = tile_wbits(h->layers, tile_nb);
      for (auto& Lp : h->layers)
        col_blocks = ensure_col_blocks(*Lp, nglob, st, tile_nb, tile_wb) && col_blocks;
      if (col_blocks) {
        int ncu = 0;
        HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->device));
        tile_rows = n2v2r_spmm_tile_rows(n, ncu, 2, tile_wb);
        tile_rows16 = n2v2r_spmm_tile_rows_b(n, ncu, N2V2R_SPMM16_WPC, tile_wb, 16);
        const int nb = tile_nb;
        std::vector<CsrBlk> hb((size_t)2 * K * nb);
        for (int k = 0; k < K; ++k) {
          const LayerDev& L = *h->layers[k];
          for (int j = 0; j < nb; ++j) {
            hb[(size_t)k * nb + j] = (L.symmetric ? L.cb : L.cb_t).blk[j];
            hb[(size_t)(K + k) * nb + j] = L.cb.blk[j];
          }
        }
        h->ews.tblk.ensure(sizeof(CsrBlk) * hb.size());
        HIPCHK(hipMemcpyAsync(h->ews.tblk.p, hb.data(), sizeof(CsrBlk) * hb.size(),
                              hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));  // hb dies here
      }
    }
    rs_form = false;
    if (h->comm && !h->dense_layers()) {
      // read per fit (tests, A/B runs): "rs" / "gather" force a form; unset: the reduce-scatter
      // when there is more than one rank (one rank's "column share" is every row: its stage 2
      // would gather from the whole Z with the row kernel, slower than the tiled gather form)
      const char* e = std::getenv("N2V2R_DIST_STAGE2");
      rs_form = e && std::strcmp(e, "rs") == 0 ? true
                : e && std::strcmp(e, "gather") == 0 ? false
                : h->world > 1;
      if (rs_form) {
        const char* ce = std::getenv("N2V2R_RS_CHUNKS");  // read per fit (tests, A/B runs)
        rs_chunks = std::max(1, std::min(SPMM_MAX_LAYERS, ce ? std::atoi(ce) : 4));
        rs_rc = (npad + rs_chunks - 1) / rs_chunks;
        rs_chunks = (int)((npad + rs_rc - 1) / rs_rc);
        if (rs_chunks <= 1) rs_rc = 0;
        for (auto& Lp : h->layers)
          ensure_colcsr(*Lp, nglob, (int64_t)h->world * npad, st, npad, h->world, rs_rc);
      }
    }
    if (pair && !col_blocks) {
      // (the column-block copies could not be built: the 8-wide row-kernel fit instead, at the
      // keep / basis the general rule would have given -- rerun the setup without the pair mode)
      n2v2r_eig_opts o2 = o;
      o2.solver_flags |= N2V2R_EIG_PANEL8;
      return run(d_, o2, theta_out, Uout, ldu);
    }
    if (pair) {
      h->ews.x16.ensure(sizeof(float) * (size_t)npad * 16);
      hc_ld = (int64_t)(c_max + 8) * 8;
      h->ews.hcol.ensure(sizeof(double) * (size_t)nb_max * hc_ld);
      h->ews.pcab.ensure(sizeof(double) * (size_t)hc_ld);
      h->ews.pth.ensure(sizeof(double) * (size_t)keep);
      hc_lo.assign(nb_max + 2, 0);
      hc_nr.assign(nb_max + 2, 0);
    }
    split2 = split2_wanted(h, b) && !col_blocks;
    pending = nullptr;
    if (split2) h->ews.s2part.ensure(sizeof(float) * (size_t)K * npad * 8);
    // chunk partials: also the streaming Gram form at b = 8 (chunks of <= 8192 rows, rounded to
    // a multiple of 8, (c + b) x b fp64 each) and the paired full passes' two-block Gram
    // (2 (c + 2b) x b per chunk; round 6: sized for one block's, the pair fell back to two
    // separate full passes past ~48 basis blocks at N = 10M -- 2 x 3.7 ms instead of one read)
    h->partial_elems = std::max<size_t>(4096ull * 1024ull, (size_t)c_max * c_max * 8);
    h->partial_elems = std::max<size_t>(h->partial_elems,
                                        (size_t)((n + 8191) / 8192 + 24) * 2 * (c_max + 2 * b) * b);
    h->partial.ensure(sizeof(double) * h->partial_elems);
    h->ews.gsmall.ensure(sizeof(double) * (size_t)c_max * c_max);
    h->ews.csmall.ensure(sizeof(float) * (size_t)c_max * c_max);
    h->ews.tri.ensure(sizeof(double) * 3 * (size_t)c_max);
    h->ews.refl.ensure(sizeof(double) * std::max<size_t>((size_t)c_max * c_max,
                                                        (size_t)c_max * (c_max / 8 + 2) * 9));
    h->ews.ytri.ensure(sizeof(double) * (size_t)c_max * keep);
    h->ews.tscr.ensure(sizeof(double) * 6 * (size_t)((keep + 63) / 64 * 64) * c_max);
    h->ews.trcoop.ensure(n2v2r_rr_tridiag_scratch_bytes(c_max));
    h->ews.btf.ensure(n2v2r_rr_bt_scratch_bytes(c_max));
    h->ews.rinv.ensure(sizeof(double) * 64 * 64);
    h->ews.fcoef.ensure(sizeof(float) * (size_t)(c_max + 64) * 64);
    h->ews.flg.ensure(sizeof(int) * 256);
    h->ews.anyflag.ensure(sizeof(int) * 4);
    h->theta.ensure(sizeof(double) * c_max);
    h->resid.ensure(sizeof(double) * c_max);
    // (kept sets past the reducing path's 192-row arrow, and bases past its 640 columns, take
    // the banded form only with the Sturm one, whose failure falls back to the dense
    // Rayleigh-Ritz on H expanded from the band)
    band_reduce = keep + 8 <= 192 && c_max <= kReduceMaxc;
    band_rr = !pair && b == 8 && !(o.solver_flags & N2V2R_EIG_DENSE_RR) &&
              c_max <= N2V2R_BAND_MAXC && (band_reduce || rr_sturm_enabled());
    if (band_rr) {
      h->ews.hband.ensure(sizeof(double) * ((size_t)(keep + b) * b + (size_t)nb_max * 2 * b * b));
      h->ews.band.ensure(sizeof(double) * (size_t)c_max * (b + 1));
      h->ews.varr.ensure(sizeof(double) * (size_t)(keep + b) * (keep + b));
      h->ews.taua.ensure(sizeof(double) * (size_t)(keep + b));
      h->ews.rrerr.ensure(sizeof(int) * 4);
      h->ews.sturm.ensure(sizeof(double) * n2v2r_rr_sturm_scratch(c_max, keep));
    }
    const bool sturm = band_rr && rr_sturm_enabled();
    part_p = h->partial.as<double>();
    part_n = h->partial_elems;
    gsm_p = h->ews.gsmall.as<double>();
    flg_p = h->ews.flg.as<int>();
    any_p = h->ews.anyflag.as<int>();
    // Lean images on a partitioned handle too: every quantity they read back (R of the restart
    // projection, the Ritz values and coefficients, the true residuals) is all-reduced first,
    // so every rank takes the same decisions.
    const bool lean =
        pair || (b == 8 && pip_fused() && band_rr && sturm && !lean_off && lean_enabled());
    {
      // default: a tenth of the residual tolerance.  The residuals stall near the level of
      // orthogonality left in the basis (~1.5x it in cfg2 sweeps: 2e-6 stalls at 3e-6); at
      // 1e-7 .. 2.5e-7 cfg2 keeps its residuals and gains alike (most passes then touch only the
      // few blocks, the kept Ritz vectors, that lost orthogonality).  N2V2R_REORTH_TOL=0: every
      // block of every full pass.
      const char* e = std::getenv("N2V2R_REORTH_TOL");
      // capped at 1e-6: a loose residual tolerance must not loosen the basis orthogonality the
      // Rayleigh-Ritz and the lean residual estimates assume
      reorth_tol = e ? (float)std::atof(e) : (float)std::min(0.1 * tol, 1e-6);
      // (the pass-level form -- all blocks or none -- gained less at the same threshold, 37.8 vs
      // 36.5 ms per cfg2 fit; its switch N2V2R_REORTH_MODE was retired in round 6)
    }
    {
      const char* e = std::getenv("N2V2R_REORTH_DEFER");  // read per fit (A/B runs)
      // lean images only: with every image kept, the Rayleigh-Ritz and the residuals read the
      // images themselves, and a deferred block's image is the uncorrected block's
      defer = !(e && e[0] == '0') && b == 8 && pip_fused() && lean;
      deferred = nullptr;
      pair_gram = true;  // (the A/B switch of the pairing retired in round 5)
      if (defer) {
        h->ews.g2.ensure(sizeof(double) * 2 * (size_t)(nb_max + 2) * 64, st);
        // R of the pair's first pass: the identity until a pass writes it
        static const double eye[64] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0,
                                       0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0,
                                       0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0,
                                       0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1};
        h->ews.pair_ra.ensure(sizeof(double) * 64, st);
        HIPCHK(hipMemcpyAsync(h->ews.pair_ra.p, eye, sizeof(eye), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
      }
    }
    h->ews.skipc.ensure(sizeof(int) * (4 + N2V2R_BAND_MAXC / 8));  // [0]: skipped, [1 + blk]
    HIPCHK(hipMemsetAsync(h->ews.skipc.p, 0, sizeof(int) * (4 + N2V2R_BAND_MAXC / 8), st));
    // R of the restart block's two passes (pair: [0, 128) the a block's, [128, 256) the b's)
    if (lean) h->ews.rres.ensure(sizeof(double) * (pair ? 256 : 128));
    double est_scale = 1.0;  // lean: true / estimated residual seen at a failed final check
    double last_true = 1e300;  // lean: the worst true residual of the previous check
    bool rr_armed = false;   // the Rayleigh-Ritz error words zeroed (then by every read-back)
    int lean_checks = 0;
    // pinned read-back per cycle: residuals, Ritz values (keep each), flags, R (8 x 8), S's last
    // rows (pair: the restart pair's R_aa, R_bb and coupling E_a^T W_b, 3 x 8 x 8, and S's last
    // 16 rows)
    const int nrr = pair ? 192 : 64, nsl = pair ? 16 : 8;
    const size_t pin_bytes = sizeof(double) * 2 * (size_t)keep + 8 * sizeof(int) +
                             sizeof(double) * nrr + sizeof(float) * nsl * (size_t)keep;

    h->ews.dbgflag.ensure(sizeof(int) * 4);
    h->ews.tflag.ensure(sizeof(double) * 2);
    poison_scratch();
    std::vector<double> wh(keep);
    std::vector<double> res2(keep);

    // start block (counter-based: the same values whatever the row partition)
    float* q0 = take();
    HIPCHK(n2v2r_launch_fill_normal(q0, b, n, seed, nullptr, nullptr, (uint64_t)row0 * b, st));
    Q.assign(1, q0);
    orthonormalize(q0, {});
    dbg(q0, n * b, false, "orthonormalised start block");
    if (pair) {
      // the start pair: a second block of deviates from another counter stream
      float* q1 = take();
      HIPCHK(n2v2r_launch_fill_normal(q1, b, n, seed ^ 0x9E3779B97F4A7C15ull, nullptr, nullptr,
                                      (uint64_t)row0 * b, st));
      orthonormalize(q1, Q);
      Q.push_back(q1);
      W.assign(1, take());
      W.push_back(take());
      apply_M_pair(Q[0], Q[1], W[0], W[1]);
    } else {
      W.assign(1, take());
      apply_M(Q[0], W[0]);
    }
    if (debug_finite()) materialize();
    dbg(W[0], n * b, false, "SpMM image of the start block");
    if ((o.solver_flags & N2V2R_EIG_TEST_FAIL_ALONE) && h->comm && h->rank == 1)
      throw StatusFail{N2V2R_ERR_INTERNAL, "test: rank 1 fails alone"};
    int apps = pair ? 2 : 1;
    int cycle = 0;
    double maxres = 0;
    int conv = 0;
    std::vector<float*> X(pb), MX(pb);
    std::vector<double> hist_res;
    int stagnated = 0;
    const double t_start = now_ms();
    static const bool trace = [] {  // N2V2R_TRACE=1: one stderr line per Rayleigh-Ritz cycle
      const char* e = std::getenv("N2V2R_TRACE");
      return e && *e && *e != '0';
    }();
    double t_rr = 0;
    for (;; ++cycle) {
      dbg_cycle = cycle;
      y_captured = false;
      const int q_start = (int)Q.size();
      // (cycle 0: armed here; later cycles: the previous cycle's read-back zeroed it)
      if (lazy && cycle == 0) HIPCHK(hipMemsetAsync(h->ews.anyflag.as<int>() + 3, 0, sizeof(int), st));
      while ((int)Q.size() < nb_max) {
        if (pair) {
          expand_pair(W[W.size() - 2], W.back(), Q, W, lazy);
          apps += 2;
          for (int i = (int)W.size() - 4; lean && i < (int)W.size() - 2; ++i)
            if (i >= q_start) {  // consumed; the cycle's input pair stays
              give(W[i]);
              W[i] = nullptr;
            }
          continue;
        }
        expand_one(W.back(), Q, Q, W, /*save_band=*/true, lazy);
        ++apps;
        if (lean && (int)W.size() - 2 > q_start - 1) {  // consumed; the cycle's input stays
          give(W[W.size() - 2]);
          W[W.size() - 2] = nullptr;
        }
      }
      flush_deferred(Q);  // (deferred full passes) the cycle's last block
      const int nq = (int)Q.size();
      const int c = nq * b;
      for (int q = 0; q < pb; ++q) {
        X[q] = take();
        MX[q] = lean ? nullptr : take();
      }
      float* E_lean = nullptr;  // lean: the restart block, built before the convergence test
      bool dense_rr = !band_rr;
      bool band_expand = false;  // dense Rayleigh-Ritz on H expanded from the band (fallback)
      bool sturm_now = sturm;  // this cycle's banded form (the reducing one after a failure)
      int rr_err = 0;
      bool th_saved = false;  // pair: the kept Ritz values copied for this cycle's assembly
      float* E_lean2 = nullptr;  // pair: the restart pair's second block
      double th_sync0 = 0, tr0_c = 0;  // host clock (N2V2R_TRACE)
    rayleigh_ritz:
      {
      // Rayleigh-Ritz, all on the GPU, into the fp32 Ritz coefficients S (c x keep, ld keep)
      // and theta (kept in HBM until the residual read-back below).
      //   banded: the band columns saved by the expansions (+ the last block's, computed
      //     here) -> arrow reduction + bulge chasing -> bisection -> band inverse iteration;
      //   dense: H = Q^T W (fp64, all-reduced) -> Householder tridiagonal -> bisection +
      //     inverse iteration on T -> compact-WY back-transform.
      double* trid = h->ews.tri.as<double>();
      materialize();  // W.back() (every other W block was stored by its expansion's Gram pass)
      const double tr0 = now_ms();
      tr0_c = tr0;
      lds_poison();
      if (!dense_rr) {
        const std::vector<float*> loc = local_of(Q);
        tn(blocks(loc, 0, (int)loc.size()), one(W.back()),
           h->ews.hband.as<double>() + band_off(nq - 1), nullptr);
        if (!rr_armed) HIPCHK(hipMemsetAsync(h->ews.rrerr.as<int>(), 0, 4 * sizeof(int), st));
        rr_armed = true;  // from here on each read-back zeroes the words it reads
        lds_poison();
        if (sturm_now) {
          HIPCHK(n2v2r_launch_rr_sturm(h->ews.hband.as<double>(), c, kry0 * b,
                                       h->theta.as<double>(), h->ews.sturm.as<double>(),
                                       h->ews.sturm.bytes / sizeof(double),
                                       h->ews.ytri.as<double>(), h->ews.csmall.as<float>(), keep,
                                       keep, h->ews.rrerr.as<int>(), st));
        } else {
          HIPCHK(n2v2r_launch_rr_band(h->ews.hband.as<double>(), c, kry0 * b, h->theta.as<double>(),
                                      h->ews.band.as<double>(), h->ews.varr.as<double>(),
                                      h->ews.taua.as<double>(), trid, trid + c_max,
                                      h->ews.refl.as<double>(), h->ews.ytri.as<double>(),
                                      h->ews.csmall.as<float>(), keep, keep,
                                      h->ews.rrerr.as<int>(), st));
        }
      } else {
        if (pair) {
          // the last pair's band columns (its images against their coupling blocks), then H
          // assembled from every saved column of this cycle and the kept Ritz values
          const int p = nq - 2, lo = pair_lo(p);
          const std::vector<float*> La(Q.begin() + lo, Q.end());
          for (int t = 0; t < 2; ++t) {
            tn(blocks(La, 0, (int)La.size()), one(W[p + t]), hcol_at(p + t), nullptr);
            hc_lo[p + t] = lo;
            hc_nr[p + t] = (int)La.size() * 8;
          }
          // (the kept Ritz values copied once per cycle: a redone Rayleigh-Ritz -- a timed-out
          // tridiagonalisation -- finds h->theta overwritten)
          if (!th_saved && kry0 > 0)
            HIPCHK(hipMemcpyAsync(h->ews.pth.p, h->theta.p, sizeof(double) * kry0 * b,
                                  hipMemcpyDeviceToDevice, st));
          th_saved = true;
          double* Hd = h->ews.gsmall.as<double>();
          HIPCHK(hipMemsetAsync(Hd, 0, sizeof(double) * (size_t)c * c, st));
          HIPCHK(n2v2r_launch_pair_h_assemble(h->ews.hcol.as<double>(), hc_ld, hc_lo.data() + kry0,
                                              hc_nr.data() + kry0, kry0, nq - kry0, kry0 * b,
                                              h->ews.pth.as<double>(), Hd, c, st));
        } else if (band_expand) {
          HIPCHK(n2v2r_launch_rr_band_expand(h->ews.hband.as<double>(), c, kry0 * b,
                                             h->theta.as<double>(), h->ews.gsmall.as<double>(), st));
        } else {
          tn(blocks(Q, 0, nq), blocks(W, 0, nq), h->ews.gsmall.as<double>(), nullptr);
        }
        dbg(h->ews.gsmall.p, (int64_t)c * c, true, "projected matrix H = Q^T W");
        lds_poison();
        // ranks that share this device (thread group): their concurrent launches of the
        // multi-workgroup form could not all be resident, so they keep the one-workgroup kernel;
        // so does a fit whose multi-workgroup launch once timed out (tri_err below)
        const bool shared_device = h->comm && h->comm->shares_device();
        const bool coop = !shared_device && !tri_single;
        tri_err = coop ? n2v2r_rr_tridiag_err(h->ews.trcoop.p, c) : nullptr;
        HIPCHK(n2v2r_launch_rr_tridiag(h->ews.gsmall.as<double>(), c, trid, trid + c_max,
                                       trid + 2 * c_max, h->ews.refl.as<double>(),
                                       coop ? h->ews.trcoop.p : nullptr, st));
        dbg(trid, c, true, "tridiagonal diagonal");
        dbg(trid + c_max, c - 1, true, "tridiagonal off-diagonal");
        lds_poison();
        HIPCHK(n2v2r_launch_rr_tri_eig(trid, trid + c_max, c, keep, h->theta.as<double>(),
                                       h->ews.ytri.as<double>(), h->ews.tscr.as<double>(), st));
        dbg(h->theta.p, keep, true, "tridiagonal eigenvalues (bisection)");
        dbg(h->ews.ytri.p, (int64_t)c * keep, true, "tridiagonal eigenvectors");
        lds_poison();
        HIPCHK(n2v2r_launch_rr_backtransform(h->ews.refl.as<double>(), trid + 2 * c_max, c,
                                             h->ews.ytri.as<double>(), keep,
                                             h->ews.csmall.as<float>(), keep,
                                             h->ews.btf.as<double>(), st));
      }
      dbg(h->theta.p, keep, true, "Ritz values");
      dbg(h->ews.csmall.p, (int64_t)c * keep, false, "Ritz coefficients S");
      t_rr += now_ms() - tr0;
      }
      // Ritz vectors X = Q S, MX = W S (keep columns, pb blocks)
      const double to0 = now_ms();
      lds_poison();
      const int per_launch = std::max(1, 128 / b);  // output blocks per ts_nn launch (<= 128 cols)
      bool ritz_done = false;
      if (b == 8 && keep <= 96 && ritz_nn_enabled()) {
        // both products in one launch, the coefficients staged once per CU
        OutBlockList ox{}, omx{};
        ox.width = omx.width = b;
        ox.count = omx.count = pb;
        for (int t = 0; t < pb; ++t) {
          ox.blk[t] = X[t];
          omx.blk[t] = MX[t];
        }
        if (lean) omx.count = 0;  // X only
        const hipError_t e = n2v2r_launch_ritz_nn(blocks(Q, 0, nq), lean ? one(nullptr) : blocks(W, 0, nq),
                                                  h->ews.csmall.as<float>(), keep, keep, ox, omx,
                                                  n, 0, st);
        if (e == hipSuccess) ritz_done = true;
        else if (e != hipErrorNotSupported) throw HipFail{e, "n2v2r_launch_ritz_nn"};
      }
      for (int q0b = 0; !ritz_done && q0b < pb; q0b += per_launch) {
        const int nt = std::min(per_launch, pb - q0b);
        OutBlockList ox{}, omx{};
        ox.width = omx.width = b;
        ox.count = omx.count = nt;
        for (int t = 0; t < nt; ++t) {
          ox.blk[t] = X[q0b + t];
          omx.blk[t] = MX[q0b + t];
        }
        // G slice: columns [q0b*b, q0b*b + nt*b) of S (ld = keep)
        const float* g = h->ews.csmall.as<float>() + q0b * b;
        HIPCHK(n2v2r_launch_ts_nn(blocks(Q, 0, nq), g, keep, nt * b, ox, one(nullptr), 1.f, 0.f, n,
                                  nullptr, nullptr, 0, st));
        if (!lean)
          HIPCHK(n2v2r_launch_ts_nn(blocks(W, 0, nq), g, keep, nt * b, omx, one(nullptr), 1.f, 0.f,
                                    n, nullptr, nullptr, 0, st));
      }
      for (int q = 0; q < pb; ++q) {
        dbg(X[q], n * b, false, "Ritz vectors X = Q S");
        if (!lean) dbg(MX[q], n * b, false, "Ritz images MX = W S");
      }
      if (lean) {
        // the restart block now (it needs nothing from the Rayleigh-Ritz stage): its first,
        // local pass leaves R with W_last - Q_loc C = Z_{m+1} R, Z_{m+1} orthonormal.  Built
        // once per cycle: a Rayleigh-Ritz fallback (goto rayleigh_ritz) reuses it and R.
        if (!E_lean && pair) {
          // the restart pair: E_a from the last pair's first image, E_b from its second against
          // the basis and E_a.  [W_a W_b] - Q C = [E_a E_b] [[R_aa, c_ab], [0, R_bb]] with
          // c_ab = E_a^T W_b: E_b's first pass's Gram rows of E_a (pcab)
          const int p = nq - 2;
          const std::vector<float*> La(Q.begin() + pair_lo(p), Q.end());
          E_lean = take();
          orthonormalize(E_lean, Q, W[p], &La, nullptr, false, h->ews.rres.as<double>());
          std::vector<float*> qe(Q), Le(La);
          qe.push_back(E_lean);
          Le.push_back(E_lean);
          E_lean2 = take();
          orthonormalize(E_lean2, qe, W[p + 1], &Le, h->ews.pcab.as<double>(), false,
                         h->ews.rres.as<double>() + 128);
          pcab_blk = (int)Le.size() - 1;  // (where E_a's rows sit in pcab)
        } else if (!E_lean) {
          E_lean = take();
          const std::vector<float*> loc = local_of(Q);
          orthonormalize(E_lean, Q, W.back(), &loc, nullptr, false, h->ews.rres.as<double>());
        }
      } else {
        HIPCHK(n2v2r_launch_resid(blocks(X, 0, pb), blocks(MX, 0, pb), h->theta.as<double>(), n,
                                  h->partial.as<double>(), h->partial_elems,
                                  h->resid.as<double>(), st));
        h->allreduce_f64(h->resid.as<double>(), keep);
      }
      h->ensure_pin(pin_bytes);
      double* pres = static_cast<double*>(h->pin);
      double* pth = pres + keep;
      int* pflag = reinterpret_cast<int*>(pth + keep);
      double* prr = reinterpret_cast<double*>(pflag + 8);   // lean: R (8 x 8; pair 3 x 8 x 8)
      float* psl = reinterpret_cast<float*>(prr + nrr);     // lean: last 8 (16) rows of S
      {
        // one pack launch + one copy: [pres | pth | pflag[8] | prr | psl] (the layout above)
        h->ews.rback.ensure(pin_bytes);
        const int wres = 0, wth = 2 * keep, wflag = 4 * keep, wrr = wflag + 8,
                  wsl = wrr + 2 * nrr;
        void* src[12];
        int dw[12], nw[12], clr[12], ns = 0;
        auto seg = [&](void* sp, int d0, int n0, int cl = 0) {
          src[ns] = sp;
          dw[ns] = d0;
          nw[ns] = n0;
          clr[ns] = cl;
          ++ns;
        };
        if (lean && pair) {
          seg(h->ews.rres.p, wrr, 128);                                 // R_aa
          seg(h->ews.rres.as<double>() + 128, wrr + 128, 128);          // R_bb
          seg(h->ews.pcab.as<double>() + (size_t)pcab_blk * 64, wrr + 256, 128);
          seg(h->ews.csmall.as<float>() + (size_t)(c - 16) * keep, wsl, 16 * keep);
        } else if (lean) {
          seg(h->ews.rres.p, wrr, 128);
          seg(h->ews.csmall.as<float>() + (size_t)(c - b) * keep, wsl, 8 * keep);
        } else {
          seg(h->resid.p, wres, 2 * keep);
        }
        seg(h->theta.p, wth, 2 * keep);
        seg(nullptr, wflag, 1);  // pflag[0]
        // the sticky refill flag and the Rayleigh-Ritz error words are zeroed as they are read:
        // they are armed for the next cycle (or a fallback Rayleigh-Ritz) without a memset
        if (lazy) seg(h->ews.anyflag.as<int>() + 3, wflag + 1, 1, 1);
        else seg(nullptr, wflag + 1, 1);
        if (!dense_rr) seg(h->ews.rrerr.p, wflag + 2, 2, 1);
        else seg(nullptr, wflag + 2, 2);
        seg(dense_rr ? tri_err : nullptr, wflag + 4, 1);  // pflag[4]
        HIPCHK(n2v2r_launch_pack_words(src, dw, nw, clr, ns, h->ews.rback.p, st));
        const size_t upto = lean ? pin_bytes : sizeof(int) * (size_t)(wflag + 8);
        HIPCHK(hipMemcpyAsync(h->pin, h->ews.rback.p, upto, hipMemcpyDeviceToHost, st));
      }
      th_sync0 = now_ms();
      HIPCHK(hipStreamSynchronize(st));
      if (trace)
        fprintf(stderr, "[n2v2r] cycle %d host: rr start %.3f, to sync %.3f, sync %.3f ms\n",
                cycle, tr0_c - t_start, th_sync0 - tr0_c, now_ms() - th_sync0);
      if (lean && pair) {
        // ||M x_j - theta_j x_j|| = ||R16 s_j(last pair)||, R16 = [[R_aa, c_ab], [0, R_bb]]
        double R16[16][16] = {};
        for (int r = 0; r < 8; ++r)
          for (int q = 0; q < 8; ++q) {
            R16[r][q] = prr[r * 8 + q];
            R16[r][8 + q] = prr[128 + r * 8 + q];
            R16[8 + r][8 + q] = prr[64 + r * 8 + q];
          }
        for (int j = 0; j < keep; ++j) {
          double acc = 0.0;
          for (int r = 0; r < 16; ++r) {
            double v = 0.0;
            for (int cc = r; cc < 16; ++cc) v += R16[r][cc] * (double)psl[cc * keep + j];
            acc += v * v;
          }
          res2[j] = acc * est_scale * est_scale;
        }
      } else if (lean) {  // ||M x_j - theta_j x_j||^2 = ||R s_j(last block)||^2 (Krylov-Schur), scaled
        for (int j = 0; j < keep; ++j) {
          double acc = 0.0;
          for (int r = 0; r < 8; ++r) {
            double v = 0.0;
            for (int cc = r; cc < 8; ++cc) v += prr[r * 8 + cc] * (double)psl[cc * keep + j];
            acc += v * v;
          }
          res2[j] = acc * est_scale * est_scale;
        }
      } else {
        std::copy(pres, pres + keep, res2.begin());
      }
      std::copy(pth, pth + keep, wh.begin());
      if (!dense_rr) rr_err = (test_band_fail || (test_sturm_fail && sturm_now)) ? 1 : pflag[2];
      if (trace && !dense_rr && sturm_now)
        fprintf(stderr, "[n2v2r] cycle %d: %d of %d Ritz vectors took a second solve\n", cycle,
                pflag[3], keep);
      int refilled = lazy ? pflag[1] : 0;
      t_ortho += now_ms() - to0;
      if (dense_rr && h->comm) {
        // each rank read its own device's error word: agree on it (max over ranks) before
        // branching, so every rank redoes the step together (a rank that alone went back to
        // rayleigh_ritz would run one more all-reduce of H than its peers)
        double* fl = h->ews.tflag.as<double>();
        const double mine = pflag[4] ? 1.0 : 0.0;
        HIPCHK(hipMemcpyAsync(fl, &mine, sizeof(double), hipMemcpyHostToDevice, st));
        h->allreduce_f64(fl, 1);
        double any_to = 0.0;
        HIPCHK(hipMemcpyAsync(&any_to, fl, sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        pflag[4] = any_to > 0.0 ? 1 : 0;
      }
      if (dense_rr && pflag[4]) {
        // the multi-workgroup tridiagonalisation's grid barrier timed out (a workgroup was not
        // resident): its output is invalid; this cycle's Rayleigh-Ritz again, and every later
        // one, with the one-workgroup kernel
        fprintf(stderr, "[n2v2r] multi-workgroup tridiagonalisation timed out at cycle %d (c %d); "
                        "one-workgroup kernel from here on\n", cycle, c);
        tri_single = true;
        ++tri_fallbacks;
        goto rayleigh_ritz;
      }
      if (rr_err && !dense_rr && sturm_now) {  // a Sturm vector failed its residual check
        if (trace) fprintf(stderr, "[n2v2r] Sturm Rayleigh-Ritz failed, reducing fallback\n");
        // the kept Ritz values the reducing path reads: the copy the Sturm assembly made
        if (kry0 > 0)
          HIPCHK(hipMemcpyAsync(h->theta.as<double>(), h->ews.sturm.as<double>() + 4,
                                sizeof(double) * kry0 * b, hipMemcpyDeviceToDevice, st));
        sturm_now = false;
        if (!band_reduce) {  // past the reducing path's arrow: dense, from the band
          dense_rr = true;
          band_expand = true;
        }
        rr_err = 0;
        ++stats_rr_fallbacks;
        goto rayleigh_ritz;
      }
      if (rr_err && !dense_rr && lean) throw LeanRetry{};  // dense H needs every image
      if (rr_err && !dense_rr) {  // the bulge chase gave up (should not happen): dense RR
        if (trace) fprintf(stderr, "[n2v2r] banded Rayleigh-Ritz failed, dense fallback\n");
        dense_rr = true;
        rr_err = 0;
        goto rayleigh_ritz;
      }
      if (test_redo && cycle == 0 && lazy) refilled = 1;  // tests: exercise the recovery
      // a non-finite Ritz pair under the lazy (two-pass) orthogonalisation: diagnostic
      // fallback only (no known cause remains; N2V2R_DEBUG_FINITE=1 names the first stage that
      // produces one).  Always reported on stderr, then the cycle's expansion is redone with
      // three passes from the kept (finite) basis before giving up below.
      if (lazy && !refilled)
        for (int j = 0; j < keep; ++j)
          if (!std::isfinite(wh[j]) || (j < d && !std::isfinite(res2[j]))) {
            fprintf(stderr,
                    "[n2v2r] WARNING: non-finite Ritz pair %d at cycle %d (c %d, b %d, %s "
                    "Rayleigh-Ritz); cycle expanded again with three passes.  Rerun with "
                    "N2V2R_DEBUG_FINITE=1 to locate the stage.\n",
                    j, cycle, c, b, dense_rr ? "dense" : "banded");
            refilled = 1;
            break;
          }
      if (refilled) {  // a second pass refilled a column: expand this cycle again, 3 passes
        if (trace) fprintf(stderr, "[n2v2r] rank-deficient block, cycle %d expanded again\n", cycle);
        give(E_lean);
        give(E_lean2);
        for (int q = 0; q < pb; ++q) {
          give(X[q]);
          give(MX[q]);
        }
        for (int q = q_start; q < nq; ++q) {
          give(Q[q]);
          give(W[q]);
        }
        apps -= nq - q_start;
        Q.resize(q_start);
        W.resize(q_start);
        lazy = false;
        --cycle;
        continue;
      }
      for (int j = 0; j < keep; ++j)  // a non-finite Ritz pair cannot recover: stop with details
        if (!std::isfinite(wh[j]) || (j < d && !std::isfinite(res2[j])))
          throw StatusFail{N2V2R_ERR_NO_CONVERGENCE,
                           "non-finite Ritz pair " + std::to_string(j) + " at cycle " +
                               std::to_string(cycle) + " (c " + std::to_string(c) + ", b " +
                               std::to_string(b) + (dense_rr ? ", dense" : ", banded") +
                               " Rayleigh-Ritz, theta " + std::to_string(wh[j]) + ")"};
      maxres = 0;
      conv = 0;
      const double th1 = std::max(wh[0], 1e-300);
      for (int j = 0; j < d; ++j) {
        const double r = std::sqrt(std::max(res2[j], 0.0)) / th1;
        maxres = std::max(maxres, r);
        if (r <= tol) ++conv;
      }
      if (trace)
        fprintf(stderr, "[n2v2r] rank %d cycle %d apps %d c %d max_res %.3e converged %d/%d %.1f ms\n",
                h->rank, cycle, apps, c, maxres, conv, d, now_ms() - t_start);
      bool done = (conv == d || cycle + 1 >= max_restarts);
      if (!done) {
        // fp32 noise floor: the true residual of W = M Q cannot fall below ~eps32 *
        // sqrt(nnz/row) * theta_1.  Stop when the best worst-residual of the last 8 cycles is
        // not 10% below the best one before them (slow but steady convergence on clustered
        // spectra keeps going) and it is within 100x of tol.
        hist_res.push_back(maxres);
        const size_t W8 = 8;
        if (hist_res.size() >= 2 * W8) {
          const double recent = *std::min_element(hist_res.end() - W8, hist_res.end());
          const double before = *std::min_element(hist_res.begin(), hist_res.end() - W8);
          if (!no_stagnation && recent > 0.9 * before && recent <= 100.0 * tol) {
            stagnated = 1;
            done = true;
          }
        }
      }
      if (lean && done) {
        // lean images: the estimates say stop; the true residuals of the d wanted vectors
        // (their images by SpMM) decide
        ++lean_checks;
        const int qd = (d + b - 1) / b;
        std::vector<float*> MV(qd);
        // one GPU, tiled SpMM, every column of the embedding covered: keep the stage-1 products
        // (N2V2R_YCAP=0, read per fit: the embedding step computes its SpMM launches; A/B, tests)
        const char* ycv = std::getenv("N2V2R_YCAP");
        const bool cap = col_blocks && !h->comm && b == 8 && qd * b == ldu &&
                         !(ycv && ycv[0] == '0');
        if (cap) h->Y.ensure(sizeof(float) * (size_t)K * npad * ldu, st);
        for (int q = 0; q < qd; ++q) {
          MV[q] = take();
          // (pair: two vector blocks per application, their stage-1 products N x 16)
          const int w = (pair && q + 1 < qd) ? 2 : 1;
          if (w == 2) {
            MV[q + 1] = take();
            apply_M_pair(X[q], X[q + 1], MV[q], MV[q + 1]);
          } else {
            apply_M(X[q], MV[q]);
          }
          materialize();
          if (cap)
            for (int k = 0; k < K; ++k)
              HIPCHK(hipMemcpy2DAsync(h->Y.as<float>() + (size_t)k * npad * ldu + (size_t)q * b,
                                      sizeof(float) * ldu, h->ews.zk[k]->as<float>(),
                                      sizeof(float) * b * w, sizeof(float) * b * w, n,
                                      hipMemcpyDeviceToDevice, st));
          q += w - 1;
        }
        y_captured = cap;
        HIPCHK(n2v2r_launch_resid(blocks(X, 0, qd), blocks(MV, 0, qd), h->theta.as<double>(), n,
                                  h->partial.as<double>(), h->partial_elems,
                                  h->resid.as<double>(), st));
        h->allreduce_f64(h->resid.as<double>(), (size_t)qd * b);
        HIPCHK(hipMemcpyAsync(pres, h->resid.as<double>(), sizeof(double) * qd * b,
                              hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (float* p : MV) give(p);
        double worst = 0.0, est_max = 0.0;
        int tconv = 0;
        for (int j = 0; j < d; ++j) {
          const double r = std::sqrt(std::max(pres[j], 0.0)) / th1;
          const double e = std::sqrt(std::max(res2[j], 0.0)) / th1;
          worst = std::max(worst, r);
          est_max = std::max(est_max, e);
          if (r <= tol) ++tconv;
        }
        // the scale that brings the worst estimate to the worst true residual (a ratio taken
        // vector by vector blew up on estimates at the fp32 noise level: 1e-12 against a true
        // 1e-7 gave a scale of 1e5, and the scaled estimates never came back below tol)
        const double ratio = est_max > 0.0 ? worst / est_max : 0.0;
        if (trace)
          fprintf(stderr, "[n2v2r] cycle %d: true max_res %.3e converged %d/%d (estimate %.3e)\n",
                  cycle, worst, tconv, d, maxres);
        maxres = worst;
        conv = tconv;
        stagnated = 0;
        if (conv < d && cycle + 1 < max_restarts) {
          // at the fp32 floor the true residual stops falling: finish within 100x tol once a
          // check shows no 10 % gain over the previous one (or after 4 checks)
          const bool flat = lean_checks >= 2 && worst > 0.9 * last_true;
          if (!no_stagnation && (flat || lean_checks >= 4) && worst <= 100.0 * tol) {
            stagnated = 1;
          } else {
            done = false;
            // the estimates (already scaled) trail the true residual by `ratio`: rescale from
            // this check (it may also shrink back towards 1 after a pessimistic one), at most
            // by 1e3 in all
            if (ratio > 0.0) est_scale = std::min(1e3, std::max(1.0, est_scale * 1.25 * ratio));
            hist_res.clear();
          }
        }
        last_true = worst;
      }
      if (done) {
        give(E_lean);
        give(E_lean2);
        break;
      }
      // restart: [X | orth(W_last) against the old basis] (thick restart)
      std::vector<float*> E, EW;
      if (lean && pair) {
        E.push_back(E_lean);
        E.push_back(E_lean2);
        EW.push_back(take());
        EW.push_back(take());
        apply_M_pair(E_lean, E_lean2, EW[0], EW[1]);
        ++apps;
      } else if (lean) {
        E.push_back(E_lean);
        EW.push_back(take());
        apply_M(E_lean, EW[0]);
      } else {
        expand_one(W.back(), Q, E, EW);
      }
      ++apps;
      for (float* p : Q) give(p);
      for (float* p : W) give(p);
      Q.assign(X.begin(), X.end());
      W.assign(MX.begin(), MX.end());
      Q.insert(Q.end(), E.begin(), E.end());
      W.insert(W.end(), EW.begin(), EW.end());
      kry0 = pb;
    }
    materialize();
    if (trace && reorth_tol != 0.f) {
      int sk[65] = {};
      HIPCHK(hipMemcpyAsync(sk, h->ews.skipc.p, sizeof(int) * 65, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      fprintf(stderr, "[n2v2r] %d full reorthogonalisation passes skipped (tol %.1e); applied "
              "per basis block:", sk[0], (double)reorth_tol);
      for (int q = 0; q < 64; ++q) fprintf(stderr, " %d", sk[1 + q]);
      fprintf(stderr, "\n");
    }
    // U = first d columns of X (row stride ldu); theta
    theta_out.assign(wh.begin(), wh.begin() + d);
    for (int q = 0; q * b < d; ++q) {
      const int cols = std::min(b, d - q * b);
      HIPCHK(hipMemcpy2DAsync(Uout + q * b, sizeof(float) * ldu, X[q], sizeof(float) * b,
                              sizeof(float) * cols, npad, hipMemcpyDeviceToDevice, st));
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
      stats->rr_fallbacks = stats_rr_fallbacks;
      stats->est_scale = est_scale;
      stats->lean_checks = lean_checks;
      stats->pool_blocks = (int)h->ews.pool.size();
      stats->spmm_form = h->dense_layers() ? 4 : col_blocks ? 5 : split2 ? 1 : 0;
      stats->stag_cap = stag_cap;
      stats->y_captured = y_captured ? 1 : 0;
      stats->tri_fallbacks = tri_fallbacks;
      stats->panel = pair ? 16 : b;
      tsum(stats);
    }
    return (conv == d || (stagnated && maxres <= stag_cap)) ? N2V2R_OK : N2V2R_ERR_NO_CONVERGENCE;
  }
};

bool col_blocks_wanted(const n2v2r_handle* h, int b) {
  if (b != 8 || h->dense_layers() || h->layers.empty()) return false;
  const char* e = std::getenv("N2V2R_SPMM_CB");
  if (e && e[0] == '1') return true;
  if (e && e[0] == '0') return false;
  // measured (tools/cb_probe.py, one layer, HIP events): row kernel / column blocks =
  // 0.56 at a 3.2 MB panel (N = 100k: the panel already fits one L2), 1.35 at 9.6 MB,
  // 1.61 at 32 MB, 1.16 at 96 MB, 0.93 at 320 MB (beyond the Infinity Cache the gathers go
  // to HBM either way and the partials only add traffic)
  // round 3: the flat-window tiled form also wins beyond the Infinity Cache -- each phase
  // gathers from one panel block, which the Infinity Cache holds even when the whole panel does
  // not (cfg5 on one GPU, 320 MB panel: 9.5 vs 11.5 ms per stage launch) -- so the window has no
  // upper end
  const double panel = 4.0 * b * (double)h->n;
  return panel > 8.0e6;
}
// layer k's local rows (nloc x d, the embedding's first d of its ldy columns) to Y + k * stride
void copy_embedding(n2v2r_handle* h, float* Y, int64_t layer_stride) {
  HIPCHK(hipSetDevice(h->device));
  for (int k = 0; k < h->K; ++k)
    HIPCHK(hipMemcpy2DAsync(Y + (size_t)k * layer_stride, sizeof(float) * h->d,
                            h->Y.as<float>() + (size_t)k * h->npad * h->ldy,
                            sizeof(float) * h->ldy, sizeof(float) * h->d, h->nloc,
                            hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
}
}  // namespace n2v2r_int

extern "C" {

int n2v2r_uase(n2v2r_handle* h, int d, const n2v2r_eig_opts* opts, n2v2r_eig_stats* stats) {
  if (h && h->multi()) return multi_uase(h, d, opts, stats);
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
    // d <= 600: the kept Ritz vectors (max(d + 16, 5 d / 4)) plus one block must fit the
    // Rayleigh-Ritz kernels' 768-column basis
    if (d < 1 || d > 600 || d >= h->n) {
      h->set_err("embedding dimension %d out of range [1, min(600, n-1)]", d);
      return N2V2R_ERR_BAD_ARG;
    }
    n2v2r_eig_opts o{};
    if (opts) o = *opts;
    if (stats) memset(stats, 0, sizeof(*stats));
    // a fit that fails part-way must not leave a stale embedding (U, Y and the capture below are
    // rewritten from here on) or stale ranking results readable
    h->have_embedding = false;
    h->ncmp = h->ncols = 0;
    h->have_borda = false;
    // the ingest's radix scratch (~24 B per entry of the largest layer that needed a transpose)
    // is kept across n2v2r_set_layer_csr calls only; the fit's buffers get the HBM back
    for (DevBuf* b : {&h->ing_keys[0], &h->ing_keys[1], &h->ing_pay[0], &h->ing_pay[1],
                      &h->ing_hist})
      b->release();
    const int ldu = ((d + 63) / 64) * 64;  // a multiple of every block width
    h->U.ensure(sizeof(float) * h->npad * ldu);
    HIPCHK(hipMemsetAsync(h->U.p, 0, sizeof(float) * h->npad * ldu, h->stream));
    std::vector<double> theta;
    int st = 0, b = 0;
    // the fit's tiled column-block configuration, reused for the embedding images below
    bool ytile = false, ycap = false;
    int ytile_rows = 0, ytile_nb = 0, ytile_wb = 0;
    for (int attempt = 0;; ++attempt) {
      Eig eig{};
      eig.h = h;
      eig.st = h->stream;
      eig.n = h->nloc;
      eig.npad = h->npad;
      eig.row0 = h->row0;
      eig.K = h->K;
      eig.stats = stats;
      eig.lean_off = attempt > 0;
      try {
        st = eig.run(d, o, theta, h->U.as<float>(), ldu);
      } catch (const Eig::LeanRetry&) {
        // lean images cannot take the dense Rayleigh-Ritz fallback: the fit again with images
        fprintf(stderr, "[n2v2r] banded Rayleigh-Ritz failed under lean images; fit rerun\n");
        HIPCHK(hipStreamSynchronize(h->stream));
        continue;
      }
      b = eig.b;
      ytile = eig.col_blocks && eig.b == 8;
      ycap = ytile && eig.y_captured;
      ytile_rows = eig.tile_rows;
      ytile_wb = eig.tile_wb;
      ytile_nb = eig.tile_nb;
      break;
    }
    // deterministic signs: largest-magnitude entry of every column of U positive
    h->keys.ensure(sizeof(unsigned long long) * 1024 * (size_t)ldu);
    h->best.ensure(sizeof(unsigned long long) * ldu);
    h->colscale.ensure(sizeof(float) * ldu);
    HIPCHK(n2v2r_launch_colmax_keys(h->U.as<float>(), ldu, h->nloc, d, h->row0,
                                    h->keys.as<unsigned long long>(), 1024 * (size_t)ldu,
                                    h->best.as<unsigned long long>(), h->stream));
    if (h->comm)
      h->comm->allreduce_max_u64(h->best.as<unsigned long long>(), ldu, h->stream);
    HIPCHK(n2v2r_launch_colmax_sign(h->best.as<unsigned long long>(), ldu, h->U.as<float>(), ldu, d,
                                    h->row0, h->nloc, h->colscale.as<float>(), h->stream));
    if (h->comm)
      h->comm->allreduce_sum_f32(h->colscale.as<float>(), ldu, h->stream);
    HIPCHK(n2v2r_launch_scale_cols(h->U.as<float>(), ldu, h->npad, h->colscale.as<float>(),
                                   h->stream));
    // Y_k = A_k^T U diag(theta)^(-1/4)  (sigma = sqrt(theta); V sqrt(sigma) = A^T U sigma^-1/2)
    h->d = d;
    h->ldy = ldu;
    h->sigma.assign(d, 0.0);
    std::vector<float> sc(ldu, 0.f);
    for (int j = 0; j < d; ++j) {
      h->sigma[j] = std::sqrt(std::max(theta[j], 0.0));
      sc[j] = h->sigma[j] > 0 ? (float)(1.0 / std::sqrt(h->sigma[j])) : 0.f;
    }
    if (ycap) {
      // the captured A_k^T X come from the Ritz vectors before the sign pass: fold each column's
      // sign (+-1, exact) into its scale
      std::vector<float> sgn(ldu, 1.f);
      HIPCHK(hipMemcpyAsync(sgn.data(), h->colscale.p, sizeof(float) * ldu, hipMemcpyDeviceToHost,
                            h->stream));
      HIPCHK(hipStreamSynchronize(h->stream));
      for (int j = 0; j < d; ++j) sc[j] *= sgn[j];
    }
    HIPCHK(hipMemcpyAsync(h->colscale.p, sc.data(), sizeof(float) * ldu, hipMemcpyHostToDevice,
                          h->stream));
    const float* ug = h->U.as<float>();
    DevBuf ugath;
    if (h->comm) {
      ugath.ensure(sizeof(float) * h->world * h->npad * ldu);
      h->gather_panel(h->U.as<float>(), ugath.as<float>(), ldu);
      ug = ugath.as<float>();
    }
    h->Y.ensure(sizeof(float) * (size_t)h->K * h->npad * ldu);
    if (h->dense_layers()) {
      for (int k = 0; k < h->K; ++k) {
        const LayerDev& L = *h->layers[k];
        // one GEMM per layer over all ldu columns (ldu <= 256: 64-column slices)
        for (int q = 0; q * 64 < ldu; ++q)
          h->dense_apply(L.dense_at(), L.lda, ug + q * 64, ldu, std::min(64, ldu - q * 64),
                         h->Y.as<float>() + (size_t)k * h->npad * ldu + q * 64, ldu, 0.f,
                         h->colscale.as<float>() + q * 64);
      }
    }
    if (!h->dense_layers() && ytile) {
      // the fit's tiled SpMM (stage-1 blocks, A_k^T) on b-column slices of U copied to a
      // contiguous panel, then one column scaling of every Y_k (the row kernel below gathers
      // 32 B out of each 512-B row of U -- a 512 MB panel at cfg4 -- and scales in-kernel)
      const int64_t ng = h->comm ? (int64_t)h->world * h->npad : h->npad;
      DevBuf& panel = h->ypanel;
      panel.ensure_raw(sizeof(float) * ng * 8);
      SpmmTileArgs a{};
      a.blk = h->ews.tblk.as<CsrBlk>();
      a.ldx = 8;
      a.ldy = ldu;
      a.n = h->nloc;
      a.K = h->K;
      a.nb = ytile_nb;
      a.sum = 0;
      a.tile_rows = ytile_rows;
      a.wbits = ytile_wb;
      for (int q = 0; !ycap && q * 8 < ldu; ++q) {
        HIPCHK(hipMemcpy2DAsync(panel.p, sizeof(float) * 8, ug + q * 8, sizeof(float) * ldu,
                                sizeof(float) * 8, ng, hipMemcpyDeviceToDevice, h->stream));
        for (int k = 0; k < h->K; ++k) {
          a.X[k] = panel.as<float>();
          a.Y[k] = h->Y.as<float>() + (size_t)k * h->npad * ldu + q * 8;
        }
        HIPCHK(n2v2r_launch_spmm_tile(a, h->stream));
      }
      for (int k = 0; k < h->K; ++k)
        HIPCHK(n2v2r_launch_scale_cols(h->Y.as<float>() + (size_t)k * h->npad * ldu, ldu,
                                       h->npad, h->colscale.as<float>(), h->stream));
      HIPCHK(hipStreamSynchronize(h->stream));  // the panel dies here
    }
    for (int q = 0; !h->dense_layers() && !ytile && q * b < ldu; ++q) {
      SpmmArgs a{};
      a.K = h->K;
      a.sum = 0;
      a.ldx = ldu;
      a.ldy = ldu;
      a.colscale = h->colscale.as<float>() + q * b;
      for (int k = 0; k < h->K; ++k) {
        a.A[k] = h->layers[k]->csr_t();
        a.X[k] = ug + q * b;
        a.Y[k] = h->Y.as<float>() + (size_t)k * h->npad * ldu + q * b;
      }
      HIPCHK(n2v2r_launch_spmm(a, b, h->stream));
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    h->have_embedding = true;
    h->ncmp = h->ncols = 0;
    if (st != N2V2R_OK)
      h->set_err("UASE did not converge: max residual %.3e (tol %.1e%s)",
                 stats ? stats->max_residual : -1.0, o.tol > 0 ? o.tol : 1e-6,
                 stats && stats->stagnated ? "; stopped flat above the fp32-floor cap" : "");
    return st;
  });
}

// local rows (row0 .. row0 + n_local) on a distributed handle
int n2v2r_get_embedding(n2v2r_handle* h, float* Y) {
  if (h && h->multi()) return multi_get_embedding(h, Y);
  return guarded(h, [&]() -> int {
    if (!h->have_embedding) {
      h->err = "No n2v2r embeddings found";
      return N2V2R_ERR_NOT_READY;
    }
    copy_embedding(h, Y, (int64_t)h->nloc * h->d);
    return N2V2R_OK;
  });
}

int n2v2r_get_left_embedding(n2v2r_handle* h, float* X) {
  if (h && h->multi()) return multi_get_left_embedding(h, X);
  return guarded(h, [&]() -> int {
    if (!h->have_embedding || h->U.p == nullptr) {
      h->err = "No n2v2r embeddings found";
      return N2V2R_ERR_NOT_READY;
    }
    HIPCHK(hipMemcpy2DAsync(X, sizeof(float) * h->d, h->U.as<float>(), sizeof(float) * h->ldy,
                            sizeof(float) * h->d, h->nloc, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    for (int64_t i = 0; i < h->nloc; ++i)
      for (int j = 0; j < h->d; ++j) X[i * h->d + j] *= (float)std::sqrt(h->sigma[j]);
    return N2V2R_OK;
  });
}

int n2v2r_get_singular_values(n2v2r_handle* h, double* s) {
  if (h && h->multi()) h = h->ranks[0];  // identical on every rank
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
    if (h->comm || h->multi()) {
      h->err = "set_embedding is single-GPU only";
      return N2V2R_ERR_BAD_ARG;
    }
    h->K = num_layers;
    h->set_partition(n);
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

}  // extern "C"

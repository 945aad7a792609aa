// Internal declarations shared by the engine's host sources (solver.cpp, layers.cpp,
// ranking.cpp, comm.cpp, multi.cpp, engine.cpp): the kernel launchers, device buffers, layer
// storage, communicators and the handle.  Not part of the C-ABI (include/n2v2r.h).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <exception>
#include <system_error>
#include <vector>

#include "../../include/n2v2r.h"
#include "../../include/n2v2r_diag.h"
#include "common.h"

// ---- kernel launchers (spmm.hip, dense.hip, rank.hip) ------------------------------------
#include "spmm_args.h"
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
int n2v2r_spmm_rpw(const SpmmArgs& args, int B);
hipError_t n2v2r_launch_row_sums(const CsrDev& A, float* out, hipStream_t stream);
hipError_t n2v2r_launch_spmm_tile(const SpmmTileArgs& a, hipStream_t stream);
hipError_t n2v2r_launch_chunk_major_keys(uint64_t* keys, int64_t nnz, int64_t npad, int W,
                                         int64_t rc, hipStream_t stream);
// paired-panel mode (pair.hip)
hipError_t n2v2r_launch_interleave16(const float* za, const float* zb, float* x16, int64_t n,
                                     hipStream_t stream);
hipError_t n2v2r_launch_pair_h_assemble(const double* hcol, int64_t ldcol, const int* lo,
                                        const int* nr, int s0, int ns, int kp,
                                        const double* theta, double* H, int c,
                                        hipStream_t stream);
int n2v2r_spmm_tile_rows(int64_t n, int ncu, int wpc, int wbits);
int n2v2r_spmm_tile_rows_b(int64_t n, int ncu, int wpc, int wbits, int b);
hipError_t n2v2r_launch_cb_count(const CsrDev& A, int64_t cw, int nb, int32_t* cnt,
                                 hipStream_t stream);
hipError_t n2v2r_launch_cb_rowptrs(const int32_t* cnt, int64_t n, int nb, int64_t nnz,
                                   int64_t* tsum, size_t tsum_elems, int64_t* rp, int32_t* wo,
                                   int wbits, hipStream_t stream);
int64_t n2v2r_cb_scan_tiles(int64_t n, int nb);
hipError_t n2v2r_launch_cb_fill(const CsrDev& A, int64_t cw, int nb, const int64_t* rp,
                                int32_t* idx, float* dat, int cbits, int wbits,
                                hipStream_t stream);
hipError_t n2v2r_launch_ts_tn(const BlockList& A, const BlockList& B, int64_t n, double* partial,
                              size_t partial_elems, double* out, const int* cond,
                              hipStream_t stream);
hipError_t n2v2r_launch_ritz_nn(const BlockList& A0, const BlockList& A1, const float* G, int ldg,
                                int cb, const OutBlockList& O0, const OutBlockList& O1, int64_t n,
                                int grid, hipStream_t stream);
hipError_t n2v2r_launch_ts_nn(const BlockList& A, const float* G, int ldg, int cb,
                              const OutBlockList& O, const BlockList& C, float alpha, float beta,
                              int64_t n, const int* cond, const int* flags, uint64_t seed,
                              hipStream_t stream);
hipError_t n2v2r_launch_pip_chol(const double* G, int c, int b, double* xinv, int* flags,
                                 int* any_flag, const int* cond, double* save, int save_row0,
                                 int save_rows, float* fout, int* sticky, double* rsave,
                                 int first, hipStream_t stream);
hipError_t n2v2r_launch_rr_band(const double* hband, int c, int kp, double* theta, double* AB,
                                double* Varr, double* taua, double* d, double* e, double* refl,
                                double* Y, float* S, int ldS, int p, int* err,
                                hipStream_t stream);
int n2v2r_rr_band_jm(int c);
// b = 8 PIP passes use the fused Cholesky + apply launch (its A/B switch retired in round 5;
// the two-launch form serves b > 8 and bases beyond 512 columns)
inline bool pip_fused() { return true; }
hipError_t n2v2r_launch_ts_tn2(const BlockList& A, const float* Za, const float* Zb, int64_t n,
                               double* partial, size_t partial_elems, double* out,
                               hipStream_t stream);
hipError_t n2v2r_launch_rmul8(const double* r2, double* r1, hipStream_t stream);
hipError_t n2v2r_launch_pair_fixup(double* g2, int nblk_all, int nq_old, double* ra,
                                   hipStream_t stream);
hipError_t n2v2r_launch_pip_fused(const BlockList& Q, const float* Zin, float* Zout,
                                  const double* G, int c, int64_t n, const int* cond, int* flags,
                                  int* any_flag, double* save, int save_row0, int save_rows,
                                  int* sticky, uint64_t seed, int64_t row0, double* rsave,
                                  float skip_tol, int* skipped, int first, hipStream_t stream);
hipError_t n2v2r_launch_pip_apply(const BlockList& QZ, const float* F, int c, int b,
                                  const OutBlockList& Z, int64_t n, const int* cond,
                                  const int* flags, uint64_t seed, int64_t row0,
                                  hipStream_t stream);
hipError_t n2v2r_launch_fill_normal(float* blk, int w, int64_t n, uint64_t seed, const int* flags,
                                    const int* cond, uint64_t ctr0, hipStream_t stream);
hipError_t n2v2r_launch_resid(const BlockList& X, const BlockList& MX, const double* theta,
                              int64_t n, double* partial, size_t partial_elems, double* out,
                              hipStream_t stream);
hipError_t n2v2r_launch_scale_cols(float* blk, int w, int64_t n, const float* s,
                                   hipStream_t stream);
hipError_t n2v2r_launch_colmax_keys(const float* U, int64_t ldu, int64_t n, int d, int64_t row0,
                                    unsigned long long* keys, size_t key_elems,
                                    unsigned long long* best, hipStream_t stream);
hipError_t n2v2r_launch_colmax_sign(const unsigned long long* best, int ncols_padded,
                                    const float* U, int64_t ldu, int d, int64_t row0, int64_t n,
                                    float* sign, hipStream_t stream);
hipError_t n2v2r_launch_distances(const float* Y, int K, int64_t n, int64_t ldy, int64_t lrows,
                                  int strategy, int layer_i, const DistPlan& plan, double* out,
                                  int64_t ldo, hipStream_t stream);
hipError_t n2v2r_launch_pairwise(const double* a, const double* b, int64_t n, int dim, int metric,
                                 double* out, hipStream_t stream);
hipError_t n2v2r_launch_borda_init(const double* vals, int64_t n, int nseg, uint64_t* keys,
                                   int32_t* idx, unsigned long long* seg_or,
                                   unsigned long long* seg_and, hipStream_t stream);
int n2v2r_radix_tiles(int64_t n);
size_t n2v2r_radix_hist_elems(int64_t n, int nseg);
hipError_t n2v2r_launch_radix_pass(const uint64_t* kin, const int32_t* pin, uint64_t* kout,
                                   int32_t* pout, int64_t n, int nseg, int shift, uint32_t* hist,
                                   hipStream_t stream);
hipError_t n2v2r_launch_borda_finish(const int32_t* sorted_idx, int64_t n, int nseg, int ncols,
                                     int32_t* pos, int64_t* borda, hipStream_t stream);
hipError_t n2v2r_launch_tie_flags(const uint64_t* sorted_keys, int64_t n, int nseg, int32_t* tied,
                                  hipStream_t stream);
hipError_t n2v2r_launch_dense_tn(const float* B, int64_t ldb, int64_t ncols, int64_t kdim,
                                 const float* X, int ldx, int b, float* Y, int64_t ldy, float beta,
                                 const float* colscale, float* work, size_t work_elems,
                                 hipStream_t stream);
hipError_t n2v2r_launch_dense_gemm(const float* A, int64_t lda, int64_t rows, int64_t kdim,
                                   const float* X, int ldx, int b, float* Y, int64_t ldy,
                                   float beta, const float* colscale, float* work,
                                   size_t work_elems, hipStream_t stream);
hipError_t n2v2r_launch_syrk_f64(const double* W, int64_t sk, int64_t si, int64_t kd, int64_t r,
                                 double* out, int64_t ldo, hipStream_t stream);
hipError_t n2v2r_launch_transpose(const float* in, int64_t ldi, int64_t rows, int64_t cols,
                                  float* out, int64_t ldo, hipStream_t stream);
hipError_t n2v2r_launch_mismatch(const float* a, const float* b, int64_t ld, int64_t rows,
                                 int64_t cols, unsigned long long* count, hipStream_t stream);
hipError_t n2v2r_launch_rr_tridiag(double* A, int c, double* d, double* e, double* tau, double* V,
                                   void* scratch, hipStream_t stream);
size_t n2v2r_rr_tridiag_scratch_bytes(int c);
int* n2v2r_rr_tridiag_err(void* scratch, int c);
hipError_t n2v2r_launch_rr_tri_eig(const double* d, const double* e, int c, int p, double* w,
                                   double* Y, double* scratch, hipStream_t stream);
hipError_t n2v2r_launch_rr_backtransform(const double* V, const double* tau, int c,
                                         const double* Y, int p, float* S, int lds, double* tfac,
                                         hipStream_t stream);
size_t n2v2r_rr_bt_scratch_bytes(int c);
hipError_t n2v2r_launch_lds_poison(hipStream_t stream);
hipError_t n2v2r_launch_nonfinite(const void* p, int64_t count, int f64, int* flag,
                                  hipStream_t stream);
hipError_t n2v2r_launch_ts_tn_zsum(const BlockList& A, int64_t n, const float* const* parts,
                                   int count, float* zout, double* partial, size_t partial_elems,
                                   double* out, hipStream_t stream);
hipError_t n2v2r_launch_pack_words(void* const* src, const int* dst_word, const int* words,
                                   const int* clear, int count, void* dst, hipStream_t stream);
hipError_t n2v2r_launch_zsum(const float* const* parts, int count, float* zout, int64_t n,
                             hipStream_t stream);
hipError_t n2v2r_launch_rr_sturm(const double* hband, int c, int kp, double* theta, double* scr,
                                 size_t scr_elems, double* Y, float* S, int ldS, int p, int* err,
                                 hipStream_t stream);
size_t n2v2r_rr_sturm_scratch(int c, int p);
hipError_t n2v2r_launch_rr_band_expand(const double* hband, int c, int kp, const double* theta,
                                       double* H, hipStream_t stream);
hipError_t n2v2r_launch_csr_scan(const int64_t* ip, const int32_t* ix, const float* dv,
                                 int64_t n_rows, int64_t n_cols, uint64_t* keys, int32_t* idx,
                                 unsigned* flags, hipStream_t stream);
hipError_t n2v2r_launch_csr_from_sorted(const uint64_t* keys, const int32_t* idx, const float* dv,
                                        int64_t nnz, int64_t n_cols, int64_t* tp, int32_t* tx,
                                        float* td, hipStream_t stream);
hipError_t n2v2r_launch_csr_compare(const int64_t* ap, const int32_t* ax, const float* av,
                                    const int64_t* bp, const int32_t* bx, const float* bv,
                                    int64_t n_rows, int64_t nnz, unsigned* flag,
                                    hipStream_t stream);
hipError_t n2v2r_launch_csr_rebase(const int64_t* ip, int64_t r0, int64_t nr, int64_t* out,
                                   hipStream_t stream);
}

// Rayleigh-Ritz at b = 8: the band Sturm / inverse-iteration form (rr_sturm.hip) unless
// N2V2R_RR=band (the reducing arrow -> chase path, also the fallback when a Sturm vector fails
// its residual check).  Read per fit.
inline bool rr_sturm_enabled() {
  const char* e = std::getenv("N2V2R_RR");
  return !(e && e[0] == 'b');
}

// Ritz vectors and images by one launch with the coefficients staged once per CU
// (ritz_nn_kernel) where it applies (its A/B switch retired in round 5)
inline bool ritz_nn_enabled() { return true; }

// Lean images (banded Sturm Rayleigh-Ritz, one GPU) unless N2V2R_LEAN_W=0.  Read per fit.
inline bool lean_enabled() {
  const char* e = std::getenv("N2V2R_LEAN_W");
  return !(e && e[0] == '0');
}


namespace n2v2r_int {

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

inline double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// Debug switches (off by default; diagnostics only, never on the bench path):
//   N2V2R_POISON=1        new allocations and, at every fit, the eigensolver's scratch are
//                         filled with 0xFF bytes (NaN) instead of zeros: a read of anything a
//                         kernel did not write this fit turns into a non-finite value;
//   N2V2R_DEBUG_FINITE=1  the eigensolver checks every stage's output for non-finite values
//                         and stops at the first stage that produced one, naming it.
inline bool env_flag(const char* name) {
  const char* e = std::getenv(name);
  return e && *e && *e != '0';
}
inline bool debug_poison() {
  static const bool v = env_flag("N2V2R_POISON");
  return v;
}
inline bool debug_finite() {
  static const bool v = env_flag("N2V2R_DEBUG_FINITE");
  return v;
}
// N2V2R_DEBUG_ORTHO=1: every orthogonalisation pass reports on stderr a block that leaves
// orthonormality (its Gram against the basis and itself), with the pass's refill flags
inline bool debug_ortho() {
  static const bool v = env_flag("N2V2R_DEBUG_ORTHO");
  return v;
}

// Device allocation owned by the handle (zero-filled on allocation: padded rows stay zero).
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
  // The zero fill is ordered on `st` (the engine stream, non-blocking w.r.t. the null stream);
  // with st == nullptr it completes before ensure() returns.
  void ensure(size_t b, hipStream_t st = nullptr) {
    if (bytes >= b && p) return;
    release();
    if (b == 0) b = 16;
    hipError_t e = hipMalloc(&p, b);
    if (e != hipSuccess) {
      p = nullptr;
      throw StatusFail{N2V2R_ERR_OUT_OF_MEMORY,
                       "hipMalloc of " + std::to_string(b) + " bytes failed"};
    }
    const int fill = debug_poison() ? 0xFF : 0;
    if (st) {
      e = hipMemsetAsync(p, fill, b, st);
    } else {
      e = hipMemset(p, fill, b);
      if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    if (e != hipSuccess) throw HipFail{e, "hipMemset"};
    bytes = b;
  }
  // scratch that every use overwrites before reading it: no zero fill, no device sync; kept
  // (and grown) across calls when owned by the handle
  void ensure_raw(size_t b) {
    if (bytes >= b && p) return;
    if (b == 0) b = 16;
    if (debug_poison()) return ensure(b);
    release();
    if (hipMalloc(&p, b) != hipSuccess) {
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
  DevBuf indptr, indices, data;        // local rows of A (CSR, global column indices)
  DevBuf t_indptr, t_indices, t_data;  // local rows of A^T when A is not symmetric
  int64_t nnz = 0, t_nnz = 0;
  int64_t n_rows = 0;                  // local rows
  bool unit = false, t_unit = false;   // all stored values 1.0f
  bool symmetric = true;
  bool loaded = false;
  // dense layer (cfg3): local rows of A and (directed) of A^T, fp32, leading dimension lda
  bool dense = false;
  DevBuf dA, dAT;
  int64_t lda = 0;
  const float* dense_a() const { return dA.as<float>(); }
  const float* dense_at() const { return symmetric ? dA.as<float>() : dAT.as<float>(); }
  CsrDev csr() const {
    return CsrDev{indptr.as<int64_t>(), indices.as<int32_t>(), data.as<float>(), n_rows, nnz,
                  unit ? 1 : 0};
  }
  CsrDev csr_t() const {
    if (symmetric) return csr();
    return CsrDev{t_indptr.as<int64_t>(), t_indices.as<int32_t>(), t_data.as<float>(), n_rows,
                  t_nnz, t_unit ? 1 : 0};
  }
  // column-block form of A and (directed) A^T for the flat tiled SpMM (built on first use)
  struct ColBlocks {
    DevBuf wo, idx, dat;   // [nb][nwin + 1] int32 window offsets (relative); entries; values
    CsrBlk blk[CB_MAX];
    int nb = 0;            // blocks (4-64; phases of the flat tiled SpMM)
    int wbits = 0;         // windows of 2^wbits rows
    int cbits = 0;         // column bits of the packed entries (0: the layer cannot be packed)
    int64_t ncols = 0;     // column count the blocks were cut for
    bool built = false;
    bool usable = false;   // every block under 2^31 entries (int32 offsets)
  };
  ColBlocks cb, cb_t;
  // partitioned handles, reduce-scatter form: this rank's columns of A, A[:, own rows], as a CSR
  // over the world x npad padded global rows with local column indices (built on first use)
  DevBuf c_indptr, c_indices, c_data;
  int64_t c_nnz = 0, c_rows = 0;
  int64_t c_rc = 0;  // rows per chunk of the chunk-major row order (0: natural order)
  bool c_built = false;
  CsrDev csr_c() const {
    return CsrDev{c_indptr.as<int64_t>(), c_indices.as<int32_t>(), c_data.as<float>(), c_rows,
                  c_nnz, (symmetric ? unit : t_unit) ? 1 : 0};
  }
  void drop_col_blocks() {  // (and every other derived form of the layer)
    for (ColBlocks* c : {&cb, &cb_t}) {
      c->wo.release();
      c->idx.release();
      c->dat.release();
      c->built = false;
    }
    c_indptr.release();
    c_indices.release();
    c_data.release();
    c_built = false;
  }
};

// column blocks of a layer for the flat tiled SpMM (layers.cpp)
void build_col_blocks(const CsrDev& A, int64_t ncols, LayerDev::ColBlocks& out, hipStream_t st,
                      int nb, int wbits);
bool ensure_col_blocks(LayerDev& L, int64_t ncols, hipStream_t st, int nb, int wbits);
int tile_wbits(const std::vector<std::unique_ptr<LayerDev>>& layers, int nb);
// (npad, W, rc > 0: rows in the chunk-major order of the pipelined reduce-scatter)
void ensure_colcsr(LayerDev& L, int64_t ncols, int64_t rows_out, hipStream_t st, int64_t npad = 0,
                   int W = 1, int64_t rc = 0);

// ---- communicators ----------------------------------------------------------------------
struct Comm {
  int rank = 0, world = 1;
  virtual ~Comm() = default;
  // recv = world x bytes, rank-major (rank r's bytes at r * bytes)
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t st) = 0;
  virtual void allreduce_sum_f64(double* buf, size_t count, hipStream_t st) = 0;
  virtual void allreduce_max_u64(unsigned long long* buf, size_t count, hipStream_t st) = 0;
  virtual void allreduce_sum_f32(float* buf, size_t count, hipStream_t st) = 0;
  // recv (count floats) = sum over ranks of their send[rank * count .. (rank + 1) * count)
  virtual void reduce_scatter_sum_f32(const float* send, float* recv, size_t count,
                                      hipStream_t st) = 0;
  virtual const char* kind() const = 0;
  // another rank of this communicator launches on this rank's device (the thread group's ranks
  // may share one GPU; RCCL ranks never do)
  virtual bool shares_device() const { return false; }
  // unblock this rank's pending collectives after a peer failed (the communicator is dead after)
  virtual void abort() {}
};

struct NcclFail {
  ncclResult_t r;
  std::string where;
};
#define NCCLCHK(expr)                                   \
  do {                                                  \
    ncclResult_t _r = (expr);                           \
    if (_r != ncclSuccess) throw NcclFail{_r, #expr};   \
  } while (0)

// RCCL communicator of one rank (comm.cpp); takes ownership of c
std::unique_ptr<Comm> make_rccl_comm(ncclComm_t c, int rank, int world);
}  // namespace n2v2r_int

// W ranks of one process on one device (threads): the partitioned algorithm, testable on one
// GPU.  Collectives: stream sync, publish a pointer, barrier, copy / fixed-order host sum.
struct n2v2r_simgroup {
  int world = 1;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  bool aborted = false;  // a rank failed: every barrier from here on throws (no rank hangs)
  std::vector<const void*> ptrs;
  std::vector<std::vector<unsigned char>> host;
  std::vector<int> dev;  // each rank's device (-1 = not created yet), under m
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const uint64_t gen = generation;
    if (aborted) throw n2v2r_int::StatusFail{N2V2R_ERR_INTERNAL, "thread group aborted"};
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen || aborted; });
      if (generation == gen)
        throw n2v2r_int::StatusFail{N2V2R_ERR_INTERNAL, "thread group aborted"};
    }
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    aborted = true;
    cv.notify_all();
  }
};

namespace n2v2r_int {
// in-process communicator of rank `rank` of the thread group g (comm.cpp)
std::unique_ptr<Comm> make_thread_comm(n2v2r_simgroup* g, int rank, int device);

// Solver buffers kept by the handle across n2v2r_uase calls (repeated fits of the same graph
// reuse every allocation; the zero-filled padding rows of pool blocks stay zero).
struct EigWorkspace {
  std::vector<std::unique_ptr<DevBuf>> pool;  // Krylov blocks, block_bytes each
  size_t block_bytes = 0;
  std::vector<std::unique_ptr<DevBuf>> zk;    // K stage-1 panels (local)
  DevBuf zg;                                  // K gathered stage-1 panels
  DevBuf rinv, flg, anyflag, gsmall, csmall;
  DevBuf rback;  // the per-cycle read-back, packed on the device before one copy to the host
  DevBuf tri, refl, ytri, tscr;               // GPU Rayleigh-Ritz: [d|e|tau], reflectors, Y_T
  DevBuf trcoop;                              // multi-workgroup tridiagonalisation scratch
  DevBuf btf;                                 // Rayleigh-Ritz back-transform: blocks' T factors
  DevBuf hband, band, varr, taua, rrerr;      // banded RR: band columns, band matrix, arrow
  DevBuf fcoef;                               // fp32 [-C R^-1; R^-1] of the apply pass
  DevBuf dbgflag;                             // N2V2R_DEBUG_FINITE result flag
  DevBuf tflag;                               // partitioned: a per-cycle flag agreed over ranks
  DevBuf s2part;                             // [K][npad][8] XCD-split second-stage outputs
  DevBuf g2, pair_ra;                         // paired full passes: the two Grams, R of the first
  DevBuf sturm;                               // Sturm Rayleigh-Ritz: assembled arrow + band
  DevBuf rres;                                // lean images: R of the restart projection
  DevBuf skipc;                               // full passes skipped (selective reorthogonalisation)
  DevBuf tblk;                                // tiled SpMM: CsrBlk [2][K][nb] (stage 1, stage 2)
  // paired-panel mode: the N x 16 panel of two blocks, the saved band columns of the projected
  // matrix (one slot of (c + 8) x 8 per basis block), the restart pair's coupling rows
  DevBuf x16, hcol, pcab, pth;
};
}  // namespace n2v2r_int

using n2v2r_int::Comm;
using n2v2r_int::DevBuf;
using n2v2r_int::LayerDev;
using n2v2r_int::EigWorkspace;
using n2v2r_int::HipFail;
using n2v2r_int::StatusFail;

struct n2v2r_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  // side stream + events for the column-block SpMM's stage-1 reduce overlap
  hipStream_t side = nullptr;
  hipEvent_t cb_ev[2 * SPMM_MAX_LAYERS] = {};
  // pinned host staging of the per-cycle read-back (residuals, Ritz values, flags): the copies
  // are asynchronous and one stream synchronisation ends the cycle (pageable targets made each
  // copy a host round trip of its own)
  void* pin = nullptr;
  size_t pin_bytes = 0;
  void ensure_pin(size_t bytes) {
    if (pin_bytes >= bytes) return;
    if (pin) (void)hipHostFree(pin);
    pin = nullptr;
    pin_bytes = 0;
    if (hipHostMalloc(&pin, bytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      throw std::bad_alloc();
    }
    pin_bytes = bytes;
  }
  std::string err;
  int K = 0;
  int64_t n = 0;        // global nodes
  // row partition (single GPU: rank 0 of 1, row0 = 0, nloc = npad = n)
  std::unique_ptr<Comm> comm;
  int rank = 0, world = 1;
  int64_t row0 = 0, nloc = 0, npad = 0;
  int64_t h2d_layer_bytes = 0;  // layer bytes this handle copied host -> device (diagnostics)
  std::vector<std::unique_ptr<LayerDev>> layers;

  // UASE results
  int d = 0;
  int ldy = 0;              // row stride of the per-layer embedding
  DevBuf Y;                 // [K][npad][ldy] fp32 (local rows)
  DevBuf U;                 // [npad][ldy] fp32 left singular vectors (local rows)
  std::vector<double> sigma;
  bool have_embedding = false;

  // rank results (global after the gather)
  int ncmp = 0, ncols = 0;
  DevBuf D;                 // [ncmp][ncols][n] fp64
  DevBuf Dloc;              // [ncmp][ncols][npad] fp64 (distributed)
  DevBuf Dgat;              // [world][npad] staging of one gathered column
  DevBuf borda;             // [ncmp][n] int64
  bool have_borda = false;  // n2v2r_rank aggregated (N2V2R_AGG_BORDA)
  // N2V2R_EIG_TIME_SPMM: event pairs around the fit's SpMM stage launches (reused across fits)
  std::vector<hipEvent_t> tev;
  double ms_dist = 0, ms_borda = 0;

  // scratch
  DevBuf partial;           // chunk partials of the tall-skinny reductions
  size_t partial_elems = 0;
  DevBuf theta;             // fp64 Ritz values
  DevBuf resid;             // fp64 residuals
  DevBuf colscale;          // fp32
  DevBuf keys, best;        // sign convention
  DevBuf gath;              // gathered panels
  EigWorkspace ews;         // eigensolver buffers, reused across fits
  DevBuf dense_work;        // split-K slabs of the dense GEMM
  size_t dense_work_elems = 0;
  bool dense_layers() const { return !layers.empty() && layers[0]->dense; }
  // Y (nloc x b, ld ldy) = beta Y + colscale .* (A_loc X_global) for dense layer rows.
  // Bt (optional, unpartitioned handles): the stored matrix whose TRANSPOSE is A (A itself when
  // symmetric, the other copy when directed): then Y = Bt^T X by dense_tn_kernel, B streaming
  // from HBM into the MFMA operands (N2V2R_DENSE_TN=0, read per call: the LDS-staged kernel)
  void dense_apply(const float* Aloc, int64_t lda, const float* X, int ldx, int b, float* Y,
                   int64_t ldy, float beta, const float* colscale, const float* Bt = nullptr) {
    const size_t need = (size_t)std::max<int64_t>(nloc, 1) * b * 16;
    if (dense_work_elems < need) {
      dense_work.ensure(sizeof(float) * need);
      dense_work_elems = need;
    }
    const char* tn = std::getenv("N2V2R_DENSE_TN");
    if (Bt && nloc == n && !(tn && tn[0] == '0')) {
      const hipError_t e = n2v2r_launch_dense_tn(Bt, lda, nloc, n, X, ldx, b, Y, ldy, beta,
                                                 colscale, dense_work.as<float>(),
                                                 dense_work_elems, stream);
      if (e == hipSuccess) return;
      if (e != hipErrorNotSupported) throw HipFail{e, "n2v2r_launch_dense_tn"};
    }
    HIPCHK(n2v2r_launch_dense_gemm(Aloc, lda, nloc, n, X, ldx, b, Y, ldy, beta, colscale,
                                   dense_work.as<float>(), dense_work_elems, stream));
  }
  DevBuf rs_keys[2], rs_idx[2], rs_pos, rs_hist, rs_or, rs_and;
  // ingest scratch (n2v2r_set_layer_csr: radix keys / payloads of the transpose, histogram,
  // flags) and the embedding's panel slice, kept across calls (a per-call hipMalloc + zero
  // fill + device sync + hipFree each time otherwise)
  DevBuf ing_keys[2], ing_pay[2], ing_hist, ing_flag;
  DevBuf ypanel;


  void set_err(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    err = buf;
  }

  void set_partition(int64_t n_global) {
    n = n_global;
    if (world <= 1) {
      row0 = 0;
      nloc = npad = n;
      return;
    }
    npad = (n + world - 1) / world;
    row0 = std::min<int64_t>(n, (int64_t)rank * npad);
    nloc = std::max<int64_t>(0, std::min<int64_t>(n, row0 + npad) - row0);
  }

  // gather a local [npad][w] panel of every rank into the global [world*npad][w] panel
  void gather_panel(const float* local, float* global, int w) {
    if (!comm) {
      if (local != global)
        HIPCHK(hipMemcpyAsync(global, local, sizeof(float) * npad * w, hipMemcpyDeviceToDevice,
                              stream));
      return;
    }
    comm->allgather(local, global, sizeof(float) * npad * w, stream);
  }
  // the same on the collective stream, started once `ready` (recorded on the engine stream)
  // has fired; `done` is recorded behind it (SpMM stage 1 of layer k + 1 runs meanwhile)
  hipStream_t cstream = nullptr;
  hipEvent_t cev[2 * SPMM_MAX_LAYERS] = {};
  void gather_panel_async(const float* local, float* global, int w, int slot) {
    if (!cstream) {
      HIPCHK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
      for (hipEvent_t& e : cev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    HIPCHK(hipEventRecord(cev[2 * slot], stream));
    HIPCHK(hipStreamWaitEvent(cstream, cev[2 * slot], 0));
    comm->allgather(local, global, sizeof(float) * npad * w, cstream);
    HIPCHK(hipEventRecord(cev[2 * slot + 1], cstream));
  }
  void gather_wait(int slot) { HIPCHK(hipStreamWaitEvent(stream, cev[2 * slot + 1], 0)); }
  // reduce-scatter on the collective stream behind what the engine stream queued so far; the
  // engine stream waits for all of them with rs_wait_all (at most SPMM_MAX_LAYERS in flight)
  hipEvent_t rev[SPMM_MAX_LAYERS + 1] = {};
  int rs_pending = 0;
  void reduce_scatter_async(const float* send, float* recv, size_t count) {
    if (!cstream) {
      HIPCHK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
      for (hipEvent_t& e : cev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (!rev[0])
      for (hipEvent_t& e : rev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(rev[rs_pending], stream));
    HIPCHK(hipStreamWaitEvent(cstream, rev[rs_pending], 0));
    comm->reduce_scatter_sum_f32(send, recv, count, cstream);
    ++rs_pending;
  }
  void rs_wait_all() {
    if (!rs_pending) return;
    HIPCHK(hipEventRecord(rev[SPMM_MAX_LAYERS], cstream));
    HIPCHK(hipStreamWaitEvent(stream, rev[SPMM_MAX_LAYERS], 0));
    rs_pending = 0;
  }
  void allreduce_f64(double* buf, size_t count) {
    if (comm) comm->allreduce_sum_f64(buf, count, stream);
  }

  // One process, N GPUs (n2v2r_create_multi, multi.cpp): this handle owns one row-partitioned
  // rank handle per device and runs every call on all of them, one host thread per rank.
  std::vector<n2v2r_handle*> ranks;
  std::unique_ptr<n2v2r_simgroup> own_group;  // the thread communicator's group (devices repeat)
  // one persistent host thread per rank, started by the first C-ABI call (multi.cpp), stopped and
  // joined by multi_destroy
  struct n2v2r_int_rank_pool* pool = nullptr;
  bool broken = false;  // a rank failed alone and the communicator was aborted
  bool multi() const { return !ranks.empty(); }
};

namespace n2v2r_int {

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
  } catch (const NcclFail& nf) {
    h->set_err("RCCL error %d (%s) at %s", (int)nf.r, ncclGetErrorString(nf.r), nf.where.c_str());
    return N2V2R_ERR_RCCL;
  } catch (const StatusFail& sf) {
    h->err = sf.msg;
    return sf.code;
  } catch (const std::bad_alloc&) {
    h->err = "host allocation failed";
    return N2V2R_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& ex) {  // e.g. std::system_error from a host thread
    h->err = std::string("host error: ") + ex.what();
    return N2V2R_ERR_INTERNAL;
  }
}

// ---- host CSR helpers (layers.cpp) ------------------------------------------------------
int host_threads();
template <class F>
void parallel_chunks(int nt, F&& fn);
bool host_indices_in_range(int64_t nnz, const int32_t* ix, int64_t n);
bool upload_rows(hipStream_t st, int64_t r0, int64_t nr, const int64_t* ip, const int32_t* ix,
                 const float* dv, DevBuf& dip, DevBuf& dix, DevBuf& ddv, int64_t& nnz_out);
// A == A^T as multisets of (row, column, value bits), by two independent 64-bit hash sums over
// the entries and over the transposed entries (host threads; layers.cpp)
bool host_csr_symmetric(int64_t n, const int64_t* ip, const int32_t* ix, const float* dv);
// rows [r0, r0 + nr) of A^T from a host CSR of A (columns r0 .. r0 + nr - 1 of A; within a row of
// A^T the entries in ascending row of A, as the GPU transpose orders them)
void host_transpose_rows(int64_t n, const int64_t* ip, const int32_t* ix, const float* dv,
                         int64_t r0, int64_t nr, std::vector<int64_t>& tip,
                         std::vector<int32_t>& tix, std::vector<float>& tdv);
// a partitioned handle's rows of a directed layer: its rows of A and of A^T, local row pointers
int set_layer_rows_directed(n2v2r_handle* h, int k, const int64_t* aip, const int32_t* aix,
                            const float* adv, const int64_t* tip, const int32_t* tix,
                            const float* tdv);

// run fn(0) .. fn(nt - 1), one host thread each.  A thread that cannot be created leaves its
// chunk (and the later ones) to the calling thread; every started thread is joined before
// returning or rethrowing, so no joinable std::thread is ever destroyed.
template <class F>
void parallel_chunks(int nt, F&& fn) {
  std::vector<std::thread> pool;
  pool.reserve(nt);
  int t = 0;
  try {
    for (; t < nt; ++t) pool.emplace_back([&fn, t] { fn(t); });
  } catch (const std::system_error&) {
  }
  std::exception_ptr err;
  try {
    for (; t < nt; ++t) fn(t);
  } catch (...) {
    err = std::current_exception();
  }
  for (auto& th : pool) th.join();
  if (err) std::rethrow_exception(err);
}
// Algorithmic HBM bytes of one CSR x panel SpMM over `rows` rows (for this
// storage format): column indices 4 B/nnz, values 4 B/nnz unless the layer is unweighted (the
// kernel then skips them), int64 row pointers, the N x b panel read once and the rows x b
// output written once.  The gathered panel rows (4 b B per nnz, served by L2 / Infinity Cache)
// are not counted.
inline double spmm_algo_bytes(int64_t nnz, bool unit, int64_t rows, int64_t panel_rows, int b) {
  return (unit ? 4.0 : 8.0) * (double)nnz + 8.0 * (double)(rows + 1) +
         4.0 * (double)(panel_rows + rows) * b;
}

// the tiled column-block SpMM wanted at panel width b (solver.cpp)
bool col_blocks_wanted(const n2v2r_handle* h, int b);
// a new single-GPU handle on `device` (engine.cpp); nullptr on failure
n2v2r_handle* new_handle(int device);
// Local embedding rows of a (rank) handle into Y with layer k's block at Y + k * layer_stride
// (solver.cpp)
void copy_embedding(n2v2r_handle* h, float* Y, int64_t layer_stride);

// ---- multi-GPU handles (multi.cpp): the C-ABI functions forward here when h->multi() --------
int multi_destroy(n2v2r_handle* h);
int multi_synchronize(n2v2r_handle* h);
int multi_set_num_layers(n2v2r_handle* h, int num_layers, int64_t n);
int multi_set_layer_csr(n2v2r_handle* h, int k, int64_t n, int64_t nnz, const int64_t* indptr,
                        const int32_t* indices, const float* data, int symmetric);
int multi_set_layer_dense(n2v2r_handle* h, int k, int64_t n, const float* A, int symmetric);
int multi_column_sums(n2v2r_handle* h, int k, float* out);
int multi_uase(n2v2r_handle* h, int d, const n2v2r_eig_opts* opts, n2v2r_eig_stats* stats);
int multi_get_embedding(n2v2r_handle* h, float* Y);
int multi_get_left_embedding(n2v2r_handle* h, float* X);
int multi_rank(n2v2r_handle* h, int strategy, const int* dims, int n_dims, const int* metrics,
               int n_metrics, int method, int* n_comparisons, int* n_cols);
}  // namespace n2v2r_int
using n2v2r_int::guarded;


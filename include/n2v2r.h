/* n2v2r.h -- C-ABI of the MI355X-native node2vec2rank fit-and-rank engine (libn2v2r_hip.so).
 *
 * Plain C types only (no torch, no HIP types).  Host pointers unless a name says "_dev".
 * One handle drives one GPU; it owns every device buffer; it is NOT thread-safe.
 * Every function returns an n2v2r_status; on failure n2v2r_last_error() has the message.
 *
 * Reference seams these entry points replace (file:line in /root/reference):
 *   - n2v2r_set_layer_csr + n2v2r_uase + n2v2r_get_embedding
 *       replace  se.UASE(csc_layers, max_embed_dim)           node2vec2rank/model.py:51-55
 *       (third-party spectral_embedding.UASE -> scipy.sparse.linalg.svds / ARPACK)
 *   - n2v2r_rank (+ n2v2r_get_distances)
 *       replaces N2V2R.__rank                                 node2vec2rank/model.py:57-96
 *       and compute_pairwise_distances                        node2vec2rank/model_utils.py:39-67
 *   - n2v2r_rank (+ n2v2r_get_borda)
 *       replaces the per-column sort of aggregate_transform   node2vec2rank/model.py:167-185
 *       and borda_aggregate_parallel / _get_ranking           node2vec2rank/model_utils.py:22-36
 *   - n2v2r_pairwise_distances: host-array form of            node2vec2rank/model_utils.py:39
 *   - n2v2r_borda_columns:      host-array form of            node2vec2rank/model_utils.py:28
 *   - n2v2r_borda_columns_ex:   + the tie order of            node2vec2rank/model.py:173-174
 *   - n2v2r_column_sums:        float32 column sums for       node2vec2rank/model.py:282-311
 */
#ifndef N2V2R_H
#define N2V2R_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  N2V2R_OK = 0,
  N2V2R_ERR_BAD_ARG = 1,            /* -> ValueError */
  N2V2R_ERR_UNSUPPORTED_METRIC = 2, /* -> NotImplementedError, model_utils.py:64-65 */
  N2V2R_ERR_NO_CONVERGENCE = 3,     /* -> ArpackNoConvergence analogue */
  N2V2R_ERR_HIP = 4,                /* -> RuntimeError */
  N2V2R_ERR_OUT_OF_MEMORY = 5,      /* -> MemoryError */
  N2V2R_ERR_NOT_READY = 6,          /* -> ValueError("No n2v2r embeddings found"), model.py:199 */
  N2V2R_ERR_UNSUPPORTED_AGG = 7,    /* -> NotImplementedError, model.py:182-183 */
  N2V2R_ERR_INTERNAL = 8,           /* -> RuntimeError (host-side failure, e.g. a thread) */
  N2V2R_ERR_RCCL = 9                /* -> RuntimeError (an RCCL collective or communicator failed) */
} n2v2r_status;

/* comp_strategy (model.py:59-84) */
enum { N2V2R_SEQUENTIAL = 0, N2V2R_ONE_VS_BEFORE = 1, N2V2R_ONE_VS_REST = 2 };
/* distance metrics (model_utils.py:55-63) */
enum { N2V2R_COSINE = 0, N2V2R_EUCLIDEAN = 1, N2V2R_CORRELATION = 2 };
/* symmetric hint for n2v2r_set_layer_csr */
enum { N2V2R_SYM_DETECT = -1, N2V2R_SYM_NO = 0, N2V2R_SYM_YES = 1 };
/* n2v2r_rank method: Borda (model.py:179-183), or distances only (the caller aggregates later
 * through n2v2r_borda_columns, as aggregate_transform recomputes from the current frames) */
enum { N2V2R_AGG_BORDA = 0, N2V2R_AGG_NONE = -1 };

/* n2v2r_eig_opts.solver_flags */
enum { N2V2R_EIG_FULL_FIRST_PASS = 1, N2V2R_EIG_DENSE_RR = 2,
       N2V2R_EIG_TEST_REDO_CYCLE = 4 /* tests: re-expand the first cycle as after a refill */,
       N2V2R_EIG_TEST_BAND_FAIL = 8 /* tests: every banded Rayleigh-Ritz result is treated as
                                       failed, so the reducing, then the dense fallback runs
                                       (and a lean-image fit reruns with images kept) */,
       N2V2R_EIG_TEST_STURM_FAIL = 32 /* tests: only the Sturm Rayleigh-Ritz result is treated
                                         as failed (the reducing band path then runs and is
                                         accepted) */,
       N2V2R_EIG_TIME_SPMM = 16 /* HIP events around every SpMM stage launch of the fit: fills
                                   n2v2r_eig_stats.gpu_ms_spmm / spmm_timed_launches (the in-fit
                                   roofline of bench.py; adds an event pair per launch) */,
       N2V2R_EIG_TEST_NO_STAGNATION = 64 /* tests: no stop on flat residuals (the fit runs until
                                            every residual meets tol or max_restarts) */,
       N2V2R_EIG_PANEL16 = 256 /* paired-panel mode on (b = 8 basis blocks, two per SpMM
                                  application as one N x 16 panel, dense Rayleigh-Ritz of the
                                  assembled band); N2V2R_EIG_PANEL8 = 512 forces it off; neither:
                                  the library's default for the graph (solver.cpp) */,
       N2V2R_EIG_PANEL8 = 512,
       N2V2R_EIG_TEST_FAIL_ALONE = 128 /* tests, multi-GPU handles: rank 1 fails alone after its
                                          first block application while its peers go on into
                                          their next collective (the abort path) */ };

typedef struct n2v2r_handle n2v2r_handle;
typedef struct n2v2r_simgroup n2v2r_simgroup;

typedef struct {
  int block;          /* Krylov block width b: 8, 16, 32 or 64 (0 = auto: 8) */
  int max_basis;      /* max basis columns before a thick restart (0 = auto) */
  int keep;           /* Ritz vectors kept at a restart (0 = auto: max(d + 16, 21d/16) for CSR
                         layers, at most 184 where the banded Rayleigh-Ritz fits; d + b for dense) */
  int max_restarts;   /* (0 = auto: 2000) */
  double tol;         /* stop when ||M x_j - theta_j x_j|| <= tol * theta_1 for j < d (<=0: 1e-6) */
  uint64_t seed;      /* start block seed */
  int solver_flags;   /* 0 = defaults.  N2V2R_EIG_FULL_FIRST_PASS: orthogonalise every new
                         block with two full block-Gram-Schmidt passes (instead of a local pass
                         against the two previous blocks + one full pass);
                         N2V2R_EIG_DENSE_RR: Rayleigh-Ritz on the dense projected matrix
                         Q^T M Q (instead of the block-tridiagonal one) */
} n2v2r_eig_opts;

typedef struct {
  int restarts;              /* Rayleigh-Ritz cycles run */
  int block_applications;    /* applications of M = sum_k A_k A_k^T to a b-wide block */
  int converged;             /* Ritz pairs (of d) that met tol */
  int basis;                 /* max basis columns used */
  double max_residual;       /* max_j<d ||M x_j - theta_j x_j|| / theta_1 */
  double ms_total, ms_spmm, ms_ortho, ms_rr_host; /* host wall-clock split (launch time for
                                                     asynchronous GPU stages) */
  int64_t spmm_launches;     /* SpMM kernel launches (for roofline accounting) */
  double spmm_algo_bytes;    /* sum over launches of the SURVEY 8(d) algorithmic bytes */
  int stagnated;             /* 1: stopped because the residuals went flat (the fp32 floor); the
                                fit is N2V2R_OK only if max_residual <= stag_cap, else
                                N2V2R_ERR_NO_CONVERGENCE */
  int rr_fallbacks;          /* Rayleigh-Ritz cycles whose Sturm/inverse-iteration vectors failed
                                the residual check and were redone by the reducing path */
  /* N2V2R_EIG_TIME_SPMM only (else 0): device time of the fit's SpMM stage launches (HIP events
   * on the engine stream), their count and their algorithmic bytes (per launch
   * form), split by stage: [0] = Z_k = A_k^T X (all layers), [1] = W = sum_k A_k Z_k */
  double gpu_ms_spmm[2];
  int64_t spmm_timed_launches[2];
  double spmm_stage_bytes[2];
  double est_scale;          /* lean images: the last true / estimated residual scale (1 = none) */
  int lean_checks;           /* lean images: true-residual checks run */
  int pool_blocks;           /* Krylov blocks the handle's solver pool holds after the fit */
  int spmm_form;             /* SpMM form of the fit: 0 row kernel, 1 row kernel with the layers
                                split over the XCDs, 2 column blocks + partial reduce, 3 tiled
                                column blocks (one launch per stage over all layers, row
                                groups), 4 dense, 5 tiled column blocks with packed flat windows
                                (the default tiled form) */
  double stag_cap;           /* the largest max_residual a stagnated fit may end with and still
                                return N2V2R_OK: 2 max(tol, sqrt(c) 2^-24), c = the basis columns
                                (the fp32 rounding floor of a Ritz vector assembled from c of them) */
  int y_captured;            /* 1: the embedding A_k^T U came from the final residual check's SpMM
                                products (no separate embedding launches) */
  int tri_fallbacks;         /* dense Rayleigh-Ritz: multi-workgroup tridiagonalisations that timed
                                out (a workgroup not resident) and were redone on one workgroup */
  int panel;                 /* columns each SpMM launch of the fit multiplies: b, or 16 in the
                                paired-panel mode (two b = 8 blocks per application of M;
                                block_applications still counts 8-wide blocks) */
} n2v2r_eig_stats;

/* lifecycle */
int n2v2r_create(int device, n2v2r_handle** out);
void n2v2r_destroy(n2v2r_handle* h);
int n2v2r_last_error(const n2v2r_handle* h, char* buf, size_t len);
const char* n2v2r_version(void);

/* Row-partitioned multi-GPU (no reference counterpart: the reference is
 * single-process).  Rank g of W owns rows [g*R, min(N,(g+1)*R)), R = ceil(N/W), of every layer,
 * of every Krylov block and of the embedding; panels are all-gathered per SpMM stage and the
 * small Gram / projection / residual reductions all-reduced.  Every rank calls every function
 * in the same order (collective semantics).  Results: n2v2r_get_embedding /
 * n2v2r_get_left_embedding return the LOCAL rows (n_local x d); distances, Borda, singular
 * values and column sums are global on every rank.
 *   RCCL, one process per GPU: rank 0 calls n2v2r_comm_unique_id, broadcasts the bytes
 *   (N2V2R_UNIQUE_ID_BYTES) over its own control plane, every rank calls n2v2r_create_rccl.
 *   Thread group, W ranks on ONE device in one process (tests): n2v2r_simgroup_create, then one
 *   thread per rank calls n2v2r_create_sim and drives its handle. */
#define N2V2R_UNIQUE_ID_BYTES 128
int n2v2r_comm_unique_id(char* out, size_t len);
int n2v2r_create_rccl(int device, int rank, int world, const char* unique_id, n2v2r_handle** out);
int n2v2r_simgroup_create(int world, n2v2r_simgroup** out);
void n2v2r_simgroup_destroy(n2v2r_simgroup* g);
int n2v2r_create_sim(int device, n2v2r_simgroup* g, int rank, n2v2r_handle** out);
int n2v2r_dist_info(const n2v2r_handle* h, int* rank, int* world, int64_t* row0, int64_t* n_local);

/* One process, n_gpus GPUs, through the same API as a single-GPU handle (one host
 * thread per GPU inside the library).  The handle row-partitions every layer, Krylov block and
 * embedding over the devices and runs each call on all of them at once; results come back
 * global (n2v2r_get_embedding: all N rows; distances, Borda, singular values as on one GPU), so
 * a caller switches by creating the handle with n2v2r_create_multi instead of n2v2r_create.
 * Collectives: RCCL over the listed devices (ncclCommInitAll) when they are distinct; when a
 * device repeats, an in-process thread group (W ranks sharing one GPU: the same partitioned
 * algorithm, for testing on fewer devices).  n2v2r_set_layer_csr with N2V2R_SYM_YES uploads to
 * each device only its rows; other layers are ingested whole by every device (each runs the GPU
 * transpose and symmetry test) before keeping its rows.  n2v2r_set_layer_csr_rows and
 * n2v2r_set_embedding are refused; n2v2r_dist_info reports (0, n_gpus, 0, N).  Every call is
 * collective inside the library; the handle is not thread-safe (as every handle).
 * Reference: the reference is single-process (model.py:18, 51-55); this is the same drop-in
 * N2V2R call (node2vec2rank_amd.model.N2V2R(..., n_gpus=N)) spread over N GPUs. */
int n2v2r_create_multi(const int* devices, int n_gpus, n2v2r_handle** out);
/* the devices of a handle (1 for a single-GPU handle); returns the count, fills up to cap */
int n2v2r_multi_devices(const n2v2r_handle* h, int* devices, int cap);

/* graph layers: K layers over the same N nodes.  CSR is copied to HBM (int64 row pointers;
 * int32 column indices; fp32 values).  The column-index range check, the transpose (stable LSD
 * radix sort of the entries by column on the GPU) and symmetric = N2V2R_SYM_DETECT (A compared
 * with A^T entry by entry on the GPU) run on the device.  Non-symmetric layers also keep A^T.
 * The transpose sorts int32 entry indices: a layer with more than 2^31 - 1 entries needs
 * symmetric = N2V2R_SYM_YES (N2V2R_ERR_BAD_ARG otherwise).
 * The first fit on one GPU adds a column-blocked copy of the entries for the tiled SpMM
 * (~4 nnz bytes, + 4 nnz of values for a weighted layer, + 4 nb (N / 2^wbits + 1) of window
 * offsets; A^T's as well when not symmetric), kept with the layer.
 * Memory: on a partitioned handle this call still uploads the WHOLE layer to every rank (and,
 * unless N2V2R_SYM_YES, sorts its transpose there, ~40 B per global entry at the peak) before
 * keeping the rank's rows; n2v2r_set_layer_csr_rows is the ingest whose memory scales with the
 * row partition. */
int n2v2r_set_num_layers(n2v2r_handle* h, int num_layers, int64_t n);
int n2v2r_set_layer_csr(n2v2r_handle* h, int k, int64_t n, int64_t nnz, const int64_t* indptr,
                        const int32_t* indices, const float* data, int symmetric);
/* dense layer (BASELINE cfg3, co-expression networks): A row-major n x n fp32 on the host.
 * Stored dense in HBM (this rank's rows; A^T rows as well unless symmetric); the Gram
 * application becomes dense MFMA GEMMs.  All layers of a handle are CSR or all dense.
 * symmetric: N2V2R_SYM_* (DETECT compares A with A^T on the GPU). */
int n2v2r_set_layer_dense(n2v2r_handle* h, int k, int64_t n, const float* A, int symmetric);
/* distributed ingest without the global CSR on every rank: the caller's own rows
 * [row0, row0 + n_rows) (must equal n2v2r_dist_info's) of a SYMMETRIC layer, indptr local
 * (starting at 0), column indices global. */
int n2v2r_set_layer_csr_rows(n2v2r_handle* h, int k, int64_t n, int64_t row0, int64_t n_rows,
                             int64_t nnz, const int64_t* indptr, const int32_t* indices,
                             const float* data);

/* UASE: top-d truncated SVD of the unfolded [A_1 | ... | A_K]; embeddings stay in HBM. */
int n2v2r_uase(n2v2r_handle* h, int d, const n2v2r_eig_opts* opts, n2v2r_eig_stats* stats);
int n2v2r_get_embedding(n2v2r_handle* h, float* Y /* K*N*d, row-major [k][n][j] */);
int n2v2r_get_left_embedding(n2v2r_handle* h, float* X /* N*d */);
int n2v2r_get_singular_values(n2v2r_handle* h, double* s /* d, descending */);
int n2v2r_set_embedding(n2v2r_handle* h, int num_layers, int64_t n, int d, const float* Y);

/* fit-and-rank tail: distances for every (comparison, dim, metric) column and their Borda
 * aggregate, all device-resident.  Columns: dims outer, metrics inner, cosine skipped at dim 1.
 * method: N2V2R_AGG_BORDA (the only aggregation, model.py:179-183) or N2V2R_AGG_NONE
 * (distances only; n2v2r_get_borda then returns N2V2R_ERR_NOT_READY). */
int n2v2r_rank(n2v2r_handle* h, int strategy, const int* dims, int n_dims, const int* metrics,
               int n_metrics, int method, int* n_comparisons, int* n_cols);
int n2v2r_get_distances(n2v2r_handle* h, int comparison, double* D /* C*N, column-major */);
int n2v2r_get_borda(n2v2r_handle* h, int comparison, int64_t* borda /* N, node order */);
int n2v2r_rank_timing(n2v2r_handle* h, double* ms_distances, double* ms_borda);

/* host-array seams */
int n2v2r_pairwise_distances(n2v2r_handle* h, const double* m1, const double* m2, int64_t n,
                             int dim, int metric, double* out);
int n2v2r_borda_columns(n2v2r_handle* h, const double* D /* C*N column-major */, int64_t n,
                        int n_cols, int64_t* borda);
int n2v2r_column_sums(n2v2r_handle* h, int k, float* out /* N */);
/* n2v2r_borda_columns with the reference's tie order within the caller's reach
 * (aggregate_transform, model.py:167-185).  The GPU sort is stable: equal values rank by
 * ascending node index.  The reference sorts each column with pandas
 * Series.sort_values(ascending=False) = numpy argsort(kind='quicksort') between two reversals
 * (model.py:173-174), whose order of EQUAL values is implementation-defined (x86-simd-sort on
 * AVX-512 hosts); on columns without exact ties every correct descending sort agrees.
 *   tied (optional, n_cols int32 out): 1 where the column holds two equal non-NaN values
 *     (-0 == +0), i.e. where its descending order is not unique; 0 elsewhere.
 *   given_cols / given_orders (optional, n_given columns): columns whose descending order the
 *     caller supplies (given_orders: n_given x n int32, row g = the node indices of column
 *     given_cols[g] best first, a permutation of 0..n-1; N2V2R_ERR_BAD_ARG otherwise) instead of
 *     the stable GPU order.  The Python front-end passes pandas' order for the tied columns only.
 * n <= 2^31 - 1. */
int n2v2r_borda_columns_ex(n2v2r_handle* h, const double* D /* C*N column-major */, int64_t n,
                           int n_cols, const int32_t* given_cols, int n_given,
                           const int32_t* given_orders, int64_t* borda, int32_t* tied);

/* bipartite projection of a non-square layer (preprocessing_utils.py:16-32): out = W^T W
 * (n x n) when on_columns, else W W^T (m x m), for a host row-major m x n fp64 W; fp64
 * arithmetic (fp64 MFMA) as the reference's float64 np.matmul, exactly symmetric output. */
int n2v2r_project(n2v2r_handle* h, int64_t m, int64_t n, const double* W, int on_columns,
                  double* out);

/* device sync */
int n2v2r_synchronize(n2v2r_handle* h);

/* Diagnostic entry points (kernel timings, single stages for tests) are declared in
 * n2v2r_diag.h: they are not part of the drop-in API. */

#ifdef __cplusplus
}
#endif

#endif /* N2V2R_H */

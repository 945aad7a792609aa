/* n2v2r_diag.h -- diagnostic entry points of libn2v2r_hip.so (kernel timings and single solver
 * stages for tests and the roofline); not part of the drop-in API in n2v2r.h and with no
 * reference counterpart.  Same conventions as n2v2r.h. */
#ifndef N2V2R_DIAG_H
#define N2V2R_DIAG_H

#include "n2v2r.h"

#ifdef __cplusplus
extern "C" {
#endif

/* SpMM kernel alone (tests + roofline): Y = A_k X (transpose = 0) or A_k^T X (1) for a host
 * N x b panel X (b = 8, 16, 32 or 64), timed with HIP events on the engine stream over `reps`
 * launches after one warm-up.  avg_ms = mean launch duration; algo_bytes = SURVEY 8(d) bytes
 * per launch (8 nnz + 4 (N+1) + 8 N b).  On a partitioned handle A_k means this rank's rows:
 * X is the global N x b panel, Y its n_local x b rows, bytes 8 nnz_loc + 4 (n_loc+1) +
 * 4 (N + n_loc) b.  Y may be NULL. */
int n2v2r_bench_spmm(n2v2r_handle* h, int k, int transpose, int b, int reps, const float* X,
                     float* Y, double* avg_ms, double* algo_bytes);
/* The flat-window tiled SpMM of layer k (A_k X, or A_k^T X) at panel width b = 8 with nb column
 * blocks (0: panel blocks of <= 2 MB, at most 32), one-GPU handles; Y (optional, n x 8) receives
 * the product.  N2V2R_ERR_BAD_ARG when the layer cannot take packed blocks. */
int n2v2r_bench_spmm_tiled(n2v2r_handle* h, int k, int transpose, int b, int nb, int reps,
                           const float* X, float* Y, double* avg_ms);

/* 1 when UASE (and n2v2r_bench_spmm) use a column-block SpMM at panel width b on this handle's
 * layers, else 0: b = 8 CSR panels beyond 8 MB (no upper bound) take the flat-window tiled form
 * (each layer's entries regrouped into column blocks of <= 2 MB of panel, 4..32 blocks chosen
 * automatically, one launch per SpMM stage walking the blocks in phases with LDS accumulators);
 * env N2V2R_SPMM_CB=1/0 forces / forbids column blocks. */
int n2v2r_spmm_col_blocks(const n2v2r_handle* h, int b);

/* Rayleigh-Ritz stage alone (tests): top-p eigenpairs of a host symmetric c x c fp64 matrix H
 * (3 <= c <= 768) through UASE's own path, all on the GPU (Householder tridiagonalisation,
 * bisection + inverse iteration on the tridiagonal, compact-WY back-transform).  w: p eigenvalues, descending; S: c x p
 * row-major fp32 eigenvectors (the Ritz coefficients UASE consumes). */
int n2v2r_rr_top(n2v2r_handle* h, int c, const double* H, int p, double* w, float* S);

/* Banded Rayleigh-Ritz stage alone (tests; block width 8, c <= 512, kp + 8 <= 192): the
 * projected matrix of a Krylov-Schur cycle given as UASE keeps it.  Basis order [X (kp
 * columns, diagonal theta_prev), E, Z_2, ...] in 8-wide blocks; hband holds band column
 * j0 = kp/8 ([X E]^T M E, (kp+8) x 8 row-major) at offset 0, then for every later block j the
 * 16 x 8 matrix [Q_{j-1} Q_j]^T M Q_j.  Entries outside the band (half-bandwidth 8) are taken
 * as zero.  Same outputs as n2v2r_rr_top. */
int n2v2r_rr_band_top(n2v2r_handle* h, int c, int kp, const double* hband, int64_t hband_len,
                      const double* theta_prev, int p, double* w, float* S);

/* Layer bytes each rank copied host -> device so far (one-GPU handle: one entry): row pointers,
 * column indices and values of every layer ingest, into per_rank[0 .. min(W, cap)).  Returns the
 * rank count W.  A multi-GPU handle slices layers on the host, so each rank's figure is about
 * 1/W of the layers' bytes (2/W for directed layers: rows of A and of A^T). */
int n2v2r_h2d_layer_bytes(const n2v2r_handle* h, int64_t* per_rank, int cap);

#ifdef __cplusplus
}
#endif

#endif /* N2V2R_DIAG_H */

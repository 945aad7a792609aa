// CSR ingest on the GPU: column-index range check, unweighted-layer detection, transpose and
// symmetry detection (replaces the host transpose / comparison that n2v2r_set_layer_csr ran
// before; the reference converts each layer with scipy's csc_matrix inside its fit,
// model.py:53, and keeps A_k^T implicitly through the unfolded matrix's transpose).
//
// Transpose: every entry (r, c) becomes a 64-bit key c << 32 | r with its entry index as the
// payload; a stable LSD radix sort over the column digits only (the entries arrive in row
// order, so ties keep ascending r) gives A^T in CSR order with every transposed row sorted by
// source row -- the same output as a serial counting sort.  Row pointers of A^T come from the
// boundaries of the sorted column keys (no atomics, no scan).  Symmetry: A == A^T entry by entry
// (row pointers, columns, float == on values, as the host check did) once A's rows are sorted;
// an unsorted A is compared through (A^T)^T.
#include "common.h"

// One wave per row: flags bit 0 = a column index outside [0, n), bit 1 = a value != 1.0f,
// bit 2 = a row whose column indices are not ascending.  keys / idx (optional) receive the
// transpose sort's input.
__global__ __launch_bounds__(256) void csr_scan_kernel(const int64_t* __restrict__ ip,
                                                       const int32_t* __restrict__ ix,
                                                       const float* __restrict__ dv, int64_t n_rows,
                                                       int64_t n_cols, uint64_t* __restrict__ keys,
                                                       int32_t* __restrict__ idx,
                                                       unsigned* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  unsigned f = 0;
  for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n_rows;
       r += nw) {
    const int64_t p0 = ip[r], p1 = ip[r + 1];
    for (int64_t p = p0 + lane; p < p1; p += 64) {
      const int32_t c = ix[p];
      const bool bad = c < 0 || (int64_t)c >= n_cols;
      f |= bad ? 1u : 0u;
      f |= (dv[p] != 1.0f) ? 2u : 0u;
      if (p > p0 && ix[p - 1] > c) f |= 4u;
      if (keys) {
        keys[p] = ((uint64_t)(uint32_t)(bad ? 0 : c) << 32) | (uint64_t)(uint32_t)r;
        idx[p] = (int32_t)p;
      }
    }
  }
  // one atomic per wave (flags are sticky bits, the order does not matter)
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) f |= (unsigned)__shfl_xor((int)f, m, 64);
  if (lane == 0 && f) atomicOr(flags, f);
}

// A^T from the sorted keys: entry q is (column c = key >> 32, source row r = key & 0xFFFFFFFF);
// row pointers from the boundaries between consecutive columns.
__global__ __launch_bounds__(256) void csr_from_sorted_kernel(const uint64_t* __restrict__ keys,
                                                              const int32_t* __restrict__ idx,
                                                              const float* __restrict__ dv,
                                                              int64_t nnz, int64_t n_cols,
                                                              int64_t* __restrict__ tp,
                                                              int32_t* __restrict__ tx,
                                                              float* __restrict__ td) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nnz) return;
  const uint64_t k = keys[q];
  const int64_t c = (int64_t)(k >> 32);
  tx[q] = (int32_t)(uint32_t)(k & 0xFFFFFFFFull);
  if (td) td[q] = dv[idx[q]];
  const int64_t prev = q > 0 ? (int64_t)(keys[q - 1] >> 32) : -1;
  for (int64_t x = prev + 1; x <= c; ++x) tp[x] = q;
  if (q == nnz - 1)
    for (int64_t x = c + 1; x <= n_cols; ++x) tp[x] = nnz;
}

// mismatch flag: bit 0 set when two CSRs with the same row count differ (row pointers, column
// indices, or values by float ==)
__global__ __launch_bounds__(256) void csr_compare_kernel(const int64_t* __restrict__ ap,
                                                          const int32_t* __restrict__ ax,
                                                          const float* __restrict__ av,
                                                          const int64_t* __restrict__ bp,
                                                          const int32_t* __restrict__ bx,
                                                          const float* __restrict__ bv,
                                                          int64_t n_rows, int64_t nnz,
                                                          unsigned* __restrict__ flag) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nt = (int64_t)gridDim.x * blockDim.x;
  bool diff = false;
  for (int64_t i = t; i <= n_rows; i += nt) diff |= ap[i] != bp[i];
  for (int64_t p = t; p < nnz; p += nt) diff |= (ax[p] != bx[p]) || !(av[p] == bv[p]);
  const unsigned long long m = __ballot(diff);
  if ((threadIdx.x & 63) == 0 && m) atomicOr(flag, 1u);
}

// rows [r0, r0 + nr) of a device CSR: row pointers rebased to 0
__global__ void csr_rebase_kernel(const int64_t* __restrict__ ip, int64_t r0, int64_t nr,
                                  int64_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r <= nr) out[r] = ip[r0 + r] - ip[r0];
}

static unsigned grid_for(int64_t work, int per_block, unsigned cap) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

extern "C" hipError_t n2v2r_launch_csr_scan(const int64_t* ip, const int32_t* ix, const float* dv,
                                            int64_t n_rows, int64_t n_cols, uint64_t* keys,
                                            int32_t* idx, unsigned* flags, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(csr_scan_kernel, dim3(grid_for(n_rows, 4, 65536)), dim3(256), 0, stream, ip,
                     ix, dv, n_rows, n_cols, keys, idx, flags);
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_csr_from_sorted(const uint64_t* keys, const int32_t* idx,
                                                   const float* dv, int64_t nnz, int64_t n_cols,
                                                   int64_t* tp, int32_t* tx, float* td,
                                                   hipStream_t stream) {
  if (nnz <= 0) return hipMemsetAsync(tp, 0, sizeof(int64_t) * (n_cols + 1), stream);
  hipLaunchKernelGGL(csr_from_sorted_kernel, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0,
                     stream, keys, idx, dv, nnz, n_cols, tp, tx, td);
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_csr_compare(const int64_t* ap, const int32_t* ax,
                                               const float* av, const int64_t* bp,
                                               const int32_t* bx, const float* bv, int64_t n_rows,
                                               int64_t nnz, unsigned* flag, hipStream_t stream) {
  const int64_t work = nnz > n_rows ? nnz : n_rows + 1;
  hipLaunchKernelGGL(csr_compare_kernel, dim3(grid_for(work, 256 * 8, 8192)), dim3(256), 0,
                     stream, ap, ax, av, bp, bx, bv, n_rows, nnz, flag);
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_csr_rebase(const int64_t* ip, int64_t r0, int64_t nr,
                                              int64_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(csr_rebase_kernel, dim3((unsigned)((nr + 1 + 255) / 256)), dim3(256), 0,
                     stream, ip, r0, nr, out);
  return hipGetLastError();
}

// Row order of a partitioned layer's column share A[:, own rows] (layers.cpp ensure_colcsr) made
// chunk-major for the pipelined reduce-scatter (solver.cpp apply_M_rs): global row j = g npad + i
// (rank g's local row i, chunk c = i / rc of nch) moves to position
// c W rc + g rows_c + (i - c rc), rows_c = min(rc, npad - c rc), so chunk c's W row blocks are one
// contiguous range of the product -- what one reduce-scatter of that chunk sends.  Applied to the
// col << 32 | row keys before the sort by column.
__global__ void chunk_major_keys_kernel(uint64_t* __restrict__ keys, int64_t nnz, int64_t npad,
                                        int W, int64_t rc) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz;
       e += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[e];
    const int64_t j = (int64_t)(k >> 32);
    const int64_t g = j / npad, i = j - g * npad;
    const int64_t c = i / rc;
    const int64_t rows_c = rc < npad - c * rc ? rc : npad - c * rc;
    const int64_t pos = c * W * rc + g * rows_c + (i - c * rc);
    keys[e] = ((uint64_t)pos << 32) | (k & 0xFFFFFFFFull);
  }
}

extern "C" hipError_t n2v2r_launch_chunk_major_keys(uint64_t* keys, int64_t nnz, int64_t npad,
                                                   int W, int64_t rc, hipStream_t stream) {
  if (nnz <= 0) return hipSuccess;
  if (W < 1 || rc < 1 || npad < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(chunk_major_keys_kernel, dim3(grid_for(nnz, 256, 8192)), dim3(256), 0, stream,
                     keys, nnz, npad, W, rc);
  return hipGetLastError();
}

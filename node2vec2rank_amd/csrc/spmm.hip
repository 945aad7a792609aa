// CSR x dense-panel SpMM for the Gram operator M = sum_k A_k A_k^T (gfx950, wave64).
//
// Layout: CSR per layer (int64 row pointers, int32 columns, fp32 values) resident in HBM;
// dense panels row-major N x B fp32 (B = 32 or 64: one 128-B / 256-B line per row).
// One wave owns one output row.  The row's column indices and values are loaded once,
// coalesced, 64 at a time, and broadcast with __shfl; the wave then gathers NPS = 64 / (B/4)
// panel rows per step, each by B/4 lanes with one 16-B load per lane, so a panel row is one
// coalesced 128/256-B segment.  Partial sums of the NPS lane groups are folded with xor
// shuffles and the B/4 lanes of group 0 store the output row with 16-B stores.
// There is no LDS staging: an ER/co-expression row's columns are uniformly random, so a
// workgroup has no panel reuse to stage; reuse comes from L2 / Infinity Cache.
//
// Algorithmic bytes per launch: 8*nnz + 4*(N+1) + 4*N*B (read) + 4*N*B (write).
#include "common.h"

#define SPMM_MAX_LAYERS 8

struct SpmmArgs {
  CsrDev A[SPMM_MAX_LAYERS];
  const float* X[SPMM_MAX_LAYERS];
  float* Y[SPMM_MAX_LAYERS];
  int64_t ldx;
  int64_t ldy;
  int K;                 // layers in this launch
  int sum;               // 1: Y[0] = sum_k A_k X_k ; 0: Y[k] = A_k X_k (grid.y = k)
  const float* colscale; // optional per-column scale of the output (nullptr = none)
};

template <int B>
__device__ __forceinline__ void spmm_row_accumulate(const CsrDev& A, const float* __restrict__ X,
                                                    int64_t ldx, int64_t row, int lane,
                                                    f32x4& acc) {
  constexpr int LPN = B / 4;      // lanes per gathered panel row
  constexpr int NPS = 64 / LPN;   // panel rows gathered per step
  const int grp = lane / LPN;
  const int sub = lane % LPN;
  const int64_t beg = A.indptr[row];
  const int64_t end = A.indptr[row + 1];
  for (int64_t base = beg; base < end; base += 64) {
    const int nn = (int)((end - base) < 64 ? (end - base) : 64);
    int colv = 0;
    float valv = 0.f;
    if (lane < nn) {
      colv = A.indices[base + lane];
      valv = A.data[base + lane];
    }
    const int steps = (nn + NPS - 1) / NPS;
    int s = 0;
    for (; s + 4 <= steps; s += 4) {
      int c0 = __shfl(colv, (s + 0) * NPS + grp, 64);
      int c1 = __shfl(colv, (s + 1) * NPS + grp, 64);
      int c2 = __shfl(colv, (s + 2) * NPS + grp, 64);
      int c3 = __shfl(colv, (s + 3) * NPS + grp, 64);
      float v0 = __shfl(valv, (s + 0) * NPS + grp, 64);
      float v1 = __shfl(valv, (s + 1) * NPS + grp, 64);
      float v2 = __shfl(valv, (s + 2) * NPS + grp, 64);
      float v3 = __shfl(valv, (s + 3) * NPS + grp, 64);
      f32x4 x0 = *reinterpret_cast<const f32x4*>(X + (int64_t)c0 * ldx + sub * 4);
      f32x4 x1 = *reinterpret_cast<const f32x4*>(X + (int64_t)c1 * ldx + sub * 4);
      f32x4 x2 = *reinterpret_cast<const f32x4*>(X + (int64_t)c2 * ldx + sub * 4);
      f32x4 x3 = *reinterpret_cast<const f32x4*>(X + (int64_t)c3 * ldx + sub * 4);
      acc += v0 * x0;
      acc += v1 * x1;
      acc += v2 * x2;
      acc += v3 * x3;
    }
    for (; s < steps; ++s) {
      int c0 = __shfl(colv, s * NPS + grp, 64);
      float v0 = __shfl(valv, s * NPS + grp, 64);
      f32x4 x0 = *reinterpret_cast<const f32x4*>(X + (int64_t)c0 * ldx + sub * 4);
      acc += v0 * x0;
    }
  }
}

template <int B>
__global__ __launch_bounds__(256) void spmm_csr_panel_kernel(SpmmArgs args) {
  constexpr int LPN = B / 4;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int k0 = args.sum ? 0 : (int)blockIdx.y;
  const int64_t n = args.A[k0].n_rows;
  if (row >= n) return;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (args.sum) {
    for (int k = 0; k < args.K; ++k)
      spmm_row_accumulate<B>(args.A[k], args.X[k], args.ldx, row, lane, acc);
  } else {
    spmm_row_accumulate<B>(args.A[k0], args.X[k0], args.ldx, row, lane, acc);
  }
#pragma unroll
  for (int m = LPN; m < 64; m <<= 1) {
    acc.x += __shfl_xor(acc.x, m, 64);
    acc.y += __shfl_xor(acc.y, m, 64);
    acc.z += __shfl_xor(acc.z, m, 64);
    acc.w += __shfl_xor(acc.w, m, 64);
  }
  if (lane < LPN) {
    if (args.colscale) {
      f32x4 sc = *reinterpret_cast<const f32x4*>(args.colscale + lane * 4);
      acc *= sc;
    }
    *reinterpret_cast<f32x4*>(args.Y[k0] + row * args.ldy + lane * 4) = acc;
  }
}

extern "C" hipError_t n2v2r_launch_spmm(const SpmmArgs& args, int B, hipStream_t stream) {
  const int64_t n = args.A[0].n_rows;
  const int waves_per_block = 4;
  dim3 grid((unsigned)((n + waves_per_block - 1) / waves_per_block), args.sum ? 1 : args.K);
  dim3 block(64 * waves_per_block);
  if (B == 32)
    hipLaunchKernelGGL(spmm_csr_panel_kernel<32>, grid, block, 0, stream, args);
  else if (B == 64)
    hipLaunchKernelGGL(spmm_csr_panel_kernel<64>, grid, block, 0, stream, args);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// Column sums of a CSR layer (DeDi, model.py:282-311): out[j] = sum_i A[i][j].  fp32
// atomics would make the order run-dependent, so the engine calls this on A^T (row sums of
// the transpose = column sums) when the layer is not symmetric.
__global__ void csr_row_sums_kernel(CsrDev A, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= A.n_rows) return;
  float s = 0.f;
  for (int64_t p = A.indptr[row] + lane; p < A.indptr[row + 1]; p += 64) s += A.data[p];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (lane == 0) out[row] = s;
}

extern "C" hipError_t n2v2r_launch_row_sums(const CsrDev& A, float* out, hipStream_t stream) {
  dim3 grid((unsigned)((A.n_rows + 3) / 4));
  hipLaunchKernelGGL(csr_row_sums_kernel, grid, dim3(256), 0, stream, A, out);
  return hipGetLastError();
}

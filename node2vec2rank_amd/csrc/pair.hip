// Kernels of the solver's paired-panel mode (solver.cpp, "pair"): the Krylov basis stays in
// 8-wide blocks (every b = 8 orthogonalisation form applies unchanged), while each application of
// M = sum_k A_k A_k^T multiplies TWO blocks at once as one N x 16 panel -- the tiled SpMM at
// 64-B panel rows (spmm16_flat_kernel), which gathers a vector column at ~0.6x the cost of the
// 32-B rows of b = 8 where the gathers miss L2 (BASELINE cfg5: 5.45 vs 4.38 ms per layer launch
// for twice the columns, profiles/r06_spmm16_cfg5.jsonl).  The projected matrix of such a basis
// is banded with half-bandwidth 16; it is assembled here, densely, from the Gram rows the local
// orthogonalisation passes saved, and handed to the dense Rayleigh-Ritz (rr.hip).
#include "common.h"

// x16 (N x 16) = [za | zb] (two N x 8 blocks): one 16-B chunk per thread, 64 consecutive chunks
// of a wave = 16 rows, i.e. 512 contiguous bytes of each source block and 1 KB of x16
__global__ __launch_bounds__(256) void interleave16_kernel(const float* __restrict__ za,
                                                           const float* __restrict__ zb,
                                                           float* __restrict__ x16, int64_t n) {
  const int64_t total = n * 4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e >> 2;
    const int q = (int)(e & 3);
    const float* src = (q < 2 ? za : zb) + r * 8 + (q & 1) * 4;
    *reinterpret_cast<f32x4*>(x16 + r * 16 + q * 4) = *reinterpret_cast<const f32x4*>(src);
  }
}

extern "C" hipError_t n2v2r_launch_interleave16(const float* za, const float* zb, float* x16,
                                                int64_t n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int64_t nb = (n * 4 + 255) / 256;
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(interleave16_kernel, dim3((unsigned)nb), dim3(256), 0, stream, za, zb, x16, n);
  return hipGetLastError();
}

// Projected matrix H = Q^T M Q (c x c, fp64, row-major; zero-filled by the caller) of a paired
// basis [X | E | Krylov blocks]:
//   * H[j][j] = theta_j for the kp kept Ritz vectors (X's block is diagonal);
//   * column block s >= kry0 (the image M q_s's first, local Gram pass saved its rows
//     lo_s .. lo_s + nr_s / 8 - 1 of the basis: g_s[r][i] = q_r^T M q_{s,i}): its entries above
//     the diagonal block go to H and, mirrored, below it; the diagonal block is symmetrised; the
//     rows past it are not used (the later column that saved them as its upper part supplies
//     them), so every entry has exactly one source.
// One workgroup per saved column block; the extra last workgroup writes theta.
struct PairHCols {
  int lo[N2V2R_MAX_BLOCKS];  // first basis block of the saved rows
  int nr[N2V2R_MAX_BLOCKS];  // saved rows (a multiple of 8)
};

__global__ __launch_bounds__(256) void pair_h_assemble_kernel(const double* __restrict__ hcol,
                                                              int64_t ldcol, PairHCols d, int s0,
                                                              int ns, int kp,
                                                              const double* __restrict__ theta,
                                                              double* __restrict__ H, int c) {
  const int t = blockIdx.x;
  if (t == ns) {
    for (int j = threadIdx.x; j < kp; j += blockDim.x) H[(int64_t)j * c + j] = theta[j];
    return;
  }
  const int s = s0 + t;
  const double* g = hcol + (int64_t)t * ldcol;
  const int r0 = d.lo[t] * 8, nr = d.nr[t], cs = s * 8;
  for (int e = threadIdx.x; e < nr * 8; e += blockDim.x) {
    const int rl = e >> 3, i = e & 7;
    const int r = r0 + rl, col = cs + i;
    const double v = g[e];
    if (r < cs) {
      H[(int64_t)r * c + col] = v;
      H[(int64_t)col * c + r] = v;
    } else if (r < cs + 8) {
      const double vt = g[(cs + i - r0) * 8 + (r - cs)];  // the transposed entry, same block
      H[(int64_t)r * c + col] = 0.5 * (v + vt);
    }
  }
}

extern "C" hipError_t n2v2r_launch_pair_h_assemble(const double* hcol, int64_t ldcol,
                                                   const int* lo, const int* nr, int s0, int ns,
                                                   int kp, const double* theta, double* H, int c,
                                                   hipStream_t stream) {
  if (ns < 0 || ns > N2V2R_MAX_BLOCKS || c <= 0 || (kp > 0 && !theta)) return hipErrorInvalidValue;
  PairHCols d{};
  for (int t = 0; t < ns; ++t) {
    if (lo[t] < 0 || nr[t] < 0 || nr[t] % 8 != 0 || lo[t] * 8 + nr[t] > c ||
        (int64_t)nr[t] * 8 > ldcol || (s0 + t) * 8 + 8 > c)
      return hipErrorInvalidValue;
    d.lo[t] = lo[t];
    d.nr[t] = nr[t];
  }
  hipLaunchKernelGGL(pair_h_assemble_kernel, dim3((unsigned)ns + 1), dim3(256), 0, stream, hcol,
                     ldcol, d, s0, ns, kp, theta, H, c);
  return hipGetLastError();
}

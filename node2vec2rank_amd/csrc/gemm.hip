// Dense layers (BASELINE cfg3: K dense fp32 N x N co-expression layers): the Gram application
// of UASE becomes two dense GEMMs per layer, Z_k = A_k^T X and W = sum_k A_k Z_k, with X an
// N x b panel.  At b = 8..64 the GEMM streams A once (N^2 fp32) and does 2 N^2 b flops, i.e.
// 4..32 flop/B: HBM-bound at small b, MFMA-bound near b = 64.
//
//   dense_gemm_kernel<NT, XT>  Y[r0:r0+rows, 0:b] (+)= A[rows x kdim] X[kdim x b]:
//     v_mfma_f32_32x32x2_f32, one wave per 32 output rows x NT*32 columns, 4 waves per WG
//     (128 rows).  The 128 x 64 A tile of a round is loaded with 16-B loads, every
//     wave-instruction 4 rows x 256 B contiguous, into registers one round ahead (in flight
//     across the current round's MFMAs), then stored to LDS (row pitch 68 floats); each lane
//     reads its row's 16 consecutive k of a group from LDS (lane half h carries k 8h..8h+7, MFMA
//     m sums k = {m, 8+m}; X's k order is permuted identically).  X staged through LDS 64
//     k-rows at a time.  Split-K over
//     grid.y when the row tiles alone cannot fill the chip, fp32 partial slabs folded by
//     dense_fold_kernel.
//   transpose_kernel       32x32 LDS tiles (A^T of a directed layer, once at ingest).
//   mismatch_kernel        counts A != A^T entries (symmetry detection at ingest).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "common.h"

#define DG_KC 64  // k columns of A (rows of X) staged per LDS round
#define DG_AP (DG_KC + 4)  // padded LDS row pitch of the A tile (16-B reads conflict-free)

// A tile rows x DG_KC: thread t loads rows u * 16 + t / 16 (u = 0..7), 16 B at k = 4 (t % 16):
// every wave-instruction reads 4 rows x 256 B contiguous (the lane-per-row form read 32 rows
// x 32 B per instruction: 0.32 of HBM at cfg3).  Clamped addresses and unconditional 16-B
// loads: all eight issue as one batch (a guarded load per element compiles to a branch and a
// wait each); out-of-range rows / k are zeroed at the LDS store (dg_store_a), so the loads stay
// in flight across the MFMAs of the previous round.
__device__ __forceinline__ void dg_load_a(const float* __restrict__ A, int64_t lda, int64_t rows,
                                          int64_t tile_r0, int64_t k0, f32x4 (&v)[8]) {
  const int t = threadIdx.x;
  const int64_t kg = k0 + (t & 15) * 4;
  const int64_t kc = kg + 4 <= lda ? kg : lda - 4;  // lda % 4 == 0: always in the row
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int64_t r = tile_r0 + u * 16 + (t >> 4);
    const int64_t rc = r < rows ? r : rows - 1;
    v[u] = *reinterpret_cast<const f32x4*>(A + rc * lda + kc);
  }
}

__device__ __forceinline__ void dg_store_a(float (*as)[DG_AP], const f32x4 (&v)[8], int64_t rows,
                                           int64_t tile_r0, int64_t k0, int64_t k_end) {
  const int t = threadIdx.x;
  const int64_t kg = k0 + (t & 15) * 4;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const bool rok = tile_r0 + u * 16 + (t >> 4) < rows;
    f32x4 w = v[u];
#pragma unroll
    for (int m = 0; m < 4; ++m) w[m] = (rok && kg + m < k_end) ? w[m] : 0.f;
    *reinterpret_cast<f32x4*>(&as[u * 16 + (t >> 4)][(t & 15) * 4]) = w;
  }
}

// (Round 4, measured and not kept: X rows loaded a round ahead with the A tile and each 16-k
// group's LDS operands read before the previous group's MFMAs: 0.447 vs 0.407 ms per cfg3
// launch, profiles/r04_dense_forms.jsonl; X staged transposed, xs[column][k], so a lane reads
// its 8 consecutive k of a 16-k group as two 16-B LDS reads like its A operands: 0.40 vs 0.39
// ms per cfg3 launch.)  xs[k][column], one LDS read per MFMA.
template <int NT>
__global__ __launch_bounds__(256) void dense_gemm_kernel(const float* __restrict__ A, int64_t lda,
                                                         int64_t rows, int64_t kdim,
                                                         int64_t kper, const float* __restrict__ X,
                                                         int ldx, int b, float* __restrict__ out,
                                                         int64_t ldo, int64_t slab) {
  constexpr int XP = NT * 32 + 4;  // padded LDS row pitch of xs
  __shared__ __attribute__((aligned(16))) float xs[DG_KC][XP];
  __shared__ __attribute__((aligned(16))) float as[128][DG_AP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int64_t tile_r0 = (int64_t)blockIdx.x * 128;
  const int64_t r0 = tile_r0 + wave * 32;
  const int64_t k_begin = (int64_t)blockIdx.y * kper;
  int64_t k_end = k_begin + kper;
  if (k_end > kdim) k_end = kdim;
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{0.f};
  // one 64-k round: the A tile from `buf` (registers) and X rows into LDS, then `buf` refilled
  // with the A tile of round `kload` (in flight across this round's MFMAs)
  auto round = [&](int64_t k0, f32x4 (&buf)[8], int64_t kload) {
    const int kn = (k_end - k0) < DG_KC ? (int)(k_end - k0) : DG_KC;
    __syncthreads();  // the previous round's LDS reads are done
    dg_store_a(as, buf, rows, tile_r0, k0, k_end);
    {
      // X rows k0 .. k0 + 63: clamped unconditional loads (one batch), masked LDS stores
      constexpr int XN = DG_KC * NT * 32 / 256;
      float xv[XN];
#pragma unroll
      for (int u = 0; u < XN; ++u) {
        const int e = threadIdx.x + 256 * u;
        const int kk = e / (NT * 32), j = e % (NT * 32);
        const int64_t kr = k0 + (kk < kn ? kk : kn - 1);
        xv[u] = X[kr * ldx + (j < b ? j : b - 1)];
      }
#pragma unroll
      for (int u = 0; u < XN; ++u) {
        const int e = threadIdx.x + 256 * u;
        const int kk = e / (NT * 32), j = e % (NT * 32);
        xs[kk][j] = (kk < kn && j < b) ? xv[u] : 0.f;
      }
    }
    __syncthreads();
    if (kload < k_end) dg_load_a(A, lda, rows, tile_r0, kload, buf);
    if (r0 < rows) {
      for (int kk = 0; kk < kn; kk += 16) {
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(&as[wave * 32 + i][kk + 8 * h]);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(&as[wave * 32 + i][kk + 8 * h + 4]);
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const float av = m < 4 ? a0[m] : a1[m - 4];
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, xs[kk + 8 * h + m][t * 32 + i],
                                                          acc[t], 0, 0, 0);
        }
      }
    }
  };
  // (two A tiles in flight -- a round's loads with two rounds of MFMAs to land -- measured
  // 0.395 vs 0.394 ms per cfg3 launch: not kept)
  f32x4 nxt[8];
  if (k_begin < k_end) dg_load_a(A, lda, rows, tile_r0, k_begin, nxt);
  for (int64_t k0 = k_begin; k0 < k_end; k0 += DG_KC) round(k0, nxt, k0 + DG_KC);
  if (r0 >= rows) return;
  float* o = out + (int64_t)blockIdx.y * slab;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = t * 32 + i;
    if (col >= b) continue;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t rr = r0 + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (rr < rows) o[rr * ldo + col] = acc[t][q];
    }
  }
}

// Y[r][j] = beta * Y[r][j] + s[j] * sum_s P[s][r][j]   (s = colscale, or 1)
__global__ void dense_fold_kernel(const float* __restrict__ P, int nsplit, int64_t slab,
                                  int64_t rows, int b, float* __restrict__ Y, int64_t ldy,
                                  float beta, const float* __restrict__ colscale) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * b) return;
  const int64_t r = e / b;
  const int j = (int)(e % b);
  float s = 0.f;
  for (int q = 0; q < nsplit; ++q) s += P[q * slab + r * b + j];
  if (colscale) s *= colscale[j];
  float* y = Y + r * ldy + j;
  *y = (beta != 0.f ? beta * *y : 0.f) + s;
}

// Y (rows x b, ld ldy) = beta * Y + colscale .* (A[rows x kdim] X[kdim x b]).  `work` holds the
// split-K slabs (>= nsplit * rows * b floats; nullptr forces nsplit = 1 and a direct write,
// allowed only with beta == 0 and no colscale).
extern "C" hipError_t n2v2r_launch_dense_gemm(const float* A, int64_t lda, int64_t rows,
                                              int64_t kdim, const float* X, int ldx, int b,
                                              float* Y, int64_t ldy, float beta,
                                              const float* colscale, float* work,
                                              size_t work_elems, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  if (b < 1 || b > 64 || lda % 4 != 0 || ((uintptr_t)A & 15) != 0) return hipErrorInvalidValue;
  const int64_t tiles = (rows + 127) / 128;
  // split K until ~2 workgroups per CU, 256-aligned k ranges, slabs within `work`
  int64_t nsplit = 1;
  if (work) {
    nsplit = (512 + tiles - 1) / tiles;
    const int64_t kmax = (kdim + 255) / 256;
    if (nsplit > kmax) nsplit = kmax;
    if (nsplit < 1) nsplit = 1;
    const int64_t cap = (int64_t)(work_elems / (size_t)(rows * b));
    if (nsplit > cap) nsplit = cap;
    if (nsplit < 1) return hipErrorInvalidValue;
  } else if (beta != 0.f || colscale) {
    return hipErrorInvalidValue;
  }
  int64_t kper = (kdim + nsplit - 1) / nsplit;
  kper = (kper + 15) & ~(int64_t)15;
  nsplit = (kdim + kper - 1) / kper;
  float* dst = work ? work : Y;
  const int64_t ldo = work ? b : ldy;
  const int64_t slab = work ? rows * b : 0;
  const dim3 grid((unsigned)tiles, (unsigned)nsplit);
#define DG_LAUNCH(NT)                                                                          \
  hipLaunchKernelGGL((dense_gemm_kernel<NT>), grid, dim3(256), 0, stream, A, lda, rows, kdim, kper, \
                     X, ldx, b, dst, ldo, slab)
  if (b <= 32)
    DG_LAUNCH(1);
  else
    DG_LAUNCH(2);
#undef DG_LAUNCH
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !work) return e;
  const int64_t elems = rows * b;
  hipLaunchKernelGGL(dense_fold_kernel, dim3((unsigned)((elems + 255) / 256)), dim3(256), 0, stream,
                     work, (int)nsplit, slab, rows, b, Y, ldy, beta, colscale);
  return hipGetLastError();
}

// ---- Y = B^T X with B row-major (round 4): the stored matrix is the MFMA's B operand ---------
// Y[n][j] = sum_k B[k][n] X[k][j] (j < b <= 32).  For a symmetric layer B = A (Y = A X); for a
// directed one the engine passes the other stored copy (A X = (A^T)^T X).  Computed as
// Y^T = X^T B: v_mfma_f32_32x32x2_f32 takes X^T as its A operand (lane l: X[k0 + l/32][l%32],
// one 4-B load per k pair shared by 4 MFMAs) and B in its natural row-major layout as the B
// operand: lane l loads B[k0 + l/32][n0 + 4 (l%32) .. + 3] with ONE 16-B load (lanes 0-31 one
// 512-B run of row k, lanes 32-63 of row k + 1) and feeds element q to MFMA q, whose output
// column c stands for n = n0 + 4c + q.  No LDS on the way in: A streams from HBM straight into
// the MFMA operands, D k pairs per stage, double-buffered (the next stage's loads in flight
// across this stage's 4 D MFMAs).  A wave owns 128 n x 32 j (4 accumulators) over a quarter of
// its workgroup's k range; the 4 quarters are summed in LDS in fixed order, split-K slabs over
// grid.y are folded by dense_fold_kernel (deterministic).  dense_gemm_kernel above stages A
// through LDS as the A operand: 0.39 ms per cfg3 launch (0.50 of HBM, MFMA busy 0.45).
// k pairs per load stage: 6 (cfg3 fit 212.1 ms) against 8 (215.9), 4 (217.4 at 3 workgroups per
// CU), 12 (222.8), 16 at one workgroup per CU (238.1); 3 workgroups per CU at 6 / 8: 212.9 /
// 219.8 (profiles/r05_dense_tn_stages.txt)
#ifndef DTN_D
#define DTN_D 6
#endif
#ifndef DTN_OCC
#define DTN_OCC 2  // workgroups per CU the register budget is sized for
#endif
template <int DT_D, int OCC, bool NTB>
__global__ __launch_bounds__(256, OCC) void dense_tn_kernel(const float* __restrict__ B, int64_t ldb,
                                                          int64_t ncols, int64_t kdim, int64_t kper,
                                                          const float* __restrict__ X, int ldx,
                                                          int b, float* __restrict__ out,
                                                          int64_t ldo, int64_t slab) {
  extern __shared__ float red[];  // [128 n][33]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar bases
  const int c = lane & 31, h = lane >> 5;
  const int64_t n0 = (int64_t)blockIdx.x * 128;
  const int64_t wk0 = (int64_t)blockIdx.y * kper;
  int64_t wk1 = wk0 + kper;
  if (wk1 > kdim) wk1 = kdim;
  // this wave's quarter of the workgroup's k range, in k pairs
  const int64_t npair_wg = (wk1 - wk0 + 1) / 2;
  const int64_t qp = (npair_wg + 3) / 4;
  const int64_t kb = wk0 + 2 * qp * wave;
  int64_t ke = kb + 2 * qp;
  if (ke > wk1) ke = wk1;
  const int64_t npair = ke > kb ? (ke - kb + 1) / 2 : 0;
  // column of this lane's 16-B B load (clamped into the row: ldb % 4 == 0, ldb >= ncols)
  int64_t nc = n0 + 4 * c;
  if (nc > ldb - 4) nc = ldb - 4;
  const int jc = c < b ? c : b - 1;
  // wave-uniform bases (scalar registers) + 32-bit per-lane element offsets: one VGPR per load
  // address instead of a 64-bit pair (the host checks (kper + 1) * ldb < 2^32)
  const float* Bw = B + kb * ldb + n0;  // (kb, n0: wave-uniform)
  const float* Xw = X + kb * ldx;
  const uint32_t ncl = (uint32_t)(nc - n0);
  const int krel_max = (int)(ke - kb) - 1;
  const uint32_t lb = (uint32_t)ldb, lx = (uint32_t)ldx;
  f32x16 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = f32x16{0.f};
  f32x4 bb0[DT_D], bb1[DT_D];
  float xb0[DT_D], xb1[DT_D];
  auto load = [&](f32x4 (&bb)[DT_D], float (&xb)[DT_D], int64_t p0) {
#pragma unroll
    for (int u = 0; u < DT_D; ++u) {
      const int kr = (int)(2 * (p0 + u)) + h;
      const uint32_t krc = (uint32_t)(kr < krel_max ? kr : krel_max);  // clamped: one batch
      const f32x4* src = reinterpret_cast<const f32x4*>(Bw + (krc * lb + ncl));
      bb[u] = NTB ? __builtin_nontemporal_load(src) : *src;
      xb[u] = Xw[krc * lx + (uint32_t)jc];  // raw: masked at the use (a select here becomes a
                                            // branch with a wait; a multiply, a wait per load)
    }
  };
  auto compute = [&](const f32x4 (&bb)[DT_D], const float (&xb)[DT_D], int64_t p0) {
#pragma unroll
    for (int u = 0; u < DT_D; ++u) {
      // X is finite (clamped loads of valid rows): 0 * x = 0 past the range
      const float xm = xb[u] * ((kb + 2 * (p0 + u) + h < ke && c < b) ? 1.f : 0.f);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(xm, bb[u][q], acc[q], 0, 0, 0);
    }
  };
  // sched_barrier(0) after each batch of loads: without it the scheduler sinks every load to
  // just before its MFMAs (load, wait vmcnt(0), 4 MFMAs: no load in flight across MFMAs)
  // (Three stages in flight, triple-buffered: 0.364 vs 0.348 ms per cfg3 launch, fit 240 vs
  // 237 ms: not kept.)
  // No early exit between the two halves: a conditional use lets the optimiser sink the next
  // half's loads below this half's MFMAs; past npair the k pairs are masked to zero instead
  // (at most DT_D wasted k pairs per wave).
  if (npair > 0) {
    load(bb0, xb0, 0);
    __builtin_amdgcn_sched_barrier(0);
    for (int64_t p0 = 0; p0 < npair; p0 += 2 * DT_D) {
      load(bb1, xb1, p0 + DT_D);
      __builtin_amdgcn_sched_barrier(0);
      compute(bb0, xb0, p0);
      load(bb0, xb0, p0 + 2 * DT_D);
      __builtin_amdgcn_sched_barrier(0);
      compute(bb1, xb1, p0 + DT_D);
    }
  }
  // acc[q][r] at lane l: Y^T[j][c] with j = (r & 3) + 8 (r >> 2) + 4 h, n = n0 + 4 c + q.
  // The 4 waves' tiles summed in wave order through ONE 128 x 33 LDS buffer (17 KB: the LDS
  // does not cap the workgroups per CU)
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float& dst = red[(4 * c + q) * 33 + (r & 3) + 8 * (r >> 2) + 4 * h];
          dst = w == 0 ? acc[q][r] : dst + acc[q][r];
        }
    }
    __syncthreads();
  }
  float* o = out + (int64_t)blockIdx.y * slab;
  for (int e = threadIdx.x; e < 128 * 32; e += 256) {
    const int nl = e >> 5, j = e & 31;
    const int64_t n = n0 + nl;
    if (n < ncols && j < b) o[n * ldo + j] = red[nl * 33 + j];
  }
}

// Y (ncols x b, ld ldy) = beta * Y + colscale .* (B[kdim x ncols]^T X[kdim x b]), b <= 32;
// `work` holds the split-K slabs (nsplit * ncols * b floats).  hipErrorNotSupported when the
// form does not apply (the caller then takes n2v2r_launch_dense_gemm on the other copy).
extern "C" hipError_t n2v2r_launch_dense_tn(const float* B, int64_t ldb, int64_t ncols,
                                           int64_t kdim, const float* X, int ldx, int b, float* Y,
                                           int64_t ldy, float beta, const float* colscale,
                                           float* work, size_t work_elems, hipStream_t stream) {
  if (ncols <= 0) return hipSuccess;
  if (b < 1 || b > 32 || !work || ldb % 4 != 0 || ldb < ncols || ((uintptr_t)B & 15) != 0 ||
      kdim < 2 || (double)(kdim + 1) * (double)(ldb > ldx ? ldb : ldx) >= 4294967296.0)
    return hipErrorNotSupported;  // (32-bit element offsets inside a wave's k range)
  const int64_t tiles = (ncols + 127) / 128;
  // ~2048 workgroups (4 rounds of 2 per CU), at least 512 k per workgroup, slabs within work.
  // (Measured and not kept: 16 / 24 k pairs per stage at one workgroup per CU, 512 VGPRs:
  // 0.38 ms vs 0.36 per cfg3 launch, profiles/r04_dense_forms.jsonl.)
  int64_t nsplit = (2048 + tiles / 2) / tiles;
  const int64_t kmax = kdim / 512;
  if (nsplit > kmax) nsplit = kmax;
  if (nsplit < 1) nsplit = 1;
  const int64_t cap = (int64_t)(work_elems / (size_t)(ncols * b));
  if (nsplit > cap) nsplit = cap;
  if (nsplit < 1) return hipErrorNotSupported;
  int64_t kper = (kdim + nsplit - 1) / nsplit;
  kper = (kper + 7) & ~(int64_t)7;
  nsplit = (kdim + kper - 1) / kper;
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void*)dense_tn_kernel<DTN_D, DTN_OCC, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 33 * 4);
    (void)hipGetLastError();
    return true;
  }();
  (void)attr;
  const dim3 grid((unsigned)tiles, (unsigned)nsplit);
  // the stored matrix (read once per launch, 1.6 GB per cfg3 layer) loaded non-temporally:
  // cfg3 fit 216.3 vs 219.5 ms (profiles/r05_dense_nt.jsonl)
  hipLaunchKernelGGL((dense_tn_kernel<DTN_D, DTN_OCC, true>), grid, dim3(256), 128 * 33 * sizeof(float),
                     stream, B, ldb, ncols, kdim, kper, X, ldx, b, work, (int64_t)b, ncols * b);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t elems = ncols * b;
  hipLaunchKernelGGL(dense_fold_kernel, dim3((unsigned)((elems + 255) / 256)), dim3(256), 0, stream,
                     work, (int)nsplit, ncols * b, ncols, b, Y, ldy, beta, colscale);
  return hipGetLastError();
}

// out[c][r] = in[r][c] for an (rows x cols) block, leading dimensions ldi / ldo
__global__ void transpose_kernel(const float* __restrict__ in, int64_t ldi, int64_t rows,
                                 int64_t cols, float* __restrict__ out, int64_t ldo) {
  __shared__ float t[32][33];
  const int64_t bx = (int64_t)blockIdx.x * 32, by = (int64_t)blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int64_t r = by + k, c = bx + tx;
    t[k][tx] = (r < rows && c < cols) ? in[r * ldi + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int64_t c = bx + k, r = by + tx;
    if (c < cols && r < rows) out[c * ldo + r] = t[tx][k];
  }
}

extern "C" hipError_t n2v2r_launch_transpose(const float* in, int64_t ldi, int64_t rows,
                                             int64_t cols, float* out, int64_t ldo,
                                             hipStream_t stream) {
  const dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, stream, in, ldi, rows, cols, out, ldo);
  return hipGetLastError();
}

// *count += #{(r, c) : a[r][c] != b[r][c]} over an (rows x cols) block
__global__ void mismatch_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                int64_t ld, int64_t rows, int64_t cols,
                                unsigned long long* count) {
  unsigned long long n = 0;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < rows * cols;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols, c = e % cols;
    n += (a[r * ld + c] != b[r * ld + c]) ? 1ull : 0ull;
  }
  for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o, 64);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(count, n);
}

extern "C" hipError_t n2v2r_launch_mismatch(const float* a, const float* b, int64_t ld,
                                            int64_t rows, int64_t cols, unsigned long long* count,
                                            hipStream_t stream) {
  hipLaunchKernelGGL(mismatch_kernel, dim3(2048), dim3(256), 0, stream, a, b, ld, rows, cols,
                     count);
  return hipGetLastError();
}

// ---- bipartite projection in fp64 (preprocessing_utils.py:16-32 multiplies in float64) -------
// out (r x r, row-major) = X^T X, X(k, i) = W[k * sk + i * si] (k < kd, i < r): W^T W with
// (sk, si) = (n, 1), W W^T with (1, n).  One workgroup per 64 x 64 output tile of the upper
// triangle (bj >= bi), written to both (bi, bj) and its mirror, so the result is exactly
// symmetric like numpy's syrk path for `W.T @ W`.  Four waves, each a 32 x 32 quarter as 2 x 2
// v_mfma_f64_16x16x4_f64 tiles; X staged through LDS in chunks of 16 k (loads ordered along
// whichever of k / i is contiguous in W); the tile goes back through LDS so both the tile and its
// mirror are stored as contiguous rows.
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void syrk_f64_kernel(const double* __restrict__ W, int64_t sk,
                                                       int64_t si, int64_t kd, int64_t r,
                                                       double* __restrict__ out, int64_t ldo,
                                                       int nt) {
  __shared__ double xa[16][68], xb[16][68];
  __shared__ double tt[64][65];
  int64_t idx = blockIdx.x;
  int bi = 0;
  while (idx >= nt - bi) {
    idx -= nt - bi;
    ++bi;
  }
  const int bj = bi + (int)idx;
  const int64_t i0 = (int64_t)bi * 64, j0 = (int64_t)bj * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = (wave & 1) * 32, wj = (wave >> 1) * 32;
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f64x4){0.0, 0.0, 0.0, 0.0};
  const bool irow = si == 1;  // i contiguous in W (W^T W), else k contiguous (W W^T)
  for (int64_t k0 = 0; k0 < kd; k0 += 16) {
#pragma unroll
    for (int rep = 0; rep < 4; ++rep) {
      const int e = tid + rep * 256;
      const int kk = irow ? (e >> 6) : (e & 15);
      const int ii = irow ? (e & 63) : (e >> 4);
      const int64_t k = k0 + kk, ia = i0 + ii, ja = j0 + ii;
      xa[kk][ii] = (k < kd && ia < r) ? W[k * sk + ia * si] : 0.0;
      xb[kk][ii] = (k < kd && ja < r) ? W[k * sk + ja * si] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 16; ks += 4) {
      double av[2], bv[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        av[t] = xa[ks + (lane >> 4)][wi + t * 16 + (lane & 15)];
        bv[t] = xb[ks + (lane >> 4)][wj + t * 16 + (lane & 15)];
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }
  // f64 16x16x4 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        tt[wi + a * 16 + (lane >> 4) + 4 * q][wj + b * 16 + (lane & 15)] = acc[a][b][q];
  __syncthreads();
  for (int e = tid; e < 64 * 64; e += 256) {
    const int ii = e >> 6, jj = e & 63;
    if (i0 + ii < r && j0 + jj < r) out[(i0 + ii) * ldo + j0 + jj] = tt[ii][jj];
  }
  if (bi != bj) {
    for (int e = tid; e < 64 * 64; e += 256) {
      const int jj = e >> 6, ii = e & 63;
      if (i0 + ii < r && j0 + jj < r) out[(j0 + jj) * ldo + i0 + ii] = tt[ii][jj];
    }
  }
}

extern "C" hipError_t n2v2r_launch_syrk_f64(const double* W, int64_t sk, int64_t si, int64_t kd,
                                            int64_t r, double* out, int64_t ldo,
                                            hipStream_t stream) {
  const int64_t nt = (r + 63) / 64;
  const int64_t tiles = nt * (nt + 1) / 2;
  if (r < 1 || kd < 1 || tiles > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(syrk_f64_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, W, sk, si, kd,
                     r, out, ldo, (int)nt);
  return hipGetLastError();
}

// Tall-skinny dense kernels for the block Krylov-Schur eigensolver (gfx950, wave64).
//
// Basis storage: blocks of N x W fp32 (W = 32 or 64), row-major, one allocation per block.
// Every product is cut into 32 x 32 MFMA tiles of v_mfma_f32_32x32x2_f32 (exact fp32
// products, fp32 accumulate; C/D map: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) +
// 4 (lane >> 5)).
//   ts_tn : G = A^T B   (ca x cb, reduction over N rows).  Per workgroup a chunk of rows;
//           4 waves split the chunk, their fp32 tiles are summed in fp64 through LDS and
//           written as a per-chunk fp64 partial; a second kernel sums the chunks in fixed
//           order (deterministic, no atomics).
//   ts_nn : O = alpha A G + beta C   (N x cb).  One wave per 32 output rows and ALL of the
//           output columns (so O may alias A or C: each wave reads only its own rows).
//           A rows are read as 16-B loads; the k order inside each 8-column group is
//           permuted consistently for A and G (lane half h carries columns 4h..4h+3).
//   chol_inv : one-workgroup fp64 Cholesky G = R^T R (+shift on breakdown) and R^{-1},
//           flagging rank-deficient columns; rows of those columns are refilled with
//           random values by fill_flagged so the next CGS pass can orthogonalise them.
#include "common.h"

// Breakdown handling of the Cholesky-QR passes.  The pivot p of column j is the squared norm of
// Z_j - Q C_j by Pythagoras (Z_j^T Z_j - C_j^T C_j), which carries an error of ~1e-8 .. 1e-7 of
// zz = Z_j^T Z_j (the fp32 data under the fp64 Gram, the basis's own loss of orthogonality).
// Below PIP_CANCEL * zz (a norm ratio of 1e-3) p is not trusted: the column is scaled by the
// clamped pivot PIP_CANCEL * zz instead (its remainder, legitimate or rounding noise, is KEPT,
// at a norm of at most ~1), the column is marked cancelled, and the next pass -- whose Gram is
// explicit for it -- normalises it.  A lazy cycle whose block went to its SpMM with a cancelled
// column is expanded again with every full pass first (the sticky flag); a pass that cancels
// asks for the pass after it (any_flag).  Refilled with random values (flagged) are only columns
// that are zero (or not finite) before the projection.  Discarding a small but legitimate
// remainder breaks the Krylov-Schur relation the lean images rely on (a converging Ritz vector
// lost its residual direction for good: BASELINE cfg3 stalled at 4e-4), and normalising an
// untrusted pivot made non-orthonormal basis vectors (an exhausted Krylov space: the rank-8
// lowrank_exact layers, whose images of the second block are rounding noise).
#ifndef PIP_CANCEL
#define PIP_CANCEL 1e-6
#endif

#include <algorithm>
#include <cstdlib>
#include <cstring>

// ----------------------------------------------------------------------------- helpers
// N(0,1) deviate from a counter (Box-Muller on two splitmix64 draws)
__device__ __forceinline__ float counter_normal(uint64_t seed, uint64_t ctr) {
  const uint64_t h1 = splitmix64(seed ^ ctr * 0x2545F4914F6CDD1Dull);
  const uint64_t h2 = splitmix64(h1);
  const double u1 = ((h1 >> 11) + 1.0) * (1.0 / 9007199254740993.0);
  const double u2 = (h2 >> 11) * (1.0 / 9007199254740992.0);
  return (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
}

// ----------------------------------------------------------------------------- ts_tn
#define TN_WAVES 4
#define TN_FLUSH 1024  // rows per fp32 partial sum before it is added to the fp64 total

// Column `col` of a block list (nullptr past the last column): per lane, so a 32-wide tile may
// span several 8/16-wide blocks.
__device__ __forceinline__ const float* blk_col_ptr(const BlockList& L, int col) {
  if (col >= L.count * L.width) return nullptr;
  return L.blk[col / L.width] + (col % L.width);
}

__global__ __launch_bounds__(256) void ts_tn_kernel(BlockList A, BlockList B, int64_t n,
                                                    int64_t rows_per_chunk, int ntj,
                                                    double* __restrict__ partial,
                                                    const int* cond) {
  if (cond && *cond == 0) return;
  __shared__ double red[TN_WAVES][16][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tile = blockIdx.y;
  const int ti = tile / ntj, tj = tile % ntj;
  const int ca = A.count * A.width, cb = B.count * B.width;
  const int i0 = ti * 32, j0 = tj * 32;
  const float* pa = blk_col_ptr(A, i0 + (lane & 31));
  const float* pb = blk_col_ptr(B, j0 + (lane & 31));
  // lanes past the last column read a valid row of column 0 and multiply by zero
  const float ma = pa ? 1.f : 0.f, mb = pb ? 1.f : 0.f;
  if (!pa) pa = A.blk[0];
  if (!pb) pb = B.blk[0];
  const int64_t lda = A.width, ldb = B.width;
  const int h = lane >> 5;
  const int64_t c0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t c1 = c0 + rows_per_chunk;
  if (c1 > n) c1 = n;
  const int64_t per_wave = (rows_per_chunk + TN_WAVES - 1) / TN_WAVES;
  int64_t r0 = c0 + wave * per_wave;
  int64_t r1 = r0 + per_wave;
  if (r1 > c1) r1 = c1;
  f32x16 acc = {0.f};
  double dacc[16];  // fp64 flush of the fp32 MFMA sums every TN_FLUSH rows: bounded fp32 sums
#pragma unroll
  for (int q = 0; q < 16; ++q) dacc[q] = 0.0;
  int64_t r = r0;
  while (r + 8 <= r1) {
    int64_t rend = r + TN_FLUSH;
    if (rend > r1) rend = r1;
    for (; r + 8 <= rend; r += 8) {
      float a0 = ma * pa[(r + 0 + h) * lda], b0 = mb * pb[(r + 0 + h) * ldb];
      float a1 = ma * pa[(r + 2 + h) * lda], b1 = mb * pb[(r + 2 + h) * ldb];
      float a2 = ma * pa[(r + 4 + h) * lda], b2 = mb * pb[(r + 4 + h) * ldb];
      float a3 = ma * pa[(r + 6 + h) * lda], b3 = mb * pb[(r + 6 + h) * ldb];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2, b2, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a3, b3, acc, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      dacc[q] += (double)acc[q];
      acc[q] = 0.f;
    }
    if (rend == r1 || r + 8 > r1) break;
  }
  for (; r < r1; r += 2) {
    const int64_t rr = r + h;
    float a = 0.f, b = 0.f;
    if (rr < r1) {
      a = ma * pa[rr * lda];
      b = mb * pb[rr * ldb];
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) red[wave][q][lane] = dacc[q] + (double)acc[q];
  __syncthreads();
  // 256 threads fold 4 waves x 1024 values in fixed order.
  double* out = partial + (int64_t)blockIdx.x * ca * cb;
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) {
    const int q = e >> 6, l = e & 63;
    const double s = red[0][q][l] + red[1][q][l] + red[2][q][l] + red[3][q][l];
    const int row = i0 + (q & 3) + 8 * (q >> 2) + 4 * (l >> 5);
    const int col = j0 + (l & 31);
    if (row < ca && col < cb) out[(int64_t)row * cb + col] = s;
  }
}

// out[e] = sum_c partial[c][e]: one wave per element, lanes stride the chunks, fixed-order
// xor-tree fold (deterministic).
__global__ __launch_bounds__(256) void reduce_chunks_kernel(const double* __restrict__ partial,
                                                            int nchunks, int64_t elems,
                                                            double* __restrict__ out,
                                                            const int* cond) {
  if (cond && *cond == 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= elems) return;
  // 4 independent loads in flight per lane (fixed summation order: deterministic)
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int c = lane;
  for (; c + 192 < nchunks; c += 256) {
    s0 += partial[(int64_t)c * elems + e];
    s1 += partial[(int64_t)(c + 64) * elems + e];
    s2 += partial[(int64_t)(c + 128) * elems + e];
    s3 += partial[(int64_t)(c + 192) * elems + e];
  }
  for (; c < nchunks; c += 64) s0 += partial[(int64_t)c * elems + e];
  double s = (s0 + s1) + (s2 + s3);
  s = wave_sum_f64(s);
  if (lane == 0) out[e] = s;
}

// Same sum, coalesced: lane = element (64 consecutive elements per workgroup, one 512-B run of
// every chunk's partial per wave-load), the 16 waves take chunks w, w + 16, ... with 4
// independent accumulators each, then fold the 16 wave sums in fixed order through LDS
// (deterministic).  The form above touches one 128-B line per lane (lanes stride the chunks),
// which made the reduce of a 144-chunk Gram ~5 us.
__global__ __launch_bounds__(1024) void reduce_cols_kernel(const double* __restrict__ partial,
                                                           int nchunks, int64_t elems,
                                                           double* __restrict__ out,
                                                           const int* cond) {
  if (cond && *cond == 0) return;
  __shared__ double red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  double s = 0.0;
  if (e < elems) {
    const double* p = partial + e;
    // batches of 16 loads per lane, all issued before the first add (one memory round trip
    // per batch instead of one per 4 loads); fixed summation order
    for (int c0 = w; c0 < nchunks; c0 += 16 * 16) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int c = c0 + 16 * u;
        v[u] = c < nchunks ? p[(int64_t)c * elems] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && e < elems) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lane];
    out[e] = t;
  }
}

// Non-temporal loads of the Krylov basis (round 4): a basis beyond the 256 MB Infinity Cache is
// streamed from HBM by every pass that reads it, so its lines are read once per pass -- nt
// dwordx4 loads stream 2 GB at 6.8 TB/s against 6.0 for plain ones on MI355X
// (profiles/r04_stream_ceiling.jsonl).  A basis that fits the cache keeps plain loads (it is
// re-read from there by the next pass).  (Its A/B switch retired in round 5.)
static bool basis_nt(int64_t n, int count) {
  return (double)n * 32.0 * (double)count > 256.0 * 1024 * 1024;
}

// out[e] = sum_c partial[c][e] for the Gram forms below: the per-element wave form for small
// Grams (<= 512 entries: the local pass's 192 spread over 48 workgroups instead of 3; 12.1 ->
// 10.8 us per local Gram + reduce at cfg2), the coalesced form otherwise (the full pass's 3136:
// 32.6 vs 33.1 us).
static hipError_t launch_reduce(const double* partial, int64_t nchunks, int64_t elems, double* out,
                                const int* cond, hipStream_t stream) {
  if (elems <= 512)
    hipLaunchKernelGGL(reduce_chunks_kernel, dim3((unsigned)((elems + 3) / 4)), dim3(256), 0,
                       stream, partial, (int)nchunks, elems, out, cond);
  else
    hipLaunchKernelGGL(reduce_cols_kernel, dim3((unsigned)((elems + 63) / 64)), dim3(1024), 0,
                       stream, partial, (int)nchunks, elems, out, cond);
  return hipGetLastError();
}

// Narrow right-hand side (one JB = 8/16-wide block B, the Gram step of the orthogonalisation
// G = [Q Z]^T Z): VALU form.  Lane owns 4 consecutive columns of A (one 16-B load per row,
// a wave covers 256 columns = 1 KB of every row), the B row is wave-uniform (scalar loads,
// read once per row instead of once per 32-column tile), 4 x JB fp32 accumulators per lane.
// The 4 waves take contiguous quarters of the workgroup's row chunk and are folded through
// LDS in fixed order into one fp64 partial per chunk; grid.y = 256-column group.
template <int JB, bool FLUSH>
__global__ __launch_bounds__(256) void ts_tn_narrow_kernel(BlockList A, const float* __restrict__ Bz,
                                                           int64_t n, int64_t rows_per_chunk,
                                                           double* __restrict__ partial,
                                                           const int* cond) {
  if (cond && *cond == 0) return;
  extern __shared__ double tn_red[];  // [4 waves][256 columns][JB]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: B rows via SMEM
  const int ca = A.count * A.width;
  const int u = blockIdx.y;               // 256-column group
  const int col0 = (u * 64 + lane) * 4;  // this lane's first column
  const bool colok = col0 < ca;
  const float* ab = colok ? A.blk[col0 / A.width] + (col0 % A.width) : A.blk[0];
  const int64_t lda = A.width;
  const int64_t c0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t c1 = c0 + rows_per_chunk;
  if (c1 > n) c1 = n;
  const int64_t per_wave = (rows_per_chunk + 3) / 4;
  int64_t r0 = c0 + wave * per_wave;
  int64_t r1 = r0 + per_wave;
  if (r1 > c1) r1 = c1;
  float acc[4][JB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j) acc[i][j] = 0.f;
  double dacc[FLUSH ? 4 : 1][FLUSH ? JB : 1];
#pragma unroll
  for (int i = 0; i < (FLUSH ? 4 : 1); ++i)
#pragma unroll
    for (int j = 0; j < (FLUSH ? JB : 1); ++j) dacc[i][j] = 0.0;
  int64_t r = r0;
  int64_t next_flush = r0 + TN_FLUSH;
  // 8 rows per step: 8 independent 16-B loads per lane in flight (the chunk grid is only
  // ~1.5 waves per SIMD at N = 100k, so the loads in flight per wave set the bandwidth)
  for (; r + 8 <= r1; r += 8) {
    if (FLUSH && r >= next_flush) {  // bounded fp32 partial sums, fp64 totals
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < JB; ++j) {
          dacc[FLUSH ? i : 0][FLUSH ? j : 0] += (double)acc[i][j];
          acc[i][j] = 0.f;
        }
      next_flush += TN_FLUSH;
    }
    f32x4 a[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
      a[t] = colok ? *reinterpret_cast<const f32x4*>(ab + (r + t) * lda) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float* zr = Bz + (r + t) * JB;
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        const float zj = zr[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] += a[t][i] * zj;
      }
    }
  }
  for (; r < r1; ++r) {
    const f32x4 a = colok ? *reinterpret_cast<const f32x4*>(ab + r * lda) : f32x4{0.f, 0.f, 0.f, 0.f};
    const float* zr = Bz + r * JB;
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const float zj = zr[j];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] += a[i] * zj;
    }
  }
  // fold the 4 waves (fixed order) and write this chunk's fp64 partial [ca][JB]
  double* mine = tn_red + (size_t)wave * 256 * JB;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j)
      mine[(lane * 4 + i) * JB + j] = (FLUSH ? dacc[FLUSH ? i : 0][FLUSH ? j : 0] : 0.0) +
                                      (double)acc[i][j];
  __syncthreads();
  double* out = partial + (int64_t)blockIdx.x * ca * JB;
  for (int e = threadIdx.x; e < 256 * JB; e += 256) {
    const int cl = e / JB;  // column within this 256-column group
    const int col = u * 256 + cl;
    if (col >= ca) continue;
    const double s = tn_red[e] + tn_red[256 * JB + e] + tn_red[2 * 256 * JB + e] +
                     tn_red[3 * 256 * JB + e];
    out[(int64_t)col * JB + (e % JB)] = s;
  }
}

// Gram step for 8-wide basis blocks and an 8-wide right-hand side (G = [Q Z]^T Z at b = 8):
// every wave-instruction reads whole 128-B lines.  A wave owns 8 blocks; lane =
// (block: 3 bits, column half h: 1 bit, row offset ro: 2 bits), so for one load the 4 lanes of
// a (block, h) pair read rows r..r+3 of that block = one 128-B line, and each lane also loads
// its row of Z (4 distinct 32-B rows per instruction, shared by all blocks).  4 row-quads per
// step (16 rows, 12 x 16-B loads per lane in flight); fp32 sums flushed to fp64 every 1024
// rows; the 4 row offsets are folded by DPP at the end and each chunk writes its fp64 partial
// [ca][8] (no LDS, no cross-wave fold).
__global__ __launch_bounds__(256) void ts_tn_lines_kernel(BlockList A, const float* __restrict__ Bz,
                                                          int64_t n, int64_t rows_per_chunk,
                                                          double* __restrict__ partial,
                                                          const int* cond) {
  if (cond && *cond == 0) return;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int blk = ((int)blockIdx.y * 4 + wave) * 8 + (lane >> 3);
  const int h = (lane >> 2) & 1, ro = lane & 3;
  const bool bok = blk < A.count;
  if (__ballot(bok) == 0) return;  // a wave past the last block
  const float* ab = (bok ? A.blk[blk] : A.blk[0]) + 4 * h;
  const int64_t c0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t c1 = c0 + rows_per_chunk;
  if (c1 > n) c1 = n;
  float acc[4][8];
  double dacc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[i][j] = 0.f;
      dacc[i][j] = 0.0;
    }
  int64_t r = c0;
  int since = 0;
  for (; r + 16 <= c1; r += 16) {
    f32x4 a[4], z0[4], z1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t rr = r + 4 * u + ro;
      a[u] = bok ? *reinterpret_cast<const f32x4*>(ab + rr * 8) : f32x4{0.f, 0.f, 0.f, 0.f};
      z0[u] = *reinterpret_cast<const f32x4*>(Bz + rr * 8);
      z1[u] = *reinterpret_cast<const f32x4*>(Bz + rr * 8 + 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] += a[u][i] * z0[u][j];
          acc[i][4 + j] += a[u][i] * z1[u][j];
        }
      }
    if (++since == 64) {  // 1024 rows: bounded fp32 partial sums
      since = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          dacc[i][j] += (double)acc[i][j];
          acc[i][j] = 0.f;
        }
    }
  }
  for (; r < c1; r += 4) {
    const int64_t rr = r + ro;
    if (rr < c1) {
      const f32x4 a1 = bok ? *reinterpret_cast<const f32x4*>(ab + rr * 8) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 y0 = *reinterpret_cast<const f32x4*>(Bz + rr * 8);
      const f32x4 y1 = *reinterpret_cast<const f32x4*>(Bz + rr * 8 + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] += a1[i] * y0[j];
          acc[i][4 + j] += a1[i] * y1[j];
        }
    }
  }
  double* out = partial + (int64_t)blockIdx.x * ((int64_t)A.count * 8) * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      double v = dacc[i][j] + (double)acc[i][j];
      // fold the 4 row offsets (lane bits 0, 1) in fixed order: quad_perm xor 1, xor 2
      const int lo1 = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0xB1, 0xF, 0xF, false);
      const int hi1 = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0xB1, 0xF, 0xF, false);
      v += __hiloint2double(hi1, lo1);
      const int lo2 = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x4E, 0xF, 0xF, false);
      const int hi2 = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x4E, 0xF, 0xF, false);
      v += __hiloint2double(hi2, lo2);
      if (bok && ro == 0) out[(int64_t)(blk * 8 + 4 * h + i) * 8 + j] = v;
    }
}

// Gram step for 8-wide basis blocks and an 8-wide right-hand side, streaming form: one wave
// per basis block and row chunk, lane = (column half h = lane >> 5, row offset rl = lane & 31),
// so every wave-instruction reads 32 consecutive 32-B rows of ONE block (1 KB contiguous; the
// line form above touched 8 blocks x 128 B per instruction, which halves the HBM rate).  Each
// lane also loads its Z row (32 B, shared by the h pair).  TS_U row-steps (128 rows) per
// iteration keep 12 x 16-B loads per lane in flight.  A chunk holds at most 8192 rows, so every
// lane sums at most 256 products per entry in fp32; the 32 row lanes are then folded in fp64
// by a fixed reduce-scatter (xor 1, 2, 4, 8, 16): after it lane rl holds entry
// v = bitrev5(rl) of its half, and the wave writes its 64 fp64 partials as one contiguous run.
// Chunks with the same rows run on one XCD (nchunks % 8 == 0, workgroup id = y * nchunks + x),
// so each XCD's L2 fetches a Z chunk once for all of its column groups.
#define TS_MAX_CHUNK 8192
template <int MASK>
__device__ __forceinline__ double xor_lanes_f64(double v) {
  // lane ^ MASK within 32-lane halves (ds_swizzle bitmask mode: and 0x1F, xor MASK)
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), 0x1F | (MASK << 10));
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), 0x1F | (MASK << 10));
  return __hiloint2double(hi, lo);
}

template <int BIT, int HALF>
__device__ __forceinline__ void rs_step(double* v, int rl) {
  // v[0..2*HALF): keep the half selected by lane bit BIT, add the partner's copy of it
  const bool up = (rl >> BIT) & 1;
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    const double mine = up ? v[k + HALF] : v[k];
    const double give = up ? v[k] : v[k + HALF];
    v[k] = mine + xor_lanes_f64<1 << BIT>(give);
  }
}

// ZSum (count > 0): the right-hand side Z is not stored yet; it is the sum of `count` per-layer
// SpMM outputs (the XCD-split second stage), summed here in fixed order.  A's last block is Z
// itself: the wave that owns it uses the sums as its A rows and stores them to `out` (the
// block Z will live in), so the pass that follows reads a materialised Z.
struct ZSum {
  const float* p[8];
  int count;
  float* out;
};

__device__ __forceinline__ void zsum_store(const ZSum& zs, int64_t off, const f32x4& v) {
  *reinterpret_cast<f32x4*>(zs.out + off) = v;
}

template <bool SUM>
__device__ __forceinline__ void zrow_load(const float* __restrict__ Bz, const ZSum& zs, int64_t rr,
                                          f32x4& z0, f32x4& z1) {
  if (!SUM) {
    z0 = *reinterpret_cast<const f32x4*>(Bz + rr * 8);
    z1 = *reinterpret_cast<const f32x4*>(Bz + rr * 8 + 4);
    return;
  }
  z0 = *reinterpret_cast<const f32x4*>(zs.p[0] + rr * 8);
  z1 = *reinterpret_cast<const f32x4*>(zs.p[0] + rr * 8 + 4);
  for (int i = 1; i < zs.count; ++i) {
    z0 += *reinterpret_cast<const f32x4*>(zs.p[i] + rr * 8);
    z1 += *reinterpret_cast<const f32x4*>(zs.p[i] + rr * 8 + 4);
  }
}

template <int TS_U, bool SUM>
__global__ __launch_bounds__(256) void ts_tn_stream_kernel(BlockList A, const float* __restrict__ Bz,
                                                           int64_t n, int64_t rows_per_chunk,
                                                           double* __restrict__ partial,
                                                           const int* cond, ZSum zs) {
  if (cond && *cond == 0) return;
  const int lane = threadIdx.x & 63;
  const int blk = (int)blockIdx.y * 4 + (threadIdx.x >> 6);
  if (blk >= A.count) return;  // wave-uniform; no block barrier below
  const int h = lane >> 5, rl = lane & 31;
  // SUM: the last block is Z (= the sums): this wave takes its A rows from them and stores them
  const bool zblk = SUM && blk == A.count - 1;
  const float* ab = (zblk ? A.blk[0] : A.blk[blk]) + 4 * h;
  const int64_t c0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t c1 = c0 + rows_per_chunk;
  if (c1 > n) c1 = n;
  float acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  int64_t r = c0;
  for (; r + 32 * TS_U <= c1; r += 32 * TS_U) {
    f32x4 a[TS_U], z0[TS_U], z1[TS_U];
#pragma unroll
    for (int u = 0; u < TS_U; ++u) {
      const int64_t rr = r + 32 * u + rl;
      if (!zblk) a[u] = *reinterpret_cast<const f32x4*>(ab + rr * 8);
      zrow_load<SUM>(Bz, zs, rr, z0[u], z1[u]);
    }
    if (zblk) {
#pragma unroll
      for (int u = 0; u < TS_U; ++u) {
        const int64_t rr = r + 32 * u + rl;
        a[u] = h ? z1[u] : z0[u];
        zsum_store(zs, rr * 8 + 4 * h, a[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < TS_U; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] += a[u][i] * z0[u][j];
          acc[i][4 + j] += a[u][i] * z1[u][j];
        }
  }
  for (; r < c1; r += 32) {
    const int64_t rr = r + rl;
    if (rr < c1) {
      f32x4 y0, y1, a1;
      zrow_load<SUM>(Bz, zs, rr, y0, y1);
      if (zblk) {
        a1 = h ? y1 : y0;
        zsum_store(zs, rr * 8 + 4 * h, a1);
      } else {
        a1 = *reinterpret_cast<const f32x4*>(ab + rr * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] += a1[i] * y0[j];
          acc[i][4 + j] += a1[i] * y1[j];
        }
    }
  }
  double v[32];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i * 8 + j] = (double)acc[i][j];
  rs_step<0, 16>(v, rl);
  rs_step<1, 8>(v, rl);
  rs_step<2, 4>(v, rl);
  rs_step<3, 2>(v, rl);
  rs_step<4, 1>(v, rl);
  // lane rl now holds entry e = bitrev5(rl) = (i, j) = (e >> 3, e & 7) of its column half
  const int e = ((rl & 1) << 4) | ((rl & 2) << 2) | (rl & 4) | ((rl & 8) >> 2) | ((rl & 16) >> 4);
  double* out = partial + (int64_t)blockIdx.x * ((int64_t)A.count * 8) * 8;
  out[(int64_t)blk * 64 + 32 * h + e] = v[0];
}

// The streaming Gram with Z's rows staged once per workgroup through LDS (the 4 waves of a
// workgroup take 4 basis blocks over the same rows, so each used to load the same 32-B Z row
// per lane and row step: twice the block's own bytes through L1).  Double-buffered, the next
// step's A rows and Z piece in flight across the barrier; same products in the same order as
// ts_tn_stream_kernel<TS_U, false> (bit-identical Grams).  N2V2R_TN_LDS=0: the unstaged form.
template <int TS_U>
__global__ __launch_bounds__(256) void ts_tn_stream_lds_kernel(BlockList A, const float* __restrict__ Bz,
                                                               int64_t n, int64_t rows_per_chunk,
                                                               double* __restrict__ partial,
                                                               const int* cond) {
  if (cond && *cond == 0) return;  // (uniform: before any barrier)
  static_assert(32 * TS_U * 2 == 256, "one staged 16-B piece per thread per row step");
  const int lane = threadIdx.x & 63;
  const int blk = (int)blockIdx.y * 4 + (threadIdx.x >> 6);
  const bool active = blk < A.count;
  const int h = lane >> 5, rl = lane & 31;
  const float* ab = A.blk[active ? blk : 0] + 4 * h;
  const int64_t c0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t c1 = c0 + rows_per_chunk;
  if (c1 > n) c1 = n;
  __shared__ f32x4 zst[2][32 * TS_U * 2];
  float acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  const int t = threadIdx.x, zr = t >> 1, zq = t & 1;
  f32x4 an[TS_U], zn = {0.f, 0.f, 0.f, 0.f};
  auto load_step = [&](int64_t rs) {
    if (active) {
#pragma unroll
      for (int u = 0; u < TS_U; ++u)
        an[u] = *reinterpret_cast<const f32x4*>(ab + (rs + 32 * u + rl) * 8);
    }
    zn = *reinterpret_cast<const f32x4*>(Bz + (rs + zr) * 8 + 4 * zq);
  };
  int64_t r = c0;
  int buf = 0;
  if (r + 32 * TS_U <= c1) load_step(r);
  for (; r + 32 * TS_U <= c1; r += 32 * TS_U, buf ^= 1) {
    f32x4 a[TS_U];
#pragma unroll
    for (int u = 0; u < TS_U; ++u) a[u] = an[u];
    zst[buf][t] = zn;
    if (r + 64 * TS_U <= c1) load_step(r + 32 * TS_U);
    __syncthreads();  // (readers of the other buffer all passed the previous barrier)
    if (active) {
#pragma unroll
      for (int u = 0; u < TS_U; ++u) {
        const int lr = 32 * u + rl;
        const f32x4 z0 = zst[buf][lr * 2], z1 = zst[buf][lr * 2 + 1];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] += a[u][i] * z0[j];
            acc[i][4 + j] += a[u][i] * z1[j];
          }
      }
    }
  }
  if (!active) return;  // past the last barrier
  for (; r < c1; r += 32) {
    const int64_t rr = r + rl;
    if (rr < c1) {
      const f32x4 y0 = *reinterpret_cast<const f32x4*>(Bz + rr * 8);
      const f32x4 y1 = *reinterpret_cast<const f32x4*>(Bz + rr * 8 + 4);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(ab + rr * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] += a1[i] * y0[j];
          acc[i][4 + j] += a1[i] * y1[j];
        }
    }
  }
  double v[32];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i * 8 + j] = (double)acc[i][j];
  rs_step<0, 16>(v, rl);
  rs_step<1, 8>(v, rl);
  rs_step<2, 4>(v, rl);
  rs_step<3, 2>(v, rl);
  rs_step<4, 1>(v, rl);
  const int e = ((rl & 1) << 4) | ((rl & 2) << 2) | (rl & 4) | ((rl & 8) >> 2) | ((rl & 16) >> 4);
  double* out = partial + (int64_t)blockIdx.x * ((int64_t)A.count * 8) * 8;
  out[(int64_t)blk * 64 + 32 * h + e] = v[0];
}

// Gram-kernel selection for 8-wide blocks: the streaming form (about 4096 waves, chunks of at
// least 256 rows); the line form where its partials would not fit (the A/B switch retired in
// round 5)
static bool tn_stream_form() { return true; }
#define TN_STREAM_WAVES 4096
#define TN_STREAM_MIN_ROWS 256

static hipError_t launch_ts_tn(const BlockList& A, const BlockList& B, int64_t n,
                               double* partial, size_t partial_elems, double* out,
                               const int* cond, const ZSum* zs, hipStream_t stream) {
  const int ca = A.count * A.width, cb = B.count * B.width;
  int64_t s_chunks = 0, s_rows = 0;
  if (B.count == 1 && B.width == 8 && A.width == 8 && tn_stream_form()) {
    // streaming form: ~TN_STREAM_WAVES (4096) waves, chunks of <= TS_MAX_CHUNK rows, nchunks % 8 == 0
    // (<= 4 blocks -- the local pass -- aim at half the waves: longer chunks, half the partials
    // to reduce; cfg4 Gram 30.1 -> 28.4 us and reduce 7.0 -> 5.0 us per pass, 1024 / 8192 worse;
    // profiles/r04_tn_small_waves.txt)
    s_chunks = ((A.count <= 4 ? TN_STREAM_WAVES / 2 : TN_STREAM_WAVES) + A.count - 1) / A.count;
    const int64_t lo = (n + TS_MAX_CHUNK - 1) / TS_MAX_CHUNK,
                  hi = (n + TN_STREAM_MIN_ROWS - 1) / TN_STREAM_MIN_ROWS;
    if (s_chunks > hi) s_chunks = hi;
    if (s_chunks < lo) s_chunks = lo;
    s_chunks = (s_chunks + 7) & ~(int64_t)7;
    s_rows = ((n + s_chunks - 1) / s_chunks + 31) & ~(int64_t)31;
    s_chunks = (n + s_rows - 1) / s_rows;
    // partials must fit the buffer; otherwise the line form below takes it
    if ((size_t)(s_chunks * ca * cb) > partial_elems || s_rows > TS_MAX_CHUNK) s_chunks = 0;
  }
  if (s_chunks > 0) {
    const int64_t elems = (int64_t)ca * cb;
    const int64_t nchunks = s_chunks, rows_per_chunk = s_rows;
    const dim3 grid((unsigned)nchunks, (unsigned)((A.count + 3) / 4));
    const ZSum none{};
    if (zs && zs->count > 0)
      hipLaunchKernelGGL((ts_tn_stream_kernel<4, true>), grid, dim3(256), 0, stream, A, B.blk[0],
                         n, rows_per_chunk, partial, cond, *zs);
    else
      hipLaunchKernelGGL((ts_tn_stream_lds_kernel<4>), grid, dim3(256), 0, stream, A, B.blk[0],
                         n, rows_per_chunk, partial, cond);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_reduce(partial, nchunks, elems, out, cond, stream);
  }
  if (zs && zs->count > 0) return hipErrorNotSupported;  // the Z sums: streaming form only
  if (B.count == 1 && B.width == 8 && A.width == 8) {
    // line form: ~2048 waves, >= 64 rows per chunk, partials within the buffer
    const int64_t elems = (int64_t)ca * cb;
    const int groups = (A.count + 7) / 8;
    int64_t nchunks = 2048 / groups;
    if (nchunks < 1) nchunks = 1;
    if (nchunks > (n + 63) / 64) nchunks = (n + 63) / 64;
    if ((size_t)(nchunks * elems) > partial_elems) nchunks = (int64_t)(partial_elems / elems);
    if (nchunks < 1) return hipErrorInvalidValue;
    int64_t rows_per_chunk = (n + nchunks - 1) / nchunks;
    rows_per_chunk = (rows_per_chunk + 15) & ~(int64_t)15;
    nchunks = (n + rows_per_chunk - 1) / rows_per_chunk;
    const dim3 grid((unsigned)nchunks, (unsigned)((groups + 3) / 4));
    hipLaunchKernelGGL(ts_tn_lines_kernel, grid, dim3(256), 0, stream, A, B.blk[0], n,
                       rows_per_chunk, partial, cond);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_reduce(partial, nchunks, elems, out, cond, stream);
  }
  if (B.count == 1 && (B.width == 8 || B.width == 16) && A.width % 4 == 0) {
    // narrow form: ~1024 workgroups of >= 256 rows, partials within the buffer
    const int64_t elems = (int64_t)ca * cb;
    int64_t nchunks = (n + 255) / 256;
    if (nchunks > 1024) nchunks = 1024;
    if ((size_t)(nchunks * elems) > partial_elems) nchunks = (int64_t)(partial_elems / elems);
    if (nchunks < 1) return hipErrorInvalidValue;
    const int64_t rows_per_chunk = (n + nchunks - 1) / nchunks;
    nchunks = (n + rows_per_chunk - 1) / rows_per_chunk;
    const int groups = (ca + 255) / 256;
    const size_t lds = sizeof(double) * 4 * 256 * B.width;
    const dim3 grid((unsigned)nchunks, (unsigned)groups);
    static bool attr = false;
    if (!attr) {  // 128 KB of LDS for the 16-wide form
      (void)hipFuncSetAttribute((const void*)ts_tn_narrow_kernel<16, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);
      (void)hipFuncSetAttribute((const void*)ts_tn_narrow_kernel<16, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);
      (void)hipGetLastError();  // a refused attribute must not surface at a later launch
      attr = true;
    }
    const bool flush = rows_per_chunk / 4 > TN_FLUSH;  // rows per wave beyond one fp32 span
#define TN_NARROW(J, F)                                                                    \
  hipLaunchKernelGGL((ts_tn_narrow_kernel<J, F>), grid, dim3(256), lds, stream, A, B.blk[0], n, \
                     rows_per_chunk, partial, cond)
    if (B.width == 8) {
      if (flush) TN_NARROW(8, true); else TN_NARROW(8, false);
    } else {
      if (flush) TN_NARROW(16, true); else TN_NARROW(16, false);
    }
#undef TN_NARROW
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_reduce(partial, nchunks, elems, out, cond, stream);
  }
  const int nti = (ca + 31) / 32, ntj = (cb + 31) / 32;
  const int ntiles = nti * ntj;
  // chunk count: ~1024 workgroups with >= 512 rows per chunk, partials within the buffer
  int64_t nchunks = (n + 511) / 512;
  int64_t cap = 1024 / ntiles;
  if (cap < 1) cap = 1;
  if (nchunks > cap) nchunks = cap;
  const int64_t elems = (int64_t)ca * cb;
  if ((size_t)(nchunks * elems) > partial_elems) nchunks = (int64_t)(partial_elems / elems);
  if (nchunks < 1) return hipErrorInvalidValue;
  int64_t rows_per_chunk = (n + nchunks - 1) / nchunks;
  rows_per_chunk = (rows_per_chunk + 7) & ~(int64_t)7;
  nchunks = (n + rows_per_chunk - 1) / rows_per_chunk;
  dim3 grid((unsigned)nchunks, (unsigned)ntiles);
  hipLaunchKernelGGL(ts_tn_kernel, grid, dim3(256), 0, stream, A, B, n, rows_per_chunk, ntj,
                     partial, cond);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_reduce(partial, nchunks, elems, out, cond, stream);
}

extern "C" hipError_t n2v2r_launch_ts_tn(const BlockList& A, const BlockList& B, int64_t n,
                                         double* partial, size_t partial_elems, double* out,
                                         const int* cond, hipStream_t stream) {
  return launch_ts_tn(A, B, n, partial, partial_elems, out, cond, nullptr, stream);
}

// G = [Q Z]^T Z with Z = sum of `count` partial panels, stored to zout (= A's last block and
// B's only block) on the way; hipErrorNotSupported when the streaming form does not apply
// (the caller then sums the partials itself)
extern "C" hipError_t n2v2r_launch_ts_tn_zsum(const BlockList& A, int64_t n, const float* const* parts,
                                              int count, float* zout, double* partial,
                                              size_t partial_elems, double* out, hipStream_t stream) {
  if (count < 1 || count > 8 || A.count < 1 || A.blk[A.count - 1] != zout) return hipErrorInvalidValue;
  ZSum zs{};
  for (int i = 0; i < count; ++i) zs.p[i] = parts[i];
  zs.count = count;
  zs.out = zout;
  BlockList B{};
  B.count = 1;
  B.width = A.width;
  B.blk[0] = zout;
  return launch_ts_tn(A, B, n, partial, partial_elems, out, nullptr, &zs, stream);
}

// ---- paired full passes (deferred reorthogonalisation, engine.cpp Eig::pair_pass) ----------
// Two right-hand sides in one read of the basis: out = [A]^T [Za Zb] as two Gram arrays,
// out[r][blk][64] (r = 0: Za, 1: Zb), each block's 8 x 8 in the layout of ts_tn_stream_kernel
// (row-major (blk * 8 + i, j)).  Same streaming form: one wave per (basis block, row chunk), a
// lane owns 4 columns of its block over rows rl, rl + 32, ..., fp32 products of at most
// TS_MAX_CHUNK / 32 rows per lane, then a fixed fp64 reduce-scatter over the 32 row lanes.
template <int TS_U, bool NT>
__global__ __launch_bounds__(256) void ts_tn_stream2_kernel(BlockList A, const float* __restrict__ Za,
                                                            const float* __restrict__ Zb, int64_t n,
                                                            int64_t rows_per_chunk,
                                                            double* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int blk = (int)blockIdx.y * 4 + (threadIdx.x >> 6);
  // the 4 waves of a workgroup read the same rows of Za / Zb for 4 basis blocks: those rows are
  // staged once through LDS (one 16-B piece per thread per 64 rows, double-buffered, one barrier
  // per step) instead of every wave loading them (each lane a 64-B Z row per row step: 4x the
  // block's own bytes through L1).  Waves past the last block stage and wait at the barriers.
  const bool active = blk < A.count;
  const int h = lane >> 5, rl = lane & 31;
  const float* ab = A.blk[active ? blk : 0] + 4 * h;
  const int64_t c0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t c1 = c0 + rows_per_chunk;
  if (c1 > n) c1 = n;
  __shared__ f32x4 zst[2][32 * TS_U * 4];
  float acc[4][16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  auto fma_row = [&](const f32x4& a, const f32x4& y0, const f32x4& y1, const f32x4& y2,
                     const f32x4& y3) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] += a[i] * y0[j];
        acc[i][4 + j] += a[i] * y1[j];
        acc[i][8 + j] += a[i] * y2[j];
        acc[i][12 + j] += a[i] * y3[j];
      }
  };
  static_assert(32 * TS_U * 4 == 256, "one staged 16-B piece per thread per row step");
  int64_t r = c0;
  const int t = threadIdx.x, zr = t >> 2, zq = t & 3;  // staged row, 16-B quarter
  const float* zsrc = (zq < 2 ? Za : Zb) + 4 * (zq & 1);
  int buf = 0;
  // the next step's A rows and Z piece are loaded before this step's products (one memory round
  // trip in flight across the barrier and the FMAs)
  f32x4 an[TS_U], zn = {0.f, 0.f, 0.f, 0.f};
  auto load_step = [&](int64_t rs) {
    if (active) {
#pragma unroll
      for (int u = 0; u < TS_U; ++u) {
        const f32x4* p = reinterpret_cast<const f32x4*>(ab + (rs + 32 * u + rl) * 8);
        an[u] = NT ? __builtin_nontemporal_load(p) : *p;
      }
    }
    zn = *reinterpret_cast<const f32x4*>(zsrc + (rs + zr) * 8);
  };
  if (r + 32 * TS_U <= c1) load_step(r);
  for (; r + 32 * TS_U <= c1; r += 32 * TS_U, buf ^= 1) {
    f32x4 a[TS_U];
#pragma unroll
    for (int u = 0; u < TS_U; ++u) a[u] = an[u];
    zst[buf][t] = zn;
    if (r + 64 * TS_U <= c1) load_step(r + 32 * TS_U);
    __syncthreads();  // (readers of the other buffer all passed the previous barrier)
    if (active) {
#pragma unroll
      for (int u = 0; u < TS_U; ++u) {
        const int lr = 32 * u + rl;
        fma_row(a[u], zst[buf][lr * 4], zst[buf][lr * 4 + 1], zst[buf][lr * 4 + 2],
                zst[buf][lr * 4 + 3]);
      }
    }
  }
  if (!active) return;  // past the last barrier
  for (; r < c1; r += 32) {
    const int64_t rr = r + rl;
    if (rr < c1) {
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(ab + rr * 8);
      fma_row(a1, *reinterpret_cast<const f32x4*>(Za + rr * 8),
              *reinterpret_cast<const f32x4*>(Za + rr * 8 + 4),
              *reinterpret_cast<const f32x4*>(Zb + rr * 8),
              *reinterpret_cast<const f32x4*>(Zb + rr * 8 + 4));
    }
  }
  // one right-hand side at a time through the fixed fp64 reduce-scatter (as ts_tn_stream_kernel:
  // lane rl ends with entry bitrev5(rl) = (i, j) of its column half), so only 32 fp64 values are
  // live at once (a 64-value fold held 144 VGPRs: 3 waves per SIMD)
  const int e = ((rl & 1) << 4) | ((rl & 2) << 2) | (rl & 4) | ((rl & 8) >> 2) | ((rl & 16) >> 4);
  double* out = partial + (int64_t)blockIdx.x * ((int64_t)A.count * 128);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    double v[32];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i * 8 + j] = (double)acc[i][8 * r + j];
    rs_step<0, 16>(v, rl);
    rs_step<1, 8>(v, rl);
    rs_step<2, 4>(v, rl);
    rs_step<3, 2>(v, rl);
    rs_step<4, 1>(v, rl);
    out[((int64_t)r * A.count + blk) * 64 + 32 * h + e] = v[0];
  }
}

// out[2][A.count][64] = [A]^T [Za Zb] (fp64, rows over ranks NOT summed here)
extern "C" hipError_t n2v2r_launch_ts_tn2(const BlockList& A, const float* Za, const float* Zb,
                                          int64_t n, double* partial, size_t partial_elems,
                                          double* out, hipStream_t stream) {
  if (A.width != 8 || A.count < 1 || n < 1) return hipErrorInvalidValue;
  const int64_t elems = (int64_t)A.count * 128;
  int64_t s_chunks = (TN_STREAM_WAVES + A.count - 1) / A.count;
  const int64_t lo = (n + TS_MAX_CHUNK - 1) / TS_MAX_CHUNK,
                hi = (n + TN_STREAM_MIN_ROWS - 1) / TN_STREAM_MIN_ROWS;
  if (s_chunks > hi) s_chunks = hi;
  if (s_chunks < lo) s_chunks = lo;
  s_chunks = (s_chunks + 7) & ~(int64_t)7;
  const int64_t s_rows = ((n + s_chunks - 1) / s_chunks + 31) & ~(int64_t)31;
  s_chunks = (n + s_rows - 1) / s_rows;
  if ((size_t)(s_chunks * elems) > partial_elems || s_rows > TS_MAX_CHUNK) return hipErrorNotSupported;
  const dim3 grid((unsigned)s_chunks, (unsigned)((A.count + 3) / 4));
  if (basis_nt(n, A.count))
    hipLaunchKernelGGL((ts_tn_stream2_kernel<2, true>), grid, dim3(256), 0, stream, A, Za, Zb, n,
                       s_rows, partial);
  else
    hipLaunchKernelGGL((ts_tn_stream2_kernel<2, false>), grid, dim3(256), 0, stream, A, Za, Zb, n,
                       s_rows, partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_reduce(partial, s_chunks, elems, out, nullptr, stream);
}

// The second pass of a pair: Zb's Gram against the CORRECTED Za' = (Za - Q Ca) Ra^{-1} from
// the pair's Gram, D = Za'^T Zb = Ra^{-T} (Za^T Zb - Ca^T Cb) (Ca, Cb: the old blocks' rows of
// the two Grams, all of them: rows a selective pass skipped are below its threshold, so their
// products are below the threshold squared), written over Za's rows of Zb's Gram.  Ra: the
// first pass's R (rsave; identity when that pass applied nothing) -- reset to the identity here
// for the next pair.  One 256-thread workgroup.
__global__ __launch_bounds__(256) void pair_fixup_kernel(double* __restrict__ g2, int nblk_all,
                                                         int nq_old, double* __restrict__ ra) {
  // LDS: Ca rows | Cb rows (nq_old * 64 fp64 each), staged with all loads of a thread in flight
  // (a thread-per-entry loop over global rows waited out one load per row: 35 us at cfg2)
  extern __shared__ double fx[];
  __shared__ double part[4][64], dr[64], rr[64];
  const int tid = threadIdx.x;
  const int nr8 = nq_old * 64;
  const double* ga = g2;                          // [nblk_all][64]: Za's Gram
  double* gb = g2 + (int64_t)nblk_all * 64;       // Zb's Gram
  if (nr8 > 0) {
    stage_to_lds<256, 16>(fx, ga, nr8, tid);
    stage_to_lds<256, 16>(fx + nr8, gb, nr8, tid);
  }
  if (tid < 64) rr[tid] = ra[tid];
  __syncthreads();
  {
    const int q = tid >> 6, e = tid & 63, i = e >> 3, j = e & 7;
    double s = 0.0;
    for (int r = q; r < nq_old * 8; r += 4) s += fx[r * 8 + i] * fx[nr8 + r * 8 + j];
    part[q][e] = s;
  }
  __syncthreads();
  if (tid < 64)  // Za^T Zb (row i of Za, column j of Zb) - Ca^T Cb, fixed order
    dr[tid] = gb[(int64_t)nq_old * 64 + tid] - ((part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]));
  __syncthreads();
  if (tid < 8) {  // column tid: forward substitution Ra^T d = dr (Ra upper triangular)
    double d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      double v = dr[k * 8 + tid];
#pragma unroll
      for (int m = 0; m < k; ++m) v -= rr[m * 8 + k] * d[m];
      d[k] = v / rr[k * 8 + k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) gb[(int64_t)nq_old * 64 + k * 8 + tid] = d[k];
  }
  if (tid < 64) ra[tid] = (tid >> 3) == (tid & 7) ? 1.0 : 0.0;  // rr holds the copy in use
}

extern "C" hipError_t n2v2r_launch_pair_fixup(double* g2, int nblk_all, int nq_old, double* ra,
                                              hipStream_t stream) {
  if (nq_old < 0 || nblk_all < nq_old + 2) return hipErrorInvalidValue;
  const size_t lds = sizeof(double) * 2 * (size_t)nq_old * 64;
  if (lds > 120 * 1024) return hipErrorInvalidValue;
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void*)pair_fixup_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
    (void)hipGetLastError();
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(pair_fixup_kernel, dim3(1), dim3(256), lds, stream, g2, nblk_all, nq_old, ra);
  return hipGetLastError();
}

// r1 <- r2 r1 (8 x 8 fp64, row-major upper triangular): the R of two passes over one block,
// (Z - Q C1) = Z1 R1 and (Z1 - Q C2) = Z2 R2 give Z - Q (C1 + C2 R1) = Z2 (R2 R1).  The lean
// residual estimates read R of the restart block; a pass that clamped a pivot (PIP_CANCEL) left
// R1 scaled, not normalised, and the second pass's R2 corrects it.  One wave.
__global__ __launch_bounds__(64) void rmul8_kernel(const double* __restrict__ r2,
                                                   double* __restrict__ r1) {
  __shared__ double a[64], b[64];
  const int tid = threadIdx.x, i = tid >> 3, j = tid & 7;
  a[tid] = r2[tid];
  b[tid] = r1[tid];
  __syncthreads();
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k) v += a[i * 8 + k] * b[k * 8 + j];
  r1[tid] = v;
}

extern "C" hipError_t n2v2r_launch_rmul8(const double* r2, double* r1, hipStream_t stream) {
  if (!r2 || !r1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rmul8_kernel, dim3(1), dim3(64), 0, stream, r2, r1);
  return hipGetLastError();
}

// out = sum of `count` partial panels (fixed order), n x 8 fp32
__global__ void zsum_kernel(ZSum zs, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one half row (16 B)
  if (e >= n * 2) return;
  f32x4 v = *reinterpret_cast<const f32x4*>(zs.p[0] + e * 4);
  for (int i = 1; i < zs.count; ++i) v += *reinterpret_cast<const f32x4*>(zs.p[i] + e * 4);
  *reinterpret_cast<f32x4*>(zs.out + e * 4) = v;
}

// The per-cycle read-back packed into one device staging block (then one copy to pinned host
// memory): up to 8 segments, each a 4-byte-word copy (src) or zero fill (src == nullptr) into
// disjoint ranges of dst.  Five separate small copies were ~4.7 us each on the GPU timeline.
// A segment with `clear` set also zeroes its source words after copying them (the per-cycle
// flags, so no separate memset launch re-arms them for the next cycle).
struct PackSegs {
  unsigned* src[12];
  int dst_word[12];
  int words[12];
  int clear[12];
  int count;
};
__global__ __launch_bounds__(256) void pack_words_kernel(PackSegs ps, unsigned* __restrict__ dst) {
  for (int s = 0; s < ps.count; ++s)
    for (int w = threadIdx.x; w < ps.words[s]; w += 256) {
      dst[ps.dst_word[s] + w] = ps.src[s] ? ps.src[s][w] : 0u;
      if (ps.src[s] && ps.clear[s]) ps.src[s][w] = 0u;
    }
}

extern "C" hipError_t n2v2r_launch_pack_words(void* const* src, const int* dst_word,
                                              const int* words, const int* clear, int count,
                                              void* dst, hipStream_t stream) {
  if (count < 1 || count > 12) return hipErrorInvalidValue;
  PackSegs ps{};
  ps.count = count;
  for (int s = 0; s < count; ++s) {
    ps.src[s] = static_cast<unsigned*>(src[s]);
    ps.dst_word[s] = dst_word[s];
    ps.words[s] = words[s];
    ps.clear[s] = clear[s];
  }
  hipLaunchKernelGGL(pack_words_kernel, dim3(1), dim3(256), 0, stream, ps,
                     static_cast<unsigned*>(dst));
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_zsum(const float* const* parts, int count, float* zout, int64_t n,
                                        hipStream_t stream) {
  if (count < 1 || count > 8) return hipErrorInvalidValue;
  ZSum zs{};
  for (int i = 0; i < count; ++i) zs.p[i] = parts[i];
  zs.count = count;
  zs.out = zout;
  const int64_t th = n * 2;
  hipLaunchKernelGGL(zsum_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, stream, zs, n);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- ts_nn
// O[r][j] = alpha * sum_k A[r][k] F[k][j] + beta * C[r][j] (j < cb), with the coefficient
// matrix F either a plain fp32 matrix (G, ld ldg) or, in "PIP" mode, built on the fly from the
// fused Gram-Schmidt/Cholesky factors: F = [-C R^{-1}; R^{-1}] with C = pip_g[0:c] (fp64,
// row-major (c+b) x b) and R^{-1} = pip_x (fp64 b x b, flagged columns already zero).
struct Coef {
  const float* G;
  int ldg;
  const double* pip_g;
  const double* pip_x;
  int pip_c;
};

__device__ __forceinline__ float coef_at(const Coef& F, int k, int j, int cb) {
  if (F.G) return F.G[(int64_t)k * F.ldg + j];
  if (k >= F.pip_c) return (float)F.pip_x[(k - F.pip_c) * cb + j];
  double v = 0.0;
  const double* crow = F.pip_g + (int64_t)k * cb;
  for (int m = 0; m <= j; ++m) v -= crow[m] * F.pip_x[m * cb + j];
  return (float)v;
}

// MFMA form for cb >= 32 (Ritz vectors X = Q S, and b = 32/64 blocks): one wave per 32 output
// rows and all output columns (NT 32-wide tiles), so O may alias A or C.  A rows are read as
// 16-B loads; the k order inside each 8-column group is permuted consistently for A and F
// (lane half h carries columns 4h..4h+3).  F is staged through LDS 64 rows at a time.
#ifndef NN_KCH
#define NN_KCH 64
#endif
#ifndef NN_WAVES
#define NN_WAVES 4  // waves per workgroup (32 rows each), sharing one staged F chunk
#endif
#define NN_T (64 * NN_WAVES)
template <int NT>
__global__ __launch_bounds__(NN_T) void ts_nn_kernel(BlockList A, Coef F, int cb, OutBlockList O,
                                                    BlockList C, float alpha, float beta,
                                                    int64_t n, const int* cond, const int* flags,
                                                    uint64_t seed, int64_t row0) {
  if (cond && *cond == 0) return;
  __shared__ __attribute__((aligned(16))) float fs[NN_KCH][NT * 32];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t r0 = ((int64_t)blockIdx.x * NN_WAVES + wave) * 32;
  const int i = lane & 31;
  const int h = lane >> 5;
  const int64_t row = r0 + i;
  const bool row_ok = row < n;
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{0.f};
  const int ca = A.count * A.width;
  // rows past n read row n-1 (valid address, results not stored); the chunk's 8 A loads are
  // issued before the F staging so they are in flight across its barriers
  const int64_t lrow = row_ok ? row : (n > 0 ? n - 1 : 0);
  const bool vec4 = F.G && (F.ldg % 4) == 0 && (cb % 4) == 0 &&
                    (reinterpret_cast<uintptr_t>(F.G) & 15) == 0;
  for (int k0 = 0; k0 < ca; k0 += NN_KCH) {
    const int kn = (ca - k0) < NN_KCH ? (ca - k0) : NN_KCH;
    f32x4 a4[NN_KCH / 8];
#pragma unroll
    for (int s8 = 0; s8 < NN_KCH / 8; ++s8) {
      int kg = k0 + 8 * s8;
      if (kg >= ca) kg = ca - 8;
      a4[s8] = *reinterpret_cast<const f32x4*>(A.blk[kg / A.width] + (kg % A.width) + 4 * h +
                                               lrow * (int64_t)A.width);
    }
    if (F.G && vec4) {  // plain coefficients, 16-B aligned: 6 float4 loads per thread in flight
      constexpr int R4 = NT * 8;  // float4 per staged row
      constexpr int PER = NN_KCH * R4 / NN_T;
      static_assert(PER >= 1 && PER * NN_T == NN_KCH * R4, "F chunk split over the threads");
      f32x4 tv[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = threadIdx.x + u * NN_T;
        const int k = e / R4, j = (e % R4) * 4;
        const bool ok = k < kn && j < cb;
        const f32x4 v = *reinterpret_cast<const f32x4*>(F.G + (ok ? (int64_t)(k0 + k) * F.ldg + j : 0));
        tv[u] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = threadIdx.x + u * NN_T;
        *reinterpret_cast<f32x4*>(&fs[e / R4][(e % R4) * 4]) = tv[u];
      }
    } else {
      __syncthreads();
      for (int e = threadIdx.x; e < NN_KCH * NT * 32; e += blockDim.x) {
        const int k = e / (NT * 32), j = e % (NT * 32);
        fs[k][j] = (k < kn && j < cb) ? coef_at(F, k0 + k, j, cb) : 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int s8 = 0; s8 < NN_KCH / 8; ++s8) {
      if (8 * s8 >= kn) break;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(
              a4[s8][m], fs[8 * s8 + 4 * h + m][t * 32 + i], acc[t], 0, 0, 0);
      }
    }
  }
  if (r0 >= n) return;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = t * 32 + i;
    const bool colok = col < cb;
    float* ob = colok ? O.blk[col / O.width] + (col % O.width) : nullptr;
    const float* cbp = (colok && beta != 0.f) ? C.blk[col / C.width] + (col % C.width) : nullptr;
    const bool refill = colok && flags && flags[col];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t rr = r0 + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (colok && rr < n) {
        float v = alpha * acc[t][q];
        if (cbp) v += beta * cbp[rr * (int64_t)C.width];
        if (refill) v = counter_normal(seed, (uint64_t)(row0 + rr) * 64 + col);
        ob[rr * (int64_t)O.width] = v;
      }
    }
  }
}

// Ritz vectors and their images in one launch: O0 = A0 F, O1 = A1 F (X = Q S, MX = W S) with the
// whole coefficient matrix F (ca x cb, cb <= 32 NT) staged in LDS ONCE per workgroup (one
// workgroup per CU, 147 KB at ca = 384, NT = 3), then every wave walks 32-row tiles with no
// block barrier: the next 64-deep k chunk of its A rows is loaded while the MFMAs of the
// current one run (ts_nn_kernel re-stages F per chunk between two barriers).  Same MFMA form
// and k permutation as ts_nn_kernel.
#define RZ_T 512  // 8 waves (2 per SIMD: one hides the other's LDS / HBM waits), one F copy
template <int NT>
__global__ __launch_bounds__(RZ_T) void ritz_nn_kernel(BlockList A0, BlockList A1, const float* G,
                                                      int ldg, int cb, OutBlockList O0,
                                                      OutBlockList O1, int64_t n) {
  extern __shared__ __attribute__((aligned(16))) float rf[];  // [ca][NT * 32]
  constexpr int LDF = NT * 32;
  const int ca = A0.count * A0.width;
  {
    // float4 staging, 8 loads in flight per thread (ldg and cb are multiples of 4: checked by
    // the launcher); columns cb .. LDF-1 zero
    constexpr int R4 = LDF / 4;
    const int tot = ca * R4;
    for (int e0 = threadIdx.x; e0 < tot; e0 += RZ_T * 8) {
      f32x4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = min(e0 + RZ_T * u, tot - 1);
        const int k = e / R4, j = (e % R4) * 4;
        t[u] = j < cb ? *reinterpret_cast<const f32x4*>(G + (int64_t)k * ldg + j)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = min(e0 + RZ_T * u, tot - 1);
        *reinterpret_cast<f32x4*>(rf + (e / R4) * LDF + (e % R4) * 4) = t[u];
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int i = lane & 31, h = lane >> 5;
  const int64_t ntile = (n + 31) / 32;
  // wave index made provably uniform (readfirstlane): the tile, the pass and so the block
  // pointers A.blk[k / 8] are then scalar values (scalar loads), not per-lane loads whose
  // waits would serialise the k chunk's data loads
  const int64_t wave0 =
      (int64_t)blockIdx.x * (RZ_T / 64) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t nwaves = (int64_t)gridDim.x * (RZ_T / 64);
  const int npass = O1.count > 0 ? 2 : 1;
  // the B operands of one 8-deep k group: F[kb + 4h + m][t * 32 + i]
  auto load_b = [&](int kb, float (&dst)[4][NT]) {
    const float* fr = rf + (kb + 4 * h) * LDF + i;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t) dst[m][t] = fr[m * LDF + t * 32];
  };
  for (int64_t tile = wave0; tile < ntile * npass; tile += nwaves) {
    const int pass = (int)(tile / ntile);
    const BlockList& A = pass ? A1 : A0;
    const OutBlockList& O = pass ? O1 : O0;
    const int64_t r0 = (tile % ntile) * 32;
    const int64_t row = r0 + i;
    const int64_t lrow = row < n ? row : n - 1;
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{0.f};
    f32x4 cur[8], nxt[8];
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      const int kg = min(8 * s8, ca - 8);
      cur[s8] = *reinterpret_cast<const f32x4*>(A.blk[kg / 8] + 4 * h + lrow * 8);
    }
    float bc[4][NT];
    load_b(0, bc);
    for (int k0 = 0; k0 < ca; k0 += 64) {
      const int kn = min(64, ca - k0);
      if (k0 + 64 < ca) {
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) {
          const int kg = min(k0 + 64 + 8 * s8, ca - 8);
          nxt[s8] = *reinterpret_cast<const f32x4*>(A.blk[kg / 8] + 4 * h + lrow * 8);
        }
      }
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8) {
        if (8 * s8 >= kn) break;
        // the next group's LDS reads are issued before this group's 4 NT MFMAs (one wave per
        // SIMD: nothing else would hide their latency); the sched barriers keep them there
        float bn[4][NT];
        load_b(min(k0 + 8 * s8 + 8, ca - 8), bn);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[s8][m], bc[m][t], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int t = 0; t < NT; ++t) bc[m][t] = bn[m][t];
      }
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8) cur[s8] = nxt[s8];
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = t * 32 + i;
      if (col >= cb) continue;
      float* ob = O.blk[col / O.width] + (col % O.width);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t rr = r0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (rr < n) ob[rr * (int64_t)O.width] = acc[t][q];
      }
    }
  }
}

// X = Q S and MX = W S (O1.count == 0: X only); hipErrorNotSupported when the coefficients do
// not fit one CU's LDS (the caller then uses n2v2r_launch_ts_nn per product)
extern "C" hipError_t n2v2r_launch_ritz_nn(const BlockList& A0, const BlockList& A1, const float* G,
                                           int ldg, int cb, const OutBlockList& O0,
                                           const OutBlockList& O1, int64_t n, int grid,
                                           hipStream_t stream) {
  if (A0.width != 8 || O0.width < 1 || cb < 1 || cb > 96 || n < 1) return hipErrorInvalidValue;
  if (ldg % 4 || cb % 4 || (reinterpret_cast<uintptr_t>(G) & 15)) return hipErrorNotSupported;
  if (O1.count > 0 && (A1.count != A0.count || A1.width != 8 || O1.width != O0.width))
    return hipErrorInvalidValue;
  const int nt = (cb + 31) / 32;
  const size_t lds = sizeof(float) * (size_t)A0.count * 8 * nt * 32;
  if (lds > 150 * 1024) return hipErrorNotSupported;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)ritz_nn_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    (void)hipFuncSetAttribute((const void*)ritz_nn_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    (void)hipFuncSetAttribute((const void*)ritz_nn_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    (void)hipGetLastError();
    attr = true;
  }
  const dim3 g((unsigned)(grid > 0 ? grid : 256));
  switch (nt) {
    case 1: hipLaunchKernelGGL(ritz_nn_kernel<1>, g, dim3(RZ_T), lds, stream, A0, A1, G, ldg, cb, O0, O1, n); break;
    case 2: hipLaunchKernelGGL(ritz_nn_kernel<2>, g, dim3(RZ_T), lds, stream, A0, A1, G, ldg, cb, O0, O1, n); break;
    default: hipLaunchKernelGGL(ritz_nn_kernel<3>, g, dim3(RZ_T), lds, stream, A0, A1, G, ldg, cb, O0, O1, n); break;
  }
  return hipGetLastError();
}

// Narrow outputs (cb <= 16, the Krylov block at b = 8/16): one thread per row, F staged in LDS
// and read as broadcasts, A rows read as 16-B loads (consecutive lanes read consecutive rows of
// a block: coalesced).  VALU FMAs; the pass is HBM-bound on A.
template <int CB>
__global__ __launch_bounds__(256) void ts_nn_rows_kernel(BlockList A, Coef F, int cb,
                                                         OutBlockList O, BlockList C, float alpha,
                                                         float beta, int64_t n, const int* cond,
                                                         const int* flags, uint64_t seed,
                                                         int64_t row0) {
  if (cond && *cond == 0) return;
  extern __shared__ __attribute__((aligned(16))) float gs[];
  const int ca = A.count * A.width;
  for (int e = threadIdx.x; e < ca * CB; e += blockDim.x) {
    const int k = e / CB, j = e % CB;
    gs[e] = (j < cb) ? coef_at(F, k, j, cb) : 0.f;
  }
  __syncthreads();
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  float acc[CB];
#pragma unroll
  for (int j = 0; j < CB; ++j) acc[j] = 0.f;
  const int w = A.width;
  int q = 0;
  if (w == CB) {  // Krylov blocks: 4 blocks (4 x CB/4 16-B loads) in flight per step
    constexpr int NL = CB / 4;
    for (; q + 4 <= A.count; q += 4) {
      f32x4 a4[4][NL];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int l = 0; l < NL; ++l)
          a4[u][l] = *reinterpret_cast<const f32x4*>(A.blk[q + u] + row * (int64_t)CB + 4 * l);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          const float* g = gs + ((q + u) * CB + 4 * l) * CB;
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[j] += a4[u][l][m] * g[m * CB + j];
        }
    }
  }
  for (; q < A.count; ++q) {
    const float* ap = A.blk[q] + row * (int64_t)w;
    for (int kk = 0; kk < w; kk += 4) {
      const f32x4 a4 = *reinterpret_cast<const f32x4*>(ap + kk);
      const float* g = gs + (q * w + kk) * CB;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < CB; ++j) acc[j] += a4[m] * g[m * CB + j];
    }
  }
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    if (j >= cb) break;
    float v = alpha * acc[j];
    if (beta != 0.f) v += beta * C.blk[j / C.width][row * (int64_t)C.width + (j % C.width)];
    if (flags && flags[j]) v = counter_normal(seed, (uint64_t)(row0 + row) * 64 + j);
    O.blk[j / O.width][row * (int64_t)O.width + (j % O.width)] = v;
  }
}

static hipError_t launch_nn(const BlockList& A, const Coef& F, int cb, const OutBlockList& O,
                            const BlockList& C, float alpha, float beta, int64_t n,
                            const int* cond, const int* flags, uint64_t seed, int64_t row0,
                            hipStream_t stream) {
  if ((A.count * A.width) % 8 != 0 || A.width % 8 != 0) return hipErrorInvalidValue;
  const size_t lds8 = sizeof(float) * (size_t)A.count * A.width * 8;
  const size_t lds16 = 2 * lds8;
  if (cb <= 8 && lds8 <= 64 * 1024) {
    hipLaunchKernelGGL(ts_nn_rows_kernel<8>, dim3((unsigned)((n + 255) / 256)), dim3(256), lds8,
                       stream, A, F, cb, O, C, alpha, beta, n, cond, flags, seed, row0);
    return hipGetLastError();
  }
  if (cb <= 16 && lds16 <= 64 * 1024) {
    hipLaunchKernelGGL(ts_nn_rows_kernel<16>, dim3((unsigned)((n + 255) / 256)), dim3(256), lds16,
                       stream, A, F, cb, O, C, alpha, beta, n, cond, flags, seed, row0);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((n + 32 * NN_WAVES - 1) / (32 * NN_WAVES)));
  switch ((cb + 31) / 32) {
    case 1: hipLaunchKernelGGL(ts_nn_kernel<1>, grid, dim3(NN_T), 0, stream, A, F, cb, O, C, alpha, beta, n, cond, flags, seed, row0); break;
    case 2: hipLaunchKernelGGL(ts_nn_kernel<2>, grid, dim3(NN_T), 0, stream, A, F, cb, O, C, alpha, beta, n, cond, flags, seed, row0); break;
    case 3: hipLaunchKernelGGL(ts_nn_kernel<3>, grid, dim3(NN_T), 0, stream, A, F, cb, O, C, alpha, beta, n, cond, flags, seed, row0); break;
    case 4: hipLaunchKernelGGL(ts_nn_kernel<4>, grid, dim3(NN_T), 0, stream, A, F, cb, O, C, alpha, beta, n, cond, flags, seed, row0); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// flags (nullptr = none): output columns j with flags[j] != 0 are written with N(0,1) deviates
// (counter-based, seed) instead of the product: the refill of rank-deficient Krylov columns.
extern "C" hipError_t n2v2r_launch_ts_nn(const BlockList& A, const float* G, int ldg, int cb,
                                         const OutBlockList& O, const BlockList& C, float alpha,
                                         float beta, int64_t n, const int* cond,
                                         const int* flags, uint64_t seed, hipStream_t stream) {
  const Coef F{G, ldg, nullptr, nullptr, 0};
  return launch_nn(A, F, cb, O, C, alpha, beta, n, cond, flags, seed, 0, stream);
}

// Z <- [Q Z] F, F = [-C R^{-1}; R^{-1}] (fp32 (c + b) x b, formed by pip_chol): the fused
// BCGS + CholQR apply.
extern "C" hipError_t n2v2r_launch_pip_apply(const BlockList& QZ, const float* Fm, int c, int b,
                                             const OutBlockList& Z, int64_t n, const int* cond,
                                             const int* flags, uint64_t seed, int64_t row0,
                                             hipStream_t stream) {
  (void)c;
  const Coef F{Fm, b, nullptr, nullptr, 0};
  BlockList none{};
  return launch_nn(QZ, F, b, Z, none, 1.f, 0.f, n, cond, flags, seed, row0, stream);
}

// ----------------------------------------------------------------------------- small ops
// fp64 -> fp32 copy of a (rows x cols) matrix with optional negation (CGS coefficients).
__global__ void f64_to_f32_kernel(const double* __restrict__ in, float* __restrict__ out,
                                  int64_t elems, float scale, const int* cond) {
  if (cond && *cond == 0) return;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < elems) out[e] = scale * (float)in[e];
}

extern "C" hipError_t n2v2r_launch_f64_to_f32(const double* in, float* out, int64_t elems,
                                              float scale, const int* cond, hipStream_t stream) {
  hipLaunchKernelGGL(f64_to_f32_kernel, dim3((unsigned)((elems + 255) / 256)), dim3(256), 0,
                     stream, in, out, elems, scale, cond);
  return hipGetLastError();
}

// Cholesky G = R^T R of a b x b fp64 Gram matrix and Rinv = R^{-1} (fp32, row-major b x b),
// one 1024-thread workgroup, every step parallel over the trailing b x b entries.
// A pivot below 1e-10 * max diag marks a rank-deficient column: its R row becomes the unit row,
// its Rinv column is zeroed and flags[j] / *any_flag are set.
__global__ __launch_bounds__(1024) void chol_inv_kernel(const double* __restrict__ G, int b,
                                                        float* __restrict__ Rinv, int* flags,
                                                        int* any_flag) {
  __shared__ double R[64][65];
  __shared__ double X[64][65];
  __shared__ double piv[64];
  __shared__ int bad[64];
  __shared__ double dmax;
  const int tid = threadIdx.x;
  const int nt = blockDim.x;
  for (int e = tid; e < b * b; e += nt) {
    const int r = e / b, c = e % b;
    R[r][c] = 0.5 * (G[r * b + c] + G[c * b + r]);
    X[r][c] = (r == c) ? 1.0 : 0.0;
  }
  if (tid < 64) bad[tid] = 0;
  __syncthreads();
  if (tid < 64) {
    double m = (tid < b) ? R[tid][tid] : 0.0;
    for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if (tid == 0) dmax = m;
  }
  __syncthreads();
  const double tiny = 1e-10 * dmax;
  // right-looking: row j of R = (row j of the Schur complement) / sqrt(pivot)
  for (int j = 0; j < b; ++j) {
    if (tid == 0) {
      const double p = R[j][j];
      if (!(p > tiny)) {
        bad[j] = 1;
        piv[j] = 0.0;
      } else {
        piv[j] = sqrt(p);
      }
    }
    __syncthreads();
    const double pj = piv[j];
    const int isbad = bad[j];
    // scale row j (c >= j)
    for (int c = j + tid; c < b; c += nt) R[j][c] = isbad ? (c == j ? 1.0 : 0.0) : (c == j ? pj : R[j][c] / pj);
    __syncthreads();
    // trailing update R[r][c] -= R[j][r] R[j][c], j < r <= c
    const int m = b - j - 1;
    for (int e = tid; e < m * m; e += nt) {
      const int r = j + 1 + e / m, c = j + 1 + e % m;
      if (c >= r) R[r][c] -= R[j][r] * R[j][c];
    }
    __syncthreads();
  }
  // Gauss-Jordan on [R | I] from the last row up: X <- R^{-1}
  for (int j = b - 1; j >= 0; --j) {
    const double inv = 1.0 / R[j][j];
    for (int c = tid; c < b; c += nt) X[j][c] *= inv;
    __syncthreads();
    for (int e = tid; e < j * b; e += nt) {
      const int r = e / b, c = e % b;
      X[r][c] -= R[r][j] * X[j][c];
    }
    __syncthreads();
  }
  int any = 0;
  for (int j = 0; j < b; ++j) any |= bad[j];
  for (int e = tid; e < b * b; e += nt) {
    const int r = e / b, c = e % b;
    Rinv[e] = bad[c] ? 0.f : (float)X[r][c];
  }
  if (tid < b) flags[tid] = bad[tid];
  if (tid == 0) *any_flag = any;
}

// Fused block classical Gram-Schmidt + Cholesky QR ("Pythagorean" form): given
// G = [Q Z]^T Z ((c + b) x b, fp64) with C = Q^T Z (first c rows) and Z^T Z (last b rows),
// P = Z^T Z - C^T C is the Gram matrix of Z - Q C.  This kernel forms P (1024 threads, the
// c-long sums split over 16 k-slices and folded in fixed order), then one wave does the
// Cholesky P = R^T R and R^{-1} (xinv, fp64 b x b).  The apply pass builds
// F = [-C R^{-1}; R^{-1}] in LDS and writes Z <- (Z - Q C) R^{-1} in ONE pass over [Q Z].
// Pivots below PIP_CANCEL of the column's own squared norm before the projection are clamped to
// it (the column is scaled, not normalised: any_flag asks for the next pass); zero columns get a
// zero xinv column and a flag (refilled).
// save (optional): rows [save_row0, save_row0 + save_rows) of G copied out (the banded
// Rayleigh-Ritz keeps the local first-pass Gram Q_loc^T W_j as its band column j).
// fout (optional): F = [-C R^{-1}; R^{-1}] as fp32 ((c + b) x b, flagged columns zero), the
// coefficient matrix of the apply pass, formed here once instead of in every apply workgroup.
__global__ __launch_bounds__(1024) void pip_chol_kernel(const double* __restrict__ G, int c, int b,
                                                        double* __restrict__ xinv, int* flags,
                                                        int* any_flag, const int* cond,
                                                        double* __restrict__ save, int save_row0,
                                                        int save_rows, float* __restrict__ fout,
                                                        int stage, int* sticky,
                                                        double* __restrict__ rsave, int first) {
  // grid.x > 1 (wide blocks, long bases): every workgroup forms P and factors it (redundant,
  // bit-identical), workgroup g writes rows [g, g + 1) * ceil((c + b) / grid.x) of F, and
  // workgroup 0 alone the other outputs
  const bool lead = blockIdx.x == 0;
  if (cond && *cond == 0) {
    if (lead && threadIdx.x < b) flags[threadIdx.x] = 0;
    if (lead && threadIdx.x == 0) *any_flag = 0;
    if (rsave && lead && threadIdx.x < b * b)
      rsave[threadIdx.x] = (int)threadIdx.x / b == (int)threadIdx.x % b ? 1.0 : 0.0;
    return;
  }
  const int fper = (c + b + gridDim.x - 1) / gridDim.x;
  const int fbeg = blockIdx.x * fper, fend = min(c + b, fbeg + fper);
  if (save && lead)
    for (int e = threadIdx.x; e < save_rows * b; e += blockDim.x)
      save[e] = G[(int64_t)save_row0 * b + e];
  // G staged through LDS when it fits (b = 8: (c + 8) x 8 doubles <= 50 KB): the P and F loops
  // below then read LDS instead of issuing dependent L2 loads
  extern __shared__ double gstage[];
  const double* Gs = G;
  if (stage) {
    const int n2 = ((c + b) * b) / 2;
    const double2* src = reinterpret_cast<const double2*>(G);
    double2* dst = reinterpret_cast<double2*>(gstage);
    for (int e0 = threadIdx.x; e0 < n2; e0 += blockDim.x * 4) {  // 4 loads in flight
      double2 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = src[min(e0 + (int)blockDim.x * u, n2 - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u) dst[min(e0 + (int)blockDim.x * u, n2 - 1)] = t[u];
    }
    if (threadIdx.x == 0 && ((c + b) * b) % 2) gstage[(c + b) * b - 1] = G[(c + b) * b - 1];
    __syncthreads();
    Gs = gstage;
  }
  __shared__ double R[64][65];
  __shared__ double X[64][65];
  __shared__ double part[16][64];
  __shared__ double piv[64];
  __shared__ int bad[64];
  __shared__ double dmax;
  const int tid = threadIdx.x;
  const int nt = blockDim.x;
  const int bb = b * b;
  if (bb <= 64) {
    const int e = tid % 64, slice = tid / 64;
    double acc = 0.0;
    if (e < bb) {
      const int i = e / b, j = e % b;
      for (int k = slice; k < c; k += 16) acc += Gs[(int64_t)k * b + i] * Gs[(int64_t)k * b + j];
    }
    part[slice][e] = acc;
    __syncthreads();
    if (tid < bb) {
      const int i = tid / b, j = tid % b;
      double s = 0.5 * (Gs[(int64_t)(c + i) * b + j] + Gs[(int64_t)(c + j) * b + i]);
      for (int sl = 0; sl < 16; ++sl) s -= part[sl][tid];
      R[i][j] = s;
    }
  } else if (stage) {
    for (int e = tid; e < bb; e += nt) {
      const int i = e / b, j = e % b;
      double s = 0.5 * (Gs[(int64_t)(c + i) * b + j] + Gs[(int64_t)(c + j) * b + i]);
      for (int k = 0; k < c; ++k) s -= Gs[(int64_t)k * b + i] * Gs[(int64_t)k * b + j];
      R[i][j] = s;
    }
  } else {
    // G beyond the staging size (b = 32 / 64 blocks, long bases: cfg3): C = Q^T Z goes through
    // LDS 4096 / b rows at a time (X's storage, not yet in use), every thread's loads of a chunk
    // in flight together, and each entry of C^T C accumulates from LDS (was: c dependent L2
    // loads per entry, ~170 us per call at c = 768, b = 32)
    double* cst = &X[0][0];
    const int rows = 4096 / b;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // entries tid + nt u, bb <= 4096
    for (int k0 = 0; k0 < c; k0 += rows) {
      const int kr = min(rows, c - k0);
      const int tot = kr * b;
      __syncthreads();
      for (int q0 = tid; q0 < tot; q0 += nt * 4) {
        double t4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t4[u] = G[(int64_t)k0 * b + min(q0 + nt * u, tot - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) cst[min(q0 + nt * u, tot - 1)] = t4[u];
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = tid + nt * u;
        if (e < bb) {
          const int i = e / b, j = e % b;
          double a0 = 0.0, a1 = 0.0;
          int k = 0;
          for (; k + 1 < kr; k += 2) {
            a0 += cst[k * b + i] * cst[k * b + j];
            a1 += cst[(k + 1) * b + i] * cst[(k + 1) * b + j];
          }
          if (k < kr) a0 += cst[k * b + i] * cst[k * b + j];
          acc[u] += a0 + a1;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + nt * u;
      if (e < bb) {
        const int i = e / b, j = e % b;
        R[i][j] = 0.5 * (G[(int64_t)(c + i) * b + j] + G[(int64_t)(c + j) * b + i]) - acc[u];
      }
    }
    __syncthreads();
  }
  for (int e = tid; e < bb; e += nt) X[e / b][e % b] = (e / b == e % b) ? 1.0 : 0.0;
  if (tid < 64) bad[tid] = 0;
  // the columns' squared norms before the projection (Z^T Z's diagonal): the pivots are clamped
  // to PIP_CANCEL of them, and zero columns (relative to the block's largest) are refilled
  __shared__ double zzd[64];
  __shared__ int canc[64];
  if (tid < b) zzd[tid] = G[(int64_t)(c + tid) * b + tid];
  if (tid < 64) canc[tid] = 0;
  __syncthreads();
  if (tid < 64) {
    double m = (tid < b) ? zzd[tid] : 0.0;
    for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if (tid == 0) dmax = 1e-30 * m;  // the zero-column floor
  }
  __syncthreads();
  if (b > 8 && bb <= nt) {
    // 8 < b <= 32: one thread per entry of the b x b matrix, the upper triangle in registers,
    // one workgroup barrier per elimination step and per substitution step (the wave-0 form
    // below serialises ~b^3 / 64 dependent LDS updates: ~110 us per call at b = 32)
    const int ei = tid / b, ej = tid % b;
    const bool own = tid < bb;
    double v = own ? R[ei][ej] : 0.0;
    const double zfloor = dmax;
    for (int k = 0; k < b; ++k) {
      // row k of R in LDS holds its values after step k - 1 (written before the barrier)
      const double d = R[k][k];
      const double zz = zzd[k];
      const bool cn = !(d > PIP_CANCEL * zz);  // (a later pass refills: see pip_fused_kernel)
      const bool isbad = !(zz > zfloor) || !(d == d) || (cn && !first);
      const bool cj = !isbad && cn;
      const double pk = isbad ? 1.0 : sqrt(cj ? PIP_CANCEL * zz : d);
      if (own && ei == k) {  // (a clamped column is decoupled: see pip_fused_kernel)
        v = (isbad || cj) ? (ej == k ? pk : 0.0) : (ej == k ? pk : v / pk);
      } else if (own && ei > k && ej >= ei && !isbad && !cj) {
        v -= (R[k][ei] / pk) * (R[k][ej] / pk);
      }
      if (tid == 0) {
        bad[k] = isbad ? 1 : 0;
        canc[k] = cj ? 1 : 0;
      }
      if (own && ei == k + 1) R[k + 1][ej] = v;  // the next pivot row (no reader this step)
      __syncthreads();
    }
    if (own && ej >= ei) R[ei][ej] = v;  // final R (upper triangle)
    __syncthreads();
    // X = R^{-1} (upper triangular) by back substitution, x = X[ei][ej] in a register: step j
    // finishes row j (scaled by 1 / R[j][j], published), then every row above subtracts it
    double x = (own && ei == ej) ? 1.0 : 0.0;
    for (int j = b - 1; j >= 0; --j) {
      if (own && ei == j) {
        x *= 1.0 / R[j][j];
        X[j][ej] = x;
      }
      __syncthreads();
      if (own && ei < j) x -= R[ei][j] * X[j][ej];
    }
  } else if (tid < 64) {
    // O(b^3), b <= 64: wave 0 alone, synchronised as a wave (LDS executes a wave's accesses in
    // order; the waits only keep the compiler from reordering), the other waves wait at the
    // barrier below -- no block-wide barrier per elimination step
    const int nw = 64;
#define PIP_WSYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
    const double zfloor = dmax;
    for (int j = 0; j < b; ++j) {
      if (tid == 0) {
        const double p = R[j][j];
        const double zz = zzd[j];
        const bool cn = !(p > PIP_CANCEL * zz);
        if (!(zz > zfloor) || !(p == p) || (cn && !first)) {
          bad[j] = 1;
          piv[j] = 0.0;
        } else {
          const bool cj = cn;
          canc[j] = cj ? 1 : 0;
          piv[j] = sqrt(cj ? PIP_CANCEL * zz : p);
        }
      }
      PIP_WSYNC();
      const double pj = piv[j];
      const int isbad = bad[j], iscanc = canc[j];
      for (int cc = j + tid; cc < b; cc += nw)
        R[j][cc] = isbad ? (cc == j ? 1.0 : 0.0)
                         : (cc == j ? pj : (iscanc ? 0.0 : R[j][cc] / pj));
      PIP_WSYNC();
      const int m = b - j - 1;
      for (int e = tid; e < m * m; e += nw) {
        const int r = j + 1 + e / m, cc = j + 1 + e % m;
        if (cc >= r) R[r][cc] -= R[j][r] * R[j][cc];
      }
      PIP_WSYNC();
    }
    for (int j = b - 1; j >= 0; --j) {
      const double inv = 1.0 / R[j][j];
      for (int cc = tid; cc < b; cc += nw) X[j][cc] *= inv;
      PIP_WSYNC();
      for (int e = tid; e < j * b; e += nw) {
        const int r = e / b, cc = e % b;
        X[r][cc] -= R[r][j] * X[j][cc];
      }
      PIP_WSYNC();
    }
#undef PIP_WSYNC
  }
  __syncthreads();
  if (lead)
    for (int e = tid; e < bb; e += nt) {
      const int r = e / b, cc = e % b;
      xinv[e] = bad[cc] ? 0.0 : X[r][cc];
      // R (upper, row-major; a refilled column's row zero): Z - Q C = Z_out R
      if (rsave) rsave[e] = (cc >= r && !bad[r]) ? R[r][cc] : 0.0;
    }
  if (lead && tid < b) flags[tid] = bad[tid];
  if (lead && tid == 0) {
    int any = 0;
    for (int j = 0; j < b; ++j) any |= bad[j] | canc[j];
    *any_flag = any;
    if (any && sticky) *sticky = 1;
  }
  if (fout && !stage && bb > 64) {
    // the same F with C through LDS in chunks (R's storage: R is spent once xinv is out), this
    // workgroup's rows [fbeg, fend) only
    double* cst = &R[0][0];
    const int rows = 4096 / b;
    const int cend = min(c, fend);
    for (int k0 = fbeg; k0 < cend; k0 += rows) {
      const int kr = min(rows, cend - k0);
      const int tot = kr * b;
      __syncthreads();
      for (int q0 = tid; q0 < tot; q0 += nt * 4) {
        double t4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t4[u] = G[(int64_t)k0 * b + min(q0 + nt * u, tot - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) cst[min(q0 + nt * u, tot - 1)] = t4[u];
      }
      __syncthreads();
      for (int e = tid; e < tot; e += nt) {
        const int kk = e / b, j = e % b;
        float v = 0.f;
        if (!bad[j]) {
          double sacc = 0.0;
          for (int m = 0; m <= j; ++m) sacc -= cst[kk * b + m] * X[m][j];
          v = (float)sacc;
        }
        fout[(int64_t)k0 * b + e] = v;
      }
    }
    for (int e = tid; e < bb; e += nt) {
      const int i = e / b, j = e % b;
      if (c + i >= fbeg && c + i < fend)
        fout[(int64_t)(c + i) * b + j] = bad[j] ? 0.f : (float)X[i][j];
    }
  } else if (fout) {  // every thread: F[k][j] = -sum_{m <= j} C[k][m] X[m][j]; F[c + i][j] = X[i][j]
    for (int e = tid + fbeg * b; e < fend * b; e += nt) {
      const int k = e / b, j = e % b;
      float v = 0.f;
      if (!bad[j]) {
        if (k >= c) {
          v = (float)X[k - c][j];
        } else {
          const double* crow = Gs + (int64_t)k * b;
          double sacc = 0.0;
          for (int m = 0; m <= j; ++m) sacc -= crow[m] * X[m][j];
          v = (float)sacc;
        }
      }
      fout[e] = v;
    }
  }
}

extern "C" hipError_t n2v2r_launch_pip_chol(const double* G, int c, int b, double* xinv,
                                            int* flags, int* any_flag, const int* cond,
                                            double* save, int save_row0, int save_rows,
                                            float* fout, int* sticky, double* rsave,
                                            int first, hipStream_t stream) {
  if (b > 64) return hipErrorInvalidValue;
  const size_t gbytes = sizeof(double) * (size_t)(c + b) * b;
  const int stage = gbytes <= 56 * 1024 ? 1 : 0;
  // wide blocks with F wanted: F's rows over up to 8 workgroups (each factors P itself)
  const int nwg = (fout && b > 8) ? std::min(8, (c + b + 127) / 128) : 1;
  hipLaunchKernelGGL(pip_chol_kernel, dim3(nwg), dim3(1024), stage ? gbytes : 0, stream, G, c, b,
                     xinv, flags, any_flag, cond, save, save_row0, save_rows, fout, stage, sticky,
                     rsave, first);
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_chol_inv(const double* G, int b, float* Rinv, int* flags,
                                            int* any_flag, hipStream_t stream) {
  if (b > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(chol_inv_kernel, dim3(1), dim3(1024), 0, stream, G, b, Rinv, flags, any_flag);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- fused PIP pass
// One launch per BCGS-PIP pass at b = 8 (replaces pip_chol + the apply): every workgroup stages
// the Gram G = [Q Z]^T Z ((c + 8) x 8 fp64, C = Q^T Z its first c rows) in LDS, forms
// P = Z^T Z - C^T C (4 k-slices, fixed fold order), factors P = R^T R and inverts R with wave 0
// lane-parallel (lane = (i, j) entry, pivots by readlane, row/column operands by shuffles: no
// block barrier per step), then streams its 256 rows: Z <- (Z - Q C) R^{-1}, flagged columns
// refilled by counter deviates.  Every workgroup forms the same R from the same G (the
// factorisation is deterministic); workgroup 0 alone writes flags / any_flag / sticky / save.
// Same pivot rule as pip_chol_kernel (PIP_CANCEL clamp; zero columns: unit row, zero R^{-1} column).
// 1 / sqrt(p), p > 0: hardware estimate + two Newton steps (full fp64 precision)
__device__ __forceinline__ double rsq_nr(double p) {
  double r = __builtin_amdgcn_rsq(p);
  r = r * fma(-0.5 * p * r, r, 1.5);
  r = r * fma(-0.5 * p * r, r, 1.5);
  return r;
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

template <int QB, int NU, bool NT>
__global__ __launch_bounds__(256) void pip_fused_kernel(BlockList Q, const float* Zin, float* Zout,
                                                        const double* __restrict__ G, int c,
                                                        int64_t n, const int* cond, int* flags,
                                                        int* any_flag, double* save, int save_row0,
                                                        int save_rows, int* sticky, uint64_t seed,
                                                        int64_t row0, double* rsave, float skip_tol,
                                                        int* skipped, int first) {
  const int tid = threadIdx.x;
  const bool lead = blockIdx.x == 0;
  if (cond && *cond == 0) {
    if (lead && tid < 8) flags[tid] = 0;
    if (lead && tid == 0) *any_flag = 0;
    return;
  }
  // one LDS array: gd (c + 8) x 8 fp64 | part 4 x 64 fp64 | cf c x 8 fp32 | rv 8 x 8 fp32 | mask
  extern __shared__ __attribute__((aligned(16))) double pf_lds[];
  double* gd = pf_lds;
  double* part = gd + (c + 8) * 8;
  float* cf = reinterpret_cast<float*>(part + 256);
  float* rv = cf + c * 8;
  int* badw = reinterpret_cast<int*>(rv + 64);
  const int ne2 = (c + 8) * 4;  // double2 count
  // all of a thread's G loads in flight before the first LDS write (a load -> wait -> write
  // loop costs one L2 round trip per 256 entries: ~7 of them at c = 384)
  for (int e0 = tid; e0 < ne2; e0 += 256 * 8) {
    double2 t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)  // clamped, unconditional: the loads cannot sink into branches
      t[u] = reinterpret_cast<const double2*>(G)[min(e0 + 256 * u, ne2 - 1)];
#pragma unroll
    for (int u = 0; u < 8; ++u)  // past the end: the last entry again, with its own value
      reinterpret_cast<double2*>(gd)[min(e0 + 256 * u, ne2 - 1)] = t[u];
  }
  __syncthreads();
  // the basis blocks this pass applies: all, or (skip_tol > 0: selective reorthogonalisation of
  // an in-place pass) those with max_ij |C_ij| / ||z_j|| > skip_tol; every workgroup decides
  // alike from the same G.  C^T C sums the applied blocks only, so R factors the applied pass.
  // (skip_tol < 0: the whole pass, all blocks or none, by |skip_tol|)
  int* blist = badw + 4;  // compact list of applied blocks (<= N2V2R_BAND_MAXC / 8)
  const int nblk = c >> 3;
  const bool skip_whole = skip_tol < 0.f;
  skip_tol = fabsf(skip_tol);
  int* bflag = reinterpret_cast<int*>(part);  // per-block verdicts (part is free until C^T C)
  if (skip_tol > 0.f) {
    // wave w tests blocks w, w + 4, ...: lane = entry (r, j) of the block's 8 x 8 C rows
    const int lane = tid & 63;
    const double thr = (double)skip_tol * (double)skip_tol *
                       fmax(gd[(c + (lane & 7)) * 8 + (lane & 7)], 1e-300);
    for (int bk = tid >> 6; bk < nblk; bk += 4) {
      const double g = gd[bk * 64 + lane];
      const unsigned long long bm = __ballot(g * g > thr);
      if (lane == 0) bflag[bk] = bm != 0ull;
    }
    __syncthreads();
  }
  // a pass that would apply no block still runs when Z's own Gram is off the identity by more
  // than skip_tol (its Cholesky step is what restores orthonormality inside the block)
  int zz_off = 0;
  if (skip_tol > 0.f && tid < 64) {
    const int i = tid >> 3, j = tid & 7;
    zz_off = __ballot(fabs(gd[(c + i) * 8 + j] - (i == j ? 1.0 : 0.0)) > (double)skip_tol) != 0ull;
  }
  if (tid < 64) {
    // wave 0 compacts the verdicts 64 blocks at a time (bases up to N2V2R_BAND_MAXC columns:
    // 80 blocks; round 4's single ballot covered 64, so blocks past 512 columns were never
    // applied)
    bool any_on = false;
    for (int c0 = 0; c0 < nblk; c0 += 64) {
      const int bk = c0 + tid;
      const bool on = bk < nblk && (skip_tol <= 0.f || bflag[bk] != 0);
      any_on |= __ballot(on) != 0ull;
    }
    const bool all = skip_whole && any_on;
    int count = 0;
    for (int c0 = 0; c0 < nblk; c0 += 64) {
      const int bk = c0 + tid;
      const bool on = bk < nblk && (all || skip_tol <= 0.f || bflag[bk] != 0);
      const unsigned long long m = __ballot(on);
      if (on) blist[count + __popcll(m & ((1ull << tid) - 1ull))] = bk;
      if (skipped && lead && on && skip_tol > 0.f) atomicAdd(skipped + 1 + bk, 1);  // histogram
      count += __popcll(m);
    }
    if (tid == 0) {
      badw[1] = count;
      badw[2] = zz_off;
      badw[3] = 0;
    }
  }
  __syncthreads();
  const int napply = badw[1];
  if (skip_tol > 0.f) {
    if (napply == 0 && !badw[2]) {
      if (lead && tid < 8) flags[tid] = 0;
      if (rsave && lead && tid < 64) rsave[tid] = (tid >> 3) == (tid & 7) ? 1.0 : 0.0;  // R = I
      if (lead && tid == 0) {
        *any_flag = 0;
        if (skipped) atomicAdd(skipped, 1);
      }
      return;
    }
  }
  if (save && lead)
    for (int e = tid; e < save_rows * 8; e += 256) save[e] = gd[save_row0 * 8 + e];
  // fp32 coefficients and C^T C of the applied blocks only (a selective pass applies ~7 of 48
  // at cfg2: the pass over all of C was 2.8 us of the launch, zeroing the skipped rows 1.0)
  for (int e = tid; e < napply * 64; e += 256) {
    const int g = blist[e >> 6] * 64 + (e & 63);
    cf[g] = (float)gd[g];
  }
  {
    const int e = tid & 63, sl = tid >> 6, i = e >> 3, j = e & 7;
    // wave sl: list entries sl, sl + 4, ...; four independent chains (rows r mod 4)
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    for (int q = sl; q < napply; q += 4) {
      const double* g = gd + blist[q] * 64;
#pragma unroll
      for (int r = 0; r < 8; r += 4) {
        a0 += g[r * 8 + i] * g[r * 8 + j];
        a1 += g[(r + 1) * 8 + i] * g[(r + 1) * 8 + j];
        a2 += g[(r + 2) * 8 + i] * g[(r + 2) * 8 + j];
        a3 += g[(r + 3) * 8 + i] * g[(r + 3) * 8 + j];
      }
    }
    part[sl * 64 + e] = (a0 + a1) + (a2 + a3);
  }
  __syncthreads();
  if (tid < 64) {  // P = Z^T Z - C^T C (each lane reads only its own part[] entries)
    const int i = tid >> 3, j = tid & 7;
    const double v = 0.5 * (gd[(c + i) * 8 + j] + gd[(c + j) * 8 + i]);
    part[tid] = v - part[tid] - part[64 + tid] - part[128 + tid] - part[192 + tid];
  }
  __syncthreads();
  if (tid < 64) {
    const int i = tid >> 3, j = tid & 7;
    // every lane factors the whole 8 x 8 P = R^T R in registers: no cross-lane traffic, and
    // pivots by rsq + Newton, so no division or square root on the chain (the lane-per-entry
    // form, two fp64 shuffles and a division per step, was 2.5 us of every launch)
    double R[8][8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int q = r; q < 8; ++q) R[r][q] = part[r * 8 + q];
    // zero columns (relative to the block's largest) are refilled; see PIP_CANCEL
    double zmax = 0.0;
#pragma unroll
    for (int r = 0; r < 8; ++r) zmax = fmax(zmax, gd[(c + r) * 8 + r]);
    const double zfloor = 1e-30 * zmax;
    int bad = 0, cancel = 0;
    double rinv[8];
    // right-looking Cholesky: row jj of R = row jj of the Schur complement / sqrt(pivot), the
    // pivot clamped to PIP_CANCEL of the column's squared norm before the projection
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const double p = R[jj][jj];
      const double zz = gd[(c + jj) * 8 + jj];
      // (a later pass: a cancelled column is what the first pass left of a remainder at the
      // rounding level, or a near-copy of another column of the block -- refilled)
      const bool cn = !(p > PIP_CANCEL * zz);
      const bool bj = !(zz > zfloor) || !(p == p) || (cn && !first);
      const bool cj = !bj && cn;
      bad |= (int)bj << jj;
      cancel |= (int)cj << jj;
      const double pe = bj ? 1.0 : (cj ? PIP_CANCEL * zz : p);
      const double r = rsq_nr(pe);
      // a clamped column is decoupled (its row's coupling entries are as untrusted as its pivot:
      // keeping them grew R^{-1} without bound over a block of cancelled columns); the next
      // pass orthogonalises the block's columns against each other
#pragma unroll
      for (int q = jj + 1; q < 8; ++q) R[jj][q] = (bj || cj) ? 0.0 : R[jj][q] * r;
      R[jj][jj] = bj ? 1.0 : pe * r;
      rinv[jj] = bj ? 1.0 : r;
#pragma unroll
      for (int a = jj + 1; a < 8; ++a)
#pragma unroll
        for (int q = a; q < 8; ++q) R[a][q] -= R[jj][a] * R[jj][q];
    }
    // R (row-major, upper): Z - Q C = Z_out R; its columns' norms give the Krylov-Schur
    // residual estimates of the lean-image solver mode
    // (a refilled column's row is zero: the projected block has no component there)
    if (rsave && lead) {
      double rij = 0.0;
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int q = r; q < 8; ++q) rij = (i == r && j == q) ? R[r][q] : rij;
      rsave[tid] = ((bad >> i) & 1) ? 0.0 : rij;
    }
    // column j of R^{-1} by back substitution; this lane keeps entry i
    double xv[8];
#pragma unroll
    for (int a = 7; a >= 0; --a) {
      double t = (a == j) ? 1.0 : 0.0;
#pragma unroll
      for (int k = a + 1; k < 8; ++k) t -= R[a][k] * xv[k];
      xv[a] = t * rinv[a];
    }
    double x = xv[0];
#pragma unroll
    for (int a = 1; a < 8; ++a) x = (i == a) ? xv[a] : x;
    rv[tid] = ((bad >> j) & 1) ? 0.f : (float)x;
    if (tid == 0) badw[0] = bad;
    if (lead) {
      if (tid < 8) flags[tid] = (bad >> tid) & 1;
      if (tid == 0) {
        *any_flag = (bad | cancel) != 0;
        if ((bad | cancel) && sticky) *sticky = 1;
      }
    }
  }
  __syncthreads();
  // rows: wave w owns rows 32 NU w .. 32 NU (w + 1) - 1 of the workgroup's 128 NU, lane =
  // (row offset ro = lane >> 1, column half h = lane & 1) over NU 32-row parts u, so one load
  // instruction reads 32 consecutive 32-B rows of a block (1 KB contiguous)
  const int lane = tid & 63, h = lane & 1, ro = lane >> 1;
  const int64_t rbase = (int64_t)blockIdx.x * (128 * NU) + (tid >> 6) * (32 * NU) + ro;
  if (rbase >= n) return;
  int64_t rw[NU];
  bool okr[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    okr[u] = rbase + 32 * u < n;
    rw[u] = okr[u] ? rbase + 32 * u : rbase;  // past the end: row rbase again, not stored
  }
  float acc[NU][8];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const f32x4 z = *reinterpret_cast<const f32x4*>(Zin + rw[u] * 8 + 4 * h);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[u][t] = h ? 0.f : z[t];
      acc[u][4 + t] = h ? z[t] : 0.f;
    }
  }
  int q = 0;
  for (; q + QB <= napply; q += QB) {  // QB blocks x NU rows (QB NU x 16-B loads) in flight
    f32x4 a4[QB][NU];
    int bi[QB];
#pragma unroll
    for (int b4 = 0; b4 < QB; ++b4) bi[b4] = __builtin_amdgcn_readfirstlane(blist[q + b4]);
#pragma unroll
    for (int b4 = 0; b4 < QB; ++b4)
#pragma unroll
      for (int u = 0; u < NU; ++u)
        a4[b4][u] = NT ? __builtin_nontemporal_load(
                             reinterpret_cast<const f32x4*>(Q.blk[bi[b4]] + rw[u] * 8 + 4 * h))
                       : *reinterpret_cast<const f32x4*>(Q.blk[bi[b4]] + rw[u] * 8 + 4 * h);
#pragma unroll
    for (int b4 = 0; b4 < QB; ++b4) {
      const float* g = cf + (bi[b4] * 8 + 4 * h) * 8;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gv = g[m * 8 + j];
#pragma unroll
          for (int u = 0; u < NU; ++u) acc[u][j] -= a4[b4][u][m] * gv;
        }
    }
  }
  for (; q < napply; ++q) {
    f32x4 a4[NU];
    const int bq = __builtin_amdgcn_readfirstlane(blist[q]);
#pragma unroll
    for (int u = 0; u < NU; ++u)
      a4[u] = NT ? __builtin_nontemporal_load(
                       reinterpret_cast<const f32x4*>(Q.blk[bq] + rw[u] * 8 + 4 * h))
                 : *reinterpret_cast<const f32x4*>(Q.blk[bq] + rw[u] * 8 + 4 * h);
    const float* g = cf + (bq * 8 + 4 * h) * 8;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gv = g[m * 8 + j];
#pragma unroll
        for (int u = 0; u < NU; ++u) acc[u][j] -= a4[u][m] * gv;
      }
  }
  const int bad = badw[0];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    // the two column halves of a row sit in adjacent lanes: fold them (quad_perm [1,0,3,2])
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[u][j] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc[u][j]), 0xB1, 0xF, 0xF, false));
    float o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int jo = 4 * h + t;
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += (j <= jo) ? acc[u][j] * rv[j * 8 + jo] : 0.f;
      o[t] = ((bad >> jo) & 1) ? counter_normal(seed, (uint64_t)(row0 + rw[u]) * 64 + jo) : sum;
    }
    if (okr[u]) *reinterpret_cast<f32x4*>(Zout + rw[u] * 8 + 4 * h) = f32x4{o[0], o[1], o[2], o[3]};
  }
}

extern "C" hipError_t n2v2r_launch_pip_fused(const BlockList& Q, const float* Zin, float* Zout,
                                             const double* G, int c, int64_t n, const int* cond,
                                             int* flags, int* any_flag, double* save,
                                             int save_row0, int save_rows, int* sticky,
                                             uint64_t seed, int64_t row0, double* rsave,
                                             float skip_tol, int* skipped, int first,
                                             hipStream_t stream) {
  if (Q.width != 8 || c != Q.count * 8) return hipErrorInvalidValue;
  // a skipped block leaves Z in place; the band save reads G before the skipped rows are zeroed
  if (skip_tol != 0.f && (Zin != Zout || save)) return hipErrorInvalidValue;
  const size_t lds = sizeof(double) * ((size_t)(c + 8) * 8 + 256) + sizeof(float) * ((size_t)c * 8 + 64) + 16 +
                     4 * (size_t)(c / 8 > 64 ? c / 8 : 64);
  if (lds > 80 * 1024 || c > N2V2R_BAND_MAXC) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {  // bases past 640 columns (two workgroups per CU still fit)
    static const hipError_t attr = [] {
      hipError_t e = hipSuccess;
      for (const void* f : {(const void*)pip_fused_kernel<4, 2, true>, (const void*)pip_fused_kernel<4, 2, false>,
                            (const void*)pip_fused_kernel<2, 4, true>, (const void*)pip_fused_kernel<2, 4, false>}) {
        const hipError_t a = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
        if (e == hipSuccess) e = a;
      }
      (void)hipGetLastError();
      return e;
    }();
    if (attr != hipSuccess) return attr;
  }
  // rows per workgroup (64 or 128 per wave); 128 rows: cfg2 flat, cfg4 +20 % (every workgroup
  // stages the (c + 8) x 8 fp64 Gram, 33 KB at c = 512)
  // 512 rows per workgroup from N = 512k rows on (the per-workgroup prologue -- Gram staging,
  // selective test, Cholesky -- amortised over twice the rows: cfg4 fit 1,632 vs 1,645 ms; at
  // cfg2's 100k rows the 196 workgroups leave CUs idle: 34.0 vs 33.1 ms)
  const int rows = n >= (int64_t)1 << 19 ? 512 : 256;
  const unsigned grid = (unsigned)((n + rows - 1) / rows);
#define PIP_LAUNCH(QB_, NU_, NT_)                                                                \
  hipLaunchKernelGGL((pip_fused_kernel<QB_, NU_, NT_>), dim3(grid ? grid : 1), dim3(256), lds, stream, Q, \
                     Zin, Zout, G, c, n, cond, flags, any_flag, save, save_row0, save_rows, sticky,  \
                     seed, row0, rsave, skip_tol, skipped, first)
  const bool nt = basis_nt(n, Q.count);
  if (rows == 256) {
    if (nt) PIP_LAUNCH(4, 2, true); else PIP_LAUNCH(4, 2, false);
  } else {
    if (nt) PIP_LAUNCH(2, 4, true); else PIP_LAUNCH(2, 4, false);
  }
#undef PIP_LAUNCH
  return hipGetLastError();
}

// Fill an N x W block with N(0,1) deviates: all columns (flags == nullptr) or only flagged ones.
__global__ void fill_normal_kernel(float* __restrict__ blk, int w, int64_t n, uint64_t seed,
                                   const int* flags, const int* cond, uint64_t ctr0) {
  if (cond && *cond == 0) return;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * w;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int col = (int)(e % w);
    if (flags && !flags[col]) continue;
    blk[e] = counter_normal(seed, ctr0 + (uint64_t)e);
  }
}

// ctr0: counter offset (global first row x w), so a row-partitioned run draws the same values
extern "C" hipError_t n2v2r_launch_fill_normal(float* blk, int w, int64_t n, uint64_t seed,
                                               const int* flags, const int* cond, uint64_t ctr0,
                                               hipStream_t stream) {
  const int64_t elems = n * w;
  int64_t nb = (elems + 255) / 256;
  if (nb > 2048) nb = 2048;
  hipLaunchKernelGGL(fill_normal_kernel, dim3((unsigned)nb), dim3(256), 0, stream, blk, w, n, seed,
                     flags, cond, ctr0);
  return hipGetLastError();
}

// Ritz residual norms: res[j] = sum_r (MX[r][j] - theta[j] X[r][j])^2 over all blocks of X/MX
// (grid.y = block), per-chunk fp64 partials then the fixed-order wave fold.
__global__ __launch_bounds__(256) void resid_kernel(BlockList X, BlockList MX,
                                                    const double* __restrict__ theta, int64_t n,
                                                    int64_t rows_per_chunk,
                                                    double* __restrict__ partial) {
  __shared__ double red[256];
  const int w = X.width;
  const int q = blockIdx.y;
  const float* xb = X.blk[q];
  const float* mb = MX.blk[q];
  const int col = threadIdx.x % w;
  const int rg = threadIdx.x / w;
  const int ngroups = blockDim.x / w;
  const int64_t c0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t c1 = c0 + rows_per_chunk;
  if (c1 > n) c1 = n;
  const double th = theta[q * w + col];
  double s = 0.0;
  for (int64_t r = c0 + rg; r < c1; r += ngroups) {
    const double v = (double)mb[r * w + col] - th * (double)xb[r * w + col];
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < w) {
    double t = 0.0;
    for (int g = 0; g < ngroups; ++g) t += red[g * w + threadIdx.x];
    const int64_t ncols = (int64_t)X.count * w;
    partial[(int64_t)blockIdx.x * ncols + q * w + threadIdx.x] = t;
  }
}

extern "C" hipError_t n2v2r_launch_resid(const BlockList& X, const BlockList& MX,
                                         const double* theta, int64_t n, double* partial,
                                         size_t partial_elems, double* out, hipStream_t stream) {
  const int64_t ncols = (int64_t)X.count * X.width;
  int64_t nchunks = (n + 1023) / 1024;
  if (nchunks > 256) nchunks = 256;
  if ((size_t)(nchunks * ncols) > partial_elems) nchunks = (int64_t)(partial_elems / ncols);
  int64_t rows = (n + nchunks - 1) / nchunks;
  nchunks = (n + rows - 1) / rows;
  hipLaunchKernelGGL(resid_kernel, dim3((unsigned)nchunks, X.count), dim3(256), 0, stream, X, MX,
                     theta, n, rows, partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_reduce(partial, nchunks, ncols, out, nullptr, stream);
}

// Scale the columns of an N x W block: blk[r][j] *= s[j]
__global__ void scale_cols_kernel(float* __restrict__ blk, int w, int64_t n,
                                  const float* __restrict__ s) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n * w) blk[e] *= s[e % w];
}

extern "C" hipError_t n2v2r_launch_scale_cols(float* blk, int w, int64_t n, const float* s,
                                              hipStream_t stream) {
  const int64_t elems = n * w;
  hipLaunchKernelGGL(scale_cols_kernel, dim3((unsigned)((elems + 255) / 256)), dim3(256), 0,
                     stream, blk, w, n, s);
  return hipGetLastError();
}

// Deterministic SVD sign convention (as sklearn's svd_flip): flip column j of U so that its
// entry of largest magnitude (smallest row on ties) is positive.  Pass 1: per (row chunk,
// 32-column tile) the packed key (|u| bits << 32 | ~row) max; pass 2: fold chunks, read the
// sign, write +-1.
__global__ __launch_bounds__(256) void colmax_partial_kernel(const float* __restrict__ U,
                                                             int64_t ldu, int64_t n, int d,
                                                             int64_t rows_per_chunk, int64_t row0,
                                                             unsigned long long* __restrict__ keys) {
  __shared__ unsigned long long red[8][32];
  const int c = threadIdx.x & 31;
  const int rl = threadIdx.x >> 5;
  const int col = blockIdx.y * 32 + c;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  int64_t r1 = r0 + rows_per_chunk;
  if (r1 > n) r1 = n;
  unsigned long long best = 0;
  if (col < d) {
    for (int64_t r = r0 + rl; r < r1; r += 8) {
      const float v = fabsf(U[r * ldu + col]);
      const unsigned long long k = ((unsigned long long)__float_as_uint(v) << 32) |
                                   (unsigned long long)(0xFFFFFFFFu - (uint32_t)(row0 + r));
      best = k > best ? k : best;
    }
  }
  red[rl][c] = best;
  __syncthreads();
  if (rl == 0) {
    for (int g = 1; g < 8; ++g) best = red[g][c] > best ? red[g][c] : best;
    keys[(int64_t)blockIdx.x * gridDim.y * 32 + col] = best;
  }
}

// fold chunk keys -> best[col] (packed |u| bits and ~global row): one wave per column, lanes
// stride the chunks, wave max (a maximum: any order gives the same key)
__global__ __launch_bounds__(256) void colmax_fold_kernel(const unsigned long long* __restrict__ keys,
                                                          int nchunks, int ncols_padded,
                                                          unsigned long long* __restrict__ best_out) {
  const int col = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (col >= ncols_padded) return;  // (wave-uniform)
  unsigned long long best = 0;
  for (int c = lane; c < nchunks; c += 64) {
    const unsigned long long k = keys[(int64_t)c * ncols_padded + col];
    best = k > best ? k : best;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long t =
        ((unsigned long long)(unsigned)__shfl_xor((int)(best >> 32), o, 64) << 32) |
        (unsigned long long)(unsigned)__shfl_xor((int)(best & 0xFFFFFFFFull), o, 64);
    best = t > best ? t : best;
  }
  if (lane == 0) best_out[col] = best;
}

// sign[col] = sign of U at the winning row if this rank owns it, else 0 (summed over ranks)
__global__ void colmax_sign_kernel(const unsigned long long* __restrict__ best, int ncols_padded,
                                   const float* __restrict__ U, int64_t ldu, int d, int64_t row0,
                                   int64_t n, float* __restrict__ sign) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= ncols_padded) return;
  if (col >= d) {
    sign[col] = row0 == 0 ? 1.f : 0.f;
    return;
  }
  const int64_t grow = (int64_t)(0xFFFFFFFFu - (uint32_t)(best[col] & 0xFFFFFFFFull));
  const int64_t r = grow - row0;
  float sgn = 0.f;
  if (r >= 0 && r < n) sgn = (U[r * ldu + col] < 0.f) ? -1.f : 1.f;
  sign[col] = sgn;
}

extern "C" hipError_t n2v2r_launch_colmax_keys(const float* U, int64_t ldu, int64_t n, int d,
                                               int64_t row0, unsigned long long* keys,
                                               size_t key_elems, unsigned long long* best,
                                               hipStream_t stream) {
  const int tiles = (d + 31) / 32;
  // ~256 rows per chunk (cfg2: 391 x 2 workgroups; 4096-row chunks kept 50 CUs busy, 139 us)
  int64_t nchunks = (n + 255) / 256;
  if (nchunks > 1024) nchunks = 1024;
  if (nchunks < 1) nchunks = 1;
  if ((size_t)(nchunks * tiles * 32) > key_elems) nchunks = (int64_t)(key_elems / (tiles * 32));
  if (nchunks < 1) return hipErrorInvalidValue;
  int64_t rows = (n + nchunks - 1) / nchunks;
  if (rows < 1) rows = 1;
  nchunks = (n + rows - 1) / rows;
  if (nchunks < 1) nchunks = 1;
  hipLaunchKernelGGL(colmax_partial_kernel, dim3((unsigned)nchunks, tiles), dim3(256), 0, stream,
                     U, ldu, n, d, rows, row0, keys);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(colmax_fold_kernel, dim3((tiles * 32 + 3) / 4), dim3(256), 0, stream,
                     keys, (int)nchunks, tiles * 32, best);
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_colmax_sign(const unsigned long long* best, int ncols_padded,
                                               const float* U, int64_t ldu, int d, int64_t row0,
                                               int64_t n, float* sign, hipStream_t stream) {
  hipLaunchKernelGGL(colmax_sign_kernel, dim3((ncols_padded + 255) / 256), dim3(256), 0, stream,
                     best, ncols_padded, U, ldu, d, row0, n, sign);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- debug
// N2V2R_DEBUG_FINITE: *flag = 1 if any of `count` fp32 (f64 == 0) or fp64 values is not finite
// (plain vector stores from the offending lanes; the host zeroes the flag and reads it back).
__global__ void nonfinite_kernel(const void* __restrict__ p, int64_t count, int f64,
                                 int* __restrict__ flag) {
  bool bad = false;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < count;
       e += (int64_t)gridDim.x * blockDim.x)
    bad |= f64 ? !isfinite(static_cast<const double*>(p)[e]) : !isfinite(static_cast<const float*>(p)[e]);
  if (bad) flag[0] = 1;
}

extern "C" hipError_t n2v2r_launch_nonfinite(const void* p, int64_t count, int f64, int* flag,
                                             hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  int64_t nb = (count + 255) / 256;
  if (nb > 1024) nb = 1024;
  hipLaunchKernelGGL(nonfinite_kernel, dim3((unsigned)nb), dim3(256), 0, stream, p, count, f64, flag);
  return hipGetLastError();
}

// N2V2R_POISON: fill the LDS of every CU with 0xFF bytes (NaN as fp32 and fp64).  LDS is not
// cleared between dispatches, so a later kernel that reads LDS it did not write (or multiplies
// stale LDS by a zero weight) turns non-finite instead of silently using an earlier kernel's data.
__global__ __launch_bounds__(256) void lds_poison_kernel(int words) {
  extern __shared__ unsigned int lds_words[];
  for (int e = threadIdx.x; e < words; e += 256) lds_words[e] = 0xFFFFFFFFu;
  __syncthreads();
  if (lds_words[(threadIdx.x * 37) % words] != 0xFFFFFFFFu) lds_words[0] = 0;  // keep the stores
}

extern "C" hipError_t n2v2r_launch_lds_poison(hipStream_t stream) {
  static const size_t bytes = [] {
    const size_t want = 160 * 1024;
    if (hipFuncSetAttribute((const void*)lds_poison_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)want) == hipSuccess)
      return want;
    (void)hipGetLastError();
    return (size_t)64 * 1024;
  }();
  // 4 workgroups per CU: every CU's whole LDS is written whichever CUs the dispatcher picks
  hipLaunchKernelGGL(lds_poison_kernel, dim3(1024), dim3(256), bytes, stream,
                     (int)(bytes / sizeof(unsigned int)));
  return hipGetLastError();
}

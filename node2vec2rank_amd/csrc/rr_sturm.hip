// Rayleigh-Ritz of the block Krylov-Schur cycle WITHOUT reducing the projected matrix: the top-p
// eigenpairs of H = Q^T M Q come straight from its arrow + band structure (gfx950, wave64).
//
// H, in the basis order [X (kp kept Ritz vectors) | E | Z_2 ... ] (8-wide blocks):
//   * diag(Theta) on X, coupled only to E:   H[i][kp + q] = G0[i][q]        (i < kp, q < 8)
//   * the Krylov part (rows kp .. c-1) is symmetric banded with half-bandwidth 8 (block
//     tridiagonal, upper-triangular couplings R_j) -- the same entries rr_chase_kernel reads.
// Eigenvalues: Sturm counts nu(x) = #eig(H) < x by symmetric Gaussian elimination of H - x I in
// natural order, no pivoting: the kp X rows first (each a scalar pivot theta_i - x whose rank-1
// Schur update lands in the 8 x 8 E block), then the band, one row per step with a 9 x 9 window
// kept in registers (unrolled by 9 so the window shift is register renaming).  Pivots smaller
// than eps ||H|| are replaced by -eps ||H|| (dstebz's rule, at the matrix's own noise level).
// The wanted eigenvalues are bracketed by a multisection over all CUs (rr_msect_kernel; round 4
// replaced one 512-point multisection workgroup per eigenvalue, its A/B switch retired round 5).
// Eigenvectors: inverse iteration on the same structure, one 64-thread workgroup per cluster
// start (its members in order): the X rows eliminated exactly (their Schur complement is an
// 8 x 8 update of the E block), then the same symmetric elimination of the band as the Sturm
// count (L D L^T, guarded pivots, no interchanges), kept in LDS with the right-hand side and
// the iterate, so lane 0's serial factor / solve chains never wait on global memory; two
// solves, classical Gram-Schmidt against the earlier members of a cluster (as
// rr_inviter_kernel).  Every vector's residual ||(H - lambda) y|| is checked; a failure (e.g.
// element growth of the unpivoted factor) sets *err and the caller runs the reducing path
// (arrow -> band -> bulge chase) instead.
// Work per Sturm count O(kp b^2 + c b^2), per eigenvector O(c b^2): the O(c^2 b) bulge chase
// (a serial chain of ~2c steps) and its back-transform are gone.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "common.h"

#define RS_W 8
#define RS_MAXC N2V2R_BAND_MAXC
#define RS_HDR 4  // scratch header: glo, ghi, tn, (unused)
#define RS_LD 10  // band row stride in the scratch (9 entries + 1 pad: 16-B aligned rows)
#define RS_PADR 10  // zero rows past c (the elimination reads up to row c + 9)

namespace {

__device__ __forceinline__ double rs_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  r = fma(r, fma(-x, r, 1.0), r);
  return r;
}

// |x| >= tiny, sign kept (zero -> -tiny, counted negative: dstebz's convention)
__device__ __forceinline__ double rs_guard(double d, double tiny) {
  return fabs(d) < tiny ? (d > 0.0 ? tiny : -tiny) : d;
}

}  // namespace

// ---- assembly -----------------------------------------------------------------------------
// scratch (fp64): [glo, ghi, tn, 0 | Xd (kp) | Xg (kp x 8) | Lb ((c - kp + RS_PADR) x RS_LD)] with
// Lb[(r - kp) * RS_LD + t] = H[r][r - 8 + t] (t = 8: the diagonal; columns < kp stored as 0;
// the RS_PADR rows past c are zero: the eliminations read them but never pivot on them).
__device__ __forceinline__ double rs_band_entry(const double* __restrict__ hband, int c, int kp,
                                                int i, int col) {
  // H[i][col] for kp <= col <= i < c, i - col <= 8 (the band part); zero outside the band
  constexpr int W = RS_W;
  if (col < kp || i - col > W || col > i) return 0.0;
  const int j0 = kp / W;
  const int base1 = (kp + W) * W;
  const int j = i / W, r = i % W;
  if (j == j0) {  // the E block: rows kp .. kp+7 of G0 = [X E]^T W_E
    const double* G = hband;
    const int cc = col - kp;
    return 0.5 * (G[(kp + r) * W + cc] + G[(kp + cc) * W + r]);
  }
  const double* G = hband + base1 + (j - j0 - 1) * 2 * W * W;
  if (col >= j * W) {
    const int cc = col - j * W;
    return 0.5 * (G[(W + r) * W + cc] + G[(W + cc) * W + r]);
  }
  const int cc = col - (j - 1) * W;  // R_j upper triangular: r <= cc
  return (r <= cc) ? G[cc * W + r] : 0.0;
}

__global__ __launch_bounds__(256) void rr_sturm_prep_kernel(const double* hband,
                                                            int c, int kp,
                                                            const double* __restrict__ theta,
                                                            double* __restrict__ scr) {
  constexpr int W = RS_W;
  __shared__ double red[3][256];
  extern __shared__ __attribute__((aligned(16))) double hb_lds[];
  const int tid = threadIdx.x;
  const int nb = c - kp;
  double* Xd = scr + RS_HDR;
  double* Xg = Xd + kp;
  double* Lb = Xg + (size_t)kp * W;
  {
    // the band store into LDS first: every entry below is read several times, and from global
    // memory each read was a dependent round trip (26 us for the launch at c = 384)
    const int hbe = (kp + W) * W + (nb / W - 1) * 2 * W * W;
    stage_to_lds<256, 8>(hb_lds, hband, hbe, tid);
    __syncthreads();
    hband = hb_lds;
  }
  for (int e = tid; e < (nb + RS_PADR) * RS_LD; e += 256) {
    const int rr = e / RS_LD, t = e % RS_LD;
    const int i = kp + rr, col = i - W + t;
    Lb[e] = (rr < nb && t <= W) ? rs_band_entry(hband, c, kp, i, col) : 0.0;
  }
  for (int e = tid; e < kp * W; e += 256) Xg[e] = hband[e];
  for (int e = tid; e < kp; e += 256) Xd[e] = theta[e];
  // Gershgorin bounds and ||H||_inf
  double lo = 1e300, hi = -1e300, tn = 0.0;
  for (int i = tid; i < c; i += 256) {
    double ctr, rad = 0.0;
    if (i < kp) {
      ctr = theta[i];
      for (int q = 0; q < W; ++q) rad += fabs(hband[i * W + q]);
    } else {
      ctr = rs_band_entry(hband, c, kp, i, i);
      for (int d = 1; d <= W; ++d) {
        if (i - d >= kp) rad += fabs(rs_band_entry(hband, c, kp, i, i - d));
        if (i + d < c) rad += fabs(rs_band_entry(hband, c, kp, i + d, i));
      }
      if (i < kp + W)
        for (int a = 0; a < kp; ++a) rad += fabs(hband[a * W + (i - kp)]);
    }
    lo = fmin(lo, ctr - rad);
    hi = fmax(hi, ctr + rad);
    tn = fmax(tn, fabs(ctr) + rad);
  }
  red[0][tid] = lo;
  red[1][tid] = hi;
  red[2][tid] = tn;
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if (tid < s) {
      red[0][tid] = fmin(red[0][tid], red[0][tid + s]);
      red[1][tid] = fmax(red[1][tid], red[1][tid + s]);
      red[2][tid] = fmax(red[2][tid], red[2][tid + s]);
    }
    __syncthreads();
  }
  if (tid == 0) {
    scr[0] = red[0][0];
    scr[1] = red[1][0];
    scr[2] = red[2][0];
    scr[3] = 0.0;
  }
}

// ---- symmetric elimination (Sturm counts and the L D L^T of inverse iteration) -------------
// The window: rows/columns k .. k+8 of the current Schur complement, lower triangle only, 45
// values in registers.  Logical index i sits at physical slot (i + S) % 9 at step S of a 9-step
// block, so the shift after a step is register renaming; WV(a, b) maps a physical pair onto the
// lower triangle (a symmetric store: only 45 registers are ever live).
#define WV(a, b) w[((a) > (b)) ? (a) : (b)][((a) > (b)) ? (b) : (a)]

// One elimination step at band row k: pivot, multipliers t_i = w_i0 / d (returned in t[1..8]
// when KEEP), rank-1 update of the trailing 8 x 8, then band row k + 9 (held in nr, loaded one
// step earlier) enters as logical row 8 of the next step and row k + 10 is loaded into nr, so a
// row's LDS latency hides behind a whole step (rows past c are zero rows of the padded scratch).
// The pivot reciprocal takes one Newton step (~2^-50 relative: far inside the count's backward
// error, and inside inverse iteration's); KEEP returns it in t[0] (the solves multiply by it).
// The next pivot's update is issued first: it is the only result the next step waits for.
template <int S, bool KEEP>
__device__ __forceinline__ double rs_step(double (&w)[9][9], double (&nr)[9], int k, int kp,
                                          const double* __restrict__ Lb, double x, double tiny,
                                          double* t) {
  constexpr int P0 = S % 9;
  constexpr int P1 = (S + 1) % 9;
  const double d = rs_guard(WV(P0, P0), tiny);
  double rd = __builtin_amdgcn_rcp(d);
  rd = fma(rd, fma(-d, rd, 1.0), rd);
  double tt[9];
  tt[1] = WV(P1, P0) * rd;
  WV(P1, P1) -= tt[1] * WV(P1, P0);
#pragma unroll
  for (int i = 2; i < 9; ++i) tt[i] = WV((i + S) % 9, P0) * rd;
#pragma unroll
  for (int i = 2; i < 9; ++i)
#pragma unroll
    for (int j = 1; j <= i; ++j) WV((i + S) % 9, (j + S) % 9) -= tt[i] * WV((j + S) % 9, P0);
  if (KEEP) {
    t[0] = rd;
#pragma unroll
    for (int i = 1; i < 9; ++i) t[i] = tt[i];
  }
#pragma unroll
  for (int j = 0; j < 9; ++j) WV(P0, (j + S + 1) % 9) = (j == 8) ? nr[j] - x : nr[j];
  const double* src = Lb + (int64_t)(k + 10 - kp) * RS_LD;
#pragma unroll
  for (int j = 0; j < 9; ++j) nr[j] = src[j];
  return d;
}

// the window for rows kp .. kp+8 of H - x I, and band row kp + 9 in nr
__device__ __forceinline__ void rs_window_init(double (&w)[9][9], double (&nr)[9], int kp,
                                               const double* __restrict__ Lb, double x) {
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      double v = Lb[(int64_t)i * RS_LD + 8 - (i - j)];
      if (i == j) v -= x;
      w[i][j] = v;
    }
#pragma unroll
  for (int j = 0; j < 9; ++j) nr[j] = Lb[(int64_t)9 * RS_LD + j];
  (void)kp;
}

// nu(x) = number of eigenvalues of H below x
__device__ __forceinline__ int rs_count(double x, int c, int kp, const double* __restrict__ Xd,
                        const double* __restrict__ Xg, const double* __restrict__ Lb,
                        double tiny) {
  double w[9][9], nr[9];
  rs_window_init(w, nr, kp, Lb, x);
  int neg = 0;
  // the X rows: pivot theta_a - x, rank-1 update of the E block (logical rows 0..7)
  for (int a = 0; a < kp; ++a) {
    const double d = rs_guard(Xd[a] - x, tiny);
    neg += d < 0.0;
    const double rd = rs_rcp(d);
    double g[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) g[q] = Xg[a * 8 + q];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const double gi = g[i] * rd;
#pragma unroll
      for (int j = 0; j <= i; ++j) w[i][j] -= gi * g[j];
    }
  }
  // whole groups of 9 steps without exit tests (one basic block: the next step's pivot chain
  // overlaps this step's trailing updates), then the tail
#define RS_CSTEP(S_) neg += rs_step<S_, false>(w, nr, k + S_, kp, Lb, x, tiny, nullptr) < 0.0;
  int k = kp;
  for (; k + 9 <= c; k += 9) {
    RS_CSTEP(0) RS_CSTEP(1) RS_CSTEP(2) RS_CSTEP(3) RS_CSTEP(4) RS_CSTEP(5) RS_CSTEP(6)
    RS_CSTEP(7) RS_CSTEP(8)
  }
#undef RS_CSTEP
#define RS_CSTEP(S_)                                                            \
  if (k + S_ >= c) break;                                                      \
  neg += rs_step<S_, false>(w, nr, k + S_, kp, Lb, x, tiny, nullptr) < 0.0;
  for (; k < c; k += 9) {
    RS_CSTEP(0) RS_CSTEP(1) RS_CSTEP(2) RS_CSTEP(3) RS_CSTEP(4) RS_CSTEP(5) RS_CSTEP(6)
    RS_CSTEP(7) RS_CSTEP(8)
  }
#undef RS_CSTEP
  return neg;
}

// ---- global multisection (all CUs) ---------------------------------------------------------
// Round 0: T = p * M points uniform on the Gershgorin interval, one count per thread over all
// p * (M / 256) workgroups.  Round r >= 1: eigenvalue j (j-th largest, ascending index
// a = c-1-j) gets its own M points inside its bracket from round r-1 (M / 256 workgroups, each
// re-deriving the bracket from the previous counts); its workgroup 0 records the bracket so
// the next round can rebuild the point set.  Counts are used through "the first point whose
// count exceeds a" (a rounding-perturbed count cannot move a bracket backwards); with no such
// point the eigenvalue lies above the last point.  rr_msect_finish_kernel turns the last round's
// counts into w[j] (bracket midpoints; rounds until the bracket is below 1e-10 ||H||).
struct RsMsect {
  int* cnt[2];     // [p * M] counts of the previous / current round
  double* brk[2];  // [p][2] brackets (round >= 1)
};

__device__ __forceinline__ double rs_pt(double lo, double hi, int k, int npts) {
  return lo + (hi - lo) * (double)(k + 1) / (double)(npts + 1);
}

// bracket of ascending index a from `npts` counts at rs_pt(lo, hi, k, npts): (x_{k-1}, x_k] for
// the first k with cnt > a, (x_{npts-1}, hi] if none (whole workgroup; the same in every thread)
__device__ __forceinline__ int rs_block_min(int v, int* red) {
  for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  v = 0x7fffffff;
  for (int w = 0; w < nw; ++w) v = min(v, red[w]);
  __syncthreads();
  return v;
}

__device__ __forceinline__ void rs_bracket(const int* __restrict__ cnt, int npts, int a, double& lo, double& hi,
                           int* red) {
  // two levels, every load of a level in flight together: the first of blockDim.x segments
  // whose last count exceeds a, then the first such point inside it
  const int nt = blockDim.x, t = threadIdx.x;
  const int seg = (npts + nt - 1) / nt;
  int sfirst = nt;
  {
    const int last = min(t * seg + seg - 1, npts - 1);
    if (t * seg < npts && cnt[last] > a) sfirst = t;
  }
  sfirst = rs_block_min(sfirst, red);
  int first = npts;
  if (sfirst < nt) {
    const int k0 = sfirst * seg;
    for (int k = k0 + t; k < min(k0 + seg, npts); k += nt)
      if (cnt[k] > a && (k == 0 || cnt[k - 1] <= a)) first = min(first, k);
    first = rs_block_min(first, red);
    if (first >= npts) first = k0;  // a rounding wobble inside the segment: its start
  }
  // no point above the eigenvalue: it lies in the top sub-interval (x_{npts-1}, hi]
  const double nlo = first > 0 ? rs_pt(lo, hi, first - 1, npts) : lo;
  const double nhi = first < npts ? rs_pt(lo, hi, first, npts) : hi;
  lo = nlo;
  hi = nhi;
}

// NT counts per workgroup per round: 256 (one wave per SIMD, M = 768 points per eigenvalue at
// p = 80: the rounds are count-issue-bound, so half the points of the 512-thread form at the
// same round count) or 512 (N2V2R_MSECT_THREADS=512, A/B)
#define RS_MS_THREADS 512  // the largest form (scratch sizing)
template <int NT>
__global__ __launch_bounds__(NT, NT / 256) void rr_msect_kernel(
    const double* __restrict__ scr, int c, int kp, int p, int M, int round, RsMsect ms) {
  extern __shared__ __attribute__((aligned(16))) double sl[];
  __shared__ int red[NT / 64];
  const int tid = threadIdx.x;
  const int nb = c - kp;
  const int total = kp + kp * RS_W + (nb + RS_PADR) * RS_LD;
  stage_to_lds<NT, 8>(sl, scr + RS_HDR, total, tid);
  const double* Xd = sl;
  const double* Xg = sl + kp;
  const double* Lb = Xg + kp * RS_W;
  const double tn = fmax(scr[2], 1e-300);
  const double tiny = 2.220446049250313e-16 * tn;
  const double glo = scr[0] - 1e-14 * tn - 1e-300, ghi = scr[1] + 1e-14 * tn + 1e-300;
  const int m = M / NT;
  const int j = blockIdx.x / m, part = blockIdx.x % m;
  const int cur = round & 1, prev = cur ^ 1;
  double x;
  int slot;
  if (round == 0) {
    slot = blockIdx.x * NT + tid;
    x = rs_pt(glo, ghi, slot, p * M);
    __syncthreads();
  } else {
    double lo, hi;
    if (round == 1) {
      lo = glo;
      hi = ghi;
      __syncthreads();
      rs_bracket(ms.cnt[prev], p * M, c - 1 - j, lo, hi, red);
    } else {
      lo = ms.brk[prev][2 * j];
      hi = ms.brk[prev][2 * j + 1];
      __syncthreads();
      rs_bracket(ms.cnt[prev] + (size_t)j * M, M, c - 1 - j, lo, hi, red);
    }
    if (part == 0 && tid == 0) {
      ms.brk[cur][2 * j] = lo;
      ms.brk[cur][2 * j + 1] = hi;
    }
    const int k = part * NT + tid;
    slot = j * M + k;
    x = rs_pt(lo, hi, k, M);
  }
  ms.cnt[cur][slot] = rs_count(x, c, kp, Xd, Xg, Lb, tiny);
}

__global__ __launch_bounds__(256) void rr_msect_finish_kernel(int c, int p, int M, int last,
                                                              RsMsect ms, double* __restrict__ w) {
  __shared__ int red[4];
  const int j = blockIdx.x;
  const int cur = last & 1;
  double lo = ms.brk[cur][2 * j], hi = ms.brk[cur][2 * j + 1];
  rs_bracket(ms.cnt[cur] + (size_t)j * M, M, c - 1 - j, lo, hi, red);
  if (threadIdx.x == 0) w[j] = 0.5 * (lo + hi);
}

// ---- eigenvectors -------------------------------------------------------------------------
// One 64-thread workgroup per cluster start (gap to eigenvalue j-1 above clus); its members in
// order.  Everything the serial chains touch lives in LDS: the assembled matrix, the factor
// (pivots d_k and multipliers t_k,1..8, nb x 9), the right-hand side f and the iterate y.  Lane
// 0 runs the factorization and the two triangular solves (serial in k); the Gram-Schmidt,
// norms and the residual check are lane-parallel.  Per member, with D_a = 1 / (theta_a - lambda)
// (guarded): the E block takes -sum_a D_a g_a g_a^T, the band is eliminated as in the Sturm
// count; solve: f_E -= G^T D f_X; L z = f_B; y_B = L^{-T} D^{-1} z; y_X = D (f_X - G y_E).
// lane 0: band elimination of B' = band - lam I - Sch (Sch: the X rows' 8 x 8 Schur complement
// on the E block, formed lane-parallel beforehand); pivots and multipliers to F (nb x 9)
__device__ __forceinline__ void rs_factor_lane(int c, int kp, const double* Lb, const double* sch, double lam,
                               double tiny, double* F) {
  double w[9][9], nr[9];
  rs_window_init(w, nr, kp, Lb, lam);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj <= i; ++jj) w[i][jj] -= sch[i * 8 + jj];
  double t[9];
  // F row k: the pivot reciprocal 1 / d_k, then the multipliers t_k,1..8
#define RS_FSTEP(S_)                                                                   \
  {                                                                                   \
    (void)rs_step<S_, true>(w, nr, k + S_, kp, Lb, lam, tiny, t);                      \
    double* fk = F + (k + S_ - kp) * 9;                                               \
    _Pragma("unroll") for (int i = 0; i < 9; ++i) fk[i] = t[i];                       \
  }
  int k = kp;
  for (; k + 9 <= c; k += 9) {  // whole groups: one basic block (see rs_count)
    RS_FSTEP(0) RS_FSTEP(1) RS_FSTEP(2) RS_FSTEP(3) RS_FSTEP(4) RS_FSTEP(5) RS_FSTEP(6)
    RS_FSTEP(7) RS_FSTEP(8)
  }
#undef RS_FSTEP
#define RS_FSTEP(S_)                                                                   \
  if (k + S_ >= c) break;                                                             \
  {                                                                                   \
    (void)rs_step<S_, true>(w, nr, k + S_, kp, Lb, lam, tiny, t);                      \
    double* fk = F + (k + S_ - kp) * 9;                                               \
    _Pragma("unroll") for (int i = 0; i < 9; ++i) fk[i] = t[i];                       \
  }
  for (; k < c; k += 9) {
    RS_FSTEP(0) RS_FSTEP(1) RS_FSTEP(2) RS_FSTEP(3) RS_FSTEP(4) RS_FSTEP(5) RS_FSTEP(6)
    RS_FSTEP(7) RS_FSTEP(8)
  }
#undef RS_FSTEP
}


// z = L^{-1} (f_B - fe) in place of f_B, then y_B = L^{-T} D^{-1} z, the chains spread over
// lanes q = lane & 7 (every lane runs them; lanes 0..7 carry the values).  (Round 2's form ran
// both chains on lane 0, eight FMAs per row: 79 vs 52 us per solve; its A/B switch
// N2V2R_INV_SOLVE was retired in round 6.)  Forward (right-looking): lane q holds r_q, the pending right-hand
// side of row k + q; per row z_k = r_0 is broadcast (readlane), the window shifts one lane
// (DPP row_shl:1) and each lane applies its own multiplier t_{k,q+1}: one FMA per row on the
// chain instead of lane 0's eight.  Backward (column form): lane j holds the partial sum of
// row k - j, y_k = z_k / d_k - acc_0 is broadcast, and every pending row adds t y_k in one FMA.
// Coefficients are read RS_PF rows ahead.
__device__ __forceinline__ double rs_dpp_shl1(double v) {  // lane l <- lane l + 1 (16-lane rows)
  // (lanes at a row's end keep their own value: callers mask lane 7 and ignore lanes >= 8)
  const int l = __double2loint(v), h = __double2hiint(v);
  const int lo = __builtin_amdgcn_update_dpp(l, l, 0x101, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(h, h, 0x101, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rs_lane0(double v) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 0);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 0);
  return __hiloint2double(hi, lo);
}
#define RS_PF 8
__device__ __forceinline__ void rs_band_solve_par(int c, int kp, const double* F, const double* fe,
                                                  double* f, double* y) {
  const int nb = c - kp;
  const int lane = threadIdx.x & 63, q = lane & 7;
  const bool last = q == 7;
  // forward: r_q = f[kp + q] - fe[q]; at row k, lane q needs t_{k,q+1} = F[k][1 + q] and lane 7
  // the entering right-hand side f[kp + k + 8] (zero past the band: f is padded by 8 + RS_PF
  // entries read as zero below).  Whole groups of RS_PF rows without exit tests; loads for the
  // next group are issued before the current group's chain and are unconditional (clamped).
  double r = f[kp + q] - fe[q];
  double tq[RS_PF], fv[RS_PF];
  auto fload = [&](int kk, double* t, double* v) {
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      const int k = kk + u;
      t[u] = F[min(k, nb - 1) * 9 + 1 + q];
      const double fx = f[kp + min(k + 8, nb - 1)];
      v[u] = (k + 8 < nb) ? fx : 0.0;
    }
  };
  fload(0, tq, fv);
  int k0 = 0;
  for (; k0 + RS_PF <= nb; k0 += RS_PF) {
    double tn[RS_PF], fn[RS_PF];
    fload(k0 + RS_PF, tn, fn);
    double zs = 0.0;  // lane u keeps z_{k0 + u}: one store per RS_PF rows, off the chain
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      const double zk = rs_lane0(r);
      zs = (lane == u) ? zk : zs;
      double nx = rs_dpp_shl1(r);
      nx = last ? fv[u] : nx;
      r = fma(-tq[u], zk, nx);
    }
    if (lane < RS_PF) f[kp + k0 + lane] = zs;
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      tq[u] = tn[u];
      fv[u] = fn[u];
    }
  }
  {
    double zs = 0.0;
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      if (k0 + u >= nb) break;
      const double zk = rs_lane0(r);
      zs = (lane == u) ? zk : zs;
      double nx = rs_dpp_shl1(r);
      nx = last ? fv[u] : nx;
      r = fma(-tq[u], zk, nx);
    }
    if (lane < RS_PF && k0 + lane < nb) f[kp + k0 + lane] = zs;
  }
  // backward: row k's solution y_k = z_k d_k^{-1} - sum_i t_{k,i} y_{k+i}; lane j holds that sum
  // for row k - j; after y_k, lane j takes lane j + 1's sum plus t_{k-1-j, j+1} y_k
  double acc = 0.0;
  double zr[RS_PF], tb[RS_PF];
  const int top = nb - 1;
  auto bload = [&](int kk, double* z, double* t) {
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      const int k = max(kk - u, 0);
      z[u] = f[kp + k] * F[k * 9];
      const int row = kk - u - 1 - q;
      const double tx = F[max(row, 0) * 9 + q + 1];
      t[u] = row >= 0 ? tx : 0.0;
    }
  };
  bload(top, zr, tb);
  int k1 = top;
  for (; k1 - RS_PF + 1 >= 0; k1 -= RS_PF) {
    double zn[RS_PF], tbn[RS_PF];
    bload(k1 - RS_PF, zn, tbn);
    double ys = 0.0;  // lane u keeps y_{k1 - u}
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      const double yk = zr[u] - rs_lane0(acc);
      ys = (lane == u) ? yk : ys;
      double sh = rs_dpp_shl1(acc);
      sh = last ? 0.0 : sh;
      acc = fma(tb[u], yk, sh);
    }
    if (lane < RS_PF) y[kp + k1 - lane] = ys;
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      zr[u] = zn[u];
      tb[u] = tbn[u];
    }
  }
  {
    double ys = 0.0;
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      if (k1 - u < 0) break;
      const double yk = zr[u] - rs_lane0(acc);
      ys = (lane == u) ? yk : ys;
      double sh = rs_dpp_shl1(acc);
      sh = last ? 0.0 : sh;
      acc = fma(tb[u], yk, sh);
    }
    if (lane < RS_PF && k1 - lane >= 0) y[kp + k1 - lane] = ys;
  }
}
#undef RS_PF

__device__ __forceinline__ double rs_wave_sum(double v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// y = (H - lam)^{-1} f: the X rows lane-parallel (dX = 1 / (theta - lam)), the band by lane 0
__device__ __forceinline__ void rs_solve(int c, int kp, const double* Xg, const double* dX, const double* F,
                         double* fe, double* f, double* y) {
  const int lane = threadIdx.x;
  if (lane < 8) {  // f_E -= G^T D f_X
    double acc = 0.0;
    for (int a = 0; a < kp; ++a) acc += Xg[a * 8 + lane] * (f[a] * dX[a]);
    fe[lane] = acc;
  }
  __syncthreads();
  rs_band_solve_par(c, kp, F, fe, f, y);
  __syncthreads();
  for (int a = lane; a < kp; a += 64) {  // y_X = D (f_X - G y_E)
    double acc = f[a];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc -= Xg[a * 8 + q] * y[kp + q];
    y[a] = acc * dX[a];
  }
  __syncthreads();
}

__global__ __launch_bounds__(64) void rr_sturm_inviter_kernel(const double* __restrict__ scr, int c,
                                                              int kp, int p, int pw,
                                                              const double* __restrict__ w,
                                                              double clus_rel,
                                                              double* __restrict__ wout,
                                                              double* __restrict__ Y,
                                                              float* __restrict__ S, int ldS,
                                                              int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) double il[];
  const int lane = threadIdx.x;
  const int j0 = blockIdx.x;
  const double tn = fmax(scr[2], 1e-300);
  const double clus = clus_rel * tn;
  if (j0 > 0 && fabs(w[j0 - 1] - w[j0]) <= clus) return;  // not a cluster start (uniform)
  const double tiny = 2.220446049250313e-16 * tn;
  const int nb = c - kp;
  const int total = kp + kp * RS_W + (nb + RS_PADR) * RS_LD;
  stage_to_lds<64, 16>(il, scr + RS_HDR, total, lane);
  const double* Xd = il;
  const double* Xg = il + kp;
  const double* Lb = Xg + kp * RS_W;
  double* F = il + ((total + 1) & ~1);
  double* f = F + nb * 9;
  double* y = f + c;
  double* dX = y + c;       // [kp] 1 / (theta_a - lam)
  double* sch = dX + kp;    // [64] the X rows' Schur complement on the E block
  double* fe = sch + 64;    // [8]
  __syncthreads();
  for (int j = j0; j < p && (j == j0 || fabs(w[j - 1] - w[j]) <= clus); ++j) {
    const double lam = w[j];
    for (int a = lane; a < kp; a += 64) dX[a] = rs_rcp(rs_guard(Xd[a] - lam, tiny));
    __syncthreads();
    {
      const int i = lane >> 3, jj = lane & 7;
      double acc = 0.0;
      for (int a = 0; a < kp; ++a) acc += Xg[a * 8 + i] * Xg[a * 8 + jj] * dX[a];
      sch[lane] = acc;
    }
    // start vector: for a wanted value j < kp, e_j (the kept Ritz vector j, which the new
    // eigenvector j is close to once the order settles) plus a small random part so no
    // component is zero; otherwise random.  From e_j one solve usually meets the
    // single-solve test below (random starts, round 2's form: 77-79 of 80 vectors per cfg2 cycle
    // took the second solve; its A/B switch N2V2R_INV_START was retired in round 6)
    const bool warm = j < kp;
    for (int i = lane; i < c; i += 64) {
      const uint64_t hsh = splitmix64(0x9E3779B97F4A7C15ull ^ ((uint64_t)j << 32) ^ (uint64_t)i);
      const double u = (double)(hsh >> 11) * (1.0 / 9007199254740992.0) - 0.5;
      f[i] = warm ? ((i == j ? 1.0 : 0.0) + 1e-4 * u) : u;
    }
    __syncthreads();
    if (lane == 0) rs_factor_lane(c, kp, Lb, sch, lam, tiny, F);
    __syncthreads();
    // r = (H - lam) y: X rows, then the band rows (+ the X couplings of the E rows); the
    // Rayleigh quotient lam + y.r refines the eigenvalue, ||(H - rq) y||^2 = r.r - (y.r)^2
    double r2 = 0.0, yr = 0.0;
    auto residual = [&]() {
      r2 = 0.0;
      yr = 0.0;
      for (int i = lane; i < c; i += 64) {
        double v;
        if (i < kp) {
          v = (Xd[i] - lam) * y[i];
#pragma unroll
          for (int q = 0; q < 8; ++q) v += Xg[i * 8 + q] * y[kp + q];
        } else {
          const int rr = i - kp;
          v = -lam * y[i];
          for (int d = -8; d <= 8; ++d) {
            const int col = rr + d;
            if (col < 0 || col >= nb) continue;
            const double h = d <= 0 ? Lb[rr * RS_LD + 8 + d] : Lb[col * RS_LD + 8 - d];
            v += h * y[kp + col];
          }
          if (rr < 8)
            for (int aa = 0; aa < kp; ++aa) v += Xg[aa * 8 + rr] * y[aa];
        }
        r2 += v * v;
        yr += v * y[i];
      }
      r2 = rs_wave_sum(r2);
      yr = rs_wave_sum(yr);
    };
    // an isolated eigenvalue whose first iterate already has a residual below 1e-7 of its gap
    // to the neighbouring wanted values (so its components along them are below 1e-7: fp32
    // orthogonality of the Ritz coefficients) skips the second solve
    double gap = 0.0;
    if (j == j0 && j + 1 < pw && j > 0) gap = fmin(w[j - 1] - lam, lam - w[j + 1]);
    else if (j == j0 && j == 0 && pw > 1) gap = lam - w[1];
    bool ok = true, done = false;
    for (int it = 0; it < 2 && ok; ++it) {
      rs_solve(c, kp, Xg, dX, F, fe, f, y);
      // classical Gram-Schmidt against the cluster's earlier members (Y columns j0 .. j-1)
      for (int q = j0; q < j; ++q) {
        double dq = 0.0;
        for (int i = lane; i < c; i += 64) dq += Y[(int64_t)i * p + q] * y[i];
        dq = rs_wave_sum(dq);
        for (int i = lane; i < c; i += 64) y[i] -= dq * Y[(int64_t)i * p + q];
        __syncthreads();
      }
      double s2 = 0.0;
      for (int i = lane; i < c; i += 64) s2 += y[i] * y[i];
      s2 = rs_wave_sum(s2);
      ok = s2 > 0.0 && isfinite(s2);
      const double inv = ok ? 1.0 / sqrt(s2) : 0.0;
      for (int i = lane; i < c; i += 64) {
        const double v = y[i] * inv;
        y[i] = v;
        f[i] = v;
      }
      __syncthreads();
      if (it == 0 && ok && gap > 0.0) {
        residual();
        if (sqrt(fmax(r2 - yr * yr, 0.0)) <= 1e-7 * gap) {  // uniform (wave sums)
          done = true;
          break;
        }
      }
    }
    if (!done) {
      residual();
      if (lane == 0) atomicAdd(&err[1], 1);  // diagnostics: vectors that took the second solve
    }
    const double res2 = fmax(r2 - yr * yr, 0.0);
    if (lane == 0) {
      wout[j] = lam + yr;
      if (!ok || !(sqrt(res2) <= 1e-8 * tn) || !isfinite(r2)) err[0] = 1;
    }
    for (int i = lane; i < c; i += 64) {
      Y[(int64_t)i * p + j] = y[i];
      S[(int64_t)i * ldS + j] = (float)y[i];
    }
    __syncthreads();
  }
}

// Dense H (c x c, fp64, row-major, ld c) from the same arrow + band structure: the dense
// Rayleigh-Ritz's input when a Sturm vector fails its check and the kept set is past the
// reducing path's arrow (kp + 8 > 192, rr_band.hip's LDS-resident arrow).  theta: the kept
// Ritz values (the copy the prep kernel made).
__global__ __launch_bounds__(256) void rr_band_expand_kernel(const double* __restrict__ hband,
                                                             int c, int kp,
                                                             const double* __restrict__ theta,
                                                             double* __restrict__ H) {
  constexpr int W = RS_W;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)c * c) return;
  const int i = (int)(idx / c), j = (int)(idx % c);
  const int lo = i < j ? i : j, hi = i < j ? j : i;
  double v;
  if (hi < kp) v = (i == j) ? theta[i] : 0.0;                          // diag(Theta)
  else if (lo < kp) v = (hi < kp + W) ? hband[lo * W + (hi - kp)] : 0.0;  // X rows -> E
  else v = rs_band_entry(hband, c, kp, hi, lo);                        // the band
  H[idx] = v;
}

extern "C" hipError_t n2v2r_launch_rr_band_expand(const double* hband, int c, int kp,
                                                 const double* theta, double* H,
                                                 hipStream_t stream) {
  if (c < 9 || c > RS_MAXC || c % RS_W || kp % RS_W || kp + RS_W > c || (kp > 0 && !theta))
    return hipErrorInvalidValue;
  const int64_t total = (int64_t)c * c;
  hipLaunchKernelGGL(rr_band_expand_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     stream, hband, c, kp, theta, H);
  return hipGetLastError();
}

static size_t rs_asm_elems(int c, int kp) {  // header + Xd + Xg + padded band rows
  return (size_t)RS_HDR + (size_t)kp * (1 + RS_W) + (size_t)(c - kp + RS_PADR) * RS_LD;
}

// scratch doubles for any kp <= c - 8: the assembly (at most RS_HDR + RS_LD (c + RS_PADR)), the
// bisection values (c), the multisection brackets (2 x p x 2) and counts (2 x p x M ints)
static int rs_msect_threads() { return 256; }  // (512, two waves per SIMD: measured, not kept)

// points per eigenvalue per round: nt x workgroups (about one workgroup per CU)
static int rs_msect_m(int p, int nt = RS_MS_THREADS) {
  int m = 256 / (p > 0 ? p : 1);
  m = m < 1 ? 1 : (m > 4 ? 4 : m);
  return nt * m;
}

extern "C" size_t n2v2r_rr_sturm_scratch(int c, int p) {
  const size_t M = (size_t)rs_msect_m(p);
  return (((size_t)RS_HDR + (size_t)RS_LD * (c + RS_PADR) + 7) & ~(size_t)7) + (size_t)c +
         4 * (size_t)p + (2 * (size_t)p * M + 1) / 2 + 8;
}

static size_t rs_inviter_lds(int c, int kp) {  // assembly + factor + f + y
  const size_t total = (size_t)kp * (1 + RS_W) + (size_t)(c - kp + RS_PADR) * RS_LD;
  return sizeof(double) * (((total + 1) & ~(size_t)1) + (size_t)(c - kp) * 9 + 2 * (size_t)c +
                           (size_t)kp + 64 + 8);
}

extern "C" hipError_t n2v2r_launch_rr_sturm(const double* hband, int c, int kp,
                                           double* theta, double* scr, size_t scr_elems,
                                           double* Y, float* S, int ldS, int p, int* err,
                                           hipStream_t stream) {
  if (c < 9 || c > RS_MAXC || c % RS_W || kp % RS_W || kp + RS_W > c || p < 1 || p > c ||
      ldS < p)
    return hipErrorInvalidValue;
  const size_t wbis_off = (rs_asm_elems(c, kp) + 7) & ~(size_t)7;
  const int nt_ms = rs_msect_threads();
  const int pm = p;  // eigenvalues bracketed (the wanted ones)
  const int M = rs_msect_m(pm, nt_ms);
  const size_t brk_off = wbis_off + (size_t)c, cnt_off = brk_off + 4 * (size_t)pm;
  if (cnt_off + ((2 * (size_t)pm * M + 1) / 2) > scr_elems || p > c)
    return hipErrorInvalidValue;  // every region inside the scratch
  double* wbis = scr + wbis_off;
  RsMsect ms;
  ms.brk[0] = scr + brk_off;
  ms.brk[1] = ms.brk[0] + 2 * pm;
  ms.cnt[0] = reinterpret_cast<int*>(scr + cnt_off);
  ms.cnt[1] = ms.cnt[0] + (size_t)pm * M;
  static bool attr = false;
  if (!attr) {  // room for the dynamic LDS checked below (the static arrays stay under 10 KB)
    hipError_t a2 = hipFuncSetAttribute((const void*)rr_sturm_inviter_kernel,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipError_t a5 = hipFuncSetAttribute((const void*)rr_sturm_prep_kernel,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    if (a2 == hipSuccess) a2 = a5;
    hipError_t a3 = hipFuncSetAttribute((const void*)rr_msect_kernel<256>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    if (a2 == hipSuccess) a2 = a3;
    (void)hipGetLastError();  // a refused attribute must not surface as a later launch error
    if (a2 != hipSuccess) return a2;
    attr = true;
  }
  const size_t asm_d = rs_asm_elems(c, kp);
  const size_t lms = sizeof(double) * (asm_d - RS_HDR);  // the multisection's assembled H
  const size_t linv = rs_inviter_lds(c, kp);
  if (lms > 150 * 1024 || linv > 150 * 1024) return hipErrorInvalidValue;
  const size_t lprep = sizeof(double) * ((size_t)(kp + RS_W) * RS_W + (size_t)((c - kp) / RS_W - 1) * 2 * RS_W * RS_W);
  if (lprep > 150 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rr_sturm_prep_kernel, dim3(1), dim3(256), lprep, stream, hband, c, kp, theta, scr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // theta holds the kept Ritz values (kp) until the prep kernel has copied them; the
  // bisection writes wbis, the inverse iteration the refined values into theta
  {
    const unsigned grid = (unsigned)(pm * (M / nt_ms));
    // rounds until the bracket is below 1e-10 ||H|| (3 at p = 80, M = 768; 4 at p = 160, M = 256)
    int rounds = 1;
    for (double wdt = 2.0 / ((double)pm * M + 1.0); wdt > 1e-10; wdt /= (double)(M + 1)) ++rounds;
    for (int r = 0; r < rounds; ++r) {
      hipLaunchKernelGGL(rr_msect_kernel<256>, dim3(grid), dim3(256), lms, stream, scr, c, kp, pm,
                         M, r, ms);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(rr_msect_finish_kernel, dim3((unsigned)pm), dim3(256), 0, stream, c, pm, M,
                       rounds - 1, ms, wbis);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(rr_sturm_inviter_kernel, dim3((unsigned)p), dim3(64), linv, stream, scr, c,
                     kp, p, pm, wbis, 1e-9, theta, Y, S, ldS, err);
  return hipGetLastError();
}

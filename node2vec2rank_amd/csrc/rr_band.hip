// Banded Rayleigh-Ritz for the block Krylov-Schur eigensolver (block width b = 8).
//
// In exact arithmetic the projected matrix of a Krylov-Schur cycle, in the basis order
// [X (kept Ritz vectors, kp columns), E, Z_2, ..., Z_m] (b-wide blocks), is
//   * block tridiagonal on the Krylov blocks: diagonal blocks Q_j^T M Q_j, sub-diagonal blocks
//     R_j = Q_j^T M Q_{j-1} upper triangular (the Cholesky factors of the orthogonalisation);
//   * diag(Theta) on X (the previous Ritz values), coupled only to E (M X = X Theta + E B).
// Every entry it needs is a by-product of the expansion: the local first orthogonalisation
// pass of block j computes [Q_{j-1} Q_j]^T W_j (or [X E]^T W_E), saved as "band column" j.
// Off-band entries are rounding noise at the fp32 level of the basis and are dropped.
//
//   rr_arrow_kernel    [[Theta, B^T], [B, A_E]] -> half-bandwidth b by an offset-b Householder
//                      reduction of its index reversal (E untouched), packed in LDS; the
//                      reflectors are kept for the back-transform of the X rows.
//   rr_chase_kernel    band (half-bandwidth 8) -> tridiagonal by bulge chasing, LDS-resident:
//                      one wave per sweep (lane = one entry of an 8 x 8 window), sweep i+1
//                      pipelined two steps behind sweep i through LDS progress counters.
//   rr_bisect_kernel, rr_inviter_kernel (rr.hip)  top-p eigenpairs of the tridiagonal.
//   rr_band_back       eigenvectors back through the chase (one sweep = a block-diagonal
//                      product of 8 x 8 reflectors, applied in parallel) and the arrow
//                      reflectors; fp32 Ritz coefficients S written.
// Cost is O(c^2 b) + O(kp^3) instead of the O(c^3) dense tridiagonalisation.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"

#define RB_W 8
#define RB_MAXC N2V2R_BAND_MAXC
#define RB_MAXNA 192
#define RB_DONE_ALL 0x3fffffff

namespace {

__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  r = fma(r, fma(-x, r, 1.0), r);
  return r;
}

// 8-term dot product as a depth-3 tree (the chase's per-step latency)
__device__ __forceinline__ double dot8(const double* a, const double* b) {
  const double p0 = fma(a[0], b[0], a[1] * b[1]), p1 = fma(a[2], b[2], a[3] * b[3]);
  const double p2 = fma(a[4], b[4], a[5] * b[5]), p3 = fma(a[6], b[6], a[7] * b[7]);
  return (p0 + p1) + (p2 + p3);
}

__device__ __forceinline__ void house_params(double x0, double sig, double& tau, double& beta,
                                             double& scale) {
  // branch-free (sig == 0: the identity reflector tau = 0, beta = x0, scale = 0); two
  // independent reciprocals (v_rcp_f64 + two Newton steps) instead of two dependent IEEE
  // divisions: the chase's per-step latency
  const double nrm = sqrt(x0 * x0 + sig);
  const double bt = (x0 >= 0.0) ? -nrm : nrm;
  const double tc = (bt - x0) * rcp_nr(bt);
  const double sc = rcp_nr(x0 - bt);
  const bool z = sig == 0.0;
  tau = z ? 0.0 : tc;
  beta = z ? x0 : bt;
  scale = z ? 0.0 : sc;
}

template <int CTRL>
__device__ __forceinline__ double rb_dpp(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// sum over the 8 lanes of a lane's row group (all 8 get it)
__device__ __forceinline__ double rb_row_sum(double v) {
  v += rb_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += rb_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += rb_dpp<0x141>(v);  // row_half_mirror
  return v;
}

// sum over the wave: 16-lane rows by DPP, then the 4 rows by two lane exchanges
__device__ __forceinline__ double rb_wave_sum(double v) {
  v = rb_row_sum(v);
  v += rb_dpp<0x140>(v);  // row_mirror: the two 8-lane halves of a row
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}


}  // namespace

// ---- arrow -> band ----------------------------------------------------------------------
// GE: (kp + 8) x 8 row-major = [X E]^T W_E (rows 0..kp-1: B^T, rows kp..: A_E).
// R = J A J in packed lower storage; step k annihilates R[k+8+1.., k] with a reflector on the
// trailing indices k+8.. (u = [0 x 7, v] over T = R[k+1.., k+1..]).  1024 threads, 4 per row of
// T (row-wise loops over the packed rows).
// Outputs: AB rows 0..na-1 (band of A' = J R J, AB[i][kd] = A'[i][i-kd]), reflectors
// Varr[k][0..m) (v_0 = 1), taua[k].
__global__ __launch_bounds__(1024) void rr_arrow_kernel(const double* __restrict__ theta, int kp,
                                                       const double* __restrict__ GE,
                                                       double* __restrict__ AB,
                                                       double* __restrict__ Varr,
                                                       double* __restrict__ taua) {
  constexpr int W = RB_W;
  extern __shared__ double lds[];
  const int na = kp + W;
  double* R = lds;                  // packed lower, row i at i (i + 1) / 2
  double* u = R + na * (na + 1) / 2;
  double* p = u + na;
  const int tid = threadIdx.x;
  for (int i = tid; i < na; i += blockDim.x) {
    const int a = na - 1 - i;
    double* row = R + i * (i + 1) / 2;
    for (int j = 0; j <= i; ++j) {
      const int bc = na - 1 - j;  // natural indices, a <= bc
      double v;
      if (bc < kp)
        v = (a == bc) ? theta[a] : 0.0;
      else if (a < kp)
        v = GE[a * W + (bc - kp)];
      else
        v = 0.5 * (GE[a * W + (bc - kp)] + GE[bc * W + (a - kp)]);
      row[j] = v;
    }
  }
  __syncthreads();
  // three block barriers per step: every wave forms the reflector itself (sig by its own wave
  // sum, no block reduction), w = p - K u is formed on the fly, and column k is rewritten only
  // after every wave has read it
  const int lane = tid & 63;
  for (int k = 0; k + W + 1 < na; ++k) {
    const int m = na - k - W;  // reflector length (>= 2)
    const int nT = na - k - 1;
    const int o = k + 1;       // T[i][j] = R[o + i][o + j]
    double part = 0.0;
    for (int t = 1 + lane; t < m; t += 64) {
      const int row = k + W + t;
      const double x = R[row * (row + 1) / 2 + k];
      part += x * x;
    }
    const double sig = rb_wave_sum(part);
    const double x0 = R[(k + W) * (k + W + 1) / 2 + k];
    double tau, beta, scale;
    house_params(x0, sig, tau, beta, scale);
    for (int t = tid; t < nT; t += blockDim.x) {
      double val = 0.0;
      if (t == W - 1) {
        val = 1.0;
      } else if (t > W - 1) {
        const int row = o + t;
        val = R[row * (row + 1) / 2 + k] * scale;
      }
      u[t] = val;
      if (t >= W - 1) Varr[(int64_t)k * na + (t - (W - 1))] = val;
    }
    if (tid == 0) taua[k] = tau;
    __syncthreads();  // B1: u complete; column k read by everyone
    for (int t = tid; t < m; t += blockDim.x) {
      const int row = k + W + t;
      R[row * (row + 1) / 2 + k] = (t == 0) ? beta : 0.0;
    }
    if (tau == 0.0) {
      __syncthreads();
      continue;
    }
    // p = tau T u over u's support j >= W-1: row part (j <= i) + column part (j > i),
    // 4 threads per row (slice sl takes j = sl mod 4), incremental packed offsets
    {
      const int ri = tid >> 2, sl = tid & 3;
      double a0 = 0.0, a1 = 0.0;
      if (ri < nT) {
        const int gi = o + ri;
        const double* rowp = R + gi * (gi + 1) / 2 + o;
        int j = W - 1 + sl;
        for (; j + 4 <= ri; j += 8) {
          a0 += rowp[j] * u[j];
          a1 += rowp[j + 4] * u[j + 4];
        }
        for (; j <= ri; j += 4) a0 += rowp[j] * u[j];
        const int j1 = (ri + 1 > W - 1) ? ri + 1 : W - 1;
        j = j1 + ((sl - j1) & 3);
        int gj = o + j;
        int off = gj * (gj + 1) / 2 + gi;  // R[gj][gi]; R[gj + 4][gi] = off + 4 gj + 10
        for (; j + 4 < nT; j += 8) {
          a0 += R[off] * u[j];
          a1 += R[off + 4 * gj + 10] * u[j + 4];
          off += 8 * gj + 36;
          gj += 8;
        }
        for (; j < nT; j += 4) {
          a0 += R[off] * u[j];
          off += 4 * gj + 10;
          gj += 4;
        }
      }
      double acc = a0 + a1;
      acc += __shfl_xor(acc, 1, 64);
      acc += __shfl_xor(acc, 2, 64);
      if (ri < nT && sl == 0) p[ri] = tau * acc;
    }
    __syncthreads();  // B2: p complete
    double pp = 0.0;
    for (int t = lane; t < nT; t += 64) pp += p[t] * u[t];
    const double K = 0.5 * tau * rb_wave_sum(pp);  // every wave, same order: same K
    {
      const int ri = tid >> 2, sl = tid & 3;
      if (ri < nT) {
        const int gi = o + ri;
        double* rowp = R + gi * (gi + 1) / 2 + o;
        const double ui = u[ri], wi = p[ri] - K * u[ri];
        int j = sl;
        for (; j + 4 <= ri; j += 8) {
          const double r0 = rowp[j] - (ui * (p[j] - K * u[j]) + wi * u[j]);
          const double r1 = rowp[j + 4] - (ui * (p[j + 4] - K * u[j + 4]) + wi * u[j + 4]);
          rowp[j] = r0;
          rowp[j + 4] = r1;
        }
        for (; j <= ri; j += 4) rowp[j] -= ui * (p[j] - K * u[j]) + wi * u[j];
      }
    }
    __syncthreads();  // B3: step done
  }
  for (int e = tid; e < na * (W + 1); e += blockDim.x) {
    const int a = e / (W + 1), kd = e % (W + 1);
    if (a - kd < 0) {
      AB[e] = 0.0;
      continue;
    }
    const int i = na - 1 - a + kd, j = na - 1 - a;  // i >= j
    AB[e] = R[i * (i + 1) / 2 + j];
  }
}

// ---- band -> tridiagonal ----------------------------------------------------------------
// L (LDS): lower band + bulge, L[row * 17 + (row - col)], distance 0..15.
// hband: band column j at offset 0 (j = kry0, (kp + 8) x 8 rows) or
// (kp + 8) * 8 + (j - kry0 - 1) * 128 ([Q_{j-1} Q_j]^T W_j, 16 x 8).
// AB (global, c x 9): rows < na were written by rr_arrow_kernel (kp > 0); the rest is
// assembled here.
// One wave per sweep, lane (r, q) = (lane / 8, lane % 8) holds entry (r, q) of the 8 x 8 window;
// row sums over q use DPP (quad_perm + row_half_mirror), the other exchanges go through a
// per-wave LDS scratch (gather of a column / transpose), so a chase step is ~4 LDS round trips.
// Step j of sweep i is written to refl[(i * jm + j) * 9] (v[0..8), tau) for the back-transform.
__device__ __forceinline__ bool rb_wait(int* done, int prev, int need, int* abort_flag) {
  if (prev < 0) return true;
  for (int it = 0;; ++it) {
    const int v = __hip_atomic_load(&done[prev], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (v >= need) return true;
    if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    if (it > (1 << 22)) {
      __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ void rb_mark(int* done, int i, int v) {
  __hip_atomic_store(&done[i], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}


// compiler barrier for LDS exchanges inside one wave (LDS executes a wave's accesses in order)
__device__ __forceinline__ void rb_cbar() { asm volatile("" ::: "memory"); }

// One wave runs 8 consecutive sweeps in lockstep: lane (g, r) = (lane / 8, lane % 8) holds row r
// of sweep g's current window (8 doubles of the off-diagonal block O and of the diagonal block
// D in registers); at lockstep time T sweep g performs its step T - 2g, so sweep g+1 always runs
// two steps behind sweep g (the dependency of the pipelined chase) and concurrently running
// steps touch disjoint entries.  Column gathers / transposes go through a per-group LDS
// scratch.  The first sweep of a group waits for the previous group (another wave) through
// done[] (steps completed per sweep).  A step is: right-apply the previous reflector to O,
// new reflector from O's first column, left-apply, two-sided update of D; step 0 is the same
// with O = the column being annihilated.
#define RB_CH_WAVES 4
__global__ __launch_bounds__(RB_CH_WAVES * 64) void rr_chase_kernel(
    const double* __restrict__ hband, int c, int kp, double* __restrict__ AB,
    double* __restrict__ dd, double* __restrict__ ee, double* __restrict__ refl, int jm,
    int* __restrict__ err) {
  constexpr int W = RB_W, S = 2 * W + 1, GS = 80;
  extern __shared__ double L[];
  __shared__ int done[RB_MAXC];
  __shared__ int abort_flag;
  __shared__ double scratch[RB_CH_WAVES * 8 * GS];
  const int tid = threadIdx.x;
  const int na = kp > 0 ? kp + W : 0;
  const int j0 = kp / W;
  const int base1 = (kp + W) * W;
  for (int e = tid; e < (c + W) * S + 2; e += blockDim.x) L[e] = 0.0;  // band, 8 zero padding rows, trash + zero slots
  for (int e = tid; e < c; e += blockDim.x) done[e] = 0;
  if (tid == 0) abort_flag = 0;
  __syncthreads();
  for (int e = tid; e < c * (W + 1); e += blockDim.x) {
    const int i = e / (W + 1), kd = e % (W + 1);
    const int col = i - kd;
    double v = 0.0;
    if (col >= 0) {
      if (i < na) {
        v = AB[e];
      } else {
        const int j = i / W, r = i % W;
        const int nloc = (j == j0) ? (kp + W) : 2 * W;
        const double* G = hband + (j == j0 ? 0 : base1 + (j - j0 - 1) * 2 * W * W);
        if (col >= j * W) {
          const int cc = col - j * W;
          v = 0.5 * (G[(nloc - W + r) * W + cc] + G[(nloc - W + cc) * W + r]);
        } else {
          const int cc = col - (j - 1) * W;  // r <= cc: R_j upper triangular
          v = G[cc * W + r];
        }
        AB[e] = v;
      }
    } else if (i >= na) {
      AB[e] = 0.0;
    }
    L[i * S + kd] = v;
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  const int nwaves = blockDim.x >> 6;
  const int g = lane >> 3, r = lane & 7;
  double* gs = scratch + (wave * 8 + g) * GS;  // [0,64) transpose, [64,72) gather / u, [72,80) p
  const int nsw = c - 2;                       // sweeps 0 .. c-3
  bool aborted = false;
  for (int G = wave; G * 8 < nsw && !aborted; G += nwaves) {
    const int i = G * 8 + g;
    bool fin = !(i < nsw);
    int s = i + 1, m = (c - 1 - i) < W ? (c - 1 - i) : W;  // rows of the previous reflector
    if (!fin && m < 2) fin = true;
    if (fin && i < c && r == 0) done[i] = RB_DONE_ALL;
    double vp[W];
#pragma unroll
    for (int t = 0; t < W; ++t) vp[t] = 0.0;
    double taup = 0.0;
    for (int T = 0;; ++T) {
      if (__ballot(!fin) == 0) break;
      const int j = T - 2 * g;
      // window of this step, in select form (inactive groups get MR = NC = 0: every access
      // then goes to the spare slot, the reflector is the identity)
      bool act = !fin && j >= 0;
      const bool first = j == 0;
      int R0 = first ? i + 1 : s + m;
      const int C0 = first ? i : s;
      int NC = first ? 1 : m;
      int MR = first ? m : ((c - R0) < W ? (c - R0) : W);
      if (act && !first && R0 >= c) {  // sweep done
        fin = true;
        act = false;
        if (r == 0) __hip_atomic_store(&done[i], RB_DONE_ALL, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // inactive groups run the step on the zero padding rows c .. c+7 (every value stays 0;
      // nothing of theirs is recorded)
      int C0e = C0;
      if (!act) {
        R0 = c;
        C0e = c - W;
        MR = 0;
        NC = W;
      }
      // the group's first sweep waits for the previous group's last sweep (another wave)
      if (act && g == 0 && i > 0) {
        for (int it = 0;; ++it) {
          const int v = __hip_atomic_load(&done[i - 1], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
          if (v >= j + 2) break;
          if (__hip_atomic_load(&abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ||
              it > (1 << 22)) {
            __hip_atomic_store(&abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            aborted = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (__ballot(aborted) != 0) {
        aborted = true;
        break;
      }
      rb_cbar();
      {
        // rows past c are the zero padding rows (no row masks); O columns t >= NC read the
        // zero slot `zslot`, masked stores go to the trash slot `spare`.  Per-lane bases:
        // O[t] at oB - t; D[t] at dB1 - t (t <= r, row R0 + r) or dB2 + t (S + 1) (t > r, row R0 + t)
        const int spare = (c + W) * S, zslot = (c + W) * S + 1;
        const int oB = (R0 + r) * S + (R0 - C0e) + r;
        const int dB1 = (R0 + r) * S + r, dB2 = R0 * S - r;
        double O[W], D[W];
#pragma unroll
        for (int t = 0; t < W; ++t) {
          O[t] = L[t < NC ? oB - t : zslot];
          D[t] = L[t <= r ? dB1 - t : dB2 + t * (S + 1)];
        }
        // right-apply the previous reflector (acts on O's columns)
        const double tt = taup * dot8(O, vp);
#pragma unroll
        for (int t = 0; t < W; ++t) O[t] -= tt * vp[t];
        // reflector from O's first column
        gs[64 + r] = O[0];
        rb_cbar();
        double x[W];
#pragma unroll
        for (int t = 0; t < W; ++t) x[t] = gs[64 + t];
        const double sig = ((x[1] * x[1] + x[2] * x[2]) + (x[3] * x[3] + x[4] * x[4])) +
                           ((x[5] * x[5] + x[6] * x[6]) + x[7] * x[7]);
        double tau2, beta2, scale2;
        house_params(x[0], sig, tau2, beta2, scale2);
        double v2[W];
#pragma unroll
        for (int t = 0; t < W; ++t) v2[t] = (t == 0) ? 1.0 : x[t] * scale2;
        const double v2r = (r == 0) ? 1.0 : O[0] * scale2;
        // one LDS round trip for both the transpose of v2r O (left-apply: u_q = sum_r v2_r
        // O[r][q]) and p = tau D v2 (two-sided update of D)
        const double pr = tau2 * dot8(D, v2);
        rb_cbar();
#pragma unroll
        for (int t = 0; t < W; ++t) gs[r * 8 + t] = v2r * O[t];
        gs[72 + r] = pr;
        rb_cbar();
        double ut[W], ps[W];
#pragma unroll
        for (int t = 0; t < W; ++t) {
          ut[t] = gs[t * 8 + r];
          ps[t] = gs[72 + t];
        }
        const double um = ((ut[0] + ut[1]) + (ut[2] + ut[3])) + ((ut[4] + ut[5]) + (ut[6] + ut[7]));
        const double ks = dot8(ps, v2);
        rb_cbar();
        gs[64 + r] = um;
        rb_cbar();
#pragma unroll
        for (int t = 0; t < W; ++t) O[t] -= tau2 * v2r * gs[64 + t];
        O[0] = (r == 0) ? beta2 : 0.0;
#pragma unroll
        for (int t = 0; t < W; ++t) L[t < NC ? oB - t : spare] = O[t];
        // two-sided update of D
        const double K = 0.5 * tau2 * ks;
        const double wr = pr - K * v2r;
#pragma unroll
        for (int t = 0; t < W; ++t) {
          D[t] -= v2r * (ps[t] - K * v2[t]) + wr * v2[t];
          L[t <= r ? dB1 - t : spare] = D[t];
        }
        if (act) {
          // record the reflector for the back-transform
          double* slot = refl + ((int64_t)i * jm + j) * 9;
          slot[r] = v2r;
          if (r == 0) slot[8] = tau2;
#pragma unroll
          for (int t = 0; t < W; ++t) vp[t] = v2[t];
          taup = tau2;
          s = R0;
          m = MR;
        }
        rb_cbar();
        if (act && r == 0)
          __hip_atomic_store(&done[i], j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      rb_cbar();
    }
    if (!aborted && !fin) fin = true;
    if (!aborted && r == 0 && i < nsw)
      __hip_atomic_store(&done[i], RB_DONE_ALL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  if (abort_flag) {
    if (tid == 0) *err = 1;
    return;
  }
  for (int i = tid; i < c; i += blockDim.x) {
    dd[i] = L[i * S];
    if (i < c - 1) ee[i] = L[(i + 1) * S + 1];
  }
}

// ---- back-transform ---------------------------------------------------------------------
// Eigenvectors z of the tridiagonal (Y, column-major c x p) -> eigenvectors of the projected
// matrix: y = B_0 B_1 ... B_{c-3} z (sweep i's reflectors act on disjoint consecutive windows
// i+1+8j.., so B_i is block diagonal: lane j applies window j), then the X rows through the
// arrow reflectors; written as fp32 S (c x p, ld ldS).  One wave per eigenvector; y is kept
// residue-major in LDS (entry t at (t % 8) * sb + t / 8, sb odd), so the 8 entries of a window
// are read by all lanes without bank conflicts; the reflectors are staged
// through LDS at a time.
// RB_BT_VW eigenvectors per workgroup (one wave each).  The reflectors (chase sweeps in chunks
// of nch sweeps, then the arrow reflectors in chunks of whole Varr rows) stream through two LDS
// buffers shared by the workgroup: while the waves apply chunk q, every thread already holds its
// part of chunk q + 1 in registers (up to RB_BT_PF 16-B loads in flight), stored to the other
// buffer after the apply.  Window accesses are branch-free (masked lanes use a spare LDS slot);
// consecutive sweeps of one wave are ordered by the wave's in-order LDS execution.
#define RB_BT_VW 4
#define RB_BT_PF 16
typedef double f64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void rb_stage_load(const double* __restrict__ src, int nd, f64x2* r) {
  const int n2 = nd >> 1;
#pragma unroll
  for (int u = 0; u < RB_BT_PF; ++u) {
    const int e = (int)threadIdx.x + u * 256;
    r[u] = reinterpret_cast<const f64x2*>(src)[e < n2 ? e : 0];
  }
}
__device__ __forceinline__ void rb_stage_store(double* dst, const double* __restrict__ src, int nd,
                                               const f64x2* r) {
  const int n2 = nd >> 1;
#pragma unroll
  for (int u = 0; u < RB_BT_PF; ++u) {
    const int e = (int)threadIdx.x + u * 256;
    if (e < n2) reinterpret_cast<f64x2*>(dst)[e] = r[u];
  }
  if ((nd & 1) && threadIdx.x == 0) dst[nd - 1] = src[nd - 1];
}

__global__ __launch_bounds__(256) void rr_band_back_kernel(const double* __restrict__ Y, int c,
                                                           int p, const double* __restrict__ refl,
                                                           int jm, int kp,
                                                           const double* __restrict__ Varr,
                                                           const double* __restrict__ taua,
                                                           float* __restrict__ S, int ldS, int nch,
                                                           int bufd) {
  constexpr int W = RB_W;
  extern __shared__ double lds[];
  const int sb = ((c + W - 1) / W + 1) | 1;  // odd, and past the last window's reach (c + 7)
  const int ys = W * sb + 8;  // per-wave y image + spare slots
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int vec = blockIdx.x * RB_BT_VW + wave;
  const bool vok = vec < p;
  double* y = lds + wave * ys;
  const int spare = W * sb + (lane & 7);
  double* tau_s = lds + RB_BT_VW * ys;               // arrow reflector taus (RB_MAXNA)
  double* buf0 = tau_s + RB_MAXNA;                   // two reflector buffers of bufd doubles
  for (int t = lane; t < ys; t += 64) y[t] = 0.0;  // zero padding past c
  rb_cbar();
  for (int t = lane; t < c; t += 64) y[(t & 7) * sb + (t >> 3)] = vok ? Y[(int64_t)vec * c + t] : 0.0;
  const int na = kp > 0 ? kp + W : 0, nref = kp > 0 ? na - W - 1 : 0;
  for (int k = tid; k < nref; k += 256) tau_s[k] = taua[k];
  const int nsw = c - 2;  // sweeps 0 .. c-3
  const int nqc = (nsw - 1) / nch + 1;
  const int ra = na > 0 ? bufd / na : 1;  // arrow reflectors per chunk
  const int nqa = nref > 0 ? (nref + ra - 1) / ra : 0;
  const int nq = nqc + nqa;
  // chunk q: chase chunks (descending sweeps) then arrow chunks (descending k)
  auto chunk = [&](int q, const double*& src, int& nd, int& lo, int& cnt) {
    if (q < nqc) {
      lo = ((nsw - 1) / nch - q) * nch;
      cnt = (nsw - lo) < nch ? (nsw - lo) : nch;
      src = refl + (int64_t)lo * jm * 9;
      nd = cnt * jm * 9;
    } else {
      const int qa = q - nqc;
      const int hi = nref - qa * ra;
      lo = hi - ra > 0 ? hi - ra : 0;
      cnt = hi - lo;
      src = Varr + (int64_t)lo * na;
      nd = cnt * na;
    }
  };
  f64x2 pf[RB_BT_PF];
  {
    const double* src;
    int nd, lo, cnt;
    chunk(0, src, nd, lo, cnt);
    rb_stage_load(src, nd, pf);
    rb_stage_store(buf0, src, nd, pf);
  }
  __syncthreads();
  for (int q = 0; q < nq; ++q) {
    double* cur = buf0 + (q & 1) * bufd;
    double* nxt = buf0 + ((q + 1) & 1) * bufd;
    const double* nsrc = refl;
    int nnd = 0, nlo, ncnt;
    if (q + 1 < nq) chunk(q + 1, nsrc, nnd, nlo, ncnt);
    rb_stage_load(nsrc, nnd, pf);  // in flight during the apply below (nothing after the last)
    const double* src;
    int nd, lo, cnt;
    chunk(q, src, nd, lo, cnt);
    if (vok && q < nqc) {
      for (int ii = cnt - 1; ii >= 0; --ii) {
        const int i = lo + ii;
        const int nsteps = (c - (i + 1) + W - 1) / W;
        const bool act = lane < nsteps;
        const int j = act ? lane : 0;
        const double* rv = cur + ((int64_t)ii * jm + j) * 9;
        const double tau = rv[8];
        double yv[W], vv[W];
        int ad[W];
#pragma unroll
        for (int t = 0; t < W; ++t) {
          // entry (i + 1 + t) + 8 j: its residue-major slot is a sweep-uniform base + j.  The last
          // window may reach past c: those slots are zero padding and the reflector entries
          // there are zero (written so by the chase), so no mask; inactive lanes use the spare
          const int it = i + 1 + t;
          ad[t] = act ? (it & 7) * sb + (it >> 3) + j : spare;
          vv[t] = rv[t];
          yv[t] = y[ad[t]];
        }
        const double dot = tau * ((fma(vv[0], yv[0], vv[1] * yv[1]) + fma(vv[2], yv[2], vv[3] * yv[3])) +
                                  (fma(vv[4], yv[4], vv[5] * yv[5]) + fma(vv[6], yv[6], vv[7] * yv[7])));
#pragma unroll
        for (int t = 0; t < W; ++t) y[ad[t]] = yv[t] - dot * vv[t];
        rb_cbar();
      }
    } else if (vok) {  // X rows: y[0..na) <- J Q J y[0..na), reflectors k = lo + cnt - 1 .. lo
      for (int k = lo + cnt - 1; k >= lo; --k) {
        const double tau = tau_s[k];
        if (tau == 0.0) continue;
        const int m = na - k - W;
        const double* vk = cur + (int64_t)(k - lo) * na;
        double dot = 0.0;
        for (int t = lane; t < m; t += 64) {
          const int idx = na - 1 - k - W - t;
          dot += vk[t] * y[(idx & 7) * sb + (idx >> 3)];
        }
        dot = wave_sum_f64(dot);
        for (int t = lane; t < m; t += 64) {
          const int idx = na - 1 - k - W - t;
          y[(idx & 7) * sb + (idx >> 3)] -= tau * dot * vk[t];
        }
        rb_cbar();
      }
    }
    rb_stage_store(nxt, nsrc, nnd, pf);
    __syncthreads();
  }
  if (vok)
    for (int t = lane; t < c; t += 64)
      S[(int64_t)t * ldS + vec] = (float)y[(t & 7) * sb + (t >> 3)];
}

extern "C" hipError_t n2v2r_launch_rr_bisect(const double* d, const double* e, int c, int p,
                                             double* w, hipStream_t stream);
extern "C" hipError_t n2v2r_launch_rr_tri_inviter(const double* d, const double* e, int c, int p,
                                                  const double* w, double* Y,
                                                  hipStream_t stream);

// reflector slots per sweep of the bulge chase
extern "C" int n2v2r_rr_band_jm(int c) { return c / RB_W + 2; }

// Banded Rayleigh-Ritz: top-p Ritz pairs from the saved band columns.  theta: in = previous
// Ritz values (kp of them, the diagonal of the X block), out = p new ones (descending).
// refl: c * jm * 9 doubles (jm = n2v2r_rr_band_jm(c)).
extern "C" hipError_t n2v2r_launch_rr_band(const double* hband, int c, int kp, double* theta,
                                           double* AB, double* Varr, double* taua, double* d,
                                           double* e, double* refl, double* Y, float* S, int ldS,
                                           int p, int* err, hipStream_t stream) {
  if (c < 3 || c > RB_MAXC || c % RB_W || kp % RB_W || kp + RB_W > RB_MAXNA || p < 1 || p > c)
    return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)rr_arrow_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 2048);
    (void)hipFuncSetAttribute((const void*)rr_chase_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 46 * 1024);
    (void)hipFuncSetAttribute((const void*)rr_band_back_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 2048);
    (void)hipGetLastError();  // a refused attribute must not surface at a later launch
    attr = true;
  }
  const int jm = n2v2r_rr_band_jm(c);
  if (kp > 0) {
    const int na = kp + RB_W;
    const size_t lds = sizeof(double) * ((size_t)na * (na + 1) / 2 + 2 * (size_t)na);
    // 4 threads per row of the trailing matrix (nT <= na - 1 rows), whole waves, >= 256
    int nthr = ((4 * na + 63) / 64) * 64;
    if (nthr < 256) nthr = 256;
    if (nthr > 1024) nthr = 1024;
    hipLaunchKernelGGL(rr_arrow_kernel, dim3(1), dim3(nthr), lds, stream, theta, kp, hband, AB,
                       Varr, taua);
    hipError_t er = hipGetLastError();
    if (er != hipSuccess) return er;
  }
  const size_t lch = sizeof(double) * ((size_t)(c + RB_W) * (2 * RB_W + 1) + 8);  // + padding rows, spare slots
  hipLaunchKernelGGL(rr_chase_kernel, dim3(1), dim3(RB_CH_WAVES * 64), lch, stream, hband, c, kp,
                     AB, d, e, refl, jm, err);
  hipError_t er = hipGetLastError();
  if (er != hipSuccess) return er;
  er = n2v2r_launch_rr_bisect(d, e, c, p, theta, stream);
  if (er != hipSuccess) return er;
  er = n2v2r_launch_rr_tri_inviter(d, e, c, p, theta, Y, stream);
  if (er != hipSuccess) return er;
  // reflector chunk: an even number of sweeps (16-B aligned sources) within the register stage
  int nch = (2 * 256 * RB_BT_PF) / (jm * 9);
  if (nch > 16) nch = 16;
  nch &= ~1;
  if (nch < 2) return hipErrorInvalidValue;
  int bufd = nch * jm * 9;
  if (kp > 0 && bufd < kp + RB_W) bufd = kp + RB_W;
  bufd = (bufd + 1) & ~1;
  if (bufd > 2 * 256 * RB_BT_PF) return hipErrorInvalidValue;
  const size_t lbt = sizeof(double) * ((size_t)RB_BT_VW * (RB_W * (((c + RB_W - 1) / RB_W + 1) | 1) + 8) +
                                       RB_MAXNA + 2 * (size_t)bufd);
  hipLaunchKernelGGL(rr_band_back_kernel, dim3((unsigned)((p + RB_BT_VW - 1) / RB_BT_VW)),
                     dim3(64 * RB_BT_VW), lbt, stream, Y, c, p, refl, jm, kp, Varr, taua, S, ldS,
                     nch, bufd);
  return hipGetLastError();
}

// Rayleigh-Ritz on the GPU for the block Krylov-Schur eigensolver: the projected matrix
// H = Q^T M Q (c x c fp64, c <= 768) never leaves the device except as its tridiagonal.
//
//   rr_tridiag_kernel    Householder reduction H = P T P^T (one workgroup of 1024 threads,
//                        H L2-resident, full symmetric storage; per step ONE fused pass
//                        reads and writes the trailing block: rank-2 update of step k +
//                        column-oriented matvec of step k+1).  Outputs d, e (T), tau and the
//                        reflectors V (row k = v_k, v_k[0] = 1).
//   (host)               eigenvalues of T by implicit QL + inverse iteration for the top p
//                        (n2v2r_host_tridiag_eig_top, eig_host.cpp): O(c p) work.
//   rr_backtransform     S = P Y for the p wanted eigenvectors Y of T: one workgroup per 8
//                        columns applies the c-2 reflectors as compact-WY blocks of 32, last
//                        block first, and writes S as the fp32 Ritz coefficient matrix
//                        (c x ld) the NN kernels consume.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "common.h"

#define RR_MAXC 768
#define RR_BT_COLS 8

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum of one double per thread (fixed order: waves folded in index order)
template <int NW>
__device__ __forceinline__ double block_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < NW; ++w) s += red[w];
  return s;
}

}  // namespace

// Fused column-oriented Householder tridiagonalisation.  H is symmetric, so p = B v is also
// B^T v = sum_r v[r] B[r][:]: lanes own columns, waves own rows, every row is read as
// coalesced 8-B loads and accumulated without cross-lane reductions.  One pass per step does
// the rank-2 update of step k AND the matvec of step k+1 (whose reflector comes from the
// updated first row, formed just before the pass): B is read once and written once per step.
//   LDS: v, w (step k), vn, p (step k+1), part[NW][c] (per-wave matvec partials).
template <int TMAX, int NT, bool PAIRS>
__global__ __launch_bounds__(NT) void rr_tridiag_kernel(double* __restrict__ A, int c,
                                                                    double* __restrict__ dd,
                                                                    double* __restrict__ ee,
                                                                    double* __restrict__ tau,
                                                                    double* __restrict__ V) {
  constexpr int NW = NT / 64;
  extern __shared__ double lds[];
  double* v = lds;              // [c]
  double* w = v + c;            // [c]
  double* vn = w + c;           // [c]
  double* p = vn + c;           // [c]
  double* part = p + c;         // [NW][c]
  __shared__ double red[NW];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  for (int64_t q = tid; q < (int64_t)c * c; q += NT) {
    const int i = (int)(q / c), j = (int)(q % c);
    if (j < i) {
      const double s = 0.5 * (A[(int64_t)i * c + j] + A[(int64_t)j * c + i]);
      A[(int64_t)i * c + j] = s;
      A[(int64_t)j * c + i] = s;
    }
  }
  __syncthreads();

  // reflector from x (length m, in `dst`, overwritten by v, v[0] = 1); returns tau, sets beta
  // Every thread owns the entries i = tid (mod NT) of dst (it wrote them, or the caller
  // synchronised), so only the block reduction needs barriers.
  auto make_reflector = [&](double* dst, int m, int k) -> double {
    double part2 = 0.0;
    for (int i = tid; i < m; i += NT)
      if (i > 0) part2 += dst[i] * dst[i];
    const double x0 = dst[0];
    const double sig = block_sum<NW>(part2, red);
    double t = 0.0, beta = x0, scale = 0.0;
    if (sig != 0.0) {
      const double nrm = sqrt(x0 * x0 + sig);
      beta = (x0 >= 0) ? -nrm : nrm;
      t = (beta - x0) / beta;
      scale = 1.0 / (x0 - beta);
    }
    double* vk = V + (int64_t)k * c;
    for (int i = tid; i < m; i += NT) {
      const double vi = (i == 0) ? 1.0 : dst[i] * scale;
      dst[i] = vi;
      vk[i] = vi;
    }
    if (tid == 0) {
      ee[k] = beta;
      tau[k] = t;
    }
    __syncthreads();
    return t;
  };

  // ---- step 0: reflector from row 0, p = tau B v with B = A[1.., 1..] (matvec only)
  int m = c - 1;
  for (int i = tid; i < m; i += NT) v[i] = A[1 + i];
  if (tid == 0) dd[0] = A[0];
  __syncthreads();  // v[0] is read by every thread
  double t = make_reflector(v, m, 0);
  {
    double acc[TMAX];
#pragma unroll
    for (int q = 0; q < TMAX; ++q) acc[q] = 0.0;
    for (int r = wave; r < m; r += NW) {
      const double* br = A + (int64_t)(1 + r) * c + 1;
      const double vr = v[r];
#pragma unroll
      for (int q = 0; q < TMAX; ++q) {
        const int j = lane + 64 * q;
        if (j < m) acc[q] += br[j] * vr;
      }
    }
#pragma unroll
    for (int q = 0; q < TMAX; ++q) {
      const int j = lane + 64 * q;
      if (j < m) part[wave * c + j] = acc[q];
    }
    __syncthreads();
    for (int j = tid; j < m; j += NT) {
      double s2 = 0.0;
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) s2 += part[wv * c + j];
      p[j] = t * s2;
    }
    __syncthreads();
  }

  for (int k = 0; k < c - 2; ++k) {
    const int o = k + 1;  // B = A[o.., o..], m = c - o rows
    // w = p - (t/2)(p.v) v
    double pp = 0.0;
    for (int i = tid; i < m; i += NT) pp += p[i] * v[i];
    const double pvv = block_sum<NW>(pp, red);
    const double half = 0.5 * t * pvv;
    for (int i = tid; i < m; i += NT) w[i] = p[i] - half * v[i];
    __syncthreads();
    // updated first row of B: diagonal d[o] and x' = B[0][1..] (the next reflector's input)
    const double* b0 = A + (int64_t)o * c + o;
    if (tid == 0) dd[o] = b0[0] - 2.0 * v[0] * w[0];
    const int mn = m - 1;
    for (int j = tid; j < mn; j += NT)
      vn[j] = b0[1 + j] - v[0] * w[1 + j] - w[0] * v[1 + j];
    __syncthreads();
    if (mn == 1) {  // k = c - 3: the last 2 x 2 block
      if (tid == 0) {
        ee[o] = vn[0];
        tau[o] = 0.0;
        const double b11 = A[(int64_t)(o + 1) * c + o + 1];
        dd[o + 1] = b11 - 2.0 * v[1] * w[1];
      }
      break;
    }
    const double tn = make_reflector(vn, mn, o);
    // fused pass over rows r = 1..m-1: B[r][1..] -= v[r] w + w[r] v; p' += vn[r-1] B'[r][1..]
    if (PAIRS) {
      // 16-B accesses: lane owns absolute column pairs (J, J+1), J even, J >= jb
      const int jb = (o + 1) & ~1;
      double vj[TMAX], wj[TMAX], acc[TMAX];
      int rel[TMAX];
#pragma unroll
      for (int q = 0; q < TMAX; ++q) {
        const int J = jb + 2 * (lane + 64 * (q >> 1)) + (q & 1);
        rel[q] = J - (o + 1);  // column 1 + rel of B; valid for 0 <= rel < mn
        const bool ok = rel[q] >= 0 && rel[q] < mn;
        vj[q] = ok ? v[1 + rel[q]] : 0.0;
        wj[q] = ok ? w[1 + rel[q]] : 0.0;
        acc[q] = 0.0;
      }
#pragma unroll 4
      for (int r = 1 + wave; r < m; r += NW) {
        double* rowp = A + (int64_t)(o + r) * c;
        const double vr = v[r], wr = w[r], vnr = vn[r - 1];
#pragma unroll
        for (int q2 = 0; q2 < TMAX; q2 += 2) {
          const int J = jb + 2 * (lane + 64 * (q2 >> 1));
          if (J < c) {
            double2 b2 = *reinterpret_cast<const double2*>(rowp + J);
            double bx = b2.x, by = b2.y;
            if (rel[q2] >= 0) {
              bx -= vr * wj[q2] + wr * vj[q2];
              acc[q2] += bx * vnr;
            }
            by -= vr * wj[q2 + 1] + wr * vj[q2 + 1];
            acc[q2 + 1] += by * vnr;
            *reinterpret_cast<double2*>(rowp + J) = make_double2(bx, by);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < TMAX; ++q)
        if (rel[q] >= 0 && rel[q] < mn) part[wave * c + rel[q]] = acc[q];
    } else {
      double vj[TMAX], wj[TMAX], acc[TMAX];
#pragma unroll
      for (int q = 0; q < TMAX; ++q) {
        const int j = 1 + lane + 64 * q;
        vj[q] = (j < m) ? v[j] : 0.0;
        wj[q] = (j < m) ? w[j] : 0.0;
        acc[q] = 0.0;
      }
#pragma unroll 4
      for (int r = 1 + wave; r < m; r += NW) {
        double* br = A + (int64_t)(o + r) * c + o + 1;
        const double vr = v[r], wr = w[r], vnr = vn[r - 1];
#pragma unroll
        for (int q = 0; q < TMAX; ++q) {
          const int j = lane + 64 * q;  // column 1 + j of B
          if (j < mn) {
            const double b = br[j] - vr * wj[q] - wr * vj[q];
            br[j] = b;
            acc[q] += b * vnr;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < TMAX; ++q) {
        const int j = lane + 64 * q;
        if (j < mn) part[wave * c + j] = acc[q];
      }
    }
    __syncthreads();
    for (int j = tid; j < mn; j += NT) {
      double s2 = 0.0;
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) s2 += part[wv * c + j];
      p[j] = tn * s2;
      v[j] = vn[j];
    }
    // no barrier: the next pp and w loops read only this thread's own entries of p and v
    t = tn;
    m = mn;
  }
}

// ---- the same reduction spread over G = PR x nt workgroups (one per CU) ---------------------
// The c x c matrix is cut into 32 x 32 tiles (nt per dimension) that stay in LDS for the whole
// launch: workgroup (pr, pc) owns the column tile pc and the row tiles pr, pr + PR, ...
// (block-cyclic, so the active trailing block stays spread as it shrinks), i.e. up to
// ceil(nt / PR) tiles (12 at c = 768, PR = 2: 99 KB).  Each step k (pivot o = k + 1):
//   every workgroup, redundantly and bit-identically, forms p = t sum_pr part[pr] (the previous
//   pass's column partials, fixed order), w = p - (t/2)(p.v) v, the updated pivot row
//   (published by its owners) -> d[o] and the next reflector vn;
//   then updates its own tiles B -= v w^T + w v^T on rows/columns >= o+1 and accumulates the
//   column partials of the next matvec B' vn, which it publishes with the new pivot row o+1.
// One grid barrier per step.  Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first
// row of the sc1 table): every published double is an agent-scope relaxed atomic store
// (global_store sc1), every storing wave waits vmcnt(0), a workgroup barrier, then ONE lane
// adds to the monotonic counter; the poller reads it with sc1 loads, the workgroup barrier
// releases the other waves, and every load of published data is an sc1 load.  Partials and the
// pivot row are double-buffered by step parity (a buffer is rewritten only two barriers after
// it was read).  The spin is bounded: a workgroup that waits ~seconds gives up, sets *err and
// writes NaN to d[0] (the caller's Ritz values then fail), so the launch always drains.
// (Measured and dropped: data-tagged 8-B granules polled by every thread instead of the
// counter -- no barrier, but 96 workgroups x 256 threads polling the same lines starved the
// producers' stores: one c = 768 call at PR = 4 timed out; the counter poll is one lane per
// workgroup.)
#define TRC_TS 32
#define TRC_LD 33
#define TRC_NT 256

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(__hip_atomic_load(reinterpret_cast<const long long*>(p),
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double x) {
  __hip_atomic_store(reinterpret_cast<long long*>(p), __double_as_longlong(x), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Sharded form (the default): workgroup b adds to the counter of its XCD group b % 8 (each on a
// 128-B line of its own), and the poll reads all 8 shards at once (lane i of wave 0 shard i) until
// each has reached its group's arrivals for this barrier: an sc1-load poll of every shard of a
// sharded counter, the valid hand-off of MI355X_MICROARCH.md's table (first row), with 1/8 of the
// atomic traffic on each line.  gen: this barrier's 1-based index.  true when the wait timed out.
__device__ __forceinline__ bool trc_grid_barrier_sharded(unsigned* ctr, unsigned gen, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {
    const int G = gridDim.x;
    const int lane = threadIdx.x;
    if (lane == 0)
      __hip_atomic_fetch_add(ctr + 32 * (1 + (blockIdx.x & 7)), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    const int gl = lane & 7;
    const unsigned want = gl < G ? gen * (unsigned)((G - gl + 7) >> 3) : 0u;
    const unsigned* c = ctr + 32 * (1 + gl);
    int f = 0;
    long it = 0;
    while (true) {
      const unsigned v = lane < 8 ? __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : want;
      if (__ballot(v < want) == 0ull) break;
      if (++it > (1l << 24)) {
        f = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) *flag = f;
  }
  __syncthreads();
  return *flag != 0;
}

__global__ __launch_bounds__(TRC_NT) void rr_tridiag_coop_kernel(
    const double* __restrict__ A, int c, int PR, double* __restrict__ dd, double* __restrict__ ee,
    double* __restrict__ tau, double* __restrict__ V, double* part /* [2][PR][c] */,
    double* rowbuf /* [2][c] */, unsigned* ctr, int* err) {
  constexpr int NW = TRC_NT / 64;
  extern __shared__ double lds[];
  const int nt = (c + TRC_TS - 1) / TRC_TS;
  const int G = gridDim.x;
  const int pc = blockIdx.x % nt, pr = blockIdx.x / nt;
  const int ntr = (nt - pr + PR - 1) / PR;  // row tiles pr + PR q, q < ntr
  double* T = lds;                                   // [ntr][32][33]
  double* v = T + (size_t)ntr * TRC_TS * TRC_LD;     // [c], global indices
  double* w = v + c;
  double* vn = w + c;
  double* p = vn + c;
  double* row = p + c;
  double* accs = row + c;                            // [8][32]
  __shared__ double red[NW];
  __shared__ int flag;
  const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;
  const int J = TRC_TS * pc + tx;  // this thread's column
  const bool lead = blockIdx.x == 0;

  auto bsum = [&](double x) -> double {
    x = wave_sum(x);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = x;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += red[q];
    return s;
  };
  // reflector from x[lo..c) in place (x[lo] = 1 after), row k of V (the leader writes it)
  auto make_reflector = [&](double* x, int lo, int k) -> double {
    double part2 = 0.0;
    for (int i = lo + 1 + tid; i < c; i += TRC_NT) part2 += x[i] * x[i];
    const double x0 = x[lo];
    const double sig = bsum(part2);
    double t = 0.0, beta = x0, scale = 0.0;
    if (sig != 0.0) {
      const double nrm = sqrt(x0 * x0 + sig);
      beta = (x0 >= 0) ? -nrm : nrm;
      t = (beta - x0) / beta;
      scale = 1.0 / (x0 - beta);
    }
    double* vk = V + (int64_t)k * c - lo;
    for (int i = lo + tid; i < c; i += TRC_NT) {
      const double vi = (i == lo) ? 1.0 : x[i] * scale;
      x[i] = vi;
      if (lead) vk[i] = vi;
    }
    if (lead && tid == 0) {
      ee[k] = beta;
      tau[k] = t;
    }
    __syncthreads();
    return t;
  };
  // the WG's tiles on rows / columns >= lo: optional rank-2 update (v, w), column partials of
  // the product with mv, published to part[par][pr][.], and the pivot row lo to rowbuf[par]
  auto pass = [&](int lo, bool upd, const double* mv, int par) {
    const bool jok = J >= lo && J < c;
    const double vJ = (upd && jok) ? v[J] : 0.0, wJ = (upd && jok) ? w[J] : 0.0;
    const int rlo = lo & (TRC_TS - 1), blo = lo / TRC_TS;
    double acc = 0.0;
    for (int q = 0; q < ntr; ++q) {
      const int bi = pr + PR * q;
      if (bi < blo) continue;
      double* tile = T + (size_t)q * TRC_TS * TRC_LD;
#pragma unroll
      for (int u = 0; u < TRC_TS / 8; ++u) {
        const int rr = ty + 8 * u, R = TRC_TS * bi + rr;
        if (R >= lo && R < c && jok) {
          double a = tile[rr * TRC_LD + tx];
          if (upd) {
            a -= v[R] * wJ + w[R] * vJ;
            tile[rr * TRC_LD + tx] = a;
          }
          acc += a * mv[R];
          if (R == lo) st_sc1(rowbuf + (size_t)par * c + J, a);
        }
      }
    }
    accs[ty * TRC_TS + tx] = acc;
    __syncthreads();
    if (ty == 0 && J < c) {
      double sacc = 0.0;
#pragma unroll
      for (int y = 0; y < 8; ++y) sacc += accs[y * TRC_TS + tx];
      st_sc1(part + ((size_t)par * PR + pr) * c + J, sacc);
    }
  };

  // tiles in: symmetrised as the one-workgroup kernel does
  for (int q = 0; q < ntr; ++q) {
    const int bi = pr + PR * q;
    double* tile = T + (size_t)q * TRC_TS * TRC_LD;
    for (int rr = ty; rr < TRC_TS; rr += 8) {
      const int R = TRC_TS * bi + rr;
      tile[rr * TRC_LD + tx] =
          (R < c && J < c) ? 0.5 * (A[(int64_t)R * c + J] + A[(int64_t)J * c + R]) : 0.0;
    }
  }
  // reflector 0 from row 0, then the first matvec (no update)
  for (int i = 1 + tid; i < c; i += TRC_NT) v[i] = 0.5 * (A[i] + A[(int64_t)i * c]);
  if (lead && tid == 0) dd[0] = A[0];
  __syncthreads();
  double t = make_reflector(v, 1, 0);
  pass(1, false, v, 0);
  unsigned nbar = 1;
  // (one counter for the whole grid instead of one per XCD group: 5.70 vs 5.15 ms per cfg3
  // call, profiles/r05_cfg3_single_bar_kernel_stats.csv; removed)
  auto grid_barrier = [&](unsigned nb) { return trc_grid_barrier_sharded(ctr, nb, &flag); };
  bool failed = grid_barrier(nbar);
  for (int k = 0; !failed; ++k) {
    const int o = k + 1, par = k & 1;
    for (int i = o + tid; i < c; i += TRC_NT) {
      double sp = 0.0;
      for (int q = 0; q < PR; ++q) sp += ld_sc1(part + ((size_t)par * PR + q) * c + i);
      p[i] = t * sp;
      row[i] = ld_sc1(rowbuf + (size_t)par * c + i);
    }
    __syncthreads();
    double pp = 0.0;
    for (int i = o + tid; i < c; i += TRC_NT) pp += p[i] * v[i];
    const double half = 0.5 * t * bsum(pp);
    for (int i = o + tid; i < c; i += TRC_NT) w[i] = p[i] - half * v[i];
    __syncthreads();
    const double vo = v[o], wo = w[o];
    if (lead && tid == 0) dd[o] = row[o] - 2.0 * vo * wo;
    for (int i = o + 1 + tid; i < c; i += TRC_NT) vn[i] = row[i] - vo * w[i] - wo * v[i];
    __syncthreads();
    if (c - o == 2) {  // the last 2 x 2 block
      if (lead && tid == 0) {
        ee[o] = vn[o + 1];
        tau[o] = 0.0;
      }
      const int R = c - 1, bi = R / TRC_TS;
      if (pc == bi && bi % PR == pr && tx == (R & 31) && ty == ((R & 31) & 7)) {
        const double b11 = T[((size_t)((bi - pr) / PR) * TRC_TS + (R & 31)) * TRC_LD + tx];
        dd[R] = b11 - 2.0 * v[R] * w[R];
      }
      break;
    }
    const double tn = make_reflector(vn, o + 1, o);
    pass(o + 1, true, vn, par ^ 1);
    // every read of v in the pass precedes the partials' barrier inside it
    for (int i = o + 1 + tid; i < c; i += TRC_NT) v[i] = vn[i];
    t = tn;
    failed = grid_barrier(++nbar);
  }
  if (failed && tid == 0) {
    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st_sc1(dd, __builtin_nan(""));
  }
}

// [2][4][c] partials | [2][c] pivot rows | counters: [0] the single counter, [1] the error
// word, the 8 shard counters at [32 (1 + g)] (a 128-B line each)
#define TRC_CTR_WORDS (32 * 9)
extern "C" size_t n2v2r_rr_tridiag_scratch_bytes(int c) {
  return sizeof(double) * ((size_t)2 * 4 * c + (size_t)2 * c) + sizeof(unsigned) * TRC_CTR_WORDS;
}

// Y: p eigenvectors of T, column-major (vector j at Y[j * c]).  S[i * lds + j] = (P Y)[i][j],
// P = H_0 H_1 ... H_{c-3}.  Blocked (compact WY): the reflectors are taken BT_NB at a time,
// last block first; for the block H_k0 ... H_k1-1 = I - W T W^T (T upper triangular, the
// forward column-wise LAPACK larft recurrence, built from the block's Gram matrix W^T W) the
// update is z <- z - W (T (W^T z)).
//   rr_bt_tfactor_kernel: the T factors of all blocks at once, one workgroup per block (they
//     depend on the reflectors alone).  Round 4: moved out of the column workgroups, which each
//     rebuilt every block's Gram and ran the serial larft rows between two barriers (1.39 ms per
//     cfg3 call, 24 blocks x ~58 us on the critical path).
//   rr_backtransform_kernel: one workgroup per RR_BT_COLS columns keeps its columns in LDS and
//     walks the blocks with the precomputed T: W^T z, U = T (W^T z), z -= W U.
// Bit-identical to the former single kernel: the same partial sums in the same order.
#define BT_NB 32
#define BT_CH 128

__global__ __launch_bounds__(256) void rr_bt_tfactor_kernel(const double* __restrict__ V,
                                                            const double* __restrict__ tau, int c,
                                                            double* __restrict__ Tg) {
  __shared__ double Wc[BT_NB][BT_CH + 1];
  __shared__ double G[BT_NB][BT_NB + 1];
  __shared__ double T[BT_NB][BT_NB + 1];
  const int tid = threadIdx.x;
  // Gram pairs (a, bb), bb < a, enumerated e = tid and tid + 256
  int ga[2], gb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    int e = tid + 256 * h, a = 1;
    while (e >= a) {  // row a holds a pairs (bb = 0 .. a-1)
      e -= a;
      ++a;
    }
    ga[h] = a;
    gb[h] = e;
  }
  const int nref = c - 2;  // reflectors 0 .. c-3 (v_k acts on indices k+1 .. c-1)
  const int kb = blockIdx.x * BT_NB;
  const int nb = (nref - kb) < BT_NB ? (nref - kb) : BT_NB;
  double g0 = 0.0, g1 = 0.0;
  for (int ich = kb + 1; ich < c; ich += BT_CH) {
    const int len = (c - ich) < BT_CH ? (c - ich) : BT_CH;
#pragma unroll 8
    for (int it = 0; it < BT_NB * BT_CH / 256; ++it) {
      const int q = tid + 256 * it;
      const int a = q / BT_CH, ii = q % BT_CH;
      const int k = kb + a, i = ich + ii;
      const bool ok = a < nb && ii < len && i >= k + 1;
      const double x = V[ok ? (int64_t)k * c + (i - k - 1) : 0];
      Wc[a][ii] = ok ? x : 0.0;
    }
    __syncthreads();
    {
      const double* a0 = Wc[ga[0] < nb ? ga[0] : 0];
      const double* b0 = Wc[gb[0]];
      const double* a1 = Wc[ga[1] < nb ? ga[1] : 0];
      const double* b1 = Wc[gb[1] < BT_NB ? gb[1] : 0];
      double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
      const int len4 = len & ~3;
      for (int ii = 0; ii < len4; ii += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          s1[u] += a0[ii + u] * b0[ii + u];
          s2[u] += a1[ii + u] * b1[ii + u];
        }
      }
      for (int ii = len4; ii < len; ++ii) {
        s1[0] += a0[ii] * b0[ii];
        s2[0] += a1[ii] * b1[ii];
      }
      if (ga[0] < nb) g0 += (s1[0] + s1[1]) + (s1[2] + s1[3]);
      if (ga[1] < nb) g1 += (s2[0] + s2[1]) + (s2[2] + s2[3]);
    }
    __syncthreads();
  }
  if (ga[0] < nb) G[gb[0]][ga[0]] = g0;
  if (ga[1] < nb) G[gb[1]][ga[1]] = g1;
  for (int q = tid; q < BT_NB * (BT_NB + 1); q += 256) (&T[0][0])[q] = 0.0;
  __syncthreads();
  // T (forward larft): lane r builds row r alone (its own LDS row, 4 partial sums),
  // T[r][i] = -tau_i sum_{q=r}^{i-1} T[r][q] G[q][i]
  if (tid < nb) {
    const int r = tid;
    T[r][r] = tau[kb + r];
    for (int i = r + 1; i < nb; ++i) {
      double sa[4] = {0.0, 0.0, 0.0, 0.0};
      int q = r;
      for (; q + 4 <= i; q += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) sa[u] += T[r][q + u] * G[q + u][i];
      }
      for (; q < i; ++q) sa[0] += T[r][q] * G[q][i];
      T[r][i] = -tau[kb + i] * ((sa[0] + sa[1]) + (sa[2] + sa[3]));
    }
  }
  __syncthreads();
  double* out = Tg + (size_t)blockIdx.x * BT_NB * BT_NB;
  for (int q = tid; q < BT_NB * BT_NB; q += 256) out[q] = T[q / BT_NB][q % BT_NB];
}

__global__ __launch_bounds__(256) void rr_backtransform_kernel(const double* __restrict__ V,
                                                               const double* __restrict__ Tg,
                                                               int c, const double* __restrict__ Y,
                                                               int p, float* __restrict__ S,
                                                               int lds) {
  __shared__ double z[RR_BT_COLS][RR_MAXC + 1];  // +1: the 8 columns fall in distinct banks
  __shared__ double Wc[BT_NB][BT_CH + 1];         // staged rows of the block's reflectors
  __shared__ double T[BT_NB][BT_NB + 1];
  __shared__ double WZ[BT_NB][RR_BT_COLS];
  __shared__ double U[BT_NB][RR_BT_COLS];
  const int tid = threadIdx.x;
  const int j0 = blockIdx.x * RR_BT_COLS;
  const int nj = (p - j0) < RR_BT_COLS ? (p - j0) : RR_BT_COLS;
  for (int q = tid; q < RR_BT_COLS * c; q += 256) {
    const int jj = q / c, i = q % c;
    z[jj][i] = (jj < nj) ? Y[(int64_t)(j0 + jj) * c + i] : 0.0;
  }
  __syncthreads();
  // thread role in the dot phase: (a, jj) = (tid / 8, tid % 8) for W^T z
  const int wa = tid / RR_BT_COLS, wj = tid % RR_BT_COLS;
  const int nref = c - 2;
  for (int kb = ((nref - 1) / BT_NB) * BT_NB; kb >= 0; kb -= BT_NB) {
    const int nb = (nref - kb) < BT_NB ? (nref - kb) : BT_NB;
    {  // this block's T (zero past nb), read before the first barrier below
      const double* tg = Tg + (size_t)(kb / BT_NB) * BT_NB * BT_NB;
      for (int q = tid; q < BT_NB * BT_NB; q += 256) T[q / BT_NB][q % BT_NB] = tg[q];
    }
    double wz = 0.0;
    for (int ich = kb + 1; ich < c; ich += BT_CH) {
      const int len = (c - ich) < BT_CH ? (c - ich) : BT_CH;
      // fixed trip count, unrolled: all 16 loads of a thread are in flight together
#pragma unroll 8
      for (int it = 0; it < BT_NB * BT_CH / 256; ++it) {
        const int q = tid + 256 * it;
        const int a = q / BT_CH, ii = q % BT_CH;
        const int k = kb + a, i = ich + ii;
        // the address is clamped in-bounds: the unrolled select may issue the load regardless
        const bool ok = a < nb && ii < len && i >= k + 1;
        const double x = V[ok ? (int64_t)k * c + (i - k - 1) : 0];
        Wc[a][ii] = ok ? x : 0.0;
      }
      __syncthreads();
      {  // (Wc is zero past len, z is read only below c)
        const double* wr = Wc[wa < nb ? wa : 0];
        const double* zr = &z[wj][ich];
        double s0[4] = {0.0, 0.0, 0.0, 0.0};
        const int len4 = len & ~3;
        for (int ii = 0; ii < len4; ii += 4) {
#pragma unroll
          for (int u = 0; u < 4; ++u) s0[u] += wr[ii + u] * zr[ii + u];
        }
        for (int ii = len4; ii < len; ++ii) s0[0] += wr[ii] * zr[ii];
        if (wa < nb) wz += (s0[0] + s0[1]) + (s0[2] + s0[3]);
      }
      __syncthreads();
    }
    if (wa < nb) WZ[wa][wj] = wz;
    __syncthreads();
    {
      // every row of U is written: rows a >= nb (the partial block, processed first) are
      // zero, not stale LDS -- the update below multiplies them by a zero w_a[i], and
      // 0 * (a NaN / Inf bit pattern left by an earlier kernel) is NaN
      double sacc = 0.0;
      if (wa < nb)
        for (int bb = wa; bb < nb; ++bb) sacc += T[wa][bb] * WZ[bb][wj];
      U[wa][wj] = sacc;
    }
    __syncthreads();
    // z[:, i] -= sum_a w_a[i] U[a][:] for i > kb
    for (int i = kb + 1 + tid; i < c; i += 256) {
      double acc[RR_BT_COLS];
#pragma unroll
      for (int jj = 0; jj < RR_BT_COLS; ++jj) acc[jj] = 0.0;
      const int amax = (i - kb - 1) < nb ? (i - kb - 1) : nb - 1;  // w_a[i] != 0 iff i >= kb+a+1
#pragma unroll 1
      for (int h = 0; h < BT_NB; h += 8) {
        double wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {  // 8 loads in flight before the FMAs
          const int a = h + u, k = kb + a;
          const bool ok = a <= amax;  // clamped address, as above
          const double x = V[ok ? (int64_t)k * c + (i - k - 1) : 0];
          wv[u] = ok ? x : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int jj = 0; jj < RR_BT_COLS; ++jj) acc[jj] += wv[u] * U[h + u][jj];
      }
#pragma unroll
      for (int jj = 0; jj < RR_BT_COLS; ++jj) z[jj][i] -= acc[jj];
    }
    __syncthreads();
  }
  for (int q = tid; q < RR_BT_COLS * c; q += 256) {
    const int i = q / RR_BT_COLS, jj = q % RR_BT_COLS;
    if (jj < nj) S[(int64_t)i * lds + j0 + jj] = (float)z[jj][i];
  }
}

// reciprocal to fp64 accuracy: v_rcp_f64 and two Newton steps (off the IEEE-division path)
__device__ __forceinline__ double inv_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  r = fma(r, fma(-x, r, 1.0), r);
  return r;
}

// ---- eigenpairs of the tridiagonal T on the GPU --------------------------------------------
// rr_bisect_kernel: one workgroup per wanted eigenvalue (j-th largest, j < p).  Multisection
// on the Gershgorin interval: each round the 256 threads evaluate the Sturm count (negative
// pivots of the LDL^T of T - x I, pivots clamped to -pivmin as LAPACK dstebz) at 256 interior
// points, the interval shrinks 257x; 7 rounds reach fp64 resolution.
#define RR_BIS_THREADS 256
__global__ __launch_bounds__(RR_BIS_THREADS) void rr_bisect_kernel(const double* __restrict__ dg,
                                                                   const double* __restrict__ eg,
                                                                   int c, int p,
                                                                   double* __restrict__ w) {
  __shared__ double d[RR_MAXC], e2[RR_MAXC];
  __shared__ int cnt[RR_BIS_THREADS];
  __shared__ double red[4][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = blockIdx.x;
  const int a = c - 1 - j;  // ascending index of the wanted eigenvalue
  double glo = 1e300, ghi = -1e300, emax = 0.0;
  for (int i = tid; i < c; i += RR_BIS_THREADS) {
    const double di = dg[i];
    const double el = i > 0 ? fabs(eg[i - 1]) : 0.0, er = i < c - 1 ? fabs(eg[i]) : 0.0;
    d[i] = di;
    e2[i] = i > 0 ? eg[i - 1] * eg[i - 1] : 0.0;
    glo = fmin(glo, di - el - er);
    ghi = fmax(ghi, di + el + er);
    emax = fmax(emax, e2[i]);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    glo = fmin(glo, __shfl_xor(glo, o, 64));
    ghi = fmax(ghi, __shfl_xor(ghi, o, 64));
    emax = fmax(emax, __shfl_xor(emax, o, 64));
  }
  if (lane == 0) {
    red[wave][0] = glo;
    red[wave][1] = ghi;
    cnt[wave] = 0;
  }
  __syncthreads();
  double lo = fmin(fmin(red[0][0], red[1][0]), fmin(red[2][0], red[3][0]));
  double hi = fmax(fmax(red[0][1], red[1][1]), fmax(red[2][1], red[3][1]));
  const double span = fmax(fabs(lo), fabs(hi));
  lo -= 2.2e-16 * span * c + 1e-300;
  hi += 2.2e-16 * span * c + 1e-300;
  const double pivmin = fmax(1e-300, 2.2e-308 * fmax(1.0, emax));
  for (int round = 0; round < 8; ++round) {
    const double x = lo + (hi - lo) * (double)(tid + 1) / (double)(RR_BIS_THREADS + 1);
    int neg = 0;
    double q = d[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    neg += q < 0.0;
    for (int i = 1; i < c; ++i) {
      q = (d[i] - x) - e2[i] * inv_nr(q);  // Newton reciprocal: shorter serial chain
      if (fabs(q) < pivmin) q = -pivmin;
      neg += q < 0.0;
    }
    __syncthreads();
    cnt[tid] = neg;  // nu(x_t) = #eigenvalues < x_t, nondecreasing in t
    __syncthreads();
    // lambda_a lies in (x_{t-1}, x_t] for the first t with nu(x_t) > a
    int first = RR_BIS_THREADS;
    for (int t = tid; t < RR_BIS_THREADS; t += RR_BIS_THREADS)
      if (cnt[t] > a && (t == 0 || cnt[t - 1] <= a)) first = t;
    for (int o = 32; o >= 1; o >>= 1) first = min(first, __shfl_xor(first, o, 64));
    __syncthreads();
    if (lane == 0) cnt[wave] = first;
    __syncthreads();
    first = min(min(cnt[0], cnt[1]), min(cnt[2], cnt[3]));
    const double step = (hi - lo) / (double)(RR_BIS_THREADS + 1);
    const double nlo = lo + step * first;
    const double nhi = (first < RR_BIS_THREADS) ? lo + step * (first + 1) : hi;
    lo = nlo;
    hi = nhi;
    if (hi - lo <= 2.2e-16 * fmax(fabs(lo), fabs(hi))) break;
  }
  if (tid == 0) w[j] = 0.5 * (lo + hi);
}

// rr_inviter_kernel: eigenvectors of T for the p wanted eigenvalues (descending).  One
// 64-thread workgroup per cluster start (gap to the previous eigenvalue > clus = 1e-9 ||T||;
// fp64 inverse iteration leaves vectors of eigenvalues delta apart orthogonal to
// ~eps ||T|| / delta, so only gaps below that need Gram-Schmidt); the cluster's members are
// computed in order.  Lane 0 runs the O(c) tridiagonal LU (partial pivoting) and the two
// inverse-iteration solves with the factors and the iterate in LDS; the whole wave does the
// Gram-Schmidt against the earlier members (classical, twice per member: one per iteration).
// Y: column-major c x p.
__global__ __launch_bounds__(64) void rr_inviter_kernel(const double* __restrict__ d,
                                                        const double* __restrict__ e, int c,
                                                        int p, const double* __restrict__ w,
                                                        double clus_rel, double* __restrict__ Y) {
  __shared__ double dgv[RR_MAXC], u1[RR_MAXC], u2[RR_MAXC], lm[RR_MAXC], x[RR_MAXC];
  __shared__ double rdg[RR_MAXC], ds[RR_MAXC], es[RR_MAXC];
  __shared__ unsigned char sw[RR_MAXC];
  __shared__ double proj[64];
  __shared__ double nrm_s;
  const int j0 = blockIdx.x;
  const int lane = threadIdx.x;
  stage_to_lds<64, 16>(ds, d, c, lane);
  stage_to_lds<64, 16>(es, e, c - 1, lane);
  if (lane == 0) es[c - 1] = 0.0;
  __syncthreads();
  double tn = 0.0;
  for (int i = lane; i < c; i += 64) {
    const double r = (i > 0 ? fabs(es[i - 1]) : 0.0) + fabs(es[i]);
    tn = fmax(tn, fabs(ds[i]) + r);
  }
  for (int o = 32; o >= 1; o >>= 1) tn = fmax(tn, __shfl_xor(tn, o, 64));
  const double clus = clus_rel * fmax(tn, 1e-300);
  if (j0 > 0 && fabs(w[j0 - 1] - w[j0]) <= clus) return;  // not a cluster start (uniform)
  const double tiny = fmax(2.220446049250313e-16 * tn, 1e-300);
  if (j0 + 1 >= p || fabs(w[j0] - w[j0 + 1]) > clus) {
    // isolated eigenvalue: the twisted factorisation T - lam I = N_r Delta_r N_r^T (top-down
    // LDL^T in lane 0 and bottom-up UDU^T in lane 1, in parallel), twist r = argmin |gamma_r|,
    // z_r = 1 and two outward product recurrences: two serial chains of c steps instead of the
    // pivoted LU and two inverse-iteration solves.  A non-finite z falls back to those below.
    const double lam = w[j0];
    if (lane == 0) {
      double D = ds[0] - lam;
      for (int i = 0; i < c - 1; ++i) {
        if (fabs(D) < tiny) D = (D < 0 ? -tiny : tiny);
        dgv[i] = D;
        const double L = es[i] * inv_nr(D);
        lm[i] = L;
        D = fma(-L, es[i], ds[i + 1] - lam);
      }
      if (fabs(D) < tiny) D = (D < 0 ? -tiny : tiny);
      dgv[c - 1] = D;
    } else if (lane == 1) {
      double Dt = ds[c - 1] - lam;
      for (int i = c - 2; i >= 0; --i) {
        if (fabs(Dt) < tiny) Dt = (Dt < 0 ? -tiny : tiny);
        u2[i + 1] = Dt;
        const double U = es[i] * inv_nr(Dt);
        u1[i] = U;
        Dt = fma(-U, es[i], ds[i] - lam);
      }
      if (fabs(Dt) < tiny) Dt = (Dt < 0 ? -tiny : tiny);
      u2[0] = Dt;
    }
    __syncthreads();
    double best = 1e308;
    int br = 0;
    for (int i = lane; i < c; i += 64) {
      const double g = fabs(dgv[i] + u2[i] - (ds[i] - lam));
      if (g < best) {
        best = g;
        br = i;
      }
    }
    for (int o = 32; o >= 1; o >>= 1) {  // argmin, ties to the lower index
      const double ob = __shfl_xor(best, o, 64);
      const int orr = __shfl_xor(br, o, 64);
      if (ob < best || (ob == best && orr < br)) {
        best = ob;
        br = orr;
      }
    }
    if (lane == 0) {
      double z = 1.0;
      x[br] = 1.0;
      for (int i = br - 1; i >= 0; --i) {
        z = -lm[i] * z;
        x[i] = z;
      }
    } else if (lane == 1) {
      double z = 1.0;
      for (int i = br; i < c - 1; ++i) {
        z = -u1[i] * z;
        x[i + 1] = z;
      }
    }
    __syncthreads();
    double s2 = 0.0;
    for (int i = lane; i < c; i += 64) s2 += x[i] * x[i];
    for (int o = 32; o >= 1; o >>= 1) s2 += __shfl_xor(s2, o, 64);
    if (isfinite(s2) && s2 > 0.0) {  // uniform
      const double inv = 1.0 / sqrt(s2);
      double* yj = Y + (int64_t)j0 * c;
      for (int i = lane; i < c; i += 64) yj[i] = x[i] * inv;
      return;
    }
    __syncthreads();
  }
  for (int j = j0; j < p && (j == j0 || fabs(w[j - 1] - w[j]) <= clus); ++j) {
    const double lam = w[j];
    for (int i = lane; i < c; i += 64) {
      const uint64_t hsh = splitmix64(0x9E3779B97F4A7C15ull ^ ((uint64_t)j << 32) ^ (uint64_t)i);
      x[i] = (double)(hsh >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    }
    if (lane == 0) {  // LU of T - lam I with partial pivoting (one extra superdiagonal)
      // branch-free steps; the pivot reciprocal (v_rcp_f64 + Newton) replaces the division on
      // the serial chain; d / e come from LDS 8 steps ahead of the chain
      double a = ds[0] - lam;
      double cc = (c > 1) ? es[0] : 0.0;
      for (int i0 = 0; i0 < c - 1; i0 += 8) {
        double dn[8], en[8], en1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u;
          dn[u] = ds[i + 1 < c ? i + 1 : c - 1];
          en[u] = es[i < c - 1 ? i : 0];
          en1[u] = (i + 1 < c - 1) ? es[i + 1] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u;
          if (i >= c - 1) break;
          const double sub = en[u], nd = dn[u] - lam, ns = en1[u];
          const bool swp = fabs(a) < fabs(sub);
          double ag = a;
          if (fabs(ag) < tiny) ag = (ag < 0 ? -tiny : tiny);
          const double piv = swp ? sub : ag;
          const double m = (swp ? a : sub) * inv_nr(piv);
          lm[i] = m;
          sw[i] = swp ? 1 : 0;
          dgv[i] = piv;
          u1[i] = swp ? nd : cc;
          u2[i] = swp ? ns : 0.0;
          const double an = swp ? fma(-m, nd, cc) : fma(-m, cc, nd);
          cc = swp ? -m * ns : ns;
          a = an;
        }
      }
      if (fabs(a) < tiny) a = (a < 0 ? -tiny : tiny);
      dgv[c - 1] = a;
    }
    __syncthreads();
    for (int i = lane; i < c; i += 64) rdg[i] = 1.0 / dgv[i];
    __syncthreads();
    // two inverse iterations: the shift is the bisection eigenvalue (fp64-accurate), so the
    // first solve already amplifies the wanted direction by ~1/eps; the second cleans up
    for (int it = 0; it < 2; ++it) {
      if (lane == 0) {
        // forward substitution with the interchanges (x[i+1..] read 8 ahead of the chain)
        double cur = x[0];
        for (int i0 = 0; i0 < c - 1; i0 += 8) {
          double xn[8], ln[8];
          int sn[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int i = i0 + u < c - 1 ? i0 + u : c - 2;
            xn[u] = x[i + 1];
            ln[u] = lm[i];
            sn[u] = sw[i];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int i = i0 + u;
            if (i >= c - 1) break;
            const double nxt = sn[u] ? cur : xn[u];
            const double cv = sn[u] ? xn[u] : cur;
            x[i] = cv;
            cur = fma(-ln[u], cv, nxt);
          }
        }
        x[c - 1] = cur;
        // back substitution with the pivot reciprocals, x[i+1], x[i+2] in registers
        double x1 = cur * rdg[c - 1];
        x[c - 1] = x1;
        double x2 = 0.0;
        if (c > 1) {
          const double v = (x[c - 2] - u1[c - 2] * x1) * rdg[c - 2];
          x[c - 2] = v;
          x2 = x1;
          x1 = v;
        }
        for (int i0 = c - 3; i0 >= 0; i0 -= 8) {
          double xv[8], a1[8], a2[8], rv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int i = i0 - u >= 0 ? i0 - u : 0;
            xv[u] = x[i];
            a1[u] = u1[i];
            a2[u] = u2[i];
            rv[u] = rdg[i];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int i = i0 - u;
            if (i < 0) break;
            const double v = fma(-a2[u], x2, fma(-a1[u], x1, xv[u])) * rv[u];
            x[i] = v;
            x2 = x1;
            x1 = v;
          }
        }
      }
      __syncthreads();
      // classical Gram-Schmidt against the earlier members of the cluster, 64 at a time
      for (int q0 = j0; q0 < j; q0 += 64) {
        const int q = q0 + lane;
        double sdot = 0.0;
        if (q < j) {
          const double* y = Y + (int64_t)q * c;
          for (int i = 0; i < c; ++i) sdot += y[i] * x[i];
        }
        proj[lane] = sdot;
        __syncthreads();
        const int nq = min(64, j - q0);
        for (int i = lane; i < c; i += 64) {
          double acc = 0.0;
          for (int t = 0; t < nq; ++t) acc += proj[t] * Y[(int64_t)(q0 + t) * c + i];
          x[i] -= acc;
        }
        __syncthreads();
      }
      double s2 = 0.0;
      for (int i = lane; i < c; i += 64) s2 += x[i] * x[i];
      for (int o = 32; o >= 1; o >>= 1) s2 += __shfl_xor(s2, o, 64);
      if (lane == 0) nrm_s = sqrt(s2);
      __syncthreads();
      double nr = nrm_s;
      if (!(nr > 0.0)) {
        for (int i = lane; i < c; i += 64) x[i] = (i == j % c) ? 1.0 : 0.0;
        nr = 1.0;
      }
      const double inv = 1.0 / nr;
      for (int i = lane; i < c; i += 64) x[i] *= inv;
      __syncthreads();
    }
    double* yj = Y + (int64_t)j * c;
    for (int i = lane; i < c; i += 64) yj[i] = x[i];
    __syncthreads();
    __threadfence_block();
  }
}

extern "C" hipError_t n2v2r_launch_rr_tri_eig(const double* d, const double* e, int c, int p,
                                              double* w, double* Y, double* scratch,
                                              hipStream_t stream) {
  (void)scratch;
  if (c < 3 || c > RR_MAXC || p < 1 || p > c) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rr_bisect_kernel, dim3((unsigned)p), dim3(RR_BIS_THREADS), 0, stream, d, e,
                     c, p, w);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(rr_inviter_kernel, dim3((unsigned)p), dim3(64), 0, stream, d, e, c, p, w,
                     1e-9, Y);
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_rr_bisect(const double* d, const double* e, int c, int p,
                                             double* w, hipStream_t stream) {
  if (c < 3 || c > RR_MAXC || p < 1 || p > c) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rr_bisect_kernel, dim3((unsigned)p), dim3(RR_BIS_THREADS), 0, stream, d, e,
                     c, p, w);
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_rr_tri_inviter(const double* d, const double* e, int c, int p,
                                                  const double* w, double* Y,
                                                  hipStream_t stream) {
  if (c < 3 || c > RR_MAXC || p < 1 || p > c) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rr_inviter_kernel, dim3((unsigned)p), dim3(64), 0, stream, d, e, c, p, w,
                     1e-9, Y);
  return hipGetLastError();
}

// scratch (device, >= n2v2r_rr_tridiag_scratch_bytes(c)): the multi-workgroup form
// (rr_tridiag_coop_kernel); NULL: the one-workgroup kernel (handles whose ranks share one device
// pass NULL: their concurrent launches could not all be resident).  N2V2R_RR_TRI=1
// forces the one-workgroup kernel.
static hipError_t launch_rr_tridiag_coop(double* A, int c, double* d, double* e, double* tau,
                                         double* V, void* scratch, hipStream_t stream) {
  const int nt = (c + TRC_TS - 1) / TRC_TS;
  // <= 12 row tiles per workgroup: <= 99 KB of tiles in LDS (4 row residues were measured no
  // faster; the N2V2R_RR_TRI_PR switch was retired in round 6)
  const int PR = nt > 12 ? 2 : 1;
  const int ntr = (nt + PR - 1) / PR;
  const size_t shmem = sizeof(double) * ((size_t)ntr * TRC_TS * TRC_LD + 5 * (size_t)c + 8 * TRC_TS);
  if (shmem > 150 * 1024) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)rr_tridiag_coop_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    (void)hipGetLastError();
    attr_set = true;
  }
  double* part = static_cast<double*>(scratch);
  double* rowbuf = part + (size_t)2 * 4 * c;
  unsigned* ctr = reinterpret_cast<unsigned*>(rowbuf + (size_t)2 * c);
  int* err = reinterpret_cast<int*>(ctr + 1);  // 1 after a timed-out grid barrier
  hipError_t er = hipMemsetAsync(ctr, 0, sizeof(unsigned) * TRC_CTR_WORDS, stream);
  if (er != hipSuccess) return er;
  // The grid barrier needs all PR x nt (<= 4 x 24) workgroups resident at once.  The grid is
  // launched only when the occupancy the runtime reports for this kernel at this LDS size times
  // the device's CUs covers it (otherwise the caller takes the one-workgroup kernel).  Should a
  // workgroup still be held back -- another kernel of this process or another one occupying CUs
  // -- the bounded spin ends the launch with *err set and d[0] = NaN; the engine reads *err with
  // the cycle's read-back (n2v2r_rr_tridiag_err) and redoes the step with the one-workgroup
  // kernel.  (Round 5 launched it with hipLaunchCooperativeKernel.  Every process that made a
  // cooperative launch then died with SIGSEGV at exit under rocprofv3's kernel trace; round 6's
  // tools/coop_exit_repro.hip does the same with one trivial cooperative kernel and no n2v2r
  // code -- a plain launch of the same kernel exits cleanly -- so the fault is the runtime's /
  // profiler's teardown of the cooperative launch, which this plain launch avoids,
  // profiles/r06_coop_exit.md.)
  const unsigned grid = (unsigned)(PR * nt);
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)rr_tridiag_coop_kernel,
                                                   TRC_NT, shmem) != hipSuccess ||
      (int64_t)per_cu * ncu < (int64_t)grid) {
    (void)hipGetLastError();
    return hipErrorInvalidValue;  // the caller falls back to the one-workgroup kernel
  }
  hipLaunchKernelGGL(rr_tridiag_coop_kernel, dim3(grid), dim3(TRC_NT), shmem, stream, A, c, PR, d,
                     e, tau, V, part, rowbuf, ctr, err);
  return hipGetLastError();
}

// the multi-workgroup tridiagonalisation's error word in its scratch: 1 after a launch whose grid
// barrier timed out (its output is then invalid), re-armed by every launch
extern "C" int* n2v2r_rr_tridiag_err(void* scratch, int c) {
  double* part = static_cast<double*>(scratch);
  unsigned* ctr = reinterpret_cast<unsigned*>(part + (size_t)2 * 4 * c + (size_t)2 * c);
  return reinterpret_cast<int*>(ctr + 1);
}

extern "C" hipError_t n2v2r_launch_rr_tridiag(double* A, int c, double* d, double* e, double* tau,
                                              double* V, void* scratch, hipStream_t stream) {
  if (c < 3 || c > RR_MAXC) return hipErrorInvalidValue;
  const char* ev = std::getenv("N2V2R_RR_TRI");  // read per call (tests switch it)
  const bool force_one = ev && std::atoi(ev) == 1;
  if (scratch && !force_one) {
    const hipError_t er = launch_rr_tridiag_coop(A, c, d, e, tau, V, scratch, stream);
    if (er != hipErrorInvalidValue) return er;
  }
  // 1024 threads up to c = 512; 512 threads (twice the registers per lane) beyond.  Even c
  // (every UASE basis: c = blocks x b): 16-B column-pair accesses.
  static bool attr_set = false;
  const int cap = 160 * 1024 - 1024;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)rr_tridiag_kernel<4, 1024, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, cap);
    (void)hipFuncSetAttribute((const void*)rr_tridiag_kernel<8, 1024, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, cap);
    (void)hipFuncSetAttribute((const void*)rr_tridiag_kernel<12, 512, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, cap);
    (void)hipFuncSetAttribute((const void*)rr_tridiag_kernel<4, 1024, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, cap);
    (void)hipFuncSetAttribute((const void*)rr_tridiag_kernel<8, 1024, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, cap);
    (void)hipFuncSetAttribute((const void*)rr_tridiag_kernel<12, 512, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, cap);
    (void)hipGetLastError();  // a refused attribute must not surface at a later launch
    attr_set = true;
  }
  const dim3 g(1);
  const bool even = (c % 2) == 0;
  const size_t l1024 = sizeof(double) * c * 20, l512 = sizeof(double) * c * 12;
#define RR_TRI_LAUNCH(TM, NT_, PR, L)                                                           \
  hipLaunchKernelGGL((rr_tridiag_kernel<TM, NT_, PR>), g, dim3(NT_), L, stream, A, c, d, e, tau, V)
  if (c <= 256) {
    if (even) RR_TRI_LAUNCH(4, 1024, true, l1024); else RR_TRI_LAUNCH(4, 1024, false, l1024);
  } else if (c <= 512) {
    if (even) RR_TRI_LAUNCH(8, 1024, true, l1024); else RR_TRI_LAUNCH(8, 1024, false, l1024);
  } else {
    if (even) RR_TRI_LAUNCH(12, 512, true, l512); else RR_TRI_LAUNCH(12, 512, false, l512);
  }
#undef RR_TRI_LAUNCH
  return hipGetLastError();
}

extern "C" size_t n2v2r_rr_bt_scratch_bytes(int c) {
  return sizeof(double) * (size_t)((c - 2 + BT_NB - 1) / BT_NB) * BT_NB * BT_NB;
}

// tfac: n2v2r_rr_bt_scratch_bytes(c) of device scratch (the blocks' T factors)
extern "C" hipError_t n2v2r_launch_rr_backtransform(const double* V, const double* tau, int c,
                                                    const double* Y, int p, float* S, int lds,
                                                    double* tfac, hipStream_t stream) {
  if (c < 3 || c > RR_MAXC || p < 1 || p > c || !tfac) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rr_bt_tfactor_kernel, dim3((unsigned)((c - 2 + BT_NB - 1) / BT_NB)),
                     dim3(256), 0, stream, V, tau, c, tfac);
  hipLaunchKernelGGL(rr_backtransform_kernel, dim3((unsigned)((p + RR_BT_COLS - 1) / RR_BT_COLS)),
                     dim3(256), 0, stream, V, tfac, c, Y, p, S, lds);
  return hipGetLastError();
}

// Ranking tail of the fit-and-rank path (gfx950, wave64):
//   distances : per-node cross-layer cosine / euclidean / correlation distances for every
//               (dim, metric) column in ONE pass over the (K, N, d) embedding
//               (model.py:57-96, model_utils.py:39-67).
//   borda     : per column a stable LSD radix sort of 64-bit order-preserving keys
//               (descending value, NaN last, ties by ascending node index), the inverse
//               permutation, and the int64 Borda sum over columns
//               (model.py:167-185, model_utils.py:22-36).
#include "common.h"

// ----------------------------------------------------------------------------- distances
#define DIST_MAX_COLS 256

struct DistPlan {
  int n_cols;
  int col_dim[DIST_MAX_COLS];     // in emission order (sorted by dim)
  int col_metric[DIST_MAX_COLS];
  int col_out[DIST_MAX_COLS];     // output column index
  int dmax;
};

__device__ __forceinline__ double clip02_keep_nan(double x) {
  if (x != x) return x;
  return x < 0.0 ? 0.0 : (x > 2.0 ? 2.0 : x);
}

// Y: [K][N][ldy] fp32.  Comparison layer i; strategy picks embed_one.  Out: [C][N] fp64.
__global__ __launch_bounds__(256) void distances_kernel(const float* __restrict__ Y, int K,
                                                        int64_t n, int64_t ldy, int64_t lrows,
                                                        int strategy, int layer_i, DistPlan plan,
                                                        double* __restrict__ out, int64_t ldo) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int64_t lstride = lrows * ldy;  // rows per layer block of Y (>= n when padded)
  const float* y2 = Y + (int64_t)layer_i * lstride + r * ldy;
  double suv = 0, suu = 0, svv = 0, sdd = 0, su = 0, sv = 0;
  int next = 0;
  // number of layers averaged into embed_one
  int k_lo = 0, k_hi = 0;  // [k_lo, k_hi) minus layer_i when one_vs_rest
  if (strategy == 0) { k_lo = layer_i - 1; k_hi = layer_i; }
  else if (strategy == 1) { k_lo = 0; k_hi = layer_i; }
  else { k_lo = 0; k_hi = K; }
  const double cnt = (strategy == 2) ? (double)(K - 1) : (double)(k_hi - k_lo);
  for (int j = 0; j < plan.dmax; ++j) {
    double u;
    if (strategy == 0) {
      u = (double)Y[(int64_t)k_lo * lstride + r * ldy + j];
    } else {
      double acc = 0.0;
      for (int k = k_lo; k < k_hi; ++k) {
        if (strategy == 2 && k == layer_i) continue;
        acc += (double)Y[(int64_t)k * lstride + r * ldy + j];
      }
      u = acc / cnt;
    }
    const double v = (double)y2[j];
    suv += u * v;
    suu += u * u;
    svv += v * v;
    const double df = u - v;
    sdd += df * df;
    su += u;
    sv += v;
    while (next < plan.n_cols && plan.col_dim[next] == j + 1) {
      const int m = plan.col_metric[next];
      double res;
      if (m == 1) {
        res = sqrt(sdd);
      } else if (m == 0) {
        res = clip02_keep_nan(1.0 - suv / sqrt(suu * svv));
      } else {
        // correlation: centre on the prefix means, then a second pass over the prefix
        // (scipy centres explicitly; the one-pass sum formula cancels)
        const int D = j + 1;
        const double mu = su / D, mv = sv / D;
        double cuv = 0, cuu = 0, cvv = 0;
        for (int q = 0; q < D; ++q) {
          double uq;
          if (strategy == 0) {
            uq = (double)Y[(int64_t)k_lo * lstride + r * ldy + q];
          } else {
            double acc = 0.0;
            for (int k = k_lo; k < k_hi; ++k) {
              if (strategy == 2 && k == layer_i) continue;
              acc += (double)Y[(int64_t)k * lstride + r * ldy + q];
            }
            uq = acc / cnt;
          }
          const double x = uq - mu, y = (double)y2[q] - mv;
          cuv += x * y;
          cuu += x * x;
          cvv += y * y;
        }
        res = clip02_keep_nan(1.0 - cuv / sqrt(cuu * cvv));
      }
      out[(int64_t)plan.col_out[next] * ldo + r] = res;
      ++next;
    }
  }
}

// The sequential strategy without correlation columns (the bench's and the reference's default):
// the same sums in the same order as distances_kernel, with each thread's two embedding rows read
// 16 dims at a time as float4 loads issued together (the scalar per-dim loads of the general form
// touch a new line per lane per load: cfg2 132 us).  Needs ldy % 4 == 0 and ldy >= dmax rounded
// up to 16 (rows padded to 64: checked by the launcher).
__global__ __launch_bounds__(256) void distances_seq_kernel(const float* __restrict__ Y,
                                                            int64_t n, int64_t ldy, int64_t lrows,
                                                            int layer_i, DistPlan plan,
                                                            double* __restrict__ out, int64_t ldo) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int64_t lstride = lrows * ldy;
  const float* y1 = Y + (int64_t)(layer_i - 1) * lstride + r * ldy;
  const float* y2 = Y + (int64_t)layer_i * lstride + r * ldy;
  double suv = 0, suu = 0, svv = 0, sdd = 0;
  int next = 0;
  for (int j0 = 0; j0 < plan.dmax; j0 += 16) {
    f32x4 a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[q] = *reinterpret_cast<const f32x4*>(y1 + j0 + 4 * q);
      b[q] = *reinterpret_cast<const f32x4*>(y2 + j0 + 4 * q);
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int j = j0 + t;
      if (j >= plan.dmax) break;
      const double u = (double)a[t >> 2][t & 3], v = (double)b[t >> 2][t & 3];
      suv += u * v;
      suu += u * u;
      svv += v * v;
      const double df = u - v;
      sdd += df * df;
      while (next < plan.n_cols && plan.col_dim[next] == j + 1) {
        const double res = plan.col_metric[next] == 1 ? sqrt(sdd)
                                                      : clip02_keep_nan(1.0 - suv / sqrt(suu * svv));
        out[(int64_t)plan.col_out[next] * ldo + r] = res;
        ++next;
      }
    }
  }
}

// Y: [K][lrows][ldy]; the first n rows are computed; column c of the output at out + c * ldo
extern "C" hipError_t n2v2r_launch_distances(const float* Y, int K, int64_t n, int64_t ldy,
                                             int64_t lrows, int strategy, int layer_i,
                                             const DistPlan& plan, double* out, int64_t ldo,
                                             hipStream_t stream) {
  bool corr = false;
  for (int c = 0; c < plan.n_cols; ++c) corr |= plan.col_metric[c] == 2;
  if (strategy == 0 && !corr && layer_i >= 1 && ldy % 4 == 0 &&
      ldy >= ((plan.dmax + 15) / 16) * 16 && (reinterpret_cast<uintptr_t>(Y) & 15) == 0)
    hipLaunchKernelGGL(distances_seq_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       stream, Y, n, ldy, lrows, layer_i, plan, out, ldo);
  else
    hipLaunchKernelGGL(distances_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                       Y, K, n, ldy, lrows, strategy, layer_i, plan, out, ldo);
  return hipGetLastError();
}

// Host-array seam: two N x dim fp64 matrices -> N distances (model_utils.py:39).
__global__ void pairwise_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                int64_t n, int dim, int metric, double* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const double* u = a + r * dim;
  const double* v = b + r * dim;
  if (metric == 1) {
    double s = 0;
    for (int j = 0; j < dim; ++j) { const double d = u[j] - v[j]; s += d * d; }
    out[r] = sqrt(s);
    return;
  }
  double mu = 0, mv = 0;
  if (metric == 2) {
    for (int j = 0; j < dim; ++j) { mu += u[j]; mv += v[j]; }
    mu /= dim;
    mv /= dim;
  }
  double suv = 0, suu = 0, svv = 0;
  for (int j = 0; j < dim; ++j) {
    const double x = u[j] - mu, y = v[j] - mv;
    suv += x * y;
    suu += x * x;
    svv += y * y;
  }
  out[r] = clip02_keep_nan(1.0 - suv / sqrt(suu * svv));
}

extern "C" hipError_t n2v2r_launch_pairwise(const double* a, const double* b, int64_t n, int dim,
                                            int metric, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(pairwise_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a,
                     b, n, dim, metric, out);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- Borda
// Segment s (one ranking column) = N fp64 values at vals + s * n.
#define RS_THREADS 256
#define RS_ITEMS 16
#define RS_TILE (RS_THREADS * RS_ITEMS)

__device__ __forceinline__ uint64_t desc_key(double x) {
  if (x != x) return ~0ull;                 // NaN last (pandas nargsort, na_position='last')
  if (x == 0.0) x = 0.0;                    // -0 == +0
  uint64_t b = (uint64_t)__double_as_longlong(x);
  const uint64_t ordered = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
  return ~ordered;                          // ascending key == descending value
}

// keys/payload init + per-segment OR / AND of the keys (to skip constant digits).
__global__ __launch_bounds__(256) void borda_init_kernel(const double* __restrict__ vals, int64_t n, int nseg,
                                  uint64_t* __restrict__ keys, int32_t* __restrict__ idx,
                                  unsigned long long* __restrict__ seg_or,
                                  unsigned long long* __restrict__ seg_and) {
  const int s = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t k = 0, kor = 0, kand = ~0ull;
  if (i < n) {
    k = desc_key(vals[(int64_t)s * n + i]);
    keys[(int64_t)s * n + i] = k;
    idx[(int64_t)s * n + i] = (int32_t)i;
    kor = k;
    kand = k;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    kor |= (uint64_t)__shfl_xor((long long)kor, m, 64);
    kand &= (uint64_t)__shfl_xor((long long)kand, m, 64);
  }
  // one atomic pair per workgroup, not per wave: 4x fewer on the segment's two words (every
  // wave's atomics on one address serialise; per-wave they made the launch ~40 us at cfg2)
  __shared__ unsigned long long wor[4], wand[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    wor[w] = kor;
    wand[w] = kand;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (int)(blockDim.x >> 6);
    for (int q = 1; q < nw; ++q) {
      kor |= wor[q];
      kand &= wand[q];
    }
    atomicOr(&seg_or[s], (unsigned long long)kor);
    atomicAnd(&seg_and[s], (unsigned long long)kand);
  }
}

__global__ __launch_bounds__(RS_THREADS) void radix_hist_kernel(const uint64_t* __restrict__ keys,
                                                                int64_t n, int shift, int ntiles,
                                                                uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const int s = blockIdx.y;
  const int t = blockIdx.x;
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t* kp = keys + (int64_t)s * n;
  const int64_t base = (int64_t)t * RS_TILE;
#pragma unroll
  for (int it = 0; it < RS_ITEMS; ++it) {
    const int64_t i = base + it * RS_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&h[(kp[i] >> shift) & 0xFF], 1u);
  }
  __syncthreads();
  // digit-major layout: hist[s][digit][tile]
  hist[((int64_t)s * 256 + threadIdx.x) * ntiles + t] = h[threadIdx.x];
}

// exclusive scan of hist[s][*][*] (256 * ntiles entries) in place, per segment, over the
// whole chip: chunk sums (RSC_TILE entries per workgroup, coalesced), a scan of the chunk sums
// per segment, then every chunk rescanned from its offset.  (Round 2 scanned a segment in one
// workgroup, each thread a contiguous run: 2.3 ms for the 3.1M-entry histogram of a 50M-entry
// ingest sort.)
#define RSC_T 256
#define RSC_IT 8
#define RSC_TILE (RSC_T * RSC_IT)

__global__ __launch_bounds__(RSC_T) void rs_chunk_sums_kernel(const uint32_t* __restrict__ hist,
                                                              int64_t len, int nchunk,
                                                              uint32_t* __restrict__ csum) {
  const int s = blockIdx.y;
  const uint32_t* hp = hist + (int64_t)s * len;
  const int64_t base = (int64_t)blockIdx.x * RSC_TILE;
  uint32_t v = 0;
#pragma unroll
  for (int u = 0; u < RSC_IT; ++u) {
    const int64_t i = base + u * RSC_T + threadIdx.x;
    v += i < len ? hp[i] : 0u;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  __shared__ uint32_t ws[RSC_T / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < RSC_T / 64; ++w) t += ws[w];
    csum[(int64_t)s * nchunk + blockIdx.x] = t;
  }
}

// exclusive scan of one segment's chunk sums in place: 1024-entry passes with a carry
__global__ __launch_bounds__(1024) void rs_chunk_offsets_kernel(uint32_t* __restrict__ csum,
                                                                int nchunk) {
  __shared__ uint32_t sh[1024];
  uint32_t* cp = csum + (int64_t)blockIdx.x * nchunk;
  uint32_t carry = 0;
  for (int c0 = 0; c0 < nchunk; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    const uint32_t v = i < nchunk ? cp[i] : 0u;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const uint32_t t = threadIdx.x >= off ? sh[threadIdx.x - off] : 0u;
      __syncthreads();
      sh[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < nchunk) cp[i] = carry + sh[threadIdx.x] - v;
    const uint32_t tot = sh[1023];
    __syncthreads();
    carry += tot;
  }
}

// one chunk rescanned in place from its offset: RSC_IT consecutive entries per thread, a
// workgroup scan of the thread sums
__global__ __launch_bounds__(RSC_T) void rs_chunk_write_kernel(uint32_t* __restrict__ hist,
                                                               int64_t len, int nchunk,
                                                               const uint32_t* __restrict__ csum) {
  const int s = blockIdx.y;
  uint32_t* hp = hist + (int64_t)s * len;
  const int64_t base = (int64_t)blockIdx.x * RSC_TILE + (int64_t)threadIdx.x * RSC_IT;
  uint32_t v[RSC_IT];
  uint32_t t = 0;
#pragma unroll
  for (int u = 0; u < RSC_IT; ++u) {
    v[u] = base + u < len ? hp[base + u] : 0u;
    t += v[u];
  }
  __shared__ uint32_t sh[RSC_T];
  sh[threadIdx.x] = t;
  __syncthreads();
  for (int off = 1; off < RSC_T; off <<= 1) {
    const uint32_t q = threadIdx.x >= off ? sh[threadIdx.x - off] : 0u;
    __syncthreads();
    sh[threadIdx.x] += q;
    __syncthreads();
  }
  uint32_t run = csum[(int64_t)s * nchunk + blockIdx.x] + sh[threadIdx.x] - t;
#pragma unroll
  for (int u = 0; u < RSC_IT; ++u) {
    if (base + u < len) hp[base + u] = run;
    run += v[u];
  }
}

__global__ __launch_bounds__(RS_THREADS) void radix_scatter_kernel(
    const uint64_t* __restrict__ kin, const int32_t* __restrict__ pin, uint64_t* __restrict__ kout,
    int32_t* __restrict__ pout, int64_t n, int shift, int ntiles,
    const uint32_t* __restrict__ offs) {
  __shared__ uint32_t cnt[4][256];
  __shared__ uint32_t run[256];
  __shared__ uint32_t gbase[256];
  const int s = blockIdx.y;
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  run[threadIdx.x] = 0;
  gbase[threadIdx.x] = offs[((int64_t)s * 256 + threadIdx.x) * ntiles + t];
  const uint64_t* kp = kin + (int64_t)s * n;
  const int32_t* pp = pin + (int64_t)s * n;
  uint64_t* ko = kout + (int64_t)s * n;
  int32_t* po = pout + (int64_t)s * n;
  const int64_t base = (int64_t)t * RS_TILE;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int it = 0; it < RS_ITEMS; ++it) {
    cnt[wave][lane] = 0;
    cnt[wave][lane + 64] = 0;
    cnt[wave][lane + 128] = 0;
    cnt[wave][lane + 192] = 0;
    __syncthreads();
    const int64_t i = base + it * RS_THREADS + threadIdx.x;
    const bool active = i < n;
    uint64_t key = 0;
    int32_t pay = 0;
    uint32_t dig = 0;
    if (active) {
      key = kp[i];
      pay = pp[i];
      dig = (uint32_t)((key >> shift) & 0xFF);
    }
    uint64_t m = __ballot(active);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (dig >> b) & 1;
      const uint64_t bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    const uint32_t rank_in_wave = (uint32_t)__popcll(m & lt_mask);
    if (active && rank_in_wave == 0) cnt[wave][dig] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = 0;
    if (active) {
      pre = run[dig];
      for (int w = 0; w < wave; ++w) pre += cnt[w][dig];
    }
    __syncthreads();
    // advance running counters (one thread per digit)
    run[threadIdx.x] += cnt[0][threadIdx.x] + cnt[1][threadIdx.x] + cnt[2][threadIdx.x] +
                        cnt[3][threadIdx.x];
    if (active) {
      const uint32_t dst = gbase[dig] + pre + rank_in_wave;
      ko[dst] = key;
      po[dst] = pay;
    }
    __syncthreads();
  }
}

// pos[s][node] = sorted position
__global__ void inverse_perm_kernel(const int32_t* __restrict__ sorted_idx, int64_t n,
                                    int32_t* __restrict__ pos) {
  const int s = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) pos[(int64_t)s * n + sorted_idx[(int64_t)s * n + j]] = (int32_t)j;
}

// borda[g][node] = sum_{c < ncols} (n - pos[g * ncols + c][node])
__global__ void borda_sum_kernel(const int32_t* __restrict__ pos, int64_t n, int ncols,
                                 int64_t* __restrict__ borda) {
  const int g = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t s = 0;
  for (int c = 0; c < ncols; ++c) s += n - (int64_t)pos[((int64_t)g * ncols + c) * n + i];
  borda[(int64_t)g * n + i] = s;
}

extern "C" hipError_t n2v2r_launch_borda_init(const double* vals, int64_t n, int nseg, uint64_t* keys,
                                              int32_t* idx, unsigned long long* seg_or,
                                              unsigned long long* seg_and, hipStream_t stream) {
  (void)hipMemsetAsync(seg_or, 0, sizeof(unsigned long long) * nseg, stream);
  (void)hipMemsetAsync(seg_and, 0xFF, sizeof(unsigned long long) * nseg, stream);
  dim3 grid((unsigned)((n + 255) / 256), nseg);
  hipLaunchKernelGGL(borda_init_kernel, grid, dim3(256), 0, stream, vals, n, nseg, keys, idx,
                     seg_or, seg_and);
  return hipGetLastError();
}

extern "C" int n2v2r_radix_tiles(int64_t n) { return (int)((n + RS_TILE - 1) / RS_TILE); }

// uint32 elements of the `hist` buffer a radix pass needs: the [nseg][256][ntiles] histogram
// plus the chunk sums of its scan
extern "C" size_t n2v2r_radix_hist_elems(int64_t n, int nseg) {
  const int64_t len = (int64_t)256 * n2v2r_radix_tiles(n);
  const int64_t nchunk = (len + RSC_TILE - 1) / RSC_TILE;
  return (size_t)nseg * (size_t)(len + nchunk);
}

extern "C" hipError_t n2v2r_launch_radix_pass(const uint64_t* kin, const int32_t* pin,
                                              uint64_t* kout, int32_t* pout, int64_t n, int nseg,
                                              int shift, uint32_t* hist, hipStream_t stream) {
  const int ntiles = n2v2r_radix_tiles(n);
  dim3 grid(ntiles, nseg);
  hipLaunchKernelGGL(radix_hist_kernel, grid, dim3(RS_THREADS), 0, stream, kin, n, shift, ntiles,
                     hist);
  const int64_t len = (int64_t)256 * ntiles;
  const int nchunk = (int)((len + RSC_TILE - 1) / RSC_TILE);
  uint32_t* csum = hist + (int64_t)nseg * len;  // n2v2r_radix_hist_elems
  hipLaunchKernelGGL(rs_chunk_sums_kernel, dim3(nchunk, nseg), dim3(RSC_T), 0, stream, hist, len,
                     nchunk, csum);
  hipLaunchKernelGGL(rs_chunk_offsets_kernel, dim3(nseg), dim3(1024), 0, stream, csum, nchunk);
  hipLaunchKernelGGL(rs_chunk_write_kernel, dim3(nchunk, nseg), dim3(RSC_T), 0, stream, hist, len,
                     nchunk, csum);
  hipLaunchKernelGGL(radix_scatter_kernel, grid, dim3(RS_THREADS), 0, stream, kin, pin, kout, pout,
                     n, shift, ntiles, hist);
  return hipGetLastError();
}

// tied[s] = 1 when the sorted keys of segment s hold two equal non-NaN keys (exact ties,
// -0 == +0): the segment's descending order is then not unique, and the reference's order for
// it is numpy quicksort's (model.py:173-174).  Lane 0 of a wave that saw one stores 1 (a plain
// vector store: every writer stores the same value).
__global__ __launch_bounds__(256) void tie_flag_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                       int32_t* __restrict__ tied) {
  const int s = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool t = false;
  if (j + 1 < n) {
    const uint64_t a = keys[(int64_t)s * n + j];
    t = a == keys[(int64_t)s * n + j + 1] && a != ~0ull;
  }
  if (__ballot(t) != 0ull && (threadIdx.x & 63) == 0) tied[s] = 1;
}

extern "C" hipError_t n2v2r_launch_tie_flags(const uint64_t* sorted_keys, int64_t n, int nseg,
                                             int32_t* tied, hipStream_t stream) {
  (void)hipMemsetAsync(tied, 0, sizeof(int32_t) * nseg, stream);
  dim3 grid((unsigned)((n + 255) / 256), nseg);
  hipLaunchKernelGGL(tie_flag_kernel, grid, dim3(256), 0, stream, sorted_keys, n, tied);
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_borda_finish(const int32_t* sorted_idx, int64_t n, int nseg,
                                                int ncols, int32_t* pos, int64_t* borda,
                                                hipStream_t stream) {
  dim3 g1((unsigned)((n + 255) / 256), nseg);
  hipLaunchKernelGGL(inverse_perm_kernel, g1, dim3(256), 0, stream, sorted_idx, n, pos);
  dim3 g2((unsigned)((n + 255) / 256), nseg / ncols);
  hipLaunchKernelGGL(borda_sum_kernel, g2, dim3(256), 0, stream, pos, n, ncols, borda);
  return hipGetLastError();
}

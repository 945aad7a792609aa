// Shared device helpers for the n2v2r HIP kernels (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#define N2V2R_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// A b-wide row-major panel: row r starts at ptr + r * ld.
struct Panel {
  float* ptr;
  int64_t ld;
};

// One CSR matrix resident in HBM (fp32 values, int32 column indices, int64 row pointers).
struct CsrDev {
  const int64_t* indptr;
  const int32_t* indices;
  const float* data;
  int64_t n_rows;
  int64_t nnz;
  int unit;  // every stored value is 1.0f (unweighted graph): the SpMM skips the value stream
};

// Up to this many basis blocks are addressed through a by-value pointer table.
#define N2V2R_MAX_BLOCKS 112
// the largest b = 8 basis the fused PIP pass (its (c + 8) x 8 Gram and c x 8 coefficients in
// LDS: 77 KB at 768), the paired passes and the banded Rayleigh-Ritz take
#define N2V2R_BAND_MAXC 768

struct BlockList {
  const float* blk[N2V2R_MAX_BLOCKS];
  int count;   // number of blocks
  int width;   // columns per block (32 or 64)
};

struct OutBlockList {
  float* blk[N2V2R_MAX_BLOCKS];
  int count;
  int width;
};

__device__ __forceinline__ float wave_shfl_xor(float v, int mask) {
  return __shfl_xor(v, mask, N2V2R_WAVE);
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, N2V2R_WAVE);
  return v;
}

// splitmix64 -> counter-based normal deviates for the Krylov start block.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Copy `total` doubles global -> LDS with NT threads, U loads in flight per thread before the
// first LDS write (a plain strided copy loop waits out one memory round trip per NT entries).
template <int NT, int U>
__device__ __forceinline__ void stage_to_lds(double* __restrict__ dst,
                                             const double* __restrict__ src, int total, int tid) {
  for (int e0 = tid; e0 < total; e0 += NT * U) {
    double t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = src[min(e0 + NT * u, total - 1)];  // clamped: no branches
#pragma unroll
    for (int u = 0; u < U; ++u) dst[min(e0 + NT * u, total - 1)] = t[u];  // same value again
  }
}

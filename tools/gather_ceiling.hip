// Calibration of the b = 8 SpMM gather ceiling on MI355X.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/gather_ceiling tools/gather_ceiling.hip
//   tools/gather_ceiling [entries_millions=100] [reps=20] [panel_MB=all] [row_bytes=all]
//
// What spmm8_flat_kernel does per stored entry, without its row structure, LDS staging and
// per-row fold: a lane pair reads the entry's 4-B column word from a streamed index array and
// gathers the entry's 32-B panel row as two 16-B loads, 4 steps of 32 entries per wave issued as
// one batch (the flat kernel's in-flight depth), 1024-thread workgroups, 2 per CU.  Panel sizes
// from 1 MB (L2-resident) to 320 MB (cfg5's, beyond the Infinity Cache), uniformly random
// columns (an ER layer's columns).  Forms:
//   stream+gather : index words from HBM, then the gathers (the flat kernel's memory work)
//   gather only   : indices from a counter hash (no index stream): the pure gather rate
//   stream only   : the index words alone (no gathers)
//   nt-stream+gather : stream + gather with non-temporal index loads (kept out of L2's way?)
//   ..., indices 1 / 2 batches ahead : the nt stream software-pipelined against the gathers
// Also at 64-B rows (b = 16 panels: a lane quad per entry).  Prints one JSON line per (form, row
// bytes, panel size): G entries/s and the index-stream GB/s.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                         \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((x ^ (x >> 31)) >> 32);
}

__global__ void fill_idx(int32_t* idx, int64_t e, uint32_t rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < e) idx[i] = (int32_t)(((uint64_t)hash32((uint64_t)i * 7919u) * rows) >> 32);
}

__global__ void narrow_idx(const int32_t* idx, uint16_t* idx16, int64_t e) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < e) idx16[i] = (uint16_t)idx[i];
}

__global__ void fill_x(float* x, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = (float)(i & 1023) * 1e-3f;
}

// MODE 0: stream + gather, 1: gather only (hashed indices), 2: stream only, 3: stream with
// non-temporal index loads + gather, 4: 2-B index words (non-temporal) + gather (rows < 65536:
// a column block's offsets), 5: 2-B index words alone.  W: panel width in
// floats (8: 32-B rows, a lane pair per entry, 32 entries per wave step; 16: 64-B rows, a lane
// quad per entry, 16 entries per step)
template <int MODE, int W>
__global__ __launch_bounds__(1024, 8) void gather_kernel(const int32_t* __restrict__ idx,
                                                         const uint16_t* __restrict__ idx16,
                                                         int64_t e, const float* __restrict__ X,
                                                         uint32_t rows, float* __restrict__ out) {
  constexpr int G = W / 4;       // lanes per entry
  constexpr int EPS = 64 / G;    // entries per wave step
  const int lane = threadIdx.x & 63;
  const int pr = lane / G, sub = lane % G;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t per = (e / nw + 4 * EPS - 1) / (4 * EPS) * (4 * EPS);  // whole 4-step chunks
  const int64_t beg = w0 * per;
  const int64_t end = beg + per < e ? beg + per : e;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t off = beg; off < end; off += 4 * EPS) {
    int wd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = off + u * EPS + pr;
      const int64_t qc = q < end ? q : end - 1;
      if (MODE == 1)
        wd[u] = (int)(((uint64_t)hash32((uint64_t)qc * 7919u) * rows) >> 32);
      else if (MODE == 3)
        wd[u] = __builtin_nontemporal_load(idx + qc);
      else if (MODE == 4 || MODE == 5)
        wd[u] = __builtin_nontemporal_load(idx16 + qc);
      else
        wd[u] = idx[qc];
    }
    if (MODE == 2 || MODE == 5) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += (float)wd[u];
      continue;
    }
    f32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      x[u] = *reinterpret_cast<const f32x4*>(X + (uint32_t)wd[u] * (uint32_t)W + sub * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += x[u];
  }
  if (acc[0] == 12345.f) out[threadIdx.x] = acc[1] + acc[2] + acc[3];  // keeps the loads alive
}

// Software-pipelined stream + gather: the index words of batch i + PD are issued right after
// batch i's gathers, so a wave waits on one memory latency per batch (the gathers) instead of
// two in series (index word -> gather).  PD = 1 or 2 batches ahead; non-temporal index loads.
template <int PD>
__global__ __launch_bounds__(1024, 8) void gather_pipe_kernel(const int32_t* __restrict__ idx,
                                                              int64_t e,
                                                              const float* __restrict__ X,
                                                              float* __restrict__ out) {
  constexpr int EPS = 32;
  const int lane = threadIdx.x & 63;
  const int pr = lane >> 1, sub = lane & 1;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t per = (e / nw + 4 * EPS - 1) / (4 * EPS) * (4 * EPS);
  const int64_t beg = w0 * per;
  const int64_t end = beg + per < e ? beg + per : e;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int wd[PD][4];
#pragma unroll
  for (int d = 0; d < PD; ++d)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = beg + d * 4 * EPS + u * EPS + pr;
      wd[d][u] = __builtin_nontemporal_load(idx + (q < end ? q : end - 1));
    }
  for (int64_t off = beg; off < end; off += 4 * EPS) {
    f32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      x[u] = *reinterpret_cast<const f32x4*>(X + (uint32_t)wd[0][u] * 8u + sub * 4);
#pragma unroll
    for (int d = 0; d + 1 < PD; ++d)
#pragma unroll
      for (int u = 0; u < 4; ++u) wd[d][u] = wd[d + 1][u];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = off + PD * 4 * EPS + u * EPS + pr;
      wd[PD - 1][u] = __builtin_nontemporal_load(idx + (q < end ? q : (end > beg ? end - 1 : beg)));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += x[u];
  }
  if (acc[0] == 12345.f) out[threadIdx.x] = acc[1] + acc[2] + acc[3];
}

// Fewer index instructions: the plain form loads each entry's word in both lanes of its pair
// (64 lane addresses for 32 words per instruction, one instruction per step).  FORM 0: a dword
// of a distinct entry per lane (one instruction per 2 steps), handed to the pairs by
// ds_bpermute; FORM 1: a dwordx2 per lane (one instruction per 4 steps), likewise.  Non-temporal.
template <int FORM>
__global__ __launch_bounds__(1024, 8) void gather_wide_kernel(const int32_t* __restrict__ idx,
                                                              int64_t e,
                                                              const float* __restrict__ X,
                                                              float* __restrict__ out) {
  constexpr int EPS = 32;
  const int lane = threadIdx.x & 63;
  const int pr = lane >> 1, sub = lane & 1;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t per = (e / nw + 4 * EPS - 1) / (4 * EPS) * (4 * EPS);
  const int64_t beg = w0 * per;
  const int64_t end = beg + per < e ? beg + per : e;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t off = beg; off < end; off += 4 * EPS) {
    int wd[4];
    if (FORM == 0) {
      int w[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int64_t q = off + i * 64 + lane;
        w[i] = __builtin_nontemporal_load(idx + (q < end ? q : end - 1));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) wd[u] = __shfl(w[u >> 1], (u & 1) * 32 + pr, 64);
    } else {
      const int64_t q = off + 2 * lane;
      typedef int i32x2 __attribute__((ext_vector_type(2)));
      const i32x2 w = __builtin_nontemporal_load(
          reinterpret_cast<const i32x2*>(idx + (q + 1 < end ? q : end - 2)));
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int src = (u * 32 + pr) >> 1;
        const int a = __shfl(w.x, src, 64), b = __shfl(w.y, src, 64);
        wd[u] = (pr & 1) ? b : a;
      }
    }
    f32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      x[u] = *reinterpret_cast<const f32x4*>(X + (uint32_t)wd[u] * 8u + sub * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += x[u];
  }
  if (acc[0] == 12345.f) out[threadIdx.x] = acc[1] + acc[2] + acc[3];
}

template <int FORM>
static double run_wide(const int32_t* idx, int64_t e, const float* X, float* out, int reps,
                       int ncu) {
  const dim3 grid((unsigned)(2 * ncu)), block(1024);
  hipLaunchKernelGGL((gather_wide_kernel<FORM>), grid, block, 0, 0, idx, e, X, out);
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((gather_wide_kernel<FORM>), grid, block, 0, 0, idx, e, X, out);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return ms / reps;
}

template <int PD>
static double run_pipe(const int32_t* idx, int64_t e, const float* X, float* out, int reps,
                       int ncu) {
  const dim3 grid((unsigned)(2 * ncu)), block(1024);
  hipLaunchKernelGGL((gather_pipe_kernel<PD>), grid, block, 0, 0, idx, e, X, out);
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((gather_pipe_kernel<PD>), grid, block, 0, 0, idx, e, X, out);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return ms / reps;
}

template <int MODE, int W>
static double run(const int32_t* idx, const uint16_t* idx16, int64_t e, const float* X,
                  uint32_t rows, float* out, int reps, int ncu) {
  const dim3 grid((unsigned)(2 * ncu)), block(1024);
  hipLaunchKernelGGL((gather_kernel<MODE, W>), grid, block, 0, 0, idx, idx16, e, X, rows, out);
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((gather_kernel<MODE, W>), grid, block, 0, 0, idx, idx16, e, X, rows, out);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t e = (int64_t)(argc > 1 ? atof(argv[1]) : 100.0) * 1000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const double only_mb = argc > 3 ? atof(argv[3]) : 0.0;  // one panel size (PMC runs)
  const int only_rb = argc > 4 ? atoi(argv[4]) : 0;       // one row width in bytes
  int ncu = 0;
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const std::vector<double> mb = {1, 2, 4, 8, 32, 160, 320};
  const uint32_t max_rows = (uint32_t)(mb.back() * 1024 * 1024 / 32);  // 32-B rows (floats: x8)
  float *X, *out;
  int32_t* idx;
  uint16_t* idx16;
  CHK(hipMalloc(&idx16, (size_t)e * 2));
  CHK(hipMalloc(&X, (size_t)max_rows * 32));
  CHK(hipMalloc(&out, 4096));
  CHK(hipMalloc(&idx, (size_t)e * 4));
  hipLaunchKernelGGL(fill_x, dim3((unsigned)(((int64_t)max_rows * 8 + 255) / 256)), dim3(256), 0,
                     0, X, (int64_t)max_rows * 8);
  for (int wsel = 0; wsel < 2; ++wsel) {
    const int W = wsel ? 16 : 8;
    if (only_rb && only_rb != 4 * W) continue;
    for (double m : mb) {
      if (only_mb > 0.0 && m != only_mb) continue;
      const uint32_t rows = (uint32_t)(m * 1024 * 1024 / (4 * W));
      hipLaunchKernelGGL(fill_idx, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, 0, idx, e,
                         rows);
      hipLaunchKernelGGL(narrow_idx, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, 0, idx,
                         idx16, e);
      CHK(hipDeviceSynchronize());
      double ts[10] = {-1.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0};
      const bool narrow = rows <= 65536;
      if (W == 8) {
        ts[0] = run<0, 8>(idx, idx16, e, X, rows, out, reps, ncu);
        ts[1] = run<1, 8>(idx, idx16, e, X, rows, out, reps, ncu);
        ts[2] = run<2, 8>(idx, idx16, e, X, rows, out, reps, ncu);
        ts[3] = run<3, 8>(idx, idx16, e, X, rows, out, reps, ncu);
        if (narrow) {
          ts[4] = run<4, 8>(idx, idx16, e, X, rows, out, reps, ncu);
          ts[5] = run<5, 8>(idx, idx16, e, X, rows, out, reps, ncu);
        }
        ts[6] = run_pipe<1>(idx, e, X, out, reps, ncu);
        ts[7] = run_pipe<2>(idx, e, X, out, reps, ncu);
        ts[8] = run_wide<0>(idx, e, X, out, reps, ncu);
        ts[9] = run_wide<1>(idx, e, X, out, reps, ncu);
      } else {
        ts[0] = run<0, 16>(idx, idx16, e, X, rows, out, reps, ncu);
        ts[1] = run<1, 16>(idx, idx16, e, X, rows, out, reps, ncu);
      }
      const char* names[10] = {"stream+gather", "gather only", "stream only",
                              "nt-stream+gather", "u16-stream+gather", "u16-stream only",
                              "nt-stream+gather, indices 1 batch ahead",
                              "nt-stream+gather, indices 2 batches ahead",
                              "nt-stream+gather, dword per lane + bpermute",
                              "nt-stream+gather, dwordx2 per lane + bpermute"};
      for (int f = 0; f < 10; ++f) {
        if (ts[f] < 0) continue;
        printf("{\"form\": \"%s\", \"row_bytes\": %d, \"panel_MB\": %g, \"entries\": %lld, "
               "\"ms\": %.4f, \"G_entries_per_s\": %.1f, \"index_GB_per_s\": %.0f}\n",
               names[f], 4 * W, m, (long long)e, ts[f], e / (ts[f] * 1e-3) / 1e9,
               f == 1 ? 0.0 : (f == 4 || f == 5 ? 2.0 : 4.0) * e / (ts[f] * 1e-3) / 1e9);
        fflush(stdout);
      }
    }
  }
  CHK(hipFree(X));
  CHK(hipFree(out));
  CHK(hipFree(idx));
  CHK(hipFree(idx16));
  return 0;
}

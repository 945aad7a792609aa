// Streaming-read ceiling on MI355X for the orthogonalisation passes (the basis blocks are read
// once per pass, 16 B per lane): plain global_load_dwordx4, non-temporal, and LDS-DMA
// (global_load_lds_dwordx4 into a per-wave ring), U loads in flight per lane, 256-thread
// workgroups at 2..8 per CU.  Reads a 2 GB array (cfg4's full basis: 512 columns x 1M rows fp32),
// prints one JSON line per form: GB/s.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_ceiling tools/stream_ceiling.hip
//   tools/stream_ceiling [GB=2] [reps=10]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) float lds_f32;

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));             \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

// MODE 0: plain, 1: non-temporal.  U 16-B loads per lane per iteration.
template <int MODE, int U>
__global__ __launch_bounds__(256) void stream_kernel(const f32x4* __restrict__ a, int64_t n4,
                                                     float* __restrict__ out) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + (int64_t)u * 256;
      const int64_t jc = j < n4 ? j : n4 - 1;
      v[u] = MODE == 1 ? __builtin_nontemporal_load(a + jc) : a[jc];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc[0] == 1234.5f) out[threadIdx.x] = acc[1] + acc[2] + acc[3];
}

__device__ __forceinline__ void glds16(const void* src, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
}

// LDS-DMA ring: each wave owns D slots of 1 KB; issue D - 1 ahead, wait vmcnt(D - 2) style
// (counted), read its own slot back and accumulate.
template <int D>
__global__ __launch_bounds__(256) void stream_glds_kernel(const f32x4* __restrict__ a, int64_t n4,
                                                          float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float ring[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((lds_f32*)ring) + (uint32_t)wave * D * 1024;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wave;
  const int64_t nchunks = (n4 + 63) / 64;  // 1-KB chunks
  const int64_t my = nchunks > w0 ? (nchunks - w0 + nw - 1) / nw : 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const f32x4* r4 = reinterpret_cast<const f32x4*>(ring) + wave * D * 64;
  auto issue = [&](int64_t t) {
    const int64_t ch = w0 + t * nw;
    const int64_t j = ch * 64 + lane;
    glds16(a + (j < n4 ? j : n4 - 1), __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(t % D) * 1024));
  };
  for (int64_t t = 0; t < D - 1 && t < my; ++t) issue(t);
  for (int64_t t = 0; t < my; ++t) {
    if (t + D - 1 < my) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(t + D - 1);
    }
    const int64_t younger = my - 1 - t < D - 1 ? my - 1 - t : D - 1;
    if (younger >= 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else if (younger == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (younger == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if (younger == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (younger == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc += r4[(t % D) * 64 + lane];
  }
  if (acc[0] == 1234.5f) out[threadIdx.x] = acc[1] + acc[2] + acc[3];
}

template <class F>
static double timeit(F launch, int reps) {
  launch();
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  CHK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) launch();
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 2.0;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t bytes = (int64_t)(gb * 1e9) / 16 * 16;
  const int64_t n4 = bytes / 16;
  int ncu = 0;
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  f32x4* a;
  float* out;
  CHK(hipMalloc(&a, bytes));
  CHK(hipMalloc(&out, 4096));
  CHK(hipMemset(a, 0, bytes));
  (void)hipFuncSetAttribute((const void*)stream_glds_kernel<8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 8 * 1024);
  auto line = [&](const char* form, int wpc, int u, double ms) {
    printf("{\"form\": \"%s\", \"wg_per_cu\": %d, \"loads_in_flight_per_lane\": %d, \"GB\": %.2f, "
           "\"ms\": %.4f, \"GB_per_s\": %.0f}\n", form, wpc, u, bytes / 1e9, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  for (int wpc : {2, 4, 8}) {
    const dim3 g((unsigned)(wpc * ncu)), blk(256);
    line("plain dwordx4", wpc, 4, timeit([&] { hipLaunchKernelGGL((stream_kernel<0, 4>), g, blk, 0, 0, a, n4, out); }, reps));
    line("plain dwordx4", wpc, 8, timeit([&] { hipLaunchKernelGGL((stream_kernel<0, 8>), g, blk, 0, 0, a, n4, out); }, reps));
    line("nt dwordx4", wpc, 8, timeit([&] { hipLaunchKernelGGL((stream_kernel<1, 8>), g, blk, 0, 0, a, n4, out); }, reps));
    line("LDS-DMA ring (8 x 1 KB per wave)", wpc, 7, timeit([&] { hipLaunchKernelGGL((stream_glds_kernel<8>), g, blk, 4 * 8 * 1024, 0, a, n4, out); }, reps));
  }
  CHK(hipFree(a));
  CHK(hipFree(out));
  return 0;
}

// Dependent-launch cost of a hipGraph replay vs back-to-back stream launches on gfx950: a chain
// of small kernels (each workgroup stores one word; 784-B argument like the engine's BlockList)
// launched directly, and the same chain captured once into a graph and replayed.
//   hipcc --offload-arch=gfx950 -O3 tools/graph_probe.hip -o tools/graph_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

struct Big {
  const float* p[96];
  int a, b;
};

__global__ void k_touch(int* out, Big b) {  // every workgroup stores one word
  if (threadIdx.x == 0) out[blockIdx.x] = b.b;
}
__global__ void k_busy(int* out, Big b) {  // ~10 us of dependent FMAs per wave
  float x = (float)threadIdx.x;
  for (int i = 0; i < b.a; ++i) x = fmaf(x, 0.999f, 1.0f);
  if (x == 12345.f) out[blockIdx.x] = b.b;
}

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main() {
  int* d;
  CHK(hipMalloc(&d, 4096 * sizeof(int)));
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  Big b{};
  const int chain = 64, reps = 20;
  for (int grid : {256, 1024}) {
    // direct launches
    for (int r = 0; r < 50; ++r) hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, st, d, b);
    CHK(hipEventRecord(e0, st));
    for (int r = 0; r < reps * chain; ++r) {
      b.b = r;
      hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, st, d, b);
    }
    CHK(hipEventRecord(e1, st));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("grid %5d direct launches      %6.2f us per kernel\n", grid, 1e3 * ms / (reps * chain));
    // one captured chain, replayed
    hipGraph_t g;
    hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < chain; ++r) {
      b.b = r;
      hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, st, d, b);
    }
    CHK(hipStreamEndCapture(st, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(ge, st));
    CHK(hipStreamSynchronize(st));
    CHK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) CHK(hipGraphLaunch(ge, st));
    CHK(hipEventRecord(e1, st));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("grid %5d graph replay (%d)   %6.2f us per kernel\n", grid, chain,
           1e3 * ms / (reps * chain));
    CHK(hipGraphExecDestroy(ge));
    CHK(hipGraphDestroy(g));
  }
  // realistic kernel lengths: a chain of ~10-us kernels, direct vs replayed
  for (int iters : {0, 2000, 4000}) {
    b.a = iters;
    const int grid = 1024;
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_busy, dim3(grid), dim3(256), 0, st, d, b);
    CHK(hipEventRecord(e0, st));
    for (int r = 0; r < reps * chain; ++r) hipLaunchKernelGGL(k_busy, dim3(grid), dim3(256), 0, st, d, b);
    CHK(hipEventRecord(e1, st));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const float direct = 1e3f * ms / (reps * chain);
    hipGraph_t g;
    hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < chain; ++r) hipLaunchKernelGGL(k_busy, dim3(grid), dim3(256), 0, st, d, b);
    CHK(hipStreamEndCapture(st, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(ge, st));
    CHK(hipStreamSynchronize(st));
    CHK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) CHK(hipGraphLaunch(ge, st));
    CHK(hipEventRecord(e1, st));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("busy %4d iters: direct %7.2f us, graph %7.2f us per kernel\n", iters, direct,
           1e3f * ms / (reps * chain));
    CHK(hipGraphExecDestroy(ge));
    CHK(hipGraphDestroy(g));
  }
  // host cost of capture + instantiate for a 300-kernel chain
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    b.a = 0;
    auto t0 = std::chrono::steady_clock::now();
    CHK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < 300; ++r) hipLaunchKernelGGL(k_touch, dim3(1024), dim3(256), 0, st, d, b);
    CHK(hipStreamEndCapture(st, &g));
    auto t1 = std::chrono::steady_clock::now();
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    auto t2 = std::chrono::steady_clock::now();
    printf("300 kernels: capture %.1f us, instantiate %.1f us\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count(),
           std::chrono::duration<double, std::micro>(t2 - t1).count());
  }
  return 0;
}

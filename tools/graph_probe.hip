// Dependent-launch cost of a hipGraph replay vs back-to-back stream launches on gfx950: a chain
// of small kernels (each workgroup stores one word; 784-B argument like the engine's BlockList)
// launched directly, and the same chain captured once into a graph and replayed.
//   hipcc --offload-arch=gfx950 -O3 tools/graph_probe.hip -o tools/graph_probe
#include <hip/hip_runtime.h>

#include <cstdio>

struct Big {
  const float* p[96];
  int a, b;
};

__global__ void k_touch(int* out, Big b) {  // every workgroup stores one word
  if (threadIdx.x == 0) out[blockIdx.x] = b.b;
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
  return 0;
}

// Dependent-launch cost on gfx950 vs kernel-argument size: an empty 256 x 256 kernel launched
// back to back with a 4-byte argument and with a 784-byte BlockList-sized argument.
//   hipcc --offload-arch=gfx950 -O3 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>

struct Big {
  const float* p[96];
  int a, b;
};

__global__ void k_small(int* out, int v) {
  if (v == 12345 && threadIdx.x == 0) out[blockIdx.x] = v;
}
__global__ void k_big(int* out, Big b) {
  if (b.a == 12345 && threadIdx.x == 0) out[blockIdx.x] = b.b;
}
__global__ void k_touch(int* out, int v) {  // every workgroup stores one word
  if (threadIdx.x == 0) out[blockIdx.x] = v;
}
__global__ void k_bigread(int* out, Big b) {  // every wave reads 8 of the pointers
  const float* q = b.p[(blockIdx.x + threadIdx.x / 64) & 7];
  if (q == nullptr && b.a == 12345) out[blockIdx.x] = 1;
}
__global__ void k_table(int* out, const Big* __restrict__ t) {  // the same through a device table
  const float* q = t->p[(blockIdx.x + threadIdx.x / 64) & 7];
  if (q == nullptr && t->a == 12345) out[blockIdx.x] = 1;
}

int main() {
  int* d;
  hipMalloc(&d, 4096 * sizeof(int));
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  Big b{};
  const int reps = 400;
  Big* tb;
  hipMalloc(&tb, sizeof(Big));
  hipMemcpy(tb, &b, sizeof(Big), hipMemcpyHostToDevice);
  for (int grid : {256, 1024, 2048}) {
    for (int form = 0; form < 5; ++form) {
      for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, st, d, 1);
      hipEventRecord(e0, st);
      for (int r = 0; r < reps; ++r) {
        if (form == 0) hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, st, d, r);
        else if (form == 1) hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, st, d, b);
        else if (form == 2) hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, st, d, r);
        else if (form == 3) hipLaunchKernelGGL(k_bigread, dim3(grid), dim3(256), 0, st, d, b);
        else hipLaunchKernelGGL(k_table, dim3(grid), dim3(256), 0, st, d, tb);
      }
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      printf("grid %5d %-24s %6.2f us per launch\n", grid,
             form == 0 ? "4-B argument" : form == 1 ? "784-B argument" : form == 2 ? "4-B arg, one store/WG" : form == 3 ? "784-B arg, 8 read" : "device table, 8 read",
             1e3 * ms / reps);
    }
  }
  return 0;
}

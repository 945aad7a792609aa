// Timing probe of the fused PIP pass (n2v2r_launch_pip_fused) outside the solver: back-to-back
// launches at cfg2 size (N = 100k rows, 8-wide blocks), HIP events around 50 launches.
//   local:   c = 16 (two blocks, every block applied), Zin != Zout (the local first pass)
//   full k:  c = 384 (48 blocks), selective (tau = 1e-7) with exactly k blocks above tau
//   all:     c = 384, every block applied (tau = 0)
// plus the cost of a 4-byte memset between launches (the dependent-boundary reference).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I node2vec2rank_amd/csrc tools/pip_probe.cpp \
//     -L node2vec2rank_amd/lib -ln2v2r_hip -Wl,-rpath,$PWD/node2vec2rank_amd/lib -o tools/pip_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "common.h"

extern "C" hipError_t n2v2r_launch_pip_fused(const BlockList& Q, const float* Zin, float* Zout,
                                             const double* G, int c, int64_t n, const int* cond,
                                             int* flags, int* any_flag, double* save,
                                             int save_row0, int save_rows, int* sticky,
                                             uint64_t seed, int64_t row0, double* rsave,
                                             float skip_tol, int* skipped, hipStream_t stream);

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

int main() {
  const int64_t n = 100000;
  const int nblk = 48, reps = 50;
  std::mt19937 rng(1);
  std::normal_distribution<float> nd;
  std::vector<float> h((size_t)n * 8);
  std::vector<float*> blk(nblk + 2);
  for (auto& p : blk) {
    for (auto& v : h) v = nd(rng);
    CK(hipMalloc(&p, sizeof(float) * n * 8));
    CK(hipMemcpy(p, h.data(), sizeof(float) * n * 8, hipMemcpyHostToDevice));
  }
  float* Z = blk[nblk];
  float* Zo = blk[nblk + 1];
  double* G;
  int *flags, *anyf, *skipped, *tiny;
  CK(hipMalloc(&G, sizeof(double) * (nblk + 1) * 64));
  CK(hipMalloc(&flags, sizeof(int) * 64));
  CK(hipMalloc(&anyf, sizeof(int) * 4));
  CK(hipMalloc(&skipped, sizeof(int) * 68));
  CK(hipMalloc(&tiny, sizeof(int)));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto setG = [&](int c, int k) {  // Z^T Z = n I; C rows of the first k blocks above tau
    std::vector<double> g((size_t)(c + 8) * 8, 0.0);
    for (int i = 0; i < 8; ++i) g[(size_t)(c + i) * 8 + i] = (double)n;
    for (int b = 0; b < k && b * 8 < c; ++b)
      for (int r = 0; r < 8; ++r)
        for (int j = 0; j < 8; ++j) g[(size_t)(b * 8 + r) * 8 + j] = 1e-3 * std::sqrt((double)n);
    CK(hipMemcpy(G, g.data(), sizeof(double) * g.size(), hipMemcpyHostToDevice));
  };
  auto run = [&](const char* name, int c, int k, float tau, bool inplace) {
    setG(c, k);
    BlockList Q{};
    Q.count = c / 8;
    Q.width = 8;
    for (int b = 0; b < Q.count; ++b) Q.blk[b] = blk[b];
    float* zo = inplace ? Z : Zo;
    auto once = [&]() {
      CK(n2v2r_launch_pip_fused(Q, Z, zo, G, c, n, nullptr, flags, anyf, nullptr, 0, 0, nullptr,
                                7, 0, nullptr, tau, tau != 0.f ? skipped : nullptr, st));
    };
    for (int r = 0; r < 5; ++r) once();
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) once();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const int applied = tau != 0.f ? k : c / 8;
    const double mb = (applied * 8.0 * 4 * n + 2.0 * 4 * 8 * n) / 1e6;
    printf("%-10s c %3d applied %2d: %7.2f us per launch, %6.1f MB streamed, %5.2f TB/s\n", name, c,
           applied, 1e3 * ms / reps, mb, mb / (1e3 * ms / reps) / 1e6);
  };
  run("local", 16, 2, 0.f, false);
  for (int k : {0, 1, 4, 7, 16, 32})
    run("full", 384, k, 1e-7f, true);
  run("all", 384, 48, 0.f, true);
  // the boundary reference: a 4-byte memset per step
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) CK(hipMemsetAsync(tiny, 0, sizeof(int), st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("memset 4 B: %.2f us per launch\n", 1e3 * ms / reps);
  return 0;
}

// Timing probe of the orthogonalisation Grams (streaming ts_tn form + chunk reduce) outside the
// solver, at cfg2 size (N = 100k rows, 8-wide blocks), 50 back-to-back launches each:
//   full:  G = [Q_0 .. Q_47 Z]^T Z (the full pass at c = 384)
//   local: G = [Q_0 Q_1 Z]^T Z with Z = P_1 + P_2 summed and stored on the way (the local pass
//          after a split SpMM stage)
// Run under `rocprofv3 --kernel-trace --stats` for per-kernel durations (Gram vs reduce); the
// event time per pair is printed too.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I node2vec2rank_amd/csrc tools/gram_probe.cpp \
//     -L node2vec2rank_amd/lib -ln2v2r_hip -Wl,-rpath,'$ORIGIN/../node2vec2rank_amd/lib' \
//     -o tools/gram_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "common.h"

extern "C" hipError_t n2v2r_launch_ts_tn(const BlockList& A, const BlockList& B, int64_t n,
                                         double* partial, size_t partial_elems, double* out,
                                         const int* cond, hipStream_t stream);
extern "C" hipError_t n2v2r_launch_ts_tn_zsum(const BlockList& A, int64_t n,
                                              const float* const* parts, int count, float* zout,
                                              double* partial, size_t partial_elems, double* out,
                                              hipStream_t stream);

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
  std::vector<float*> blk(nblk + 3);
  for (auto& p : blk) {
    for (auto& v : h) v = nd(rng);
    CK(hipMalloc(&p, sizeof(float) * n * 8));
    CK(hipMemcpy(p, h.data(), sizeof(float) * n * 8, hipMemcpyHostToDevice));
  }
  float* Z = blk[nblk];
  const size_t pe = 4096ull * 1024ull;
  double *part, *G;
  CK(hipMalloc(&part, sizeof(double) * pe));
  CK(hipMalloc(&G, sizeof(double) * (nblk + 1) * 64));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](const char* name, auto&& once) {
    for (int r = 0; r < 5; ++r) once();
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) once();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-8s %7.2f us per Gram + reduce\n", name, 1e3 * ms / reps);
  };
  BlockList A{}, B{};
  A.width = B.width = 8;
  A.count = nblk + 1;
  for (int b = 0; b < nblk; ++b) A.blk[b] = blk[b];
  A.blk[nblk] = Z;
  B.count = 1;
  B.blk[0] = Z;
  timed("full", [&]() { CK(n2v2r_launch_ts_tn(A, B, n, part, pe, G, nullptr, st)); });
  BlockList L{};
  L.width = 8;
  L.count = 3;
  L.blk[0] = blk[0];
  L.blk[1] = blk[1];
  L.blk[2] = Z;
  const float* parts[2] = {blk[nblk + 1], blk[nblk + 2]};
  timed("local", [&]() {
    CK(n2v2r_launch_ts_tn_zsum(L, n, parts, 2, Z, part, pe, G, st));
  });
  return 0;
}

// Single-wave dependent-chain latencies on gfx950 (cycles per step by s_memtime): fp64 FMA,
// readlane -> fp64 FMA, DPP row_shl -> fp64 FMA, ds_bpermute -> fp64 FMA, LDS load -> FMA.
//   hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o tools/lat_probe && ./tools/lat_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define N 4096

__device__ __forceinline__ double lane0(double v) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 0);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 0);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double shl1(double v) {
  const int l = __double2loint(v), h = __double2hiint(v);
  return __hiloint2double(__builtin_amdgcn_update_dpp(h, h, 0x101, 0xF, 0xF, false),
                          __builtin_amdgcn_update_dpp(l, l, 0x101, 0xF, 0xF, false));
}
__device__ __forceinline__ double bperm(double v, int src) {
  return __hiloint2double(__builtin_amdgcn_ds_bpermute(src * 4, __double2hiint(v)),
                          __builtin_amdgcn_ds_bpermute(src * 4, __double2loint(v)));
}

__device__ __forceinline__ double rs_dpp_shl1(double v) {  // lane l <- lane l + 1 (16-lane rows)
  // (lanes at a row's end keep their own value: callers mask lane 7 and ignore lanes >= 8)
  const int l = __double2loint(v), h = __double2hiint(v);
  const int lo = __builtin_amdgcn_update_dpp(l, l, 0x101, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(h, h, 0x101, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rs_lane0(double v) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 0);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 0);
  return __hiloint2double(hi, lo);
}
#define RS_PF 8
__device__ __forceinline__ void rs_band_solve_par(int c, int kp, const double* F, const double* fe,
                                                  double* f, double* y) {
  const int nb = c - kp;
  const int lane = threadIdx.x & 63, q = lane & 7;
  const bool last = q == 7;
  // forward: r_q = f[kp + q] - fe[q]; at row k, lane q needs t_{k,q+1} = F[k][1 + q] and lane 7
  // the entering right-hand side f[kp + k + 8] (zero past the band: f is padded by 8 + RS_PF
  // entries read as zero below).  Whole groups of RS_PF rows without exit tests; loads for the
  // next group are issued before the current group's chain and are unconditional (clamped).
  double r = f[kp + q] - fe[q];
  double tq[RS_PF], fv[RS_PF];
  auto fload = [&](int kk, double* t, double* v) {
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      const int k = kk + u;
      t[u] = F[min(k, nb - 1) * 9 + 1 + q];
      const double fx = f[kp + min(k + 8, nb - 1)];
      v[u] = (k + 8 < nb) ? fx : 0.0;
    }
  };
  fload(0, tq, fv);
  int k0 = 0;
  for (; k0 + RS_PF <= nb; k0 += RS_PF) {
    double tn[RS_PF], fn[RS_PF];
    fload(k0 + RS_PF, tn, fn);
    double zs = 0.0;  // lane u keeps z_{k0 + u}: one store per RS_PF rows, off the chain
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      const double zk = rs_lane0(r);
      zs = (lane == u) ? zk : zs;
      double nx = rs_dpp_shl1(r);
      nx = last ? fv[u] : nx;
      r = fma(-tq[u], zk, nx);
    }
    if (lane < RS_PF) f[kp + k0 + lane] = zs;
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      tq[u] = tn[u];
      fv[u] = fn[u];
    }
  }
  {
    double zs = 0.0;
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      if (k0 + u >= nb) break;
      const double zk = rs_lane0(r);
      zs = (lane == u) ? zk : zs;
      double nx = rs_dpp_shl1(r);
      nx = last ? fv[u] : nx;
      r = fma(-tq[u], zk, nx);
    }
    if (lane < RS_PF && k0 + lane < nb) f[kp + k0 + lane] = zs;
  }
  // backward: row k's solution y_k = z_k d_k^{-1} - sum_i t_{k,i} y_{k+i}; lane j holds that sum
  // for row k - j; after y_k, lane j takes lane j + 1's sum plus t_{k-1-j, j+1} y_k
  double acc = 0.0;
  double zr[RS_PF], tb[RS_PF];
  const int top = nb - 1;
  auto bload = [&](int kk, double* z, double* t) {
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      const int k = max(kk - u, 0);
      z[u] = f[kp + k] * F[k * 9];
      const int row = kk - u - 1 - q;
      const double tx = F[max(row, 0) * 9 + q + 1];
      t[u] = row >= 0 ? tx : 0.0;
    }
  };
  bload(top, zr, tb);
  int k1 = top;
  for (; k1 - RS_PF + 1 >= 0; k1 -= RS_PF) {
    double zn[RS_PF], tbn[RS_PF];
    bload(k1 - RS_PF, zn, tbn);
    double ys = 0.0;  // lane u keeps y_{k1 - u}
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      const double yk = zr[u] - rs_lane0(acc);
      ys = (lane == u) ? yk : ys;
      double sh = rs_dpp_shl1(acc);
      sh = last ? 0.0 : sh;
      acc = fma(tb[u], yk, sh);
    }
    if (lane < RS_PF) y[kp + k1 - lane] = ys;
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      zr[u] = zn[u];
      tb[u] = tbn[u];
    }
  }
  {
    double ys = 0.0;
#pragma unroll
    for (int u = 0; u < RS_PF; ++u) {
      if (k1 - u < 0) break;
      const double yk = zr[u] - rs_lane0(acc);
      ys = (lane == u) ? yk : ys;
      double sh = rs_dpp_shl1(acc);
      sh = last ? 0.0 : sh;
      acc = fma(tb[u], yk, sh);
    }
    if (lane < RS_PF && k1 - lane >= 0) y[kp + k1 - lane] = ys;
  }
}
#undef RS_PF

__global__ void solve_probe(long long* cyc, double* out) {
  __shared__ double F[320 * 9 + 64];
  __shared__ double f[400], y[400], fe[8];
  const int lane = threadIdx.x;
  for (int i = lane; i < 320 * 9; i += 64) F[i] = (i % 9 == 0) ? 0.5 : 0.01 / (1 + i % 7);
  for (int i = lane; i < 400; i += 64) f[i] = 1.0 / (1 + i);
  if (lane < 8) fe[lane] = 0.0;
  __syncthreads();
  long long t0 = clock64();
  rs_band_solve_par(80 + 304, 80, F, fe, f, y);
  long long t1 = clock64();
  __syncthreads();
  if (lane == 0) cyc[0] = t1 - t0;
  out[lane] = y[100 + lane];
}

__global__ void probe(double* out, long long* cyc, double a, double b) {
  __shared__ double lds[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lds[i] = 1.0 / (i + 1);
  __syncthreads();
  double x = a + lane;
  long long t0, t1;
  // 0: fp64 FMA chain
  t0 = clock64();
  for (int i = 0; i < N; ++i) x = fma(x, b, a);
  t1 = clock64();
  cyc[0] = t1 - t0;
  // 1: readlane -> FMA
  t0 = clock64();
  for (int i = 0; i < N; ++i) x = fma(lane0(x), b, a);
  t1 = clock64();
  cyc[1] = t1 - t0;
  // 2: DPP shift -> FMA
  t0 = clock64();
  for (int i = 0; i < N; ++i) x = fma(shl1(x), b, a);
  t1 = clock64();
  cyc[2] = t1 - t0;
  // 3: ds_bpermute -> FMA
  t0 = clock64();
  for (int i = 0; i < N; ++i) x = fma(bperm(x, (lane + 9) & 63), b, a);
  t1 = clock64();
  cyc[3] = t1 - t0;
  // 4: dependent LDS load (index from the value) -> FMA
  int idx = lane;
  t0 = clock64();
  for (int i = 0; i < N; ++i) {
    x = fma(lds[idx & 1023], b, x);
    idx = (int)(x * 0.0) + ((idx + 7) & 1023);
  }
  t1 = clock64();
  cyc[4] = t1 - t0;
  // 5: readlane + DPP + cndmask + FMA (the forward-solve step)
  t0 = clock64();
  for (int i = 0; i < N; ++i) {
    const double z = lane0(x);
    double nx = shl1(x);
    nx = ((lane & 7) == 7) ? a : nx;
    x = fma(-b, z, nx);
  }
  t1 = clock64();
  cyc[5] = t1 - t0;
  out[lane] = x;
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&cyc, 8 * sizeof(long long));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, cyc, 0.5, 0.999);
    hipDeviceSynchronize();
  }
  long long h[8];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[6] = {"fma_f64", "readlane+fma", "dpp+fma", "bpermute+fma", "lds_load+fma",
                          "solve_step"};
  for (int i = 0; i < 6; ++i) printf("%-14s %7.1f cycles/step\n", names[i], (double)h[i] / N);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(solve_probe, dim3(1), dim3(64), 0, 0, cyc, out);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  printf("band solve (nb 304, fwd + bwd): %lld cycles = %.1f per row-step\n", h[0], h[0] / 608.0);
  return 0;
}

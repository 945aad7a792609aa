// CSR x dense-panel SpMM for the Gram operator M = sum_k A_k A_k^T (gfx950, wave64).
//
// Layout: CSR per layer (int64 row pointers, int32 columns, fp32 values) resident in HBM;
// dense panels row-major N x B fp32 (B = 8, 16, 32 or 64: a 32..256-B segment per row).
// A wave owns RPW output rows (a group of 64/RPW lanes per row, RPW picked from the mean row
// length).  A row's column indices and values are loaded once, coalesced, one group-width at a
// time, and broadcast with __shfl; the group then gathers panel rows, each by B/4 lanes with
// one 16-B load per lane, so a panel row is one coalesced 32..256-B segment.  Partial sums are
// folded with xor shuffles inside the group and its first B/4 lanes store the output row with
// 16-B stores.
// There is no LDS staging: an ER/co-expression row's columns are uniformly random, so a
// workgroup has no panel reuse to stage; reuse comes from L2 / Infinity Cache.
//
// Algorithmic bytes per launch (this format): 8*nnz (4*nnz for an unweighted
// layer: no value stream) + 8*(N+1) (int64 row pointers) + 4*N*B (panel read once) + 4*N*B
// (output written); the gathered panel rows (4*B per nnz) come from L2 / Infinity Cache.
#include "common.h"

#include <cstdlib>

#include "spmm_args.h"

// XCD-split task space: the layer of this workgroup and its index / count among the
// workgroups of that layer (grid.x a multiple of 8; workgroup i runs on XCD i mod 8)
__device__ __forceinline__ void split_slot(int K, int& k, int64_t& wg, int64_t& nwg) {
  const int xcd = blockIdx.x & 7;
  k = (xcd * K) >> 3;
  const int x0 = (k * 8 + K - 1) / K, x1 = ((k + 1) * 8 + K - 1) / K;
  wg = (int64_t)(blockIdx.x >> 3) * (x1 - x0) + (xcd - x0);
  nwg = (int64_t)(gridDim.x >> 3) * (x1 - x0);
}

// RPW rows per wave: each row owns a group of L = 64 / RPW lanes; inside the group LPN = B / 4
// lanes gather one panel row (one 16-B load each) and NPS = L / LPN panel rows are gathered
// per step.  Short rows (ER / k-NN graphs: tens of nnz) then keep several rows' gathers in
// flight per wave instead of leaving most lanes idle.
template <int B, int RPW>
__device__ __forceinline__ void spmm_row_accumulate(const CsrDev& A, const float* __restrict__ X,
                                                    int64_t ldx, int64_t row, bool row_ok,
                                                    int lane, f32x4& acc) {
  constexpr int L = 64 / RPW;
  constexpr int LPN = B / 4;
  constexpr int NPS = L / LPN;
  static_assert(NPS >= 1, "row group narrower than one panel row");
  const int g = lane / L;
  const int li = lane % L;
  const int sub = li % LPN;
  const int srcbase = g * L + li / LPN;
  int64_t beg = 0, end = 0;
  if (row_ok) {
    beg = A.indptr[row];
    end = A.indptr[row + 1];
  }
  // the wave loops until its longest row is done
  int64_t len = end - beg;
  int64_t maxlen = len;
#pragma unroll
  for (int m = L; m < 64; m <<= 1) {
    const int64_t o = __shfl_xor(maxlen, m, 64);
    maxlen = o > maxlen ? o : maxlen;
  }
  for (int64_t off = 0; off < maxlen; off += L) {
    int colv = 0;
    float valv = 0.f;
    if (off + li < len) {
      colv = A.indices[beg + off + li];
      valv = A.unit ? 1.f : A.data[beg + off + li];  // unweighted layers: no value stream
    }
    int64_t rem = maxlen - off;
    const int nn = (int)(rem < L ? rem : L);
    const int steps = (nn + NPS - 1) / NPS;
    int s = 0;
    for (; s + 2 <= steps; s += 2) {
      const int c0 = __shfl(colv, srcbase + (s + 0) * NPS, 64);
      const int c1 = __shfl(colv, srcbase + (s + 1) * NPS, 64);
      const float v0 = __shfl(valv, srcbase + (s + 0) * NPS, 64);
      const float v1 = __shfl(valv, srcbase + (s + 1) * NPS, 64);
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(X + (int64_t)c0 * ldx + sub * 4);
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(X + (int64_t)c1 * ldx + sub * 4);
      acc += v0 * x0;
      acc += v1 * x1;
    }
    if (s < steps) {
      const int c0 = __shfl(colv, srcbase + s * NPS, 64);
      const float v0 = __shfl(valv, srcbase + s * NPS, 64);
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(X + (int64_t)c0 * ldx + sub * 4);
      acc += v0 * x0;
    }
  }
}

template <int B, int RPW>
__global__ __launch_bounds__(256) void spmm_csr_panel_kernel(SpmmArgs args) {
  constexpr int L = 64 / RPW;
  constexpr int LPN = B / 4;
  const int lane = threadIdx.x & 63;
  const int k0 = args.sum ? 0 : (int)blockIdx.y;
  const int64_t n = args.A[k0].n_rows;
  const int li = lane % L;
  // grid-stride over row groups: a bounded number of long-lived workgroups (measured 4-7 %
  // faster than one short workgroup per 4 x RPW rows)
  const int64_t nwaves_total = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t wid = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
       wid * RPW < n; wid += nwaves_total) {
    const int64_t row = wid * RPW + lane / L;
    const bool row_ok = row < n;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (args.sum) {
      for (int k = 0; k < args.K; ++k)
        spmm_row_accumulate<B, RPW>(args.A[k], args.X[k], args.ldx, row, row_ok, lane, acc);
    } else {
      spmm_row_accumulate<B, RPW>(args.A[k0], args.X[k0], args.ldx, row, row_ok, lane, acc);
    }
#pragma unroll
    for (int m = LPN; m < L; m <<= 1) {
      acc.x += __shfl_xor(acc.x, m, 64);
      acc.y += __shfl_xor(acc.y, m, 64);
      acc.z += __shfl_xor(acc.z, m, 64);
      acc.w += __shfl_xor(acc.w, m, 64);
    }
    if (row_ok && li < LPN) {
      if (args.colscale) {
        f32x4 sc = *reinterpret_cast<const f32x4*>(args.colscale + li * 4);
        acc *= sc;
      }
      *reinterpret_cast<f32x4*>(args.Y[k0] + row * args.ldy + li * 4) = acc;
    }
  }
}

// B = 8, software-pipelined: a wave walks its tasks (row group, layer) in order and, while the
// current task's panel rows are being gathered, already has the next task's row pointers and
// first SP8_PF x L column indices (and values) in flight.  A row's gathers thus wait on one
// dependent load (the gather itself) instead of three (row pointer -> index -> gather); rows
// longer than SP8_PF x L finish in an unpipelined tail loop.  Same lane layout and summation
// order per row as spmm_csr_panel_kernel<8, RPW> (column halves in lane pairs, NPS panel rows
// per step, the row group's partial sums folded by xor shuffles).
#define SP8_PF 2
template <int RPW>
__global__ __launch_bounds__(256) void spmm8_pipe_kernel(SpmmArgs args) {
  constexpr int L = 64 / RPW, NPS = L / 2;
  const int lane = threadIdx.x & 63;
  const int g = lane / L, li = lane % L, sub = li & 1;
  const int srcbase = g * L + (li >> 1);
  const int K = args.sum ? args.K : 1;
  int kfix = args.sum ? 0 : (int)blockIdx.y;
  int64_t wg = blockIdx.x, nwg = gridDim.x;
  if (args.split) split_slot(args.K, kfix, wg, nwg);
  const int64_t n = args.A[kfix].n_rows;
  const int64_t ngroups = (n + RPW - 1) / RPW;
  const int64_t gstride = nwg * (blockDim.x / 64);
  int64_t grp = wg * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (grp >= ngroups) return;
  int k = 0;
  // current task
  int64_t row = grp * RPW + g;
  int64_t beg = 0, len = 0;
  int idx[SP8_PF];
  float val[SP8_PF];
  {
    const CsrDev& A = args.A[kfix + k];
    if (row < n) {
      beg = A.indptr[row];
      len = A.indptr[row + 1] - beg;
    }
#pragma unroll
    for (int p = 0; p < SP8_PF; ++p) {
      const bool in = p * L + li < len;
      idx[p] = in ? A.indices[beg + p * L + li] : 0;
      val[p] = in ? (A.unit ? 1.f : A.data[beg + p * L + li]) : 0.f;
    }
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (;;) {
    // next task: next layer of this row group (sum mode), else the next row group
    int nk = k + 1;
    int64_t ngrp = grp;
    if (nk == K) {
      nk = 0;
      ngrp = grp + gstride;
    }
    const bool has_next = ngrp < ngroups;
    const int64_t nrow = ngrp * RPW + g;
    const CsrDev& An = args.A[kfix + nk];
    // 1. the next task's row pointers
    int64_t nbeg = 0, nend = 0;
    if (has_next && nrow < n) {
      nbeg = An.indptr[nrow];
      nend = An.indptr[nrow + 1];
    }
    // 2. the current task's gathers (prefetched indices)
    const CsrDev& A = args.A[kfix + k];
    const float* X = args.X[kfix + k];
    int64_t maxlen = len;
#pragma unroll
    for (int m = L; m < 64; m <<= 1) {
      const int64_t o = __shfl_xor(maxlen, m, 64);
      maxlen = o > maxlen ? o : maxlen;
    }
#pragma unroll
    for (int s = 0; s < 2 * SP8_PF; ++s) {
      if (s * NPS >= maxlen) break;
      const int c0 = __shfl(idx[s >> 1], srcbase + (s & 1) * NPS, 64);
      const float v0 = __shfl(val[s >> 1], srcbase + (s & 1) * NPS, 64);
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(X + (int64_t)c0 * args.ldx + sub * 4);
      acc += v0 * x0;
    }
    // 3. the next task's first column indices / values
    const int64_t nlen = nend - nbeg;
    int nidx[SP8_PF];
    float nval[SP8_PF];
#pragma unroll
    for (int p = 0; p < SP8_PF; ++p) {
      const bool in = p * L + li < nlen;
      nidx[p] = in ? An.indices[nbeg + p * L + li] : 0;
      nval[p] = in ? (An.unit ? 1.f : An.data[nbeg + p * L + li]) : 0.f;
    }
    // 4. long rows: the rest of the current task, unpipelined
    for (int64_t off = SP8_PF * L; off < maxlen; off += L) {
      int colv = 0;
      float valv = 0.f;
      if (off + li < len) {
        colv = A.indices[beg + off + li];
        valv = A.unit ? 1.f : A.data[beg + off + li];
      }
      const int64_t rem = maxlen - off;
      const int nn = (int)(rem < L ? rem : L);
      for (int s = 0; s * NPS < nn; ++s) {
        const int c0 = __shfl(colv, srcbase + s * NPS, 64);
        const float v0 = __shfl(valv, srcbase + s * NPS, 64);
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(X + (int64_t)c0 * args.ldx + sub * 4);
        acc += v0 * x0;
      }
    }
    if (k == K - 1) {  // row complete: fold the row group, store
#pragma unroll
      for (int m = 2; m < L; m <<= 1) {
        acc.x += __shfl_xor(acc.x, m, 64);
        acc.y += __shfl_xor(acc.y, m, 64);
        acc.z += __shfl_xor(acc.z, m, 64);
        acc.w += __shfl_xor(acc.w, m, 64);
      }
      if (row < n && li < 2) {
        if (args.colscale) {
          const f32x4 sc = *reinterpret_cast<const f32x4*>(args.colscale + li * 4);
          acc *= sc;
        }
        *reinterpret_cast<f32x4*>(args.Y[kfix] + row * args.ldy + li * 4) = acc;
      }
      acc = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (!has_next) break;
    k = nk;
    grp = ngrp;
    row = nrow;
    beg = nbeg;
    len = nlen;
#pragma unroll
    for (int p = 0; p < SP8_PF; ++p) {
      idx[p] = nidx[p];
      val[p] = nval[p];
    }
  }
}

// B = 8, one lane per entry: lane li of a row's L-lane group takes entries li, li + L, ... and
// gathers the whole 32-B panel row itself (two 16-B loads), so a wave-instruction serves 64
// entries (the two-lanes-per-row form serves 32) and no index / value shuffles are needed.
// Two group-widths per step keep 4 loads per lane in flight; entries past the row end read
// panel row 0 and multiply by 0 (clamped addresses: the loads issue as one batch).  The L
// partial sums of a row are folded by an xor butterfly.
template <int RPW>
__global__ __launch_bounds__(256) void spmm8_lane_kernel(SpmmArgs args) {
  constexpr int L = 64 / RPW;
  const int lane = threadIdx.x & 63;
  const int g = lane / L, li = lane % L;
  const int K = args.sum ? args.K : 1;
  const int kfix = args.sum ? 0 : (int)blockIdx.y;
  const int64_t n = args.A[kfix].n_rows;
  const int64_t ngroups = (n + RPW - 1) / RPW;
  const int64_t gstride = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t grp = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); grp < ngroups;
       grp += gstride) {
    const int64_t row = grp * RPW + g;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const CsrDev& A = args.A[kfix + k];
      const float* X = args.X[kfix + k];
      int64_t beg = 0, len = 0;
      if (row < n) {
        beg = A.indptr[row];
        len = A.indptr[row + 1] - beg;
      }
      int64_t maxlen = len;
#pragma unroll
      for (int m = L; m < 64; m <<= 1) {
        const int64_t o = __shfl_xor(maxlen, m, 64);
        maxlen = o > maxlen ? o : maxlen;
      }
      for (int64_t off = 0; off < maxlen; off += 2 * L) {
        const bool in0 = off + li < len, in1 = off + L + li < len;
        const int c0 = in0 ? A.indices[beg + off + li] : 0;
        const int c1 = in1 ? A.indices[beg + off + L + li] : 0;
        float v0 = in0 ? 1.f : 0.f, v1 = in1 ? 1.f : 0.f;
        if (!A.unit) {
          v0 = in0 ? A.data[beg + off + li] : 0.f;
          v1 = in1 ? A.data[beg + off + L + li] : 0.f;
        }
        const float* x0 = X + (int64_t)c0 * args.ldx;
        const float* x1 = X + (int64_t)c1 * args.ldx;
        const f32x4 x00 = *reinterpret_cast<const f32x4*>(x0);
        const f32x4 x01 = *reinterpret_cast<const f32x4*>(x0 + 4);
        const f32x4 x10 = *reinterpret_cast<const f32x4*>(x1);
        const f32x4 x11 = *reinterpret_cast<const f32x4*>(x1 + 4);
        a0 += v0 * x00;
        a1 += v0 * x01;
        a0 += v1 * x10;
        a1 += v1 * x11;
      }
    }
#pragma unroll
    for (int m = 1; m < L; m <<= 1) {
      a0.x += __shfl_xor(a0.x, m, 64);
      a0.y += __shfl_xor(a0.y, m, 64);
      a0.z += __shfl_xor(a0.z, m, 64);
      a0.w += __shfl_xor(a0.w, m, 64);
      a1.x += __shfl_xor(a1.x, m, 64);
      a1.y += __shfl_xor(a1.y, m, 64);
      a1.z += __shfl_xor(a1.z, m, 64);
      a1.w += __shfl_xor(a1.w, m, 64);
    }
    if (row < n && li < 2) {
      f32x4 o = li ? a1 : a0;
      if (args.colscale) o *= *reinterpret_cast<const f32x4*>(args.colscale + li * 4);
      *reinterpret_cast<f32x4*>(args.Y[kfix] + row * args.ldy + li * 4) = o;
    }
  }
}

static int spmm8_form() {  // N2V2R_SPMM8=lane: the one-lane-per-entry kernel (A/B runs)
  static const int v = [] {
    const char* s = getenv("N2V2R_SPMM8");
    return (s && s[0] == 'l') ? 1 : 0;
  }();
  return v;
}

// B = 8 uses the pipelined kernel unless N2V2R_SPMM_PIPE=0 (A/B runs)
static bool spmm8_pipelined() {
  static const bool v = [] {
    const char* s = getenv("N2V2R_SPMM_PIPE");
    return !(s && s[0] == '0');
  }();
  return v;
}

template <int B, int RPW>
static void launch_spmm_t(const SpmmArgs& args, hipStream_t stream) {
  const int64_t n = args.A[0].n_rows;
  const int64_t waves = (n + RPW - 1) / RPW;
  int64_t wgs = (waves + 3) / 4;
  const int64_t cap = (int64_t)N2V2R_SPMM_WGS / (args.sum ? 1 : args.K);
  if (wgs > cap) wgs = cap;
  dim3 grid((unsigned)wgs, args.sum ? 1 : args.K);
  if (args.split) grid = dim3((unsigned)N2V2R_SPMM_WGS, 1);
  if constexpr (B == 8) {
    if (spmm8_form() == 1) {
      hipLaunchKernelGGL((spmm8_lane_kernel<RPW>), grid, dim3(256), 0, stream, args);
      return;
    }
  }
  if constexpr (B == 8 && RPW >= 2) {
    if (spmm8_pipelined()) {
      hipLaunchKernelGGL((spmm8_pipe_kernel<RPW>), grid, dim3(256), 0, stream, args);
      return;
    }
  }
  hipLaunchKernelGGL((spmm_csr_panel_kernel<B, RPW>), grid, dim3(256), 0, stream, args);
}

// rows per wave from the mean row length: a row group of L lanes gathers L / (B/4) panel rows
// per step; aim for ~3-4 steps per row.
template <int B>
static void launch_spmm_b(const SpmmArgs& args, hipStream_t stream) {
  double avg = 0.0;
  int kk = args.sum ? args.K : args.K;
  for (int k = 0; k < kk; ++k) avg += (double)args.A[k].nnz / (double)(args.A[k].n_rows > 0 ? args.A[k].n_rows : 1);
  avg /= (kk > 0 ? kk : 1);
  constexpr int LPN = B / 4;
  const double want_l = LPN * avg / 3.5;
  int rpw = 1;
  while (rpw < 8 && 64 / (rpw * 2) >= LPN && 64.0 / (rpw * 2) >= want_l) rpw *= 2;
  static const int rpw_env = [] {  // N2V2R_SPMM_RPW: rows per wave override (tuning runs)
    const char* s = getenv("N2V2R_SPMM_RPW");
    return s ? atoi(s) : 0;
  }();
  if (rpw_env == 1 || rpw_env == 2 || rpw_env == 4 || rpw_env == 8) rpw = rpw_env;
  switch (rpw) {
    case 8: if constexpr (64 / 8 >= LPN) { launch_spmm_t<B, 8>(args, stream); break; } [[fallthrough]];
    case 4: if constexpr (64 / 4 >= LPN) { launch_spmm_t<B, 4>(args, stream); break; } [[fallthrough]];
    case 2: launch_spmm_t<B, 2>(args, stream); break;
    default: launch_spmm_t<B, 1>(args, stream); break;
  }
}

extern "C" hipError_t n2v2r_launch_spmm(const SpmmArgs& args_in, int B, hipStream_t stream) {
  if (args_in.split && (B != 8 || args_in.sum || args_in.K > 8)) return hipErrorInvalidValue;
  SpmmArgs args = args_in;
  // the XCD split lives in the pipelined kernel; other b = 8 forms (A/B switches) write the
  // same per-layer outputs with grid.y = layer
  if (args.split && (!spmm8_pipelined() || spmm8_form() != 0)) args.split = 0;
  if (B == 8)
    launch_spmm_b<8>(args, stream);
  else if (B == 16)
    launch_spmm_b<16>(args, stream);
  else if (B == 32)
    launch_spmm_b<32>(args, stream);
  else if (B == 64)
    launch_spmm_b<64>(args, stream);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// ---- XCD-local column blocks (b = 8, panels larger than the L2s) -------------------------
// At N = 1M a b = 8 panel is 32 MB: it lives in the Infinity Cache, and every 32-B gather
// pulls a whole line over the fabric, so the gathers run at Infinity-Cache line bandwidth.
// The column-block form splits each layer's columns into CB_NB = 8 equal ranges and keeps one
// CSR per range (same row order, entries of a row in their original order).  Workgroup i runs
// on XCD i mod 8 (round-robin dispatch), so XCD j only gathers from panel rows of column block
// j (N/8 x 32 B = 4 MB at N = 1M): the gathers hit that XCD's L2.  Each block writes its own
// partial output (N x 8 fp32); cb_reduce sums the partials in fixed block order (then layer
// order), so the result is deterministic.  Extra traffic: 2 x 8 x N x 32 B of partials per
// layer launch.
// b = 8 row accumulation for the column blocks: block rows are short (N avg-deg / 8 entries),
// so the index loads of two group-widths are issued together before the gathers (one
// index -> gather latency per 2L entries instead of per L).  Same per-lane entry order as
// spmm_row_accumulate<8, RPW>.
template <int RPW>
__device__ __forceinline__ void cb_row_accumulate(const CsrBlk& A, const float* __restrict__ X,
                                                  int64_t ldx, int64_t row, bool row_ok,
                                                  int lane, f32x4& acc) {
  constexpr int L = 64 / RPW;
  constexpr int NPS = L / 2;  // panel rows per step (2 lanes per 32-B panel row)
  const int g = lane / L;
  const int li = lane % L;
  const int sub = li & 1;
  const int srcbase = g * L + (li >> 1);
  int64_t beg = 0, end = 0;
  if (row_ok) {
    beg = A.base + A.rp[row];
    end = A.base + A.rp[row + 1];
  }
  const int64_t len = end - beg;
  int64_t maxlen = len;
#pragma unroll
  for (int m = L; m < 64; m <<= 1) {
    const int64_t o = __shfl_xor(maxlen, m, 64);
    maxlen = o > maxlen ? o : maxlen;
  }
  for (int64_t off = 0; off < maxlen; off += 2 * L) {
    int cv[2] = {0, 0};
    float vv[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t p = off + u * L + li;
      if (p < len) {
        cv[u] = A.indices[beg + p];
        vv[u] = A.unit ? 1.f : A.data[beg + p];
      }
    }
    const int64_t rem = maxlen - off;
    const int nn = (int)(rem < 2 * L ? rem : 2 * L);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s * NPS >= nn) break;
      const int u = s >> 1;  // L / NPS = 2 steps per group-width
      const int c0 = __shfl(cv[u], srcbase + (s & 1) * NPS, 64);
      const float v0 = __shfl(vv[u], srcbase + (s & 1) * NPS, 64);
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(X + (int64_t)c0 * ldx + sub * 4);
      acc += v0 * x0;
    }
  }
}

// Two row groups of one column block at once (the tiled kernel): both groups' row pointers,
// then both groups' first two group-widths of column indices, then all their gathers, issued
// as batches -- clamped addresses and zero weights instead of guarded loads, so no load waits
// behind a branch (entries past a row's end gather panel row `beg` or 0 with weight 0: the
// sums are bit-identical).  Rows longer than 2L entries finish in a plain loop.
template <int RPW>
__device__ __forceinline__ void cb_rows2_accumulate(const CsrBlk& A, const float* __restrict__ X,
                                                    int64_t ldx, int64_t rowA, bool okA,
                                                    int64_t rowB, bool okB, int lane,
                                                    f32x4& accA, f32x4& accB) {
  constexpr int L = 64 / RPW;
  constexpr int NPS = L / 2;
  const int g = lane / L;
  const int li = lane % L;
  const int sub = li & 1;
  const int srcbase = g * L + (li >> 1);
  const int64_t rA = okA ? rowA : 0, rB = okB ? rowB : 0;
  const int32_t a0 = A.rp[rA], a1 = A.rp[rA + 1], b0 = A.rp[rB], b1 = A.rp[rB + 1];
  const int64_t begA = A.base + a0, begB = A.base + b0;
  const int64_t lenA = okA ? (int64_t)(a1 - a0) : 0, lenB = okB ? (int64_t)(b1 - b0) : 0;
  int64_t mx = lenA > lenB ? lenA : lenB;
#pragma unroll
  for (int m = L; m < 64; m <<= 1) {
    const int64_t o = __shfl_xor(mx, m, 64);
    mx = o > mx ? o : mx;
  }
  // first 2L entries of both rows, unconditionally (index 0 of the block's entries when past
  // the end; A.nnz >= 1 whenever any row of the block has an entry, else mx == 0 below)
  int cA[2], cB[2];
  float vA[2], vB[2];
  if (mx > 0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t p = u * L + li;
      const int64_t qa = p < lenA ? begA + p : A.base;
      const int64_t qb = p < lenB ? begB + p : A.base;
      cA[u] = A.indices[qa];
      cB[u] = A.indices[qb];
      vA[u] = p < lenA ? (A.unit ? 1.f : A.data[qa]) : 0.f;
      vB[u] = p < lenB ? (A.unit ? 1.f : A.data[qb]) : 0.f;
    }
    f32x4 xa[4], xb[4];
    float wa[4], wb[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int u = s >> 1;
      const int src = srcbase + (s & 1) * NPS;
      const int ca = __shfl(cA[u], src, 64), cb = __shfl(cB[u], src, 64);
      wa[s] = __shfl(vA[u], src, 64);
      wb[s] = __shfl(vB[u], src, 64);
      xa[s] = *reinterpret_cast<const f32x4*>(X + (int64_t)ca * ldx + sub * 4);
      xb[s] = *reinterpret_cast<const f32x4*>(X + (int64_t)cb * ldx + sub * 4);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      accA += wa[s] * xa[s];
      accB += wb[s] * xb[s];
    }
  }
  // long rows: the rest one group-width at a time
  for (int64_t off = 2 * L; off < mx; off += L) {
    const int64_t p = off + li;
    const int ca = p < lenA ? A.indices[begA + p] : 0;
    const float va = p < lenA ? (A.unit ? 1.f : A.data[begA + p]) : 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int src = srcbase + s * NPS;
      const int c0 = __shfl(ca, src, 64);
      const float w0 = __shfl(va, src, 64);
      accA += w0 * *reinterpret_cast<const f32x4*>(X + (int64_t)c0 * ldx + sub * 4);
    }
    const int cb = p < lenB ? A.indices[begB + p] : 0;
    const float vb = p < lenB ? (A.unit ? 1.f : A.data[begB + p]) : 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int src = srcbase + s * NPS;
      const int c1 = __shfl(cb, src, 64);
      const float w1 = __shfl(vb, src, 64);
      accB += w1 * *reinterpret_cast<const f32x4*>(X + (int64_t)c1 * ldx + sub * 4);
    }
  }
}

template <int RPW>
__global__ __launch_bounds__(256) void spmm8_cb_kernel(SpmmCbArgs a) {
  constexpr int L = 64 / RPW;
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x & (CB_NB - 1);
  const int64_t t = blockIdx.x / CB_NB;
  const int64_t nwg = gridDim.x / CB_NB;
  const CsrBlk& A = a.A[j];
  const int64_t n = A.n_rows;
  const int li = lane % L;
  float* __restrict__ P = a.P + (int64_t)j * a.pstride;
  const int64_t nw = nwg * (blockDim.x / 64);
  for (int64_t wid = t * (blockDim.x / 64) + (threadIdx.x >> 6); wid * RPW < n; wid += nw) {
    const int64_t row = wid * RPW + lane / L;
    const bool row_ok = row < n;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    cb_row_accumulate<RPW>(A, a.X, a.ldx, row, row_ok, lane, acc);
#pragma unroll
    for (int m = 2; m < L; m <<= 1) {
      acc.x += __shfl_xor(acc.x, m, 64);
      acc.y += __shfl_xor(acc.y, m, 64);
      acc.z += __shfl_xor(acc.z, m, 64);
      acc.w += __shfl_xor(acc.w, m, 64);
    }
    if (row_ok && li < 2) *reinterpret_cast<f32x4*>(P + row * 8 + li * 4) = acc;
  }
}

// rows per wave of the column-block kernels from the mean entries per block row (largest
// block): aim for ~3-4 gather steps of L/2 panel rows per row group
extern "C" int n2v2r_cb_rpw(const CsrBlk* A, int nb, int64_t n) {
  double avg = 0.0;
  for (int j = 0; j < nb; ++j) {
    const double m = (double)A[j].nnz / (double)(n > 0 ? n : 1);
    avg = m > avg ? m : avg;
  }
  int rpw = 1;
  while (rpw < 16 && 64.0 / (rpw * 2) / 2.0 * 3.5 >= avg) rpw *= 2;
  return rpw;
}

extern "C" hipError_t n2v2r_launch_spmm_cb(const SpmmCbArgs& a, hipStream_t stream) {
  const int64_t n = a.A[0].n_rows;
  int rpw = n2v2r_cb_rpw(a.A, CB_NB, n);
  static const int rpw_env = [] {  // N2V2R_CB_RPW / N2V2R_CB_WGS: tuning runs
    const char* s = getenv("N2V2R_CB_RPW");
    return s ? atoi(s) : 0;
  }();
  static const int wgs_env = [] {
    const char* s = getenv("N2V2R_CB_WGS");
    return s ? atoi(s) : 0;
  }();
  if (rpw_env == 1 || rpw_env == 2 || rpw_env == 4 || rpw_env == 8 || rpw_env == 16 ||
      rpw_env == 32)
    rpw = rpw_env;
  const int64_t waves = (n + rpw - 1) / rpw;
  int64_t per = (waves + 3) / 4;  // workgroups per block
  const int64_t cap = (wgs_env >= CB_NB ? wgs_env : N2V2R_SPMM_WGS) / CB_NB;
  if (per > cap) per = cap;
  if (per < 1) per = 1;
  dim3 grid((unsigned)(per * CB_NB));
#define CB_LAUNCH(R) hipLaunchKernelGGL((spmm8_cb_kernel<R>), grid, dim3(256), 0, stream, a)
  switch (rpw) {
    case 32: CB_LAUNCH(32); break;
    case 16: CB_LAUNCH(16); break;
    case 8: CB_LAUNCH(8); break;
    case 4: CB_LAUNCH(4); break;
    case 2: CB_LAUNCH(2); break;
    default: CB_LAUNCH(1); break;
  }
#undef CB_LAUNCH
  return hipGetLastError();
}

// ---- row tiles x column-block phases (b = 8, panels of 8-160 MB) ---------------------------
// The column-block SpMM above writes 8 partial outputs per layer launch (2 x 8 x 32 B per row
// of extra HBM traffic, then a reduce launch).  Here every workgroup owns a tile of rows whose
// accumulators stay in LDS (tile x 32 B: 62.5 KB at N = 1M with 2 workgroups per CU) and walks
// the column blocks in a fixed order 0..7 (the phases), gathering only from panel block p in
// phase p.  All workgroups start together and their rows carry equal work (ER / uniform
// graphs), so at any time the chip gathers from one 4 MB panel block, which every XCD's L2
// holds: the gathers hit L2 as in the column-block form, and each output row is written once.
// Sum mode (stage 2) accumulates the K layers into one output; otherwise (stage 1) each layer's
// output is written after its 8 phases.  Each row belongs to one wave (fixed row groups), so
// the LDS read-modify-writes need no barrier or atomic; per row the order is (layer, block,
// entry) -- deterministic.

// PAIR = 0 (N2V2R_TILE_FLAT=0; the flat-window kernel below is the default tiled form): one
// row group per wave step (cb_row_accumulate), 2 workgroups (32 waves) per CU.  PAIR = 2 (N2V2R_TILE_PAIR=2, A/B): two row groups per step with clamped batched loads
// (two load chains per wave, cb_rows2_accumulate), 1 workgroup (16 waves) per CU with twice the
// rows: cfg4 0.815 vs 0.795 ms per stage launch.  A one-group clamped form at 32 waves per CU
// spilled 14-18 VGPRs (64-register cap) and ran 0.995 ms.
template <int RPW, int PAIR>
__global__ __launch_bounds__(1024, PAIR == 2 ? 4 : 8) void spmm8_tile_kernel(SpmmTileArgs a) {
  constexpr int L = 64 / RPW;
  extern __shared__ f32x4 tacc[];  // [tile_rows][2]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nwave = blockDim.x >> 6;
  const int li = lane % L;
  const int64_t r0 = (int64_t)blockIdx.x * a.tile_rows;
  const int64_t rem = a.n - r0;
  const int nrows = (int)(rem < a.tile_rows ? rem : a.tile_rows);
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  for (int grp = wave; grp * RPW < nrows; grp += nwave) {
    const int lr = grp * RPW + lane / L;
    if (lr < nrows && li < 2) tacc[lr * 2 + li] = zero;
  }
  for (int k = 0; k < a.K; ++k) {
    const float* X = a.X[k];
    for (int p = 0; p < a.nb; ++p) {
      const CsrBlk A = a.blk[k * a.nb + p];
      // PAIR row groups per step (grp, grp + nwave): PAIR independent load chains per wave
      for (int grp = wave; grp * RPW < nrows; grp += (PAIR == 2 ? 2 : 1) * nwave) {
        const int lrA = grp * RPW + lane / L, lrB = lrA + nwave * RPW;
        const bool okA = lrA < nrows, okB = PAIR == 2 && lrB < nrows;
        f32x4 accA = zero, accB = zero;
        if constexpr (PAIR == 0)
          cb_row_accumulate<RPW>(A, X, a.ldx, r0 + lrA, okA, lane, accA);
        else
          cb_rows2_accumulate<RPW>(A, X, a.ldx, r0 + lrA, okA, r0 + lrB, okB, lane, accA, accB);
#pragma unroll
        for (int m = 2; m < L; m <<= 1) {
          accA.x += __shfl_xor(accA.x, m, 64);
          accA.y += __shfl_xor(accA.y, m, 64);
          accA.z += __shfl_xor(accA.z, m, 64);
          accA.w += __shfl_xor(accA.w, m, 64);
          if constexpr (PAIR == 2) {
            accB.x += __shfl_xor(accB.x, m, 64);
            accB.y += __shfl_xor(accB.y, m, 64);
            accB.z += __shfl_xor(accB.z, m, 64);
            accB.w += __shfl_xor(accB.w, m, 64);
          }
        }
        if (okA && li < 2) tacc[lrA * 2 + li] += accA;
        if (PAIR == 2 && okB && li < 2) tacc[lrB * 2 + li] += accB;
      }
      // the workgroup's waves move to the next panel block together (drifting waves would
      // want several blocks in L2 at once); each wave only touches its own rows' LDS entries
      __syncthreads();
    }
    if (!a.sum || k == a.K - 1) {
      float* Y = a.Y[a.sum ? 0 : k];
      for (int grp = wave; grp * RPW < nrows; grp += nwave) {
        const int lr = grp * RPW + lane / L;
        if (lr < nrows && li < 2) {
          *reinterpret_cast<f32x4*>(Y + (r0 + lr) * a.ldy + li * 4) = tacc[lr * 2 + li];
          tacc[lr * 2 + li] = zero;
        }
      }
    }
  }
}

// Packed flat windows (form 1): a wave owns windows of CB_WIN = 32 rows of the tile; a window's
// entries in column block p are one contiguous run of the block's index array (rows are in
// order), so the wave walks that run 32 entries per step -- lane pair i takes entry i, reads its
// packed word (row in window, column in block), gathers the 32-B panel row as two 16-B halves
// and stages weight x row in a 1-KB per-wave LDS slot; then lane pair r (owner of window row r)
// adds the staged entries of its row in entry order to a register accumulator, and after the
// window's last step adds that to the row's LDS accumulator.  Every lane gathers an entry
// whatever the row lengths are (the row-group form idles the lanes of short rows: a block row
// averages 6 entries at cfg4, the longest of a 16-row group ~12), and a window reads its row
// pointers with one load.  No atomics: one wave owns each window, so every sum has a fixed
// order (per row: layer, block, entry).  Index words and gathers of up to 4 steps are issued as
// one batch.  (A first form added every entry with ds_add_f32 into the row accumulators: 4.4 vs
// 0.8 ms per cfg4 stage launch -- LDS float atomics on shared addresses serialise.)  Measured
// at cfg4: 0.896 ms per stage launch with 8 column blocks (4 MB panel blocks: 31 % of the
// gathers miss L2), 0.748 ms with 16 (2 MB blocks; the default), against 0.807 / 0.923 ms for
// the row-group form at 8 / 16 blocks, whose rows get shorter with every block.
// a wave-uniform pointer loaded from memory, moved to SGPRs and tagged as global: loads through
// it become global_load with a scalar base (a flat pointer's loads count on lgkmcnt too, so
// every wait for them would also wait for the LDS traffic)
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* uniform_global(const T* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const __attribute__((address_space(1))) T*)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
  return ((int64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

// NS steps of 32 entries of one window: index words and gathers of all NS steps issued as
// straight-line batches, then per step: stage, and the row owners fold their entries
// NTL: the index / value stream loaded non-temporally (so it does not displace panel lines in
// L2; N2V2R_FLAT_NT=1, A/B)
template <int NS, bool UNIT, bool NTL, bool FOLD = true>
__device__ __forceinline__ void flat_steps(const __attribute__((address_space(1))) int32_t* ind,
                                           const __attribute__((address_space(1))) float* dat,
                                           int64_t beg, int off, int left,
                                           const __attribute__((address_space(1))) float* Xb,
                                           uint32_t ldx, int32_t cmask, int pr, int sub,
                                           int rs, int re, f32x4* stage, f32x4& acc) {
  int wd[NS];
  float v[NS];
  f32x4 x[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int q = u * 32 + pr;
    const int64_t e = beg + off + (q < left ? q : 0);
    if constexpr (NTL) {
      wd[u] = __builtin_nontemporal_load(ind + e);
      v[u] = UNIT ? 1.f : __builtin_nontemporal_load(dat + e);
    } else {
      wd[u] = ind[e];
      v[u] = UNIT ? 1.f : dat[e];
    }
  }
#pragma unroll
  for (int u = 0; u < NS; ++u)
    x[u] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
        Xb + ((uint32_t)(wd[u] & cmask) * ldx + sub * 4));
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    stage[pr * 2 + sub] = v[u] * x[u];  // entries past the end are never read
    if constexpr (!FOLD) {  // timing probe (N2V2R_FLAT_NOFOLD=1): wrong sums, no fold loop
      acc += stage[pr * 2 + sub];
      continue;
    }
    const int s0 = off + u * 32;
    const int lo = (rs > s0 ? rs : s0) - s0;
    const int hi = (re < s0 + 32 ? re : s0 + 32) - s0;
    for (int j = lo; j < hi; ++j) acc += stage[j * 2 + sub];
  }
}

template <bool NTL, bool FOLD = true>
__global__ __launch_bounds__(1024, 8) void spmm8_flat_kernel(SpmmTileArgs a) {
  // [tile_rows][8] row accumulators, then a 1-KB staging slot per wave
  extern __shared__ float tacf[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwave = blockDim.x >> 6;
  const int pr = lane >> 1, sub = lane & 1;
  const int64_t r0 = (int64_t)blockIdx.x * a.tile_rows;
  const int64_t rem = a.n - r0;
  const int nrows = (int)(rem < a.tile_rows ? rem : a.tile_rows);
  const int nwin = (nrows + CB_WIN - 1) / CB_WIN;
  const uint32_t ldx = (uint32_t)a.ldx;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4* tacc = reinterpret_cast<f32x4*>(tacf);
  f32x4* stage = reinterpret_cast<f32x4*>(tacf + (size_t)a.tile_rows * 8) + wave * 64;
  // zero / write back by the same window -> wave map as the adds (no barrier needed).  Measured
  // and not kept (cfg4 layer launch 0.367 ms): windows handed out per phase from an LDS
  // counter (0.557 ms), the next window's row pointers loaded before the current window's
  // entries (0.367 ms, flat); 512-thread workgroups with half the tile rows, 4 per CU
  // (0.448 ms)
  for (int w = wave; w < nwin; w += nwave) {
    const int lr = w * CB_WIN + pr;
    if (lr < nrows) tacc[lr * 2 + sub] = zero;
  }
  for (int k = 0; k < a.K; ++k) {
    const float* X = a.X[k];
    for (int p = 0; p < a.nb; ++p) {
      const CsrBlk& A = a.blk[k * a.nb + p];
      const int cbits = __builtin_amdgcn_readfirstlane(A.cbits);
      const int unit = __builtin_amdgcn_readfirstlane(A.unit);
      const auto rp = uniform_global(A.rp);
      const auto ind = uniform_global(A.indices);
      const auto dat = uniform_global(A.data);
      const int64_t base = uniform_i64(A.base);
      const int64_t col0 = uniform_i64(A.col0);
      const int32_t cmask = (1 << cbits) - 1;
      const auto Xb = uniform_global(X + col0 * a.ldx);
      for (int w = wave; w < nwin; w += nwave) {
        const int wr = w * CB_WIN;
        const int we = wr + CB_WIN < nrows ? wr + CB_WIN : nrows;
        // the window's row boundaries: lane pair r holds rows wr + r's [rs, re)
        const int rr = wr + pr < we ? wr + pr : we;
        const int32_t ps = rp[r0 + rr];
        const int32_t pe = rp[r0 + (wr + pr < we ? wr + pr + 1 : we)];
        const int32_t e0 = __builtin_amdgcn_readfirstlane(ps);
        const int len = __builtin_amdgcn_readlane(pe, 2 * (we - wr - 1)) - e0;
        const int rs = ps - e0, re = pe - e0;
        const int64_t beg = base + e0;
        f32x4 acc = zero;
#define FLAT_STEPS(U)                                                                          \
  for (int off = 0; off < len; off += 128) {                                                   \
    const int left = len - off;                                                                \
    if (left > 96)                                                                             \
      flat_steps<4, U, NTL, FOLD>(ind, dat, beg, off, left, Xb, ldx, cmask, pr, sub, rs, re, stage, acc); \
    else if (left > 64)                                                                        \
      flat_steps<3, U, NTL, FOLD>(ind, dat, beg, off, left, Xb, ldx, cmask, pr, sub, rs, re, stage, acc); \
    else if (left > 32)                                                                        \
      flat_steps<2, U, NTL, FOLD>(ind, dat, beg, off, left, Xb, ldx, cmask, pr, sub, rs, re, stage, acc); \
    else                                                                                       \
      flat_steps<1, U, NTL, FOLD>(ind, dat, beg, off, left, Xb, ldx, cmask, pr, sub, rs, re, stage, acc); \
  }
        if (unit) {
          FLAT_STEPS(true)
        } else {
          FLAT_STEPS(false)
        }
#undef FLAT_STEPS
        if (wr + pr < we) tacc[(wr + pr) * 2 + sub] += acc;
      }
      __syncthreads();  // all waves on the same panel block (see spmm8_tile_kernel)
    }
    if (!a.sum || k == a.K - 1) {
      float* Y = a.Y[a.sum ? 0 : k];
      for (int w = wave; w < nwin; w += nwave) {
        const int lr = w * CB_WIN + pr;
        if (lr < nrows) {
          *reinterpret_cast<f32x4*>(Y + (r0 + lr) * a.ldy + sub * 4) = tacc[lr * 2 + sub];
          tacc[lr * 2 + sub] = zero;
        }
      }
    }
  }
}

// ---- the packed flat-window form at b = 16 ---------------------------------------------------
// The same windows, column-block phases and packed entries as spmm8_flat_kernel, with 64-B panel
// rows: a lane quad (q = lane / 4) gathers one entry's row as four 16-B pieces, so a wave step
// takes 16 entries, and quad q owns window rows q and q + 16 (two register accumulators).  An
// entry still costs one scattered line access (the bound of the b = 8 form) but
// carries 16 columns instead of 8, so a vector application costs about half the line accesses.
template <int NS, bool UNIT>
__device__ __forceinline__ void flat16_steps(const __attribute__((address_space(1))) int32_t* ind,
                                             const __attribute__((address_space(1))) float* dat,
                                             int64_t beg, int off, int left,
                                             const __attribute__((address_space(1))) float* Xb,
                                             uint32_t ldx, int32_t cmask, int q, int sub, int rs0,
                                             int re0, int rs1, int re1, f32x4* stage, f32x4& acc0,
                                             f32x4& acc1) {
  int wd[NS];
  float v[NS];
  f32x4 x[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int t = u * 16 + q;
    const int64_t e = beg + off + (t < left ? t : 0);
    wd[u] = ind[e];
    v[u] = UNIT ? 1.f : dat[e];
  }
#pragma unroll
  for (int u = 0; u < NS; ++u)
    x[u] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
        Xb + ((uint32_t)(wd[u] & cmask) * ldx + sub * 4));
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    stage[q * 4 + sub] = v[u] * x[u];  // entries past the end are never read
    const int s0 = off + u * 16;
    const int lo0 = (rs0 > s0 ? rs0 : s0) - s0, hi0 = (re0 < s0 + 16 ? re0 : s0 + 16) - s0;
    for (int j = lo0; j < hi0; ++j) acc0 += stage[j * 4 + sub];
    const int lo1 = (rs1 > s0 ? rs1 : s0) - s0, hi1 = (re1 < s0 + 16 ? re1 : s0 + 16) - s0;
    for (int j = lo1; j < hi1; ++j) acc1 += stage[j * 4 + sub];
  }
}

__global__ __launch_bounds__(1024, 8) void spmm16_flat_kernel(SpmmTileArgs a) {
  // [tile_rows][16] row accumulators, then a 1-KB staging slot per wave
  extern __shared__ float tacf[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwave = blockDim.x >> 6;
  const int pr = lane >> 1;            // row-pointer lanes: pair pr holds window row pr
  const int q = lane >> 2, sub = lane & 3;  // entry / row-owner quad, 16-B piece
  const int64_t r0 = (int64_t)blockIdx.x * a.tile_rows;
  const int64_t rem = a.n - r0;
  const int nrows = (int)(rem < a.tile_rows ? rem : a.tile_rows);
  const int nwin = (nrows + CB_WIN - 1) / CB_WIN;
  const uint32_t ldx = (uint32_t)a.ldx;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4* tacc = reinterpret_cast<f32x4*>(tacf);
  f32x4* stage = reinterpret_cast<f32x4*>(tacf + (size_t)a.tile_rows * 16) + wave * 64;
  for (int w = wave; w < nwin; w += nwave) {
    const int lr = w * CB_WIN + q;
    if (lr < nrows) tacc[lr * 4 + sub] = zero;
    if (lr + 16 < nrows) tacc[(lr + 16) * 4 + sub] = zero;
  }
  for (int k = 0; k < a.K; ++k) {
    const float* X = a.X[k];
    for (int p = 0; p < a.nb; ++p) {
      const CsrBlk& A = a.blk[k * a.nb + p];
      const int cbits = __builtin_amdgcn_readfirstlane(A.cbits);
      const int unit = __builtin_amdgcn_readfirstlane(A.unit);
      const auto rp = uniform_global(A.rp);
      const auto ind = uniform_global(A.indices);
      const auto dat = uniform_global(A.data);
      const int64_t base = uniform_i64(A.base);
      const int64_t col0 = uniform_i64(A.col0);
      const int32_t cmask = (1 << cbits) - 1;
      const auto Xb = uniform_global(X + col0 * a.ldx);
      for (int w = wave; w < nwin; w += nwave) {
        const int wr = w * CB_WIN;
        const int we = wr + CB_WIN < nrows ? wr + CB_WIN : nrows;
        const int rr = wr + pr < we ? wr + pr : we;
        const int32_t ps = rp[r0 + rr];
        const int32_t pe = rp[r0 + (wr + pr < we ? wr + pr + 1 : we)];
        const int32_t e0 = __builtin_amdgcn_readfirstlane(ps);
        const int len = __builtin_amdgcn_readlane(pe, 2 * (we - wr - 1)) - e0;
        // this quad's rows q and q + 16: their [start, end) from the pointer lanes 2q, 2q + 32
        const int rs0 = __shfl(ps, 2 * q, 64) - e0, re0 = __shfl(pe, 2 * q, 64) - e0;
        const int rs1 = __shfl(ps, 2 * q + 32, 64) - e0, re1 = __shfl(pe, 2 * q + 32, 64) - e0;
        const int64_t beg = base + e0;
        f32x4 acc0 = zero, acc1 = zero;
#define FLAT16_STEPS(U)                                                                        \
  for (int off = 0; off < len; off += 48) {                                                    \
    const int left = len - off;                                                                \
    if (left > 32)                                                                             \
      flat16_steps<3, U>(ind, dat, beg, off, left, Xb, ldx, cmask, q, sub, rs0, re0, rs1, re1, \
                         stage, acc0, acc1);                                                   \
    else if (left > 16)                                                                        \
      flat16_steps<2, U>(ind, dat, beg, off, left, Xb, ldx, cmask, q, sub, rs0, re0, rs1, re1, \
                         stage, acc0, acc1);                                                   \
    else                                                                                       \
      flat16_steps<1, U>(ind, dat, beg, off, left, Xb, ldx, cmask, q, sub, rs0, re0, rs1, re1, \
                         stage, acc0, acc1);                                                   \
  }
        if (unit) {
          FLAT16_STEPS(true)
        } else {
          FLAT16_STEPS(false)
        }
#undef FLAT16_STEPS
        if (wr + q < we) tacc[(wr + q) * 4 + sub] += acc0;
        if (wr + q + 16 < we) tacc[(wr + q + 16) * 4 + sub] += acc1;
      }
      __syncthreads();  // all waves on the same panel block (see spmm8_tile_kernel)
    }
    if (!a.sum || k == a.K - 1) {
      float* Y = a.Y[a.sum ? 0 : k];
      for (int w = wave; w < nwin; w += nwave) {
        const int lr = w * CB_WIN + q;
        if (lr < nrows) {
          *reinterpret_cast<f32x4*>(Y + (r0 + lr) * a.ldy + sub * 4) = tacc[lr * 4 + sub];
          tacc[lr * 4 + sub] = zero;
        }
        if (lr + 16 < nrows) {
          *reinterpret_cast<f32x4*>(Y + (r0 + lr + 16) * a.ldy + sub * 4) =
              tacc[(lr + 16) * 4 + sub];
          tacc[(lr + 16) * 4 + sub] = zero;
        }
      }
    }
  }
}

// rows per tile for the tiled form: `wpc` workgroups (1024 threads each) per CU sharing its
// 160 KB of LDS (32 B of accumulators per row); a multiple of CB_WIN (the packed windows)
extern "C" int n2v2r_spmm_tile_rows(int64_t n, int ncu, int wpc) {
  int64_t t = (n + wpc * (int64_t)ncu - 1) / (wpc * (int64_t)ncu);
  t = (t + CB_WIN - 1) / CB_WIN * CB_WIN;
  const int64_t cap = (wpc == 1 ? 4096 : 2048);
  if (t > cap) t = cap;
  return (int)t;
}

extern "C" hipError_t n2v2r_launch_spmm_tile(const SpmmTileArgs& a, int rpw, hipStream_t stream) {
  if (a.K < 1 || a.K > 8 || a.tile_rows < 16 || a.n <= 0) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.n + a.tile_rows - 1) / a.tile_rows);
  if (a.b == 16) {  // 64 B of accumulators per row + a 1-KB staging slot per wave
    const size_t flds = sizeof(float) * 16 * (size_t)a.tile_rows + 16 * 1024;
    if (a.form != 1 || a.tile_rows % CB_WIN != 0 || flds > 80 * 1024) return hipErrorInvalidValue;
    static const bool fattr = [] {
      (void)hipFuncSetAttribute((const void*)spmm16_flat_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipGetLastError();
      return true;
    }();
    (void)fattr;
    hipLaunchKernelGGL(spmm16_flat_kernel, dim3(grid), dim3(1024), flds, stream, a);
    return hipGetLastError();
  }
  if (a.b != 0 && a.b != 8) return hipErrorInvalidValue;
  const size_t lds = sizeof(float) * 8 * (size_t)a.tile_rows;
  if (a.form < 0 || a.form > 2 || a.tile_rows % CB_WIN != 0) return hipErrorInvalidValue;
  if (a.form == 1) {  // + a 1-KB staging slot per wave
    const size_t flds = lds + 16 * 1024;
    static const bool fattr = [] {
      (void)hipFuncSetAttribute((const void*)spmm8_flat_kernel<false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipFuncSetAttribute((const void*)spmm8_flat_kernel<true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipGetLastError();
      return true;
    }();
    (void)fattr;
    static const bool ntl = [] {
      const char* e = getenv("N2V2R_FLAT_NT");
      return e && e[0] == '1';
    }();
    if (flds > 80 * 1024) return hipErrorInvalidValue;
    static const bool nofold = [] {  // timing probe only: the fold loop skipped, sums wrong
      const char* e = getenv("N2V2R_FLAT_NOFOLD");
      if (e && e[0] == '1')
        (void)hipFuncSetAttribute((const void*)spmm8_flat_kernel<false, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      return e && e[0] == '1';
    }();
    if (nofold)
      hipLaunchKernelGGL((spmm8_flat_kernel<false, false>), dim3(grid), dim3(1024), flds, stream, a);
    else if (ntl)
      hipLaunchKernelGGL(spmm8_flat_kernel<true>, dim3(grid), dim3(1024), flds, stream, a);
    else
      hipLaunchKernelGGL(spmm8_flat_kernel<false>, dim3(grid), dim3(1024), flds, stream, a);
    return hipGetLastError();
  }
  if (lds > 64 * 1024) {
    static bool attr = false;
    if (!attr) {
      for (const void* f : {(const void*)spmm8_tile_kernel<32, 2>, (const void*)spmm8_tile_kernel<16, 2>,
                            (const void*)spmm8_tile_kernel<8, 2>, (const void*)spmm8_tile_kernel<4, 2>,
                            (const void*)spmm8_tile_kernel<2, 2>})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipGetLastError();
      attr = true;
    }
  }
#define TILE_LAUNCH(R)                                                                     \
  if (a.form == 2)                                                                         \
    hipLaunchKernelGGL((spmm8_tile_kernel<R, 2>), dim3(grid), dim3(1024), lds, stream, a); \
  else                                                                                     \
    hipLaunchKernelGGL((spmm8_tile_kernel<R, 0>), dim3(grid), dim3(1024), lds, stream, a)
  switch (rpw) {
    case 32: TILE_LAUNCH(32); break;
    case 16: TILE_LAUNCH(16); break;
    case 8: TILE_LAUNCH(8); break;
    case 4: TILE_LAUNCH(4); break;
    default: TILE_LAUNCH(2); break;
  }
#undef TILE_LAUNCH
  return hipGetLastError();
}

// out[r] = colscale .* sum_{p < nparts} P[p][r] (rows of 8 fp32, fixed part order)
// out row r = sum_p P[p] row r, p in order (the fixed order keeps results bit-identical to the
// column-block partials' summation in every form).  NP > 0: all NP loads of a thread issued
// before the first add (the runtime-count loop waited out one memory round trip per partial:
// ~1.2 TB/s at N = 1M); NP = 0: any count.
template <int NP>
__global__ __launch_bounds__(256) void cb_reduce_kernel(const float* __restrict__ P, int nparts,
                                                        int64_t pstride, int64_t n,
                                                        float* __restrict__ out, int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one float4 each
  if (i >= n * 2) return;
  const int64_t r = i >> 1;
  const int h = (int)(i & 1);
  const float* src = P + r * 8 + h * 4;
  f32x4 s;
  if constexpr (NP > 0) {
    f32x4 v[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) v[p] = *reinterpret_cast<const f32x4*>(src + p * pstride);
    s = v[0];
#pragma unroll
    for (int p = 1; p < NP; ++p) s += v[p];
  } else {
    s = *reinterpret_cast<const f32x4*>(src);
    for (int p = 1; p < nparts; ++p) s += *reinterpret_cast<const f32x4*>(src + p * pstride);
  }
  *reinterpret_cast<f32x4*>(out + r * ldo + h * 4) = s;
}

extern "C" hipError_t n2v2r_launch_cb_reduce(const float* P, int nparts, int64_t pstride,
                                             int64_t n, float* out, int64_t ldo,
                                             hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t thr = n * 2;
  const dim3 g((unsigned)((thr + 255) / 256));
  // the runtime-count loop by default: the stage-1 reduces run beside the next layer's block
  // launch, where the unrolled form's burst of loads slowed that launch more than it saved
  // (cfg4 2353 vs 2205 ms per step); unrolled for the stage-2 sum only: 2209 vs 2206.
  // N2V2R_CB_REDUCE_UNROLL=1 / 2: always / stage-2 sums (K x 8 partials) only (A/B).
  static const int unroll_mode = [] {
    const char* e = getenv("N2V2R_CB_REDUCE_UNROLL");
    return e ? atoi(e) : 0;
  }();
  const bool unrolled = unroll_mode == 1 || (unroll_mode == 2 && nparts >= 16);
  if (!unrolled)
    hipLaunchKernelGGL(cb_reduce_kernel<0>, g, dim3(256), 0, stream, P, nparts, pstride, n, out, ldo);
  else if (nparts == 8)
    hipLaunchKernelGGL(cb_reduce_kernel<8>, g, dim3(256), 0, stream, P, nparts, pstride, n, out, ldo);
  else if (nparts == 16)
    hipLaunchKernelGGL(cb_reduce_kernel<16>, g, dim3(256), 0, stream, P, nparts, pstride, n, out, ldo);
  else if (nparts == 24)
    hipLaunchKernelGGL(cb_reduce_kernel<24>, g, dim3(256), 0, stream, P, nparts, pstride, n, out, ldo);
  else
    hipLaunchKernelGGL(cb_reduce_kernel<0>, g, dim3(256), 0, stream, P, nparts, pstride, n, out, ldo);
  return hipGetLastError();
}

// Column-block split, step 1: cnt[j * n + r] = entries of row r in column block j
// (block j = columns [j * cw, (j + 1) * cw)); NB blocks (8, 16 or 32).
template <int NB>
__global__ void cb_count_kernel(CsrDev A, int64_t cw, int32_t* __restrict__ cnt) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= A.n_rows) return;
  int c[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) c[j] = 0;
  for (int64_t p = A.indptr[r]; p < A.indptr[r + 1]; ++p) {
    const int jb = (int)(A.indices[p] / cw);
#pragma unroll
    for (int j = 0; j < NB; ++j) c[j] += jb == j;
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) cnt[(int64_t)j * A.n_rows + r] = c[j];
}

// step 2 (after the host scan): scatter each row's entries to rp[j][r] + running count,
// keeping their order inside the row.
// cbits > 0: packed entries ((r % CB_WIN) << cbits | (col - block start)) for the flat form.
template <int NB>
__global__ void cb_fill_kernel(CsrDev A, int64_t cw, const int64_t* __restrict__ rp,
                               int32_t* __restrict__ idx, float* __restrict__ dat, int cbits) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= A.n_rows) return;
  int64_t pos[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) pos[j] = rp[(int64_t)j * (A.n_rows + 1) + r];
  for (int64_t p = A.indptr[r]; p < A.indptr[r + 1]; ++p) {
    const int32_t col = A.indices[p];
    const int jb = (int)(col / cw);
    int64_t q = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (jb == j) q = pos[j]++;
    idx[q] = cbits ? (int32_t)(((r % CB_WIN) << cbits) | (col - (int64_t)jb * cw)) : col;
    if (!A.unit) dat[q] = A.data[p];
  }
}

// Row pointers of the column blocks from the counts, on the GPU: an exclusive scan of the
// counts flattened block-major (cnt[j][r]) gives every entry's absolute position in the
// block-major entry array, rp[j][r] (int64, [nb][n + 1]); rp[j][n] = rp[j + 1][0] (nnz for the
// last block); rp32[j][r] = rp[j][r] - rp[j][0] (int32, relative to the block's base).
#define SCAN_T 256
#define SCAN_IT 8
#define SCAN_TILE (SCAN_T * SCAN_IT)

__global__ __launch_bounds__(SCAN_T) void scan_tile_sums_kernel(const int32_t* __restrict__ in,
                                                                int64_t len,
                                                                int64_t* __restrict__ tsum) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  int64_t s = 0;
#pragma unroll
  for (int u = 0; u < SCAN_IT; ++u) {
    const int64_t i = base + u * SCAN_T + threadIdx.x;
    if (i < len) s += in[i];
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  __shared__ int64_t ws[SCAN_T / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < SCAN_T / 64; ++w) t += ws[w];
    tsum[blockIdx.x] = t;
  }
}

// exclusive scan of the tile sums in place, one workgroup, chunks of 1024 with a carry
__global__ __launch_bounds__(1024) void scan_tile_offsets_kernel(int64_t* __restrict__ tsum,
                                                                 int64_t ntiles) {
  __shared__ int64_t sh[1024];
  int64_t carry = 0;
  for (int64_t c0 = 0; c0 < ntiles; c0 += 1024) {
    const int64_t i = c0 + threadIdx.x;
    const int64_t v = i < ntiles ? tsum[i] : 0;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int64_t t = threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
      __syncthreads();
      sh[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < ntiles) tsum[i] = carry + sh[threadIdx.x] - v;
    const int64_t tot = sh[1023];
    __syncthreads();
    carry += tot;
  }
}

// exclusive positions of one tile: thread-local running sums over SCAN_IT consecutive counts,
// a workgroup scan of the thread sums, the tile's offset; element e = j * n + r -> rp[j][r]
__global__ __launch_bounds__(SCAN_T) void scan_tile_write_kernel(const int32_t* __restrict__ in,
                                                                 int64_t n, int nb,
                                                                 const int64_t* __restrict__ toff,
                                                                 int64_t* __restrict__ rp) {
  const int64_t len = (int64_t)nb * n;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_IT;
  int32_t v[SCAN_IT];
  int64_t s = 0;
#pragma unroll
  for (int u = 0; u < SCAN_IT; ++u) {
    v[u] = base + u < len ? in[base + u] : 0;
    s += v[u];
  }
  __shared__ int64_t sh[SCAN_T];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {
    const int64_t t = threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
    __syncthreads();
    sh[threadIdx.x] += t;
    __syncthreads();
  }
  int64_t run = toff[blockIdx.x] + sh[threadIdx.x] - s;
#pragma unroll
  for (int u = 0; u < SCAN_IT; ++u) {
    const int64_t e = base + u;
    if (e < len) {
      const int64_t j = e / n, r = e - j * n;
      rp[j * (n + 1) + r] = run;
    }
    run += v[u];
  }
}

__global__ void cb_rp_finish_kernel(int64_t* __restrict__ rp, int32_t* __restrict__ rp32,
                                    int64_t n, int nb, int64_t nnz) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)nb * (n + 1)) return;
  const int64_t j = e / (n + 1), r = e - j * (n + 1);
  int64_t v;
  if (r == n) v = j + 1 < nb ? rp[(j + 1) * (n + 1)] : nnz;
  else v = rp[e];
  if (r == n) rp[e] = v;
  rp32[e] = (int32_t)(v - rp[j * (n + 1)]);
}

extern "C" hipError_t n2v2r_launch_cb_rowptrs(const int32_t* cnt, int64_t n, int nb, int64_t nnz,
                                              int64_t* tsum, size_t tsum_elems, int64_t* rp,
                                              int32_t* rp32, hipStream_t stream) {
  const int64_t len = (int64_t)nb * n;
  const int64_t ntiles = (len + SCAN_TILE - 1) / SCAN_TILE;
  if (ntiles < 1 || (size_t)ntiles > tsum_elems) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scan_tile_sums_kernel, dim3((unsigned)ntiles), dim3(SCAN_T), 0, stream, cnt,
                     len, tsum);
  hipLaunchKernelGGL(scan_tile_offsets_kernel, dim3(1), dim3(1024), 0, stream, tsum, ntiles);
  hipLaunchKernelGGL(scan_tile_write_kernel, dim3((unsigned)ntiles), dim3(SCAN_T), 0, stream, cnt,
                     n, nb, tsum, rp);
  const int64_t tot = (int64_t)nb * (n + 1);
  hipLaunchKernelGGL(cb_rp_finish_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     stream, rp, rp32, n, nb, nnz);
  return hipGetLastError();
}

extern "C" int64_t n2v2r_cb_scan_tiles(int64_t n, int nb) {
  return ((int64_t)nb * n + SCAN_TILE - 1) / SCAN_TILE;
}

extern "C" hipError_t n2v2r_launch_cb_count(const CsrDev& A, int64_t cw, int nb, int32_t* cnt,
                                            hipStream_t stream) {
  if (A.n_rows <= 0) return hipSuccess;
  const dim3 g((unsigned)((A.n_rows + 255) / 256));
  if (nb == 4) hipLaunchKernelGGL(cb_count_kernel<4>, g, dim3(256), 0, stream, A, cw, cnt);
  else if (nb == 8) hipLaunchKernelGGL(cb_count_kernel<8>, g, dim3(256), 0, stream, A, cw, cnt);
  else if (nb == 16) hipLaunchKernelGGL(cb_count_kernel<16>, g, dim3(256), 0, stream, A, cw, cnt);
  else if (nb == 32) hipLaunchKernelGGL(cb_count_kernel<32>, g, dim3(256), 0, stream, A, cw, cnt);
  else if (nb == 64) hipLaunchKernelGGL(cb_count_kernel<64>, g, dim3(256), 0, stream, A, cw, cnt);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_cb_fill(const CsrDev& A, int64_t cw, int nb, const int64_t* rp,
                                           int32_t* idx, float* dat, int cbits,
                                           hipStream_t stream) {
  if (A.n_rows <= 0) return hipSuccess;
  const dim3 g((unsigned)((A.n_rows + 255) / 256));
#define FILL(NB) hipLaunchKernelGGL(cb_fill_kernel<NB>, g, dim3(256), 0, stream, A, cw, rp, idx, dat, cbits)
  if (nb == 4) FILL(4);
  else if (nb == 8) FILL(8);
  else if (nb == 16) FILL(16);
  else if (nb == 32) FILL(32);
  else if (nb == 64) FILL(64);
  else return hipErrorInvalidValue;
#undef FILL
  return hipGetLastError();
}

// Column sums of a CSR layer (DeDi, model.py:282-311): out[j] = sum_i A[i][j].  fp32
// atomics would make the order run-dependent, so the engine calls this on A^T (row sums of
// the transpose = column sums) when the layer is not symmetric.
__global__ void csr_row_sums_kernel(CsrDev A, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= A.n_rows) return;
  float s = 0.f;
  for (int64_t p = A.indptr[row] + lane; p < A.indptr[row + 1]; p += 64) s += A.data[p];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (lane == 0) out[row] = s;
}

extern "C" hipError_t n2v2r_launch_row_sums(const CsrDev& A, float* out, hipStream_t stream) {
  dim3 grid((unsigned)((A.n_rows + 3) / 4));
  hipLaunchKernelGGL(csr_row_sums_kernel, grid, dim3(256), 0, stream, A, out);
  return hipGetLastError();
}

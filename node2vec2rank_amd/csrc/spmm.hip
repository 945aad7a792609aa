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
#include <mutex>

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

template <int B, int RPW>
static void launch_spmm_t(const SpmmArgs& args, hipStream_t stream) {
  const int64_t n = args.A[0].n_rows;
  const int64_t waves = (n + RPW - 1) / RPW;
  int64_t wgs = (waves + 3) / 4;
  const int64_t cap = (int64_t)N2V2R_SPMM_WGS / (args.sum ? 1 : args.K);
  if (wgs > cap) wgs = cap;
  dim3 grid((unsigned)wgs, args.sum ? 1 : args.K);
  if constexpr (B == 8 && RPW >= 2) {
    if (args.split) grid = dim3((unsigned)N2V2R_SPMM_WGS, 1);
    hipLaunchKernelGGL((spmm8_pipe_kernel<RPW>), grid, dim3(256), 0, stream, args);
  } else {
    // the XCD split lives in the pipelined kernel; here the same per-layer outputs come from
    // grid.y = layer
    SpmmArgs a = args;
    a.split = 0;
    hipLaunchKernelGGL((spmm_csr_panel_kernel<B, RPW>), grid, dim3(256), 0, stream, a);
  }
}

// rows per wave from the mean row length: a row group of L lanes gathers L / (B/4) panel rows
// per step; aim for ~3-4 steps per row.
static int auto_rpw(const SpmmArgs& args, int B) {
  double avg = 0.0;
  int kk = args.sum ? args.K : args.K;
  for (int k = 0; k < kk; ++k) avg += (double)args.A[k].nnz / (double)(args.A[k].n_rows > 0 ? args.A[k].n_rows : 1);
  avg /= (kk > 0 ? kk : 1);
  const int LPN = B / 4;
  const double want_l = LPN * avg / 3.5;
  int rpw = 1;
  while (rpw < 8 && 64 / (rpw * 2) >= LPN && 64.0 / (rpw * 2) >= want_l) rpw *= 2;
  return rpw;
}

extern "C" int n2v2r_spmm_rpw(const SpmmArgs& args, int B) { return auto_rpw(args, B); }

template <int B>
static void launch_spmm_b(const SpmmArgs& args, hipStream_t stream) {
  constexpr int LPN = B / 4;
  const int rpw = args.rpw > 0 ? args.rpw : auto_rpw(args, B);
  switch (rpw) {
    case 8: if constexpr (64 / 8 >= LPN) { launch_spmm_t<B, 8>(args, stream); break; } [[fallthrough]];
    case 4: if constexpr (64 / 4 >= LPN) { launch_spmm_t<B, 4>(args, stream); break; } [[fallthrough]];
    case 2: launch_spmm_t<B, 2>(args, stream); break;
    default: launch_spmm_t<B, 1>(args, stream); break;
  }
}

extern "C" hipError_t n2v2r_launch_spmm(const SpmmArgs& args_in, int B, hipStream_t stream) {
  if (args_in.split && (B != 8 || args_in.sum || args_in.K > 8)) return hipErrorInvalidValue;
  const SpmmArgs& args = args_in;
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

// ---- row tiles x column-block phases (b = 8, panels beyond an XCD's L2) -------------------
// Every workgroup owns a tile of rows whose accumulators stay in LDS (tile x 32 B) and walks each
// layer's column blocks in a fixed order (the phases), gathering only from panel block p in
// phase p.  All workgroups start together and their rows carry equal work (ER / uniform graphs),
// so at any time the chip gathers from one panel block of <= 2 MB, which every XCD's L2 holds.
// Sum mode (stage 2) accumulates the K layers into one output; otherwise (stage 1) each layer's
// output is written after its phases.  Per row the order is (layer, block, entry): deterministic.
// (Round 2-3 forms measured against it and removed in round 4: 8 partial outputs per layer + a
// reduce launch, 2.2 s per cfg4 step; row groups per wave, 0.807 ms per stage launch at 8
// blocks; two row groups per step at one workgroup per CU, 0.815 ms)

// Packed flat windows: a wave owns windows of W = 2^wbits rows of the tile (32 at cfg4, 64 at
// cfg5's sparser blocks); a window's entries in column block p are one contiguous run of the
// block's index array (rows in order), located by two window offsets (scalar loads: the block
// keeps no per-row pointers).  The wave walks the run 32 entries per step -- lane pair i takes
// entry i, reads its packed word (row in window, column in block), gathers the 32-B panel row as
// two 16-B halves and stages weight x row in a 1-KB per-wave LDS slot.  Then, per step, the first
// lane pair of each row's segment (rows are in entry order and every entry names its row, so a
// segment starts where the row differs from the previous entry's: one bpermute and one ballot)
// sums the segment's staged entries in entry order and adds the sum to the row's LDS accumulator.
// Every lane gathers an entry whatever the row lengths are.  No atomics: one wave owns each
// window, so every sum has a fixed order (per row: layer, block, step, entry).  Index words and
// gathers of up to 4 steps are issued as one batch.  (A first form added every entry with
// ds_add_f32 into the row accumulators: 4.4 vs 0.8 ms per cfg4 stage launch -- LDS float atomics
// on shared addresses serialise.  Rounds 3-4 located each row's entries by per-row block
// pointers, [nb][N + 1] int32 read by every launch: 64 MB per cfg4 layer launch, 1.28 GB at
// cfg5, more than the index words there.)  Measured at cfg4 (round 3, row pointers): 0.896 ms per
// stage launch with 8 column blocks (4 MB panel blocks: 31 % of the gathers miss L2), 0.748 ms
// with 16 (2 MB blocks; the default), against 0.807 / 0.923 ms for a row-group form at 8 / 16
// blocks, whose rows get shorter with every block.
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

// NS steps of 32 entries of one window run: index words and gathers of all NS steps issued as
// straight-line batches, then per step: stage, and each row segment's first lane pair folds the
// segment into the row's accumulator (tw: the window's first row)
template <int NS, bool UNIT, bool NT>
__device__ __forceinline__ void flat_steps(const __attribute__((address_space(1))) int32_t* ind,
                                           const __attribute__((address_space(1))) float* dat,
                                           int64_t beg, int off, int left,
                                           const __attribute__((address_space(1))) float* Xb,
                                           uint32_t ldx, int32_t cmask, int cbits, int lane,
                                           f32x4* stage, f32x4* tw) {
  const int pr = lane >> 1, sub = lane & 1;
  int wd[NS];
  float v[NS];
  f32x4 x[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int q = u * 32 + pr;
    const int64_t e = beg + off + (q < left ? q : 0);
    wd[u] = NT ? __builtin_nontemporal_load(ind + e) : ind[e];
    v[u] = UNIT ? 1.f : (NT ? __builtin_nontemporal_load(dat + e) : dat[e]);
  }
#pragma unroll
  for (int u = 0; u < NS; ++u)
    x[u] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
        Xb + ((uint32_t)(wd[u] & cmask) * ldx + sub * 4));
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    stage[pr * 2 + sub] = v[u] * x[u];  // entries past the end are never read
    const int nval = left - u * 32;     // valid entries of this step (>= 1; may exceed 32)
    const int ri = wd[u] >> cbits;      // row in window
    const int rprev = __shfl(ri, lane - 2, 64);
    const bool start = pr < nval && (pr == 0 || rprev != ri);
    const unsigned long long m = __ballot(start);
    if (start) {
      const unsigned long long rest = pr == 31 ? 0ull : (m >> (2 * pr + 2));
      const int end = rest ? pr + 1 + (__builtin_ctzll(rest) >> 1) : (nval < 32 ? nval : 32);
      f32x4 acc = stage[pr * 2 + sub];
      for (int j = pr + 1; j < end; ++j) acc += stage[j * 2 + sub];
      tw[ri * 2 + sub] += acc;
    }
  }
}

// flat_steps for a register-resident window of 64 rows (spmm8_flat_kernel<true>): lane pair pr
// keeps rows pr (a0) and pr + 32 (a1), its half `sub`.  The segment sums are formed exactly as
// in flat_steps (same entries, same order); each then reaches its row's owner through the
// wave's staging slot, whose products are consumed by then: per half of the window, every lane
// pair zeroes its slot, the segment heads of that half write their sums into their rows' slots,
// and every owner adds its slot (0 for rows without entries in the step) -- no atomics, and
// each row's sum keeps its order, so the result is bit-identical to the LDS-resident form.
template <int NS, bool UNIT, bool NT>
__device__ __forceinline__ void flat_steps_v(const __attribute__((address_space(1))) int32_t* ind,
                                             const __attribute__((address_space(1))) float* dat,
                                             int64_t beg, int off, int left,
                                             const __attribute__((address_space(1))) float* Xb,
                                             uint32_t ldx, int32_t cmask, int cbits, int lane,
                                             f32x4* stage_, f32x4& a0, f32x4& a1) {
  const int pr = lane >> 1, sub = lane & 1;
  // every access to the slot volatile: lanes hand values to each other through it, so the
  // compiler may neither reorder these accesses nor forward a lane's own store to its load
  volatile f32x4* stage = stage_;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  int wd[NS];
  float v[NS];
  f32x4 x[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int q = u * 32 + pr;
    const int64_t e = beg + off + (q < left ? q : 0);
    wd[u] = NT ? __builtin_nontemporal_load(ind + e) : ind[e];
    v[u] = UNIT ? 1.f : (NT ? __builtin_nontemporal_load(dat + e) : dat[e]);
  }
#pragma unroll
  for (int u = 0; u < NS; ++u)
    x[u] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
        Xb + ((uint32_t)(wd[u] & cmask) * ldx + sub * 4));
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    stage[pr * 2 + sub] = v[u] * x[u];
    const int nval = left - u * 32;
    const int ri = wd[u] >> cbits;
    const int rprev = __shfl(ri, lane - 2, 64);
    const bool start = pr < nval && (pr == 0 || rprev != ri);
    const unsigned long long m = __ballot(start);
    f32x4 acc = zero;
    if (start) {
      const unsigned long long rest = pr == 31 ? 0ull : (m >> (2 * pr + 2));
      const int end = rest ? pr + 1 + (__builtin_ctzll(rest) >> 1) : (nval < 32 ? nval : 32);
      acc = stage[pr * 2 + sub];
      for (int j = pr + 1; j < end; ++j) acc += stage[j * 2 + sub];
    }
    stage[pr * 2 + sub] = zero;
    if (start && ri < 32) stage[ri * 2 + sub] = acc;
    a0 += stage[pr * 2 + sub];
    stage[pr * 2 + sub] = zero;
    if (start && ri >= 32) stage[(ri - 32) * 2 + sub] = acc;
    a1 += stage[pr * 2 + sub];
  }
}

// NT: index / value words loaded non-temporally (read once; the panel gathers keep L2)
// VW (launches of more than one round of resident tiles, 64-row windows): every wave also owns
// one 64-row window whose accumulators stay in its registers (8 VGPRs), behind the tile's
// LDS-resident rows -- a tile of tile_rows + 16 x 64 rows, so fewer rounds.  At cfg5 an L2 line
// serves 4 deg r / N gathers per round (r: rows in flight per XCD; profiles/r06_tile_nb128_pmc.md),
// so more rows in flight are fewer misses.
template <bool VW>
__global__ __launch_bounds__(1024, 8) void spmm8_flat_kernel(SpmmTileArgs a) {
  constexpr bool NT = true;
  // [tile_rows][8] row accumulators, then a 1-KB staging slot per wave
  extern __shared__ float tacf[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwave = blockDim.x >> 6;
  const int pr = lane >> 1, sub = lane & 1;
  const int wbits = __builtin_amdgcn_readfirstlane(a.wbits);
  const int W = 1 << wbits;
  const int tile_all = a.tile_rows + (VW ? nwave * 64 : 0);  // (VW: wbits = 6)
  const int64_t r0 = (int64_t)blockIdx.x * tile_all;
  const int64_t gw0 = r0 >> wbits;  // the tile's first window (tile_rows is a multiple of W)
  const int64_t rem = a.n - r0;
  const int nrows = (int)(rem < tile_all ? rem : tile_all);
  const int nwin_all = (nrows + W - 1) >> wbits;
  const int nwin_l = a.tile_rows >> wbits;  // LDS-resident windows of a full tile
  const int nwin = nwin_all < nwin_l ? nwin_all : nwin_l;
  // VW: this wave's register window (local rows vr0 .. vr0 + 63)
  const int vwin = nwin_l + wave;
  const bool vown = VW && vwin < nwin_all;
  const int vr0 = vwin << wbits;
  f32x4 va0 = {0.f, 0.f, 0.f, 0.f}, va1 = {0.f, 0.f, 0.f, 0.f};
  const uint32_t ldx = (uint32_t)a.ldx;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4* tacc = reinterpret_cast<f32x4*>(tacf);
  f32x4* stage = reinterpret_cast<f32x4*>(tacf + (size_t)a.tile_rows * 8) + wave * 64;
  // zero / write back by the same window -> wave map as the adds (no barrier needed).  Measured
  // and not kept (round 3-4, with per-row pointers; cfg4 layer launch 0.367 ms): windows handed
  // out per phase from an LDS counter (0.557 ms), the next window's row pointers loaded before
  // the current window's entries (flat); 512-thread workgroups with half the tile rows, 4 per CU
  // (0.448 ms); a wave owning one contiguous span of 4 windows walked as one run: 0.393 ms.
  // Round 5 (window offsets): two consecutive 64-row windows walked as one run, 0.351-0.356 vs
  // 0.351-0.353 ms, fit 1,441 vs 1,424 ms (profiles/r05_span2_ab.jsonl)
  for (int w = wave; w < nwin; w += nwave)
    for (int rr = pr; rr < W; rr += 32) {
      const int lr = (w << wbits) + rr;
      if (lr < nrows) tacc[lr * 2 + sub] = zero;
    }
  for (int k = 0; k < a.K; ++k) {
    const float* X = a.X[k];
    for (int p = 0; p < a.nb; ++p) {
      const CsrBlk& A = a.blk[k * a.nb + p];
      const int cbits = __builtin_amdgcn_readfirstlane(A.cbits);
      const int unit = __builtin_amdgcn_readfirstlane(A.unit);
      const auto wo = uniform_global(A.wo);
      const auto ind = uniform_global(A.indices);
      const auto dat = uniform_global(A.data);
      const int64_t base = uniform_i64(A.base);
      const int64_t col0 = uniform_i64(A.col0);
      const int32_t cmask = (1 << cbits) - 1;
      const auto Xb = uniform_global(X + col0 * a.ldx);
      for (int w = wave; w < nwin; w += nwave) {
        const int32_t e0 = wo[gw0 + w];
        const int len = wo[gw0 + w + 1] - e0;
        const int64_t beg = base + e0;
        f32x4* tw = tacc + ((size_t)w << wbits) * 2;
// (VW: at most 2 steps per batch -- the register window's 8 VGPRs within the 64 of 8 waves per
// SIMD; cfg5's runs are ~30 entries per window and block, one step)
#define FLAT_STEPS(U)                                                                          \
  for (int off = 0; off < len; off += (VW ? 64 : 128)) {                                       \
    const int left = len - off;                                                                \
    if (!VW && left > 96)                                                                      \
      flat_steps<VW ? 1 : 4, U, NT>(ind, dat, beg, off, left, Xb, ldx, cmask, cbits, lane, stage, tw); \
    else if (!VW && left > 64)                                                                 \
      flat_steps<VW ? 1 : 3, U, NT>(ind, dat, beg, off, left, Xb, ldx, cmask, cbits, lane, stage, tw); \
    else if (left > 32)                                                                        \
      flat_steps<2, U, NT>(ind, dat, beg, off, left, Xb, ldx, cmask, cbits, lane, stage, tw);  \
    else                                                                                       \
      flat_steps<1, U, NT>(ind, dat, beg, off, left, Xb, ldx, cmask, cbits, lane, stage, tw);  \
  }
        if (unit) {
          FLAT_STEPS(true)
        } else {
          FLAT_STEPS(false)
        }
#undef FLAT_STEPS
      }
      if (VW && vown) {
        const int32_t e0 = wo[gw0 + vwin];
        const int len = wo[gw0 + vwin + 1] - e0;
        const int64_t beg = base + e0;
#define FLAT_STEPS_V(U)                                                                        \
  for (int off = 0; off < len; off += 64) {                                                    \
    const int left = len - off;                                                                \
    if (left > 32)                                                                             \
      flat_steps_v<2, U, NT>(ind, dat, beg, off, left, Xb, ldx, cmask, cbits, lane, stage, va0, va1); \
    else                                                                                       \
      flat_steps_v<1, U, NT>(ind, dat, beg, off, left, Xb, ldx, cmask, cbits, lane, stage, va0, va1); \
  }
        if (unit) {
          FLAT_STEPS_V(true)
        } else {
          FLAT_STEPS_V(false)
        }
#undef FLAT_STEPS_V
      }
      // the workgroup's waves move to the next panel block together.  (No barrier: 0.57 vs
      // 0.36 ms per cfg4 layer launch; a bounded skew -- a wave starts phase g once all have
      // finished g - 2, LDS counters -- 0.393 vs 0.354 ms, fit 1,714 vs 1,603 ms,
      // profiles/r04_flat_sync.jsonl: the L2 locality of lockstep phases is worth the idling)
      // (XCD phase alignment -- a workgroup starts phase g once the workgroups of its XCD have
      // finished g - 1 - s, counters in HBM: 1.11 / 1.24 / 1.34 vs 0.72 ms per cfg4 stage launch
      // at s = 2 / 1 / 0, profiles/r05_xsync_ab.jsonl; removed)
      __syncthreads();
    }
    if (!a.sum || k == a.K - 1) {
      float* Y = a.Y[a.sum ? 0 : k];
      for (int w = wave; w < nwin; w += nwave)
        for (int rr = pr; rr < W; rr += 32) {
          const int lr = (w << wbits) + rr;
          if (lr < nrows) {
            *reinterpret_cast<f32x4*>(Y + (r0 + lr) * a.ldy + sub * 4) = tacc[lr * 2 + sub];
            tacc[lr * 2 + sub] = zero;
          }
        }
      if (VW && vown) {
        if (vr0 + pr < nrows)
          *reinterpret_cast<f32x4*>(Y + (r0 + vr0 + pr) * a.ldy + sub * 4) = va0;
        if (vr0 + pr + 32 < nrows)
          *reinterpret_cast<f32x4*>(Y + (r0 + vr0 + pr + 32) * a.ldy + sub * 4) = va1;
        va0 = zero;
        va1 = zero;
      }
    }
  }
}

// b = 16 panels (64-B rows): a lane quad per entry (lane = (entry q = lane >> 2, quarter
// sub = lane & 3), each lane one 16-B load), 16 entries per wave step, up to 4 steps per batch
// (8 spilled 24 VGPRs at the 8-waves-per-SIMD register budget).  A lane-pair form (32 entries
// per step, two 16-B loads of one row per lane, the halves staged and folded in turn) ran
// 0.57-0.59 ms against this form's 0.52-0.56 per cfg4 layer launch: not kept.
// The same packed blocks, windows, segment fold and fixed summation order as flat_steps; one
// gathered row is still one L2 request, so a vector column costs about half of b = 8's
// (the gather microbenchmark: 162 vs 182 G entries/s at 64- vs 32-B rows, tools/gather_ceiling.hip).
template <int NS, bool UNIT, bool NT>
__device__ __forceinline__ void flat16_steps(const __attribute__((address_space(1))) int32_t* ind,
                                             const __attribute__((address_space(1))) float* dat,
                                             int64_t beg, int off, int left,
                                             const __attribute__((address_space(1))) float* Xb,
                                             uint32_t ldx, int32_t cmask, int cbits, int lane,
                                             f32x4* stage, f32x4* tw) {
  const int q = lane >> 2, sub = lane & 3;
  int wd[NS];
  float v[NS];
  f32x4 x[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int qq = u * 16 + q;
    const int64_t e = beg + off + (qq < left ? qq : 0);
    wd[u] = NT ? __builtin_nontemporal_load(ind + e) : ind[e];
    v[u] = UNIT ? 1.f : (NT ? __builtin_nontemporal_load(dat + e) : dat[e]);
  }
#pragma unroll
  for (int u = 0; u < NS; ++u)
    x[u] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
        Xb + ((uint32_t)(wd[u] & cmask) * ldx + sub * 4));
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    stage[q * 4 + sub] = v[u] * x[u];  // entries past the end are never read
    const int nval = left - u * 16;     // valid entries of this step (>= 1; may exceed 16)
    const int ri = wd[u] >> cbits;      // row in window
    const int rprev = __shfl(ri, lane - 4, 64);
    const bool start = q < nval && (q == 0 || rprev != ri);
    const unsigned long long m = __ballot(start);
    if (start) {
      const unsigned long long rest = q == 15 ? 0ull : (m >> (4 * q + 4));
      const int end = rest ? q + 1 + (__builtin_ctzll(rest) >> 2) : (nval < 16 ? nval : 16);
      f32x4 acc = stage[q * 4 + sub];
      for (int j = q + 1; j < end; ++j) acc += stage[j * 4 + sub];
      tw[ri * 4 + sub] += acc;
    }
  }
}

// WPC: workgroups per CU.  2: 1024-row tiles (64 KB of accumulators), 8 waves per SIMD, up to
// 4 steps per batch; 1: 2048-row tiles (128 KB), 4 waves per SIMD with twice the registers, up to
// 8 steps per batch (the same loads in flight per SIMD, half the phase barriers per row)
template <int WPC>
__global__ __launch_bounds__(1024, WPC == 1 ? 4 : 8) void spmm16_flat_kernel(SpmmTileArgs a) {
  constexpr bool NT = true;
  constexpr int MAXNS = WPC == 1 ? 8 : 4;
  // [tile_rows][16] row accumulators, then a 1-KB staging slot per wave
  extern __shared__ float tacf[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwave = blockDim.x >> 6;
  const int q = lane >> 2, sub = lane & 3;
  const int wbits = __builtin_amdgcn_readfirstlane(a.wbits);
  const int W = 1 << wbits;
  const int64_t r0 = (int64_t)blockIdx.x * a.tile_rows;
  const int64_t gw0 = r0 >> wbits;
  const int64_t rem = a.n - r0;
  const int nrows = (int)(rem < a.tile_rows ? rem : a.tile_rows);
  const int nwin = (nrows + W - 1) >> wbits;
  const uint32_t ldx = (uint32_t)a.ldx;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4* tacc = reinterpret_cast<f32x4*>(tacf);
  f32x4* stage = reinterpret_cast<f32x4*>(tacf + (size_t)a.tile_rows * 16) + wave * 64;
  for (int w = wave; w < nwin; w += nwave)
    for (int rr = q; rr < W; rr += 16) {
      const int lr = (w << wbits) + rr;
      if (lr < nrows) tacc[lr * 4 + sub] = zero;
    }
  for (int k = 0; k < a.K; ++k) {
    const float* X = a.X[k];
    for (int p = 0; p < a.nb; ++p) {
      const CsrBlk& A = a.blk[k * a.nb + p];
      const int cbits = __builtin_amdgcn_readfirstlane(A.cbits);
      const int unit = __builtin_amdgcn_readfirstlane(A.unit);
      const auto wo = uniform_global(A.wo);
      const auto ind = uniform_global(A.indices);
      const auto dat = uniform_global(A.data);
      const int64_t base = uniform_i64(A.base);
      const int64_t col0 = uniform_i64(A.col0);
      const int32_t cmask = (1 << cbits) - 1;
      const auto Xb = uniform_global(X + col0 * a.ldx);
      for (int w = wave; w < nwin; w += nwave) {
        const int32_t e0 = wo[gw0 + w];
        const int len = wo[gw0 + w + 1] - e0;
        const int64_t beg = base + e0;
        f32x4* tw = tacc + ((size_t)w << wbits) * 4;
#define F16S(NS_, U) flat16_steps<(NS_), U, NT>(ind, dat, beg, off, left, Xb, ldx, cmask, cbits, lane, stage, tw)
#define FLAT16_STEPS(U)                                                                          \
  for (int off = 0; off < len; off += 16 * MAXNS) {                                              \
    const int left = len - off;                                                                  \
    const int ns = (left + 15) >> 4;                                                             \
    if (MAXNS > 4 && ns >= 8) F16S(MAXNS > 4 ? 8 : 1, U);                                        \
    else if (MAXNS > 4 && ns == 7) F16S(MAXNS > 4 ? 7 : 1, U);                                   \
    else if (MAXNS > 4 && ns == 6) F16S(MAXNS > 4 ? 6 : 1, U);                                   \
    else if (MAXNS > 4 && ns == 5) F16S(MAXNS > 4 ? 5 : 1, U);                                   \
    else if (ns >= 4) F16S(4, U);                                                                \
    else if (ns == 3) F16S(3, U);                                                                \
    else if (ns == 2) F16S(2, U);                                                                \
    else F16S(1, U);                                                                             \
  }
        if (unit) {
          FLAT16_STEPS(true)
        } else {
          FLAT16_STEPS(false)
        }
#undef FLAT16_STEPS
#undef F16S
      }
      __syncthreads();
    }
    if (!a.sum || k == a.K - 1) {
      float* Y = a.Y[a.sum ? 0 : k];
      // split output (paired mode): lane quarter sub < 2 writes Y[0]'s row, sub >= 2 Y2's
      const bool split = a.sum && a.Y2;
      float* Yq = split ? (sub < 2 ? Y : a.Y2) : Y;
      const int64_t ld = split ? 8 : a.ldy;
      const int co = split ? (sub & 1) * 4 : sub * 4;
      for (int w = wave; w < nwin; w += nwave)
        for (int rr = q; rr < W; rr += 16) {
          const int lr = (w << wbits) + rr;
          if (lr < nrows) {
            *reinterpret_cast<f32x4*>(Yq + (r0 + lr) * ld + co) = tacc[lr * 4 + sub];
            tacc[lr * 4 + sub] = zero;
          }
        }
    }
  }
}

// rows per tile for the tiled form: `wpc` workgroups (1024 threads each) per CU sharing its
// 160 KB of LDS (32 B of accumulators per row), at most 2048 (4096 at one per CU); a multiple of
// the window rows 2^wbits.  When the rows need more than one round of resident workgroups
// (cfg5: 10M rows, ~10 rounds), the tiles are sized so that every round is full.
extern "C" int n2v2r_spmm_tile_rows_b(int64_t n, int ncu, int wpc, int wbits, int b);
extern "C" int n2v2r_spmm_tile_rows(int64_t n, int ncu, int wpc, int wbits) {
  return n2v2r_spmm_tile_rows_b(n, ncu, wpc, wbits, 8);
}

// (b = 16: 64 B of accumulators per row, half the rows)
extern "C" int n2v2r_spmm_tile_rows_b(int64_t n, int ncu, int wpc, int wbits, int b) {
  const int64_t slots = wpc * (int64_t)ncu;
  // (b = 16: 1024 rows, 80 KB with the staging slots, two per CU: 0.549 ms per cfg4 layer
  // launch against 0.60-0.63 at 960 / 768 / 512 rows)
  const int64_t cap = (wpc == 1 ? 4096 : 2048) * 8 / (b == 16 ? 16 : 8);
  const int64_t w = (int64_t)1 << wbits;
  const int64_t rounds = (n + slots * cap - 1) / (slots * cap);
  int64_t t = (n + slots * rounds - 1) / (slots * rounds);
  t = (t + w - 1) / w * w;
  if (t > cap) t = cap / w * w;
  return (int)t;
}

// The register-window form when the LDS-only tiles take more than one round of resident
// workgroups (occupancy x CUs of the current device, queried once per LDS size).
// N2V2R_SPMM_VW (read per launch): 0 off; 2 (tests) on at any size.
static bool flat_vw_wanted(unsigned grid, size_t flds, int* resident) {
  const char* env = std::getenv("N2V2R_SPMM_VW");
  if (env && env[0] == '0') return false;
  const bool force = env && env[0] == '2';
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  static std::mutex mu;
  static size_t occ_flds[64] = {};
  static int slots[64] = {};
  std::lock_guard<std::mutex> lk(mu);
  if (occ_flds[dev] != flds) {
    int per_cu = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)spmm8_flat_kernel<false>,
                                                     1024, flds) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
      (void)hipGetLastError();
      per_cu = 0;
    }
    slots[dev] = per_cu * ncu;
    occ_flds[dev] = flds;
  }
  *resident = slots[dev];
  return slots[dev] > 0 && (force || grid > (unsigned)slots[dev]);
}

extern "C" hipError_t n2v2r_launch_spmm_tile(const SpmmTileArgs& a, hipStream_t stream) {
  if (a.K < 1 || a.K > 8 || a.n <= 0 || a.wbits < CB_WIN_BITS_MIN || a.wbits > CB_WIN_BITS_MAX ||
      a.tile_rows < (1 << a.wbits) || a.tile_rows % (1 << a.wbits) != 0)
    return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.n + a.tile_rows - 1) / a.tile_rows);
  const int width = a.width ? a.width : 8;
  if (width != 8 && width != 16) return hipErrorInvalidValue;
  // 4 b B of accumulators per row + a 1-KB staging slot per wave
  const size_t flds = sizeof(float) * width * (size_t)a.tile_rows + 16 * 1024;
  // (b = 16 tiles beyond 1024 rows: one workgroup per CU, up to 144 KB)
  const bool wide16 = width == 16 && a.tile_rows > 1024;
  if (flds > (wide16 ? 144 : 80) * 1024) return hipErrorInvalidValue;
  static const bool fattr = [] {
    (void)hipFuncSetAttribute((const void*)spmm8_flat_kernel<false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipFuncSetAttribute((const void*)spmm8_flat_kernel<true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipFuncSetAttribute((const void*)spmm16_flat_kernel<2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipFuncSetAttribute((const void*)spmm16_flat_kernel<1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024);
    (void)hipGetLastError();
    return true;
  }();
  (void)fattr;
  if (width == 16) {
    if (wide16)
      hipLaunchKernelGGL(spmm16_flat_kernel<1>, dim3(grid), dim3(1024), flds, stream, a);
    else
      hipLaunchKernelGGL(spmm16_flat_kernel<2>, dim3(grid), dim3(1024), flds, stream, a);
    return hipGetLastError();
  }
  // (Non-temporal index / value loads: cfg4 layer launch 0.354 vs 0.363 ms, fit 1,599 vs
  // 1,609 ms, profiles/r04_flat_nt.jsonl; no phase barrier: 0.57 vs 0.36 ms,
  // profiles/r04_flat_bar.jsonl -- the A/B switches of those runs are gone.)
  // more tiles than one round of resident workgroups (cfg5): tiles with register windows
  // Tiles: the caller's LDS rows + 1,024 register rows per workgroup (cfg5: 1,984 + 1,024, 4.14-
  // 4.16 vs 4.38-4.39 ms per layer launch; 2,048 + 1,024: 4.21-4.22; tiles that fill each of 7
  // rounds, 1,792 + 1,024: 4.21 -- rows in flight win; profiles/r06_register_windows.jsonl), or,
  // when one round of resident workgroups holds every row, tiles that fill exactly one round (the
  // 8-GPU row partition's 1.25M rows per rank).
  int resident = 0;
  if (a.wbits == 6 && flat_vw_wanted(grid, flds, &resident)) {
    const int64_t vrows = 16 * 64, cap_all = 2048 + vrows, per = resident;
    int64_t lds = a.tile_rows;
    if (a.n <= per * cap_all) {
      int64_t t_all = (a.n + per - 1) / per;
      t_all = (t_all + 63) / 64 * 64;
      lds = t_all - vrows;
      lds = lds < 64 ? 64 : (lds + 63) / 64 * 64;
      if (lds > 2048) lds = 2048;
    }
    SpmmTileArgs av = a;
    av.tile_rows = (int)lds;
    const size_t fv = sizeof(float) * 8 * (size_t)lds + 16 * 1024;
    const unsigned gv = (unsigned)((a.n + lds + vrows - 1) / (lds + vrows));
    hipLaunchKernelGGL(spmm8_flat_kernel<true>, dim3(gv), dim3(1024), fv, stream, av);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(spmm8_flat_kernel<false>, dim3(grid), dim3(1024), flds, stream, a);
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
// cbits > 0: packed entries ((r % 2^wbits) << cbits | (col - block start)) for the flat form.
template <int NB>
__global__ void cb_fill_kernel(CsrDev A, int64_t cw, const int64_t* __restrict__ rp,
                               int32_t* __restrict__ idx, float* __restrict__ dat, int cbits,
                               int wbits) {
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
    idx[q] = cbits ? (int32_t)(((r & ((1 << wbits) - 1)) << cbits) | (col - (int64_t)jb * cw))
                   : col;
    if (!A.unit) dat[q] = A.data[p];
  }
}

// Row pointers of the column blocks from the counts, on the GPU: an exclusive scan of the
// counts flattened block-major (cnt[j][r]) gives every entry's absolute position in the
// block-major entry array, rp[j][r] (int64, [nb][n + 1], a build temporary); rp[j][n] =
// rp[j + 1][0] (nnz for the last block).  What the blocks keep: the window offsets
// wo[j][w] = rp[j][min(w 2^wbits, n)] - rp[j][0] (int32, [nb][ceil(n / 2^wbits) + 1]).
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

__global__ void cb_rp_finish_kernel(int64_t* __restrict__ rp, int64_t n, int nb, int64_t nnz) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nb) return;
  rp[j * (n + 1) + n] = j + 1 < nb ? rp[(j + 1) * (n + 1)] : nnz;
}

__global__ void cb_wo_kernel(const int64_t* __restrict__ rp, int64_t n, int nb, int wbits,
                             int64_t nnz, int32_t* __restrict__ wo) {
  const int64_t nw1 = ((n + (1 << wbits) - 1) >> wbits) + 1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)nb * nw1) return;
  const int64_t j = e / nw1, w = e - j * nw1;
  const int64_t r = (w << wbits) < n ? (w << wbits) : n;
  const int64_t v = r == n ? (j + 1 < nb ? rp[(j + 1) * (n + 1)] : nnz) : rp[j * (n + 1) + r];
  wo[e] = (int32_t)(v - rp[j * (n + 1)]);
}

extern "C" hipError_t n2v2r_launch_cb_rowptrs(const int32_t* cnt, int64_t n, int nb, int64_t nnz,
                                              int64_t* tsum, size_t tsum_elems, int64_t* rp,
                                              int32_t* wo, int wbits, hipStream_t stream) {
  const int64_t len = (int64_t)nb * n;
  const int64_t ntiles = (len + SCAN_TILE - 1) / SCAN_TILE;
  if (ntiles < 1 || (size_t)ntiles > tsum_elems) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scan_tile_sums_kernel, dim3((unsigned)ntiles), dim3(SCAN_T), 0, stream, cnt,
                     len, tsum);
  hipLaunchKernelGGL(scan_tile_offsets_kernel, dim3(1), dim3(1024), 0, stream, tsum, ntiles);
  hipLaunchKernelGGL(scan_tile_write_kernel, dim3((unsigned)ntiles), dim3(SCAN_T), 0, stream, cnt,
                     n, nb, tsum, rp);
  hipLaunchKernelGGL(cb_rp_finish_kernel, dim3((unsigned)((nb + 63) / 64)), dim3(64), 0, stream,
                     rp, n, nb, nnz);
  const int64_t tot = (int64_t)nb * (((n + (1 << wbits) - 1) >> wbits) + 1);
  hipLaunchKernelGGL(cb_wo_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, rp,
                     n, nb, wbits, nnz, wo);
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
  else if (nb == 128) hipLaunchKernelGGL(cb_count_kernel<128>, g, dim3(256), 0, stream, A, cw, cnt);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" hipError_t n2v2r_launch_cb_fill(const CsrDev& A, int64_t cw, int nb, const int64_t* rp,
                                           int32_t* idx, float* dat, int cbits, int wbits,
                                           hipStream_t stream) {
  if (A.n_rows <= 0) return hipSuccess;
  const dim3 g((unsigned)((A.n_rows + 255) / 256));
#define FILL(NB) hipLaunchKernelGGL(cb_fill_kernel<NB>, g, dim3(256), 0, stream, A, cw, rp, idx, dat, cbits, wbits)
  if (nb == 4) FILL(4);
  else if (nb == 8) FILL(8);
  else if (nb == 16) FILL(16);
  else if (nb == 32) FILL(32);
  else if (nb == 64) FILL(64);
  else if (nb == 128) FILL(128);
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

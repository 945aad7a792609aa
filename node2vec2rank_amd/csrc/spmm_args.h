// Launch arguments of the CSR x panel SpMM (spmm.hip), shared with the engine.
#pragma once

#include "common.h"

#define SPMM_MAX_LAYERS 8
#ifndef N2V2R_SPMM_WGS
#define N2V2R_SPMM_WGS 2048  // workgroups per launch (8 per CU); rows are grid-strided
#endif

struct SpmmArgs {
  CsrDev A[SPMM_MAX_LAYERS];
  const float* X[SPMM_MAX_LAYERS];
  float* Y[SPMM_MAX_LAYERS];
  int64_t ldx;
  int64_t ldy;
  int K;                 // layers in this launch
  int sum;               // 1: Y[0] = sum_k A_k X_k ; 0: Y[k] = A_k X_k (grid.y = k)
  const float* colscale; // optional per-column scale of the output (nullptr = none)
  int split;             // (b = 8, sum = 0, K <= 8) Y[k] = A_k X_k with grid.y = 1 and the
                         // layers split over the XCDs: workgroup i runs layer (i mod 8) K / 8,
                         // so each XCD's L2 holds one layer's panel
};

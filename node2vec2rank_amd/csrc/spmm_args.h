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
  int rpw;               // rows per wave of the row kernels (0: from the mean row length); a
                         // launch over a row range of a matrix passes the whole matrix's choice
                         // so every row is summed exactly as in one launch over all rows
  int split;             // (b = 8, sum = 0, K <= 8) Y[k] = A_k X_k with grid.y = 1 and the
                         // layers split over the XCDs: workgroup i runs layer (i mod 8) K / 8,
                         // so each XCD's L2 holds one layer's panel
};

// ---- column blocks (b = 8 panels beyond 8 MB: the flat-window tiled SpMM) --------------------
#define CB_NB 8      // default column blocks when a caller names none (the fit picks 4-32)
#define CB_MAX 128   // column blocks per layer at most (N2V2R_SPMM_TILE_NB)
#define CB_WIN_BITS_MIN 5  // windows of 2^wbits rows: 32 ..
#define CB_WIN_BITS_MAX 7  //                          .. 128 (row-in-window bits of a packed entry)
// b = 16 flat tiles: workgroups per CU (2: 1024-row tiles; 1: 2048-row tiles, spmm16_flat_kernel)
#ifndef N2V2R_SPMM16_WPC
#define N2V2R_SPMM16_WPC 2
#endif

// One column block of a layer, packed for the flat tiled form: entry = (row % W) << cbits |
// (column - col0), W = 2^wbits rows per window, in the layer's shared index array starting at
// `base`.  The rows of a window have their entries in this block as ONE contiguous run (rows in
// order), so the block keeps no per-row pointers: wo[w] .. wo[w + 1] (relative to base) is
// window w's run, and each entry names its own row.  (Round 4 kept int32 row pointers
// [n_rows + 1] per block: 4 MB per block at cfg4 and 40 MB at cfg5 read by every launch.)
struct CsrBlk {
  const int32_t* wo;       // ceil(n_rows / W) + 1 window offsets, relative to base
  const int32_t* indices;  // shared by the blocks of a layer
  const float* data;       // shared (nullptr when unit)
  int64_t base;
  int64_t n_rows;
  int64_t nnz;
  int unit;
  int cbits;               // column bits of a packed entry (the row-in-window bits sit above)
  int64_t col0;            // first column of the block
};

struct SpmmTileArgs {  // row tiles x column-block phases (spmm8/16_flat_kernel)
  const CsrBlk* blk;   // device array [K][nb]
  const float* X[SPMM_MAX_LAYERS];  // panel per layer (gathered, global rows)
  float* Y[SPMM_MAX_LAYERS];        // output per layer (sum: Y[0])
  int64_t ldx, ldy;
  int64_t n;           // rows
  int K;
  int nb;              // column blocks (phases) per layer
  int sum;
  int tile_rows;       // a multiple of the window rows 2^wbits
  int wbits;           // window rows = 2^wbits (CB_WIN_BITS_MIN..MAX), as the blocks were packed
  int width;           // panel width b: 8 (spmm8_flat_kernel) or 16 (spmm16_flat_kernel); 0 = 8
  // width 16, sum mode: non-null splits the output -- columns 0-7 to Y[0], 8-15 to Y2, both
  // N x 8 (ld 8): the two 8-wide basis blocks of the solver's paired mode (pair.hip)
  float* Y2;
};

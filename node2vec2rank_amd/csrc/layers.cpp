// Layer ingest: CSR / dense layers to HBM (range check, GPU transpose and symmetry test, row
// slices of partitioned handles), the column-block copies of the flat tiled SpMM, the
// column sums (DeDi) and the bipartite projection.
#include "engine.h"

using namespace n2v2r_int;

namespace n2v2r_int {
// Split a CSR into nb column blocks of ceil(ncols / nb) columns, packed for the flat tiled SpMM
// (spmm.hip): per-row block counts on the GPU, a device scan into entry positions, the window
// offsets of windows of 2^wbits rows, and a scatter keeping each row's entries in order.  One-off
// per layer; not part of a fit's timed work.  cbits stays 0 (the layer not packable) when the
// column bits of a block and the row-in-window bits do not fit 31 bits.
void build_col_blocks(const CsrDev& A, int64_t ncols, LayerDev::ColBlocks& out, hipStream_t st,
                      int nb, int wbits) {
  const int64_t n = A.n_rows;
  const int64_t cw = (ncols + nb - 1) / nb;
  int cbits = 1;
  while (((int64_t)1 << cbits) < cw) ++cbits;
  out.ncols = ncols;
  out.nb = nb;
  out.wbits = wbits;
  out.cbits = cbits + wbits <= 31 ? cbits : 0;
  out.built = true;
  out.usable = false;
  if (n <= 0 || out.cbits == 0) return;
  // per-row block counts, then every entry position by a device scan (no host round trip)
  DevBuf cnt, rp64, tsum;
  cnt.ensure(sizeof(int32_t) * nb * n, st);
  HIPCHK(n2v2r_launch_cb_count(A, cw, nb, cnt.as<int32_t>(), st));
  const int64_t ntiles = n2v2r_cb_scan_tiles(n, nb);
  tsum.ensure(sizeof(int64_t) * ntiles, st);
  rp64.ensure(sizeof(int64_t) * nb * (n + 1), st);
  const int64_t nw1 = ((n + ((int64_t)1 << wbits) - 1) >> wbits) + 1;
  out.wo.ensure(sizeof(int32_t) * nb * nw1, st);
  HIPCHK(n2v2r_launch_cb_rowptrs(cnt.as<int32_t>(), n, nb, A.nnz, tsum.as<int64_t>(),
                                 (size_t)ntiles, rp64.as<int64_t>(), out.wo.as<int32_t>(), wbits,
                                 st));
  // block bases and ends: rp[j][0], rp[j][n]
  std::vector<int64_t> ends(2 * (size_t)nb);
  for (int j = 0; j < nb; ++j) {
    HIPCHK(hipMemcpyAsync(&ends[2 * j], rp64.as<int64_t>() + (size_t)j * (n + 1),
                          sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&ends[2 * j + 1], rp64.as<int64_t>() + (size_t)j * (n + 1) + n,
                          sizeof(int64_t), hipMemcpyDeviceToHost, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  if (ends[2 * (nb - 1) + 1] != A.nnz || ends[0] != 0)
    throw StatusFail{N2V2R_ERR_INTERNAL, "column-block split lost entries"};
  for (int j = 0; j < nb; ++j)
    if (ends[2 * j + 1] - ends[2 * j] > (int64_t)INT32_MAX) return;  // int32 offsets: row kernel
  out.idx.ensure(sizeof(int32_t) * std::max<int64_t>(A.nnz, 1), st);
  if (!A.unit) out.dat.ensure(sizeof(float) * std::max<int64_t>(A.nnz, 1), st);
  HIPCHK(n2v2r_launch_cb_fill(A, cw, nb, rp64.as<int64_t>(), out.idx.as<int32_t>(),
                              A.unit ? nullptr : out.dat.as<float>(), out.cbits, wbits, st));
  HIPCHK(hipStreamSynchronize(st));
  for (int j = 0; j < nb; ++j)
    out.blk[j] = CsrBlk{out.wo.as<int32_t>() + (size_t)j * nw1, out.idx.as<int32_t>(),
                        A.unit ? nullptr : out.dat.as<float>(), ends[2 * j], n,
                        ends[2 * j + 1] - ends[2 * j], A.unit, out.cbits, (int64_t)j * cw};
  out.usable = true;
}

// false when a block would exceed int32 offsets or the packed bits do not fit (then the row
// kernel runs)
bool ensure_col_blocks(LayerDev& L, int64_t ncols, hipStream_t st, int nb, int wbits) {
  auto stale = [&](const LayerDev::ColBlocks& c) {
    return !c.built || c.ncols != ncols || c.nb != nb || c.wbits != wbits;
  };
  if (stale(L.cb)) build_col_blocks(L.csr(), ncols, L.cb, st, nb, wbits);
  if (!L.symmetric && stale(L.cb_t)) build_col_blocks(L.csr_t(), ncols, L.cb_t, st, nb, wbits);
  return L.cb.usable && L.cb.cbits && (L.symmetric || (L.cb_t.usable && L.cb_t.cbits));
}

// Window rows of the flat tiled SpMM: 64 (wbits 6).  Layer launches, round 5 sweeps
// (profiles/r05_tile_cfg4.jsonl, r05_tile_cfg5.jsonl): cfg4 (16 blocks, ~3 entries per row and
// block) 0.356 / 0.348 / 0.357 ms at windows of 32 / 64 / 128 rows; cfg5 (64 blocks, ~0.5)
// 5.13 / 4.36 / 4.79 ms -- longer runs per window and block until a wave's windows get too
// few to balance.  N2V2R_SPMM_WBITS (5..7) overrides (read per call).
int tile_wbits(const std::vector<std::unique_ptr<LayerDev>>& layers, int nb) {
  (void)layers;
  (void)nb;
  if (const char* e = std::getenv("N2V2R_SPMM_WBITS")) {
    const int v = std::atoi(e);
    if (v >= CB_WIN_BITS_MIN && v <= CB_WIN_BITS_MAX) return v;
  }
  return 6;
}

// A[:, own rows] of a partitioned layer as a CSR over rows_out (>= N) global rows, columns local:
// the transpose of the rank's rows of A^T (A's own columns), by the ingest's GPU transpose (the
// stable LSD radix sort of col << 32 | row keys over the column digits).  Stage 2 of the
// reduce-scatter form gathers from this rank's Z rows only.  One-off per layer.
void ensure_colcsr(LayerDev& L, int64_t ncols, int64_t rows_out, hipStream_t st, int64_t npad,
                   int W, int64_t rc) {
  if (rc <= 0 || rc >= npad) rc = 0;  // one chunk: the natural row order
  if (L.c_built && L.c_rows == rows_out && L.c_rc == rc) return;
  const CsrDev s = L.csr_t();
  const int64_t nnz = s.nnz;
  if (nnz > (int64_t)INT32_MAX)
    throw StatusFail{N2V2R_ERR_BAD_ARG, "a rank's layer block over 2^31 - 1 entries"};
  L.c_indptr.ensure(sizeof(int64_t) * (rows_out + 1));
  L.c_indices.ensure(sizeof(int32_t) * std::max<int64_t>(nnz, 1));
  if (!s.unit) L.c_data.ensure(sizeof(float) * std::max<int64_t>(nnz, 1));
  if (nnz == 0) {
    HIPCHK(n2v2r_launch_csr_from_sorted(nullptr, nullptr, nullptr, 0, rows_out,
                                        L.c_indptr.as<int64_t>(), nullptr, nullptr, st));
  } else {
    DevBuf keys[2], pay[2], hist, flag;
    for (int i = 0; i < 2; ++i) {
      keys[i].ensure(sizeof(uint64_t) * nnz);
      pay[i].ensure(sizeof(int32_t) * nnz);
    }
    flag.ensure(sizeof(unsigned) * 4, st);
    HIPCHK(hipMemsetAsync(flag.p, 0, sizeof(unsigned) * 4, st));
    HIPCHK(n2v2r_launch_csr_scan(s.indptr, s.indices, s.data, s.n_rows, ncols,
                                 keys[0].as<uint64_t>(), pay[0].as<int32_t>(),
                                 flag.as<unsigned>(), st));
    if (rc > 0)
      HIPCHK(n2v2r_launch_chunk_major_keys(keys[0].as<uint64_t>(), nnz, npad, W, rc, st));
    hist.ensure(sizeof(uint32_t) * n2v2r_radix_hist_elems(nnz, 1));
    int bits = 1;
    const int64_t span = rc > 0 ? rows_out : ncols;
    while (bits < 31 && ((int64_t)1 << bits) < span) ++bits;
    int cur = 0;
    for (int sh = 32; sh < 32 + bits; sh += 8) {
      HIPCHK(n2v2r_launch_radix_pass(keys[cur].as<uint64_t>(), pay[cur].as<int32_t>(),
                                     keys[cur ^ 1].as<uint64_t>(), pay[cur ^ 1].as<int32_t>(),
                                     nnz, 1, sh, hist.as<uint32_t>(), st));
      cur ^= 1;
    }
    HIPCHK(n2v2r_launch_csr_from_sorted(keys[cur].as<uint64_t>(), pay[cur].as<int32_t>(), s.data,
                                        nnz, rows_out, L.c_indptr.as<int64_t>(),
                                        L.c_indices.as<int32_t>(),
                                        s.unit ? nullptr : L.c_data.as<float>(), st));
    HIPCHK(hipStreamSynchronize(st));  // the sort scratch dies here
  }
  L.c_nnz = nnz;
  L.c_rows = rows_out;
  L.c_rc = rc;
  L.c_built = true;
}

// ---- host CSR helpers -------------------------------------------------------------------
int host_threads() {
  return (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
}

// every value exactly 1.0f (an unweighted layer: its value array need not cross PCIe -- the
// device copy is filled with 1.0f instead); large layers in up to 16 host threads
bool host_all_ones(int64_t nnz, const float* dv) {
  auto ok = [&](int64_t p0, int64_t p1) {
    bool good = true;
    for (int64_t p = p0; p < p1; ++p) good &= dv[p] == 1.0f;
    return good;
  };
  int nt = host_threads();
  if (nnz < (int64_t)1 << 22) nt = 1;
  if (nt == 1) return ok(0, nnz);
  std::vector<char> res(nt, 1);
  const int64_t per = (nnz + nt - 1) / nt;
  parallel_chunks(nt, [&](int t) {
    const int64_t p0 = std::min<int64_t>(nnz, t * per);
    res[t] = ok(p0, std::min<int64_t>(nnz, p0 + per)) ? 1 : 0;
  });
  for (char c : res)
    if (!c) return false;
  return true;
}

// every column index in [0, n); large layers are checked in up to 16 host threads
bool host_indices_in_range(int64_t nnz, const int32_t* ix, int64_t n) {
  auto ok = [&](int64_t p0, int64_t p1) {
    bool good = true;
    for (int64_t p = p0; p < p1; ++p) good &= (ix[p] >= 0) & ((int64_t)ix[p] < n);
    return good;
  };
  int nt = host_threads();
  if (nnz < (int64_t)1 << 22) nt = 1;
  if (nt == 1) return ok(0, nnz);
  std::vector<char> res(nt, 1);
  const int64_t per = (nnz + nt - 1) / nt;
  parallel_chunks(nt, [&](int t) {
    const int64_t p0 = std::min<int64_t>(nnz, t * per);
    res[t] = ok(p0, std::min<int64_t>(nnz, p0 + per)) ? 1 : 0;
  });
  for (char c : res)
    if (!c) return false;
  return true;
}

// upload rows [r0, r0 + nr) of a CSR (global column indices kept) into (ip, ix, dv) buffers;
// returns whether every uploaded value is 1.0f (an unweighted graph: the SpMM skips values)
bool upload_rows(hipStream_t st, int64_t r0, int64_t nr, const int64_t* ip, const int32_t* ix,
                 const float* dv, DevBuf& dip, DevBuf& dix, DevBuf& ddv, int64_t& nnz_out) {
  const int64_t p0 = ip[r0], p1 = ip[r0 + nr];
  nnz_out = p1 - p0;
  const bool unit = host_all_ones(nnz_out, dv + p0);
  std::vector<int64_t> lip(nr + 1);
  for (int64_t r = 0; r <= nr; ++r) lip[r] = ip[r0 + r] - p0;
  dip.ensure(sizeof(int64_t) * (nr + 1));
  dix.ensure(sizeof(int32_t) * std::max<int64_t>(nnz_out, 1));
  ddv.ensure(sizeof(float) * std::max<int64_t>(nnz_out, 1));
  HIPCHK(hipMemcpyAsync(dip.p, lip.data(), sizeof(int64_t) * (nr + 1), hipMemcpyHostToDevice, st));
  if (nnz_out) {
    HIPCHK(hipMemcpyAsync(dix.p, ix + p0, sizeof(int32_t) * nnz_out, hipMemcpyHostToDevice, st));
    if (unit)  // (0x3F800000 = 1.0f)
      HIPCHK(hipMemsetD32Async((hipDeviceptr_t)ddv.p, 0x3F800000, (size_t)nnz_out, st));
    else
      HIPCHK(hipMemcpyAsync(ddv.p, dv + p0, sizeof(float) * nnz_out, hipMemcpyHostToDevice, st));
  }
  HIPCHK(hipStreamSynchronize(st));  // lip dies here
  return unit;
}

namespace {
inline uint64_t mix64(uint64_t z) {  // splitmix64's finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
}  // namespace

// Multiset equality of {(r, c, v)} and {(c, r, v)} by two hash sums each (mod 2^64): a
// non-symmetric layer passes with probability ~2^-128.  Values compare by their bits (-0 and +0
// differ, which only makes a layer count as directed: the slower, always correct path).
bool host_csr_symmetric(int64_t n, const int64_t* ip, const int32_t* ix, const float* dv) {
  int nt = host_threads();
  const int64_t nnz = ip[n];
  if (nnz < (int64_t)1 << 20) nt = 1;
  std::vector<uint64_t> acc((size_t)nt * 4, 0);
  const int64_t per = (n + nt - 1) / nt;
  parallel_chunks(nt, [&](int t) {
    const int64_t r0 = std::min<int64_t>(n, t * per), r1 = std::min<int64_t>(n, r0 + per);
    uint64_t a1 = 0, a2 = 0, b1 = 0, b2 = 0;
    for (int64_t r = r0; r < r1; ++r)
      for (int64_t p = ip[r]; p < ip[r + 1]; ++p) {
        uint32_t vb;
        std::memcpy(&vb, dv + p, sizeof(vb));
        const uint64_t c = (uint32_t)ix[p], rr = (uint64_t)r;
        const uint64_t kf = (rr << 32) | c, kt = (c << 32) | rr;
        a1 += mix64(mix64(kf + 0x9E3779B97F4A7C15ull) ^ vb);
        b1 += mix64(mix64(kt + 0x9E3779B97F4A7C15ull) ^ vb);
        a2 += mix64(mix64(kf ^ 0xD1B54A32D192ED03ull) + ((uint64_t)vb << 17));
        b2 += mix64(mix64(kt ^ 0xD1B54A32D192ED03ull) + ((uint64_t)vb << 17));
      }
    acc[(size_t)t * 4 + 0] = a1;
    acc[(size_t)t * 4 + 1] = a2;
    acc[(size_t)t * 4 + 2] = b1;
    acc[(size_t)t * 4 + 3] = b2;
  });
  uint64_t s[4] = {0, 0, 0, 0};
  for (int t = 0; t < nt; ++t)
    for (int i = 0; i < 4; ++i) s[i] += acc[(size_t)t * 4 + i];
  return s[0] == s[2] && s[1] == s[3];
}

void host_transpose_rows(int64_t n, const int64_t* ip, const int32_t* ix, const float* dv,
                         int64_t r0, int64_t nr, std::vector<int64_t>& tip,
                         std::vector<int32_t>& tix, std::vector<float>& tdv) {
  tip.assign((size_t)nr + 1, 0);
  const uint64_t span = (uint64_t)nr;
  for (int64_t r = 0; r < n; ++r)
    for (int64_t p = ip[r]; p < ip[r + 1]; ++p) {
      const uint64_t c = (uint64_t)((int64_t)ix[p] - r0);
      if (c < span) ++tip[c + 1];
    }
  for (int64_t i = 0; i < nr; ++i) tip[i + 1] += tip[i];
  tix.resize((size_t)std::max<int64_t>(tip[nr], 1));
  tdv.resize((size_t)std::max<int64_t>(tip[nr], 1));
  std::vector<int64_t> pos(tip.begin(), tip.end() - 1);
  for (int64_t r = 0; r < n; ++r)
    for (int64_t p = ip[r]; p < ip[r + 1]; ++p) {
      const uint64_t c = (uint64_t)((int64_t)ix[p] - r0);
      if (c < span) {
        const int64_t q = pos[c]++;
        tix[q] = (int32_t)r;
        tdv[q] = dv[p];
      }
    }
}

int set_layer_rows_directed(n2v2r_handle* h, int k, const int64_t* aip, const int32_t* aix,
                            const float* adv, const int64_t* tip, const int32_t* tix,
                            const float* tdv) {
  return guarded(h, [&]() -> int {
    const int64_t nr = h->nloc;
    if (k < 0 || k >= h->K || aip[0] != 0 || tip[0] != 0) return N2V2R_ERR_BAD_ARG;
    for (int64_t r = 0; r < nr; ++r)
      if (aip[r + 1] < aip[r]) {
        h->set_err("layer %d: indptr not monotone", k);
        return N2V2R_ERR_BAD_ARG;
      }
    if (!host_indices_in_range(aip[nr], aix, h->n)) {
      h->set_err("layer %d: column index out of range", k);
      return N2V2R_ERR_BAD_ARG;
    }
    for (int j = 0; j < h->K; ++j)
      if (j != k && h->layers[j]->loaded && h->layers[j]->dense) {
        h->err = "layers must be all CSR or all dense";
        return N2V2R_ERR_BAD_ARG;
      }
    LayerDev& L = *h->layers[k];
    L.dense = false;
    L.loaded = false;
    L.drop_col_blocks();
    L.n_rows = nr;
    L.unit = upload_rows(h->stream, 0, nr, aip, aix, adv, L.indptr, L.indices, L.data, L.nnz);
    L.t_unit = upload_rows(h->stream, 0, nr, tip, tix, tdv, L.t_indptr, L.t_indices, L.t_data,
                           L.t_nnz);
    h->h2d_layer_bytes += 16 * (nr + 1) + (L.unit ? 4 : 8) * L.nnz + (L.t_unit ? 4 : 8) * L.t_nnz;
    L.symmetric = false;
    L.loaded = true;
    h->have_embedding = false;
    return N2V2R_OK;
  });
}
}  // namespace n2v2r_int

extern "C" {

int n2v2r_set_num_layers(n2v2r_handle* h, int num_layers, int64_t n) {
  if (h && h->multi()) return multi_set_num_layers(h, num_layers, n);
  return guarded(h, [&]() -> int {
    if (num_layers < 1 || n < 1 || n > (int64_t)INT32_MAX) {
      h->set_err("bad layer count %d or node count %lld", num_layers, (long long)n);
      return N2V2R_ERR_BAD_ARG;
    }
    if (num_layers > SPMM_MAX_LAYERS) {
      h->set_err("at most %d layers are supported", SPMM_MAX_LAYERS);
      return N2V2R_ERR_BAD_ARG;
    }
    h->K = num_layers;
    h->set_partition(n);
    h->layers.clear();
    for (int k = 0; k < num_layers; ++k) h->layers.emplace_back(new LayerDev());
    h->have_embedding = false;
    h->ncmp = h->ncols = 0;
    return N2V2R_OK;
  });
}

int n2v2r_set_layer_csr(n2v2r_handle* h, int k, int64_t n, int64_t nnz, const int64_t* indptr,
                        const int32_t* indices, const float* data, int symmetric) {
  if (h && h->multi()) return multi_set_layer_csr(h, k, n, nnz, indptr, indices, data, symmetric);
  return guarded(h, [&]() -> int {
    if (k < 0 || k >= h->K || n != h->n || nnz < 0 || !indptr || (nnz > 0 && (!indices || !data))) {
      h->set_err("bad CSR arguments for layer %d", k);
      return N2V2R_ERR_BAD_ARG;
    }
    if (indptr[0] != 0 || indptr[n] != nnz) {
      h->set_err("layer %d: indptr must start at 0 and end at nnz", k);
      return N2V2R_ERR_BAD_ARG;
    }
    // the GPU transpose (and the symmetry test built on it) sorts int32 entry indices: a layer
    // that needs it is limited to 2^31 - 1 entries; N2V2R_SYM_YES layers are not
    if (symmetric != N2V2R_SYM_YES && nnz > (int64_t)INT32_MAX) {
      h->set_err("layer %d: more than 2^31 - 1 entries need symmetric = N2V2R_SYM_YES (the GPU "
                 "transpose / symmetry test sorts int32 entry indices)", k);
      return N2V2R_ERR_BAD_ARG;
    }
    for (int64_t r = 0; r < n; ++r)
      if (indptr[r + 1] < indptr[r]) {
        h->set_err("layer %d: indptr not monotone", k);
        return N2V2R_ERR_BAD_ARG;
      }
    for (int j = 0; j < h->K; ++j)
      if (j != k && h->layers[j]->loaded && h->layers[j]->dense) {
        h->err = "layers must be all CSR or all dense";
        return N2V2R_ERR_BAD_ARG;
      }
    LayerDev& L = *h->layers[k];
    L.dense = false;
    L.loaded = false;
    L.drop_col_blocks();
    L.n_rows = h->nloc;
    const hipStream_t st = h->stream;
    // the whole layer to HBM (on one GPU straight into the layer's buffers; a partitioned
    // handle keeps its row slice and the slice of the transpose)
    const bool whole = !h->comm;
    DevBuf gip, gix, gdv;
    DevBuf& dip = whole ? L.indptr : gip;
    DevBuf& dix = whole ? L.indices : gix;
    DevBuf& ddv = whole ? L.data : gdv;
    dip.ensure(sizeof(int64_t) * (n + 1));
    dix.ensure(sizeof(int32_t) * std::max<int64_t>(nnz, 1));
    ddv.ensure(sizeof(float) * std::max<int64_t>(nnz, 1));
    HIPCHK(hipMemcpyAsync(dip.p, indptr, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, st));
    const bool ones = nnz > 0 && host_all_ones(nnz, data);  // unweighted: no value upload
    if (nnz) {
      HIPCHK(hipMemcpyAsync(dix.p, indices, sizeof(int32_t) * nnz, hipMemcpyHostToDevice, st));
      if (ones)
        HIPCHK(hipMemsetD32Async((hipDeviceptr_t)ddv.p, 0x3F800000, (size_t)nnz, st));
      else
        HIPCHK(hipMemcpyAsync(ddv.p, data, sizeof(float) * nnz, hipMemcpyHostToDevice, st));
    }
    h->h2d_layer_bytes += 8 * (n + 1) + (ones ? 4 : 8) * nnz;
    const bool need_t = symmetric != N2V2R_SYM_YES;
    DevBuf* keys = h->ing_keys;
    DevBuf* pay = h->ing_pay;
    DevBuf& hist = h->ing_hist;
    DevBuf& flag = h->ing_flag;
    flag.ensure_raw(sizeof(unsigned) * 4);
    HIPCHK(hipMemsetAsync(flag.p, 0, sizeof(unsigned) * 4, st));
    if (need_t && nnz) {
      keys[0].ensure_raw(sizeof(uint64_t) * nnz);
      pay[0].ensure_raw(sizeof(int32_t) * nnz);
    }
    HIPCHK(n2v2r_launch_csr_scan(dip.as<int64_t>(), dix.as<int32_t>(), ddv.as<float>(), n, n,
                                 need_t && nnz ? keys[0].as<uint64_t>() : nullptr,
                                 need_t && nnz ? pay[0].as<int32_t>() : nullptr,
                                 flag.as<unsigned>(), st));
    unsigned fl = 0;
    HIPCHK(hipMemcpyAsync(&fl, flag.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (fl & 1u) {
      h->set_err("layer %d: column index out of range", k);
      return N2V2R_ERR_BAD_ARG;
    }
    const bool unit = !(fl & 2u);
    const bool sorted = !(fl & 4u);
    // A^T = the entries stably sorted by column (LSD radix over the column digits only)
    auto transpose = [&](const int64_t* ip_, const int32_t* ix_, const float* dv_, bool have_keys,
                         DevBuf& tp, DevBuf& tx, DevBuf& td) {
      tp.ensure(sizeof(int64_t) * (n + 1));
      tx.ensure(sizeof(int32_t) * std::max<int64_t>(nnz, 1));
      if (!unit) td.ensure(sizeof(float) * std::max<int64_t>(nnz, 1));
      if (nnz == 0) {
        HIPCHK(n2v2r_launch_csr_from_sorted(nullptr, nullptr, nullptr, 0, n, tp.as<int64_t>(),
                                            nullptr, nullptr, st));
        return;
      }
      keys[0].ensure_raw(sizeof(uint64_t) * nnz);
      pay[0].ensure_raw(sizeof(int32_t) * nnz);
      keys[1].ensure_raw(sizeof(uint64_t) * nnz);
      pay[1].ensure_raw(sizeof(int32_t) * nnz);
      if (!have_keys)
        HIPCHK(n2v2r_launch_csr_scan(ip_, ix_, dv_, n, n, keys[0].as<uint64_t>(),
                                     pay[0].as<int32_t>(), flag.as<unsigned>() + 1, st));
      hist.ensure_raw(sizeof(uint32_t) * n2v2r_radix_hist_elems(nnz, 1));
      int bits = 1;
      while (bits < 31 && ((int64_t)1 << bits) < n) ++bits;
      int cur = 0;
      for (int sh = 32; sh < 32 + bits; sh += 8) {
        HIPCHK(n2v2r_launch_radix_pass(keys[cur].as<uint64_t>(), pay[cur].as<int32_t>(),
                                       keys[cur ^ 1].as<uint64_t>(), pay[cur ^ 1].as<int32_t>(),
                                       nnz, 1, sh, hist.as<uint32_t>(), st));
        cur ^= 1;
      }
      HIPCHK(n2v2r_launch_csr_from_sorted(keys[cur].as<uint64_t>(), pay[cur].as<int32_t>(), dv_,
                                          nnz, n, tp.as<int64_t>(), tx.as<int32_t>(),
                                          unit ? nullptr : td.as<float>(), st));
    };
    bool sym = symmetric == N2V2R_SYM_YES;
    DevBuf gtp, gtx, gtd;
    DevBuf& tp = whole ? L.t_indptr : gtp;
    DevBuf& tx = whole ? L.t_indices : gtx;
    DevBuf& td = whole ? L.t_data : gtd;
    if (need_t) {
      transpose(dip.as<int64_t>(), dix.as<int32_t>(), ddv.as<float>(), true, tp, tx, td);
      if (symmetric == N2V2R_SYM_DETECT) {
        // unit layers compare their (absent) values as equal: both sides read A's values
        const float* tv = unit ? ddv.as<float>() : td.as<float>();
        HIPCHK(hipMemsetAsync(flag.as<unsigned>() + 2, 0, sizeof(unsigned), st));
        if (sorted) {
          HIPCHK(n2v2r_launch_csr_compare(dip.as<int64_t>(), dix.as<int32_t>(), ddv.as<float>(),
                                          tp.as<int64_t>(), tx.as<int32_t>(), tv, n, nnz,
                                          flag.as<unsigned>() + 2, st));
        } else {  // A's rows sorted = (A^T)^T
          DevBuf sp_, sx, sv;
          transpose(tp.as<int64_t>(), tx.as<int32_t>(), tv, false, sp_, sx, sv);
          HIPCHK(n2v2r_launch_csr_compare(sp_.as<int64_t>(), sx.as<int32_t>(),
                                          unit ? ddv.as<float>() : sv.as<float>(),
                                          tp.as<int64_t>(), tx.as<int32_t>(), tv, n, nnz,
                                          flag.as<unsigned>() + 2, st));
          HIPCHK(hipStreamSynchronize(st));
        }
        unsigned mism = 0;
        HIPCHK(hipMemcpyAsync(&mism, flag.as<unsigned>() + 2, sizeof(unsigned),
                              hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        sym = mism == 0;
      }
    }
    HIPCHK(hipStreamSynchronize(st));  // the sort scratch dies here
    keys[0].release();
    keys[1].release();
    pay[0].release();
    pay[1].release();
    // this rank's rows of A and (not symmetric) of A^T
    auto slice = [&](DevBuf& sip, DevBuf& six, DevBuf& sdv, bool copy_values, DevBuf& oip,
                     DevBuf& oix, DevBuf& odv, int64_t& onnz) {
      int64_t p0 = 0, p1 = 0;
      HIPCHK(hipMemcpyAsync(&p0, sip.as<int64_t>() + h->row0, sizeof(int64_t),
                            hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(&p1, sip.as<int64_t>() + h->row0 + h->nloc, sizeof(int64_t),
                            hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      onnz = p1 - p0;
      oip.ensure(sizeof(int64_t) * (h->nloc + 1));
      oix.ensure(sizeof(int32_t) * std::max<int64_t>(onnz, 1));
      odv.ensure(sizeof(float) * std::max<int64_t>(onnz, 1));
      HIPCHK(n2v2r_launch_csr_rebase(sip.as<int64_t>(), h->row0, h->nloc, oip.as<int64_t>(), st));
      if (onnz) {
        HIPCHK(hipMemcpyAsync(oix.p, six.as<int32_t>() + p0, sizeof(int32_t) * onnz,
                              hipMemcpyDeviceToDevice, st));
        if (copy_values)
          HIPCHK(hipMemcpyAsync(odv.p, sdv.as<float>() + p0, sizeof(float) * onnz,
                                hipMemcpyDeviceToDevice, st));
      }
      HIPCHK(hipStreamSynchronize(st));
    };
    if (whole) {
      L.nnz = nnz;
      L.t_nnz = nnz;
      if (sym) {
        L.t_indptr.release();
        L.t_indices.release();
        L.t_data.release();
      }
    } else {
      slice(gip, gix, gdv, true, L.indptr, L.indices, L.data, L.nnz);
      if (!sym) slice(gtp, gtx, gtd, !unit, L.t_indptr, L.t_indices, L.t_data, L.t_nnz);
    }
    L.unit = unit;
    L.t_unit = unit;
    L.symmetric = sym;
    L.loaded = true;
    h->have_embedding = false;
    return N2V2R_OK;
  });
}

int n2v2r_set_layer_dense(n2v2r_handle* h, int k, int64_t n, const float* A, int symmetric) {
  if (h && h->multi()) return multi_set_layer_dense(h, k, n, A, symmetric);
  return guarded(h, [&]() -> int {
    if (k < 0 || k >= h->K || n != h->n || !A) {
      h->set_err("bad dense arguments for layer %d", k);
      return N2V2R_ERR_BAD_ARG;
    }
    for (int j = 0; j < h->K; ++j)
      if (j != k && h->layers[j]->loaded && !h->layers[j]->dense) {
        h->err = "layers must be all CSR or all dense";
        return N2V2R_ERR_BAD_ARG;
      }
    LayerDev& L = *h->layers[k];
    L.dense = true;
    L.n_rows = h->nloc;
    L.lda = (n + 63) / 64 * 64;
    const int64_t nl = std::max<int64_t>(h->nloc, 1);
    L.dA.ensure(sizeof(float) * nl * L.lda);
    HIPCHK(hipMemcpy2D(L.dA.p, sizeof(float) * L.lda, A + h->row0 * n, sizeof(float) * n,
                       sizeof(float) * n, h->nloc, hipMemcpyHostToDevice));
    bool sym = symmetric == N2V2R_SYM_YES;
    if (!sym) {
      // A^T rows [row0, row0 + nloc) = columns of A: a partitioned handle stages all of A once
      // (one GPU: the rows already uploaded are all of A)
      DevBuf full;
      const float* src = L.dA.as<float>();
      if (h->comm) {
        full.ensure(sizeof(float) * n * L.lda);
        HIPCHK(hipMemcpy2D(full.p, sizeof(float) * L.lda, A, sizeof(float) * n,
                           sizeof(float) * n, n, hipMemcpyHostToDevice));
        src = full.as<float>();
      }
      L.dAT.ensure(sizeof(float) * nl * L.lda);
      HIPCHK(n2v2r_launch_transpose(src + h->row0, L.lda, n, h->nloc, L.dAT.as<float>(), L.lda,
                                    h->stream));
      if (symmetric == N2V2R_SYM_DETECT) {
        DevBuf cnt;
        cnt.ensure(sizeof(unsigned long long));
        HIPCHK(n2v2r_launch_mismatch(L.dA.as<float>(), L.dAT.as<float>(), L.lda, h->nloc, n,
                                     cnt.as<unsigned long long>(), h->stream));
        unsigned long long mism = 0;
        HIPCHK(hipMemcpyAsync(&mism, cnt.p, sizeof(mism), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        sym = mism == 0;
      }
      HIPCHK(hipStreamSynchronize(h->stream));
      if (sym) L.dAT.release();
    }
    L.symmetric = sym;
    L.loaded = true;
    h->have_embedding = false;
    return N2V2R_OK;
  });
}

int n2v2r_set_layer_csr_rows(n2v2r_handle* h, int k, int64_t n, int64_t row0, int64_t n_rows,
                             int64_t nnz, const int64_t* indptr, const int32_t* indices,
                             const float* data) {
  return guarded(h, [&]() -> int {
    if (h->multi()) {
      h->err = "n2v2r_set_layer_csr_rows: a multi-GPU handle takes whole layers (it slices them)";
      return N2V2R_ERR_BAD_ARG;
    }
    if (k < 0 || k >= h->K || n != h->n || row0 != h->row0 || n_rows != h->nloc || nnz < 0 ||
        !indptr || (nnz > 0 && (!indices || !data)) || indptr[0] != 0 || indptr[n_rows] != nnz) {
      h->set_err("bad local CSR rows for layer %d (expected rows [%lld, %lld))", k,
                 (long long)h->row0, (long long)(h->row0 + h->nloc));
      return N2V2R_ERR_BAD_ARG;
    }
    for (int64_t r = 0; r < n_rows; ++r)  // a non-monotone block would hand the SpMM bad spans
      if (indptr[r + 1] < indptr[r]) {
        h->set_err("layer %d: indptr not monotone", k);
        return N2V2R_ERR_BAD_ARG;
      }
    if (!host_indices_in_range(nnz, indices, n)) {
      h->set_err("layer %d: column index out of range", k);
      return N2V2R_ERR_BAD_ARG;
    }
    for (int j = 0; j < h->K; ++j)
      if (j != k && h->layers[j]->loaded && h->layers[j]->dense) {
        h->err = "layers must be all CSR or all dense";
        return N2V2R_ERR_BAD_ARG;
      }
    LayerDev& L = *h->layers[k];
    L.dense = false;
    L.drop_col_blocks();
    L.n_rows = h->nloc;
    L.unit = upload_rows(h->stream, 0, n_rows, indptr, indices, data, L.indptr, L.indices, L.data,
                         L.nnz);
    h->h2d_layer_bytes += 8 * (n_rows + 1) + (L.unit ? 4 : 8) * L.nnz;
    L.symmetric = true;
    L.loaded = true;
    h->have_embedding = false;
    return N2V2R_OK;
  });
}

// float32 column sums of layer k for all N nodes (row sums of the local rows of A^T, gathered)
int n2v2r_column_sums(n2v2r_handle* h, int k, float* out) {
  if (h && h->multi()) return multi_column_sums(h, k, out);
  return guarded(h, [&]() -> int {
    if (k < 0 || k >= h->K || !out || !h->layers[k]->loaded) return N2V2R_ERR_BAD_ARG;
    DevBuf o, g;
    o.ensure(sizeof(float) * h->npad);
    if (h->layers[k]->dense) {
      DevBuf ones;
      ones.ensure(sizeof(float) * h->n);
      std::vector<float> one(h->n, 1.f);
      HIPCHK(hipMemcpy(ones.p, one.data(), sizeof(float) * h->n, hipMemcpyHostToDevice));
      h->dense_apply(h->layers[k]->dense_at(), h->layers[k]->lda, ones.as<float>(), 1, 1,
                     o.as<float>(), 1, 0.f, nullptr);
    } else {
      HIPCHK(n2v2r_launch_row_sums(h->layers[k]->csr_t(), o.as<float>(), h->stream));
    }
    const float* src = o.as<float>();
    if (h->comm) {
      g.ensure(sizeof(float) * h->world * h->npad);
      h->comm->allgather(o.p, g.p, sizeof(float) * h->npad, h->stream);
      src = g.as<float>();
    }
    HIPCHK(hipMemcpyAsync(out, src, sizeof(float) * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

// Bipartite projection (replaces bipartite_to_unipartite_projection, preprocessing_utils.py:16-32,
// which network_transform applies to non-square layers, :130-132): out = W^T W (n x n,
// on_columns) or W W^T (m x m) for a host row-major m x n fp64 W, in fp64 as the reference's
// float64 np.matmul (syrk_f64_kernel: v_mfma_f64_16x16x4_f64, exactly symmetric output).
int n2v2r_project(n2v2r_handle* h, int64_t m, int64_t n, const double* W, int on_columns,
                  double* out) {
  if (h && h->multi()) h = h->ranks[0];  // no collective: rank 0's GPU
  return guarded(h, [&]() -> int {
    if (m < 1 || n < 1 || !W || !out) return N2V2R_ERR_BAD_ARG;
    DevBuf w, o;
    w.ensure(sizeof(double) * m * n);
    HIPCHK(hipMemcpyAsync(w.p, W, sizeof(double) * m * n, hipMemcpyHostToDevice, h->stream));
    // columns: X = W (k = row of W, i = column); rows: X = W^T (k = column, i = row)
    const int64_t r = on_columns ? n : m, kd = on_columns ? m : n;
    const int64_t sk = on_columns ? n : 1, si = on_columns ? 1 : n;
    o.ensure(sizeof(double) * r * r);
    HIPCHK(n2v2r_launch_syrk_f64(w.as<double>(), sk, si, kd, r, o.as<double>(), r, h->stream));
    HIPCHK(hipMemcpyAsync(out, o.p, sizeof(double) * r * r, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return N2V2R_OK;
  });
}

}  // extern "C"

// Host-side Rayleigh-Ritz solver for the block Krylov-Schur eigensolver: the top-p
// eigenpairs of a small dense symmetric fp64 matrix H (c x c, c <= ~1024).
//
//   1. Householder tridiagonalisation H = Q T Q^T (reflectors kept below the subdiagonal)
//   2. implicit QL (eigenvalues only) on T, the p largest kept
//   3. inverse iteration on T (tridiagonal LU with partial pivoting), modified Gram-Schmidt
//      inside clusters of near-degenerate eigenvalues (|lambda_i - lambda_j| <= 1e-7 ||T||)
//   4. back-transformation Z <- Q Z by the stored reflectors
// Cost ~ (4/3) c^3 + 2 c^2 p flops: only the wanted vectors are formed.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

// Solve (T - lambda I) x = b in place (b -> x) by Gaussian elimination with partial pivoting
// on the tridiagonal (d, e): the factorisation grows one extra superdiagonal.
void tri_shift_solve(int n, const double* d, const double* e, double lambda, double tiny,
                     double* b, std::vector<double>& wk) {
  wk.resize(5 * (size_t)n);
  double* dg = wk.data();        // diagonal of U
  double* u1 = dg + n;           // first superdiagonal of U
  double* u2 = u1 + n;           // second superdiagonal of U
  double* lm = u2 + n;           // multipliers
  double* swp = lm + n;          // 1.0 where rows i, i+1 were interchanged
  // working copies of the current row
  double a = d[0] - lambda;      // current diagonal candidate
  double c = (n > 1) ? e[0] : 0.0;  // current super
  for (int i = 0; i < n - 1; ++i) {
    const double sub = e[i];           // T[i+1][i]
    const double nd = d[i + 1] - lambda;
    const double ns = (i + 1 < n - 1) ? e[i + 1] : 0.0;
    if (std::fabs(a) >= std::fabs(sub)) {
      if (std::fabs(a) < tiny) a = (a < 0 ? -tiny : tiny);
      const double m = sub / a;
      lm[i] = m;
      swp[i] = 0.0;
      dg[i] = a;
      u1[i] = c;
      u2[i] = 0.0;
      a = nd - m * c;
      c = ns;
    } else {
      // swap rows i and i+1
      const double m = a / sub;
      lm[i] = m;
      swp[i] = 1.0;
      dg[i] = sub;
      u1[i] = nd;
      u2[i] = ns;
      a = c - m * nd;
      c = -m * ns;
    }
  }
  if (std::fabs(a) < tiny) a = (a < 0 ? -tiny : tiny);
  dg[n - 1] = a;
  // forward substitution with the row interchanges
  for (int i = 0; i < n - 1; ++i) {
    if (swp[i] != 0.0) std::swap(b[i], b[i + 1]);
    b[i + 1] -= lm[i] * b[i];
  }
  // back substitution
  b[n - 1] /= dg[n - 1];
  if (n > 1) b[n - 2] = (b[n - 2] - u1[n - 2] * b[n - 1]) / dg[n - 2];
  for (int i = n - 3; i >= 0; --i) b[i] = (b[i] - u1[i] * b[i + 1] - u2[i] * b[i + 2]) / dg[i];
}

}  // namespace

// Top-p eigenpairs of the symmetric tridiagonal T = tridiag(e, d, e) (d: n, e: n-1).
// w[p] descending; Y: p x n, row j = unit eigenvector of w[j] (column-major n x p).
extern "C" int n2v2r_host_tridiag_eig_top(int n, const double* d_in, const double* e_in, int p,
                                          double* w, double* Y) {
  if (n <= 0 || p <= 0 || p > n) return 1;
  std::vector<double> d(d_in, d_in + n), e(std::max(n - 1, 1), 0.0);
  for (int i = 0; i < n - 1; ++i) e[i] = e_in[i];
  // --- 2. all eigenvalues of T by implicit QL (no vectors), keep the p largest --------
  const double eps = 2.220446049250313e-16;
  double tnorm = 0.0;
  for (int i = 0; i < n; ++i) {
    const double r = (i > 0 ? std::fabs(e[i - 1]) : 0.0) + (i < n - 1 ? std::fabs(e[i]) : 0.0);
    tnorm = std::max(tnorm, std::fabs(d[i]) + r);
  }
  {
    std::vector<double> dd(d), ee(n, 0.0);
    for (int i = 0; i < n - 1; ++i) ee[i] = e[i];
    for (int l = 0; l < n; ++l) {
      int iter = 0;
      int m;
      do {
        for (m = l; m < n - 1; ++m) {
          const double s = std::fabs(dd[m]) + std::fabs(dd[m + 1]);
          if (std::fabs(ee[m]) <= eps * s) break;
        }
        if (m != l) {
          if (++iter > 60) break;
          double g = (dd[l + 1] - dd[l]) / (2.0 * ee[l]);
          double r = std::sqrt(g * g + 1.0);
          g = dd[m] - dd[l] + ee[l] / (g + (g >= 0 ? std::fabs(r) : -std::fabs(r)));
          double s = 1.0, c = 1.0, pp = 0.0;
          int i;
          bool underflow = false;
          for (i = m - 1; i >= l; --i) {
            double f = s * ee[i];
            const double bb = c * ee[i];
            r = std::sqrt(f * f + g * g);  // |f|, |g| << 1e150 here: no hypot needed
            ee[i + 1] = r;
            if (r == 0.0) {
              dd[i + 1] -= pp;
              ee[m] = 0.0;
              underflow = true;
              break;
            }
            s = f / r;
            c = g / r;
            g = dd[i + 1] - pp;
            r = (dd[i] - g) * s + 2.0 * c * bb;
            pp = s * r;
            dd[i + 1] = g + pp;
            g = c * r - bb;
          }
          if (underflow) continue;
          dd[l] -= pp;
          ee[l] = g;
          ee[m] = 0.0;
        }
      } while (m != l);
    }
    std::sort(dd.begin(), dd.end(), [](double a, double b) { return a > b; });
    for (int j = 0; j < p; ++j) w[j] = dd[j];
  }

  // --- 3. inverse iteration ----------------------------------------------------------
  std::vector<double> x(n), wk;
  double* T = Y;  // column j at T[j*n]
  // fp64 inverse iteration leaves vectors of eigenvalues delta apart orthogonal to
  // ~eps ||T|| / delta, so only near-degenerate ones (delta <= 1e-7 ||T||) need Gram-Schmidt;
  // LAPACK's 1e-3 ||T|| lumps the whole bulk edge of a Krylov projection into one cluster.
  const double clus = 1e-7 * std::max(tnorm, 1e-300);
  const double tiny = std::max(eps * tnorm, 1e-300);
  int cluster_start = 0;
  uint64_t seed = 0x9E3779B97F4A7C15ull;
  for (int j = 0; j < p; ++j) {
    if (j > 0 && std::fabs(w[j - 1] - w[j]) > clus) cluster_start = j;
    // perturb identical eigenvalues slightly, as dstein does
    double lam = w[j];
    for (int i = 0; i < n; ++i) {
      seed = seed * 6364136223846793005ull + 1442695040888963407ull;
      x[i] = ((double)(seed >> 11) / 9007199254740992.0) - 0.5;
    }
    for (int it = 0; it < 3; ++it) {
      tri_shift_solve(n, d.data(), e.data(), lam, tiny, x.data(), wk);
      // MGS against the previous members of the cluster
      for (int q = cluster_start; q < j; ++q) {
        const double* tq = &T[(size_t)q * n];
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += tq[i] * x[i];
        for (int i = 0; i < n; ++i) x[i] -= s * tq[i];
      }
      double nr = 0.0;
      for (int i = 0; i < n; ++i) nr += x[i] * x[i];
      nr = std::sqrt(nr);
      if (!(nr > 0)) {
        x[j % n] = 1.0;
        nr = 1.0;
      }
      for (int i = 0; i < n; ++i) x[i] /= nr;
    }
    std::memcpy(&T[(size_t)j * n], x.data(), sizeof(double) * n);
  }

  return 0;
}

// A: n x n row-major symmetric (destroyed).  Returns 0 on success.
// w[p]: eigenvalues, descending.  Z: n x p row-major, column j = eigenvector of w[j].
extern "C" int n2v2r_host_sym_eig_top(int n, double* A, int p, double* w, double* Z) {
  if (n <= 0 || p <= 0 || p > n) return 1;
  std::vector<double> d(n), e(std::max(n - 1, 1), 0.0), tau(std::max(n - 1, 1), 0.0);
  std::vector<double> v(n), pv(n), wv(n);
  // --- 1. tridiagonalisation on the lower triangle (dsytd2-style) -----------------
  // Row-major lower storage: row i holds A[i][0..i].  The reflector of step k is stored in
  // column k below the subdiagonal (A[k+2..n-1][k]).
  for (int k = 0; k < n - 2; ++k) {
    const int m = n - k - 1;  // length of x = A[k+1:, k]
    const int o = k + 1;
    double* col = &v[0];
    for (int i = 0; i < m; ++i) col[i] = A[(size_t)(o + i) * n + k];
    double sig = 0.0;
    for (int i = 1; i < m; ++i) sig += col[i] * col[i];
    const double x0 = col[0];
    d[k] = A[(size_t)k * n + k];
    if (sig == 0.0) {
      tau[k] = 0.0;
      e[k] = x0;
      continue;
    }
    const double nrm = std::sqrt(x0 * x0 + sig);
    const double beta = (x0 >= 0) ? -nrm : nrm;
    const double t = (beta - x0) / beta;
    const double scale = 1.0 / (x0 - beta);
    col[0] = 1.0;
    for (int i = 1; i < m; ++i) col[i] *= scale;
    tau[k] = t;
    e[k] = beta;
    for (int i = 1; i < m; ++i) A[(size_t)(o + i) * n + k] = col[i];
    // p = A22 v using the lower triangle: one pass per row (dot for j<i, axpy into p_j)
    double* __restrict__ pvp = pv.data();
    const double* __restrict__ cv = col;
    for (int i = 0; i < m; ++i) pvp[i] = 0.0;
    for (int i = 0; i < m; ++i) {
      const double* __restrict__ row = &A[(size_t)(o + i) * n + o];
      const double vi = cv[i];
      double s = 0.0;
#pragma omp simd reduction(+ : s)
      for (int j = 0; j < i; ++j) {
        s += row[j] * cv[j];
        pvp[j] += row[j] * vi;
      }
      pvp[i] += s + row[i] * vi;
    }
    double pvv = 0.0;
    for (int i = 0; i < m; ++i) {
      pv[i] *= t;
      pvv += pv[i] * col[i];
    }
    const double half = 0.5 * t * pvv;
    for (int i = 0; i < m; ++i) wv[i] = pv[i] - half * col[i];
    // A22 -= v w^T + w v^T on the lower triangle
    const double* __restrict__ wvp = wv.data();
    for (int i = 0; i < m; ++i) {
      double* __restrict__ row = &A[(size_t)(o + i) * n + o];
      const double vi = cv[i], wi = wvp[i];
#pragma omp simd
      for (int j = 0; j <= i; ++j) row[j] -= vi * wvp[j] + wi * cv[j];
    }
  }
  if (n >= 2) {
    d[n - 2] = A[(size_t)(n - 2) * n + (n - 2)];
    e[n - 2] = A[(size_t)(n - 1) * n + (n - 2)];
    tau[n - 2] = 0.0;
  }
  d[n - 1] = A[(size_t)(n - 1) * n + (n - 1)];

  // --- 2./3. eigenpairs of T -------------------------------------------------------
  std::vector<double> T(n * (size_t)p);  // column j at T[j*n]
  if (n2v2r_host_tridiag_eig_top(n, d.data(), e.data(), p, w, T.data()) != 0) return 1;

  // --- 4. back-transformation: z <- H_0 H_1 ... H_{n-3} z ------------------------------
  for (int k = n - 3; k >= 0; --k) {
    if (tau[k] == 0.0) continue;
    const int m = n - k - 1;
    v[0] = 1.0;
    for (int i = 1; i < m; ++i) v[i] = A[(size_t)(k + 1 + i) * n + k];
    for (int j = 0; j < p; ++j) {
      double* z = &T[(size_t)j * n + (k + 1)];
      double s = 0.0;
      for (int i = 0; i < m; ++i) s += v[i] * z[i];
      s *= tau[k];
      for (int i = 0; i < m; ++i) z[i] -= s * v[i];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < p; ++j) Z[(size_t)i * p + j] = T[(size_t)j * n + i];
  return 0;
}

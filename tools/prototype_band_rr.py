"""Design prototype (NOT product, NOT oracle): numpy model of the banded Rayleigh-Ritz.

In a block Krylov-Schur cycle the projected matrix H = Q^T M Q is, in exact arithmetic,
block tridiagonal (b x b blocks, upper-triangular sub-diagonal blocks R_j = Q_j^T M Q_{j-1})
plus an arrow: the kept Ritz block X (diagonal Theta) couples only to the first new block E.
This prototype checks the reduction the GPU kernels implement:
  1. arrow -> band: offset-b Householder reduction of [[Theta, B^T], [B, A_E]] in reversed
     index order (E untouched), so [X P, E, Z_2, ...] is a band matrix of half-bandwidth b;
  2. band -> tridiagonal by bulge chasing (one reflector of length <= b per step, sweep i
     annihilates column i; step j of sweep i+1 may run once step j+1 of sweep i is done);
  3. eigenvalues of the tridiagonal, eigenvectors by inverse iteration on the BAND matrix
     (partial-pivoting band LU), X part mapped back through the arrow reflectors.
Run: python tools/prototype_band_rr.py
"""
import numpy as np


def house(x):
    """v (v[0] = 1), tau, beta with (I - tau v v^T) x = beta e_0."""
    x0 = x[0]
    sig = float(np.dot(x[1:], x[1:]))
    v = np.zeros_like(x)
    v[0] = 1.0
    if sig == 0.0:
        return v, 0.0, x0
    nrm = np.sqrt(x0 * x0 + sig)
    beta = -nrm if x0 >= 0 else nrm
    tau = (beta - x0) / beta
    v[1:] = x[1:] / (x0 - beta)
    return v, tau, beta


def arrow_to_band(theta, BT, AE, b):
    """A = [[diag(theta), BT], [BT^T, AE]] (n_a = keep + b) -> (A' band(b), reflectors) with
    A' = P^T A P, P acting on the X part only.  Done on R = J A J (reversed order)."""
    keep = len(theta)
    na = keep + b
    A = np.zeros((na, na))
    A[:keep, :keep] = np.diag(theta)
    A[:keep, keep:] = BT
    A[keep:, :keep] = BT.T
    A[keep:, keep:] = 0.5 * (AE + AE.T)
    R = A[::-1, ::-1].copy()
    refl = []
    for k in range(0, na - b - 1):
        x = R[k + b:, k].copy()
        if len(x) < 2:
            break
        v, tau, beta = house(x)
        u = np.zeros(na)
        u[k + b:] = v
        p = tau * (R @ u)
        K = 0.5 * tau * np.dot(p, u)
        w = p - K * u
        R -= np.outer(u, w) + np.outer(w, u)
        R[k + b, k] = R[k, k + b] = beta
        R[k + b + 1:, k] = 0.0
        R[k, k + b + 1:] = 0.0
        refl.append((k + b, v, tau))
    return R[::-1, ::-1].copy(), refl


def apply_arrow_back(refl, na, y):
    """S[:na] = P y[:na], P = J Q J, Q = H_0 H_1 ... (reversed coordinates)."""
    z = y[:na][::-1].copy()
    for s, v, tau in reversed(refl):
        z[s:] -= tau * v * np.dot(v, z[s:])
    out = y.copy()
    out[:na] = z[::-1]
    return out


def band_to_tridiag(Aband_full, w):
    """Bulge chasing on a dense copy (only band + bulge entries ever nonzero)."""
    A = Aband_full.copy()
    n = A.shape[0]
    for i in range(n - 2):
        m = min(w, n - 1 - i)
        if m < 2:
            continue
        x = A[i + 1:i + 1 + m, i].copy()
        v, tau, beta = house(x)
        A[i + 1:i + 1 + m, i] = 0.0
        A[i, i + 1:i + 1 + m] = 0.0
        A[i + 1, i] = A[i, i + 1] = beta
        s = i + 1
        D = A[s:s + m, s:s + m]
        p = tau * D @ v
        K = 0.5 * tau * np.dot(p, v)
        ww = p - K * v
        A[s:s + m, s:s + m] = D - np.outer(v, ww) - np.outer(ww, v)
        while True:
            r0 = s + m
            if r0 >= n:
                break
            mr = min(w, n - r0)
            O = A[r0:r0 + mr, s:s + m].copy()
            # bandwidth check: nothing outside the chased window
            assert np.all(A[r0 + mr:, s:s + m] == 0.0)
            O = O - tau * np.outer(O @ v, v)
            v2, tau2, beta2 = house(O[:, 0].copy())
            O = O - tau2 * np.outer(v2, v2 @ O)
            O[:, 0] = 0.0
            O[0, 0] = beta2
            A[r0:r0 + mr, s:s + m] = O
            A[s:s + m, r0:r0 + mr] = O.T
            D = A[r0:r0 + mr, r0:r0 + mr]
            p = tau2 * D @ v2
            K = 0.5 * tau2 * np.dot(p, v2)
            ww = p - K * v2
            A[r0:r0 + mr, r0:r0 + mr] = D - np.outer(v2, ww) - np.outer(ww, v2)
            v, tau, s, m = v2, tau2, r0, mr
    d = np.diag(A).copy()
    e = np.diag(A, -1).copy()
    off = A - np.diag(d) - np.diag(e, -1) - np.diag(e, 1)
    return d, e, np.abs(off).max()


def band_lu_solve(A, lam, w, rhs_list):
    """Partial-pivoting LU of (A - lam I) restricted to the band (dense storage, band logic)."""
    n = A.shape[0]
    U = A - lam * np.eye(n)
    piv = np.arange(n)
    L = np.zeros((n, w))
    perm = []
    tiny = 2.2e-16 * np.abs(A).max()
    for k in range(n):
        hi = min(n, k + w + 1)
        p = k + int(np.argmax(np.abs(U[k:hi, k])))
        perm.append(p)
        if p != k:
            U[[k, p], k:min(n, k + 2 * w + 1)] = U[[p, k], k:min(n, k + 2 * w + 1)]
        if abs(U[k, k]) < tiny:
            U[k, k] = tiny
        for r in range(k + 1, hi):
            l = U[r, k] / U[k, k]
            L[k, r - k - 1] = l
            U[r, k:min(n, k + 2 * w + 1)] -= l * U[k, k:min(n, k + 2 * w + 1)]
    outs = []
    for rhs in rhs_list:
        x = rhs.copy()
        for k in range(n):
            p = perm[k]
            if p != k:
                x[k], x[p] = x[p], x[k]
            hi = min(n, k + w + 1)
            x[k + 1:hi] -= L[k, :hi - k - 1] * x[k]
        for k in range(n - 1, -1, -1):
            hi = min(n, k + 2 * w + 1)
            x[k] = (x[k] - np.dot(U[k, k + 1:hi], x[k + 1:hi])) / U[k, k]
        outs.append(x)
    return outs


def band_rr(theta_prev, hloc, kry0_blocks, nblocks, b, keep_out):
    """Band Rayleigh-Ritz from the saved local Grams.  hloc[j] = [Q_loc]^T W_j (rows: local
    blocks' columns, b columns).  Returns top keep_out (theta, S) in the basis order."""
    c = nblocks * b
    kp = kry0_blocks * b
    A = np.zeros((c, c))
    for j in range(kry0_blocks, nblocks):
        G = hloc[j]
        o = j * b
        A[o:o + b, o:o + b] = 0.5 * (G[-b:] + G[-b:].T)
        if j > kry0_blocks:
            Hup = np.triu(G[:b].T)  # H[j, j-1] = (Q_{j-1}^T W_j)^T, upper triangular part
            A[o:o + b, o - b:o] = Hup
            A[o - b:o, o:o + b] = Hup.T
    refl = []
    if kp > 0:
        G = hloc[kry0_blocks]
        Ared, refl = arrow_to_band(theta_prev, G[:kp], G[kp:], b)
        na = kp + b
        A[:na, :na] = Ared
    # band check
    n = c
    for i in range(n):
        for j in range(n):
            if abs(i - j) > b:
                assert A[i, j] == 0.0
    d, e, offmax = band_to_tridiag(A, b)
    T = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
    th = np.linalg.eigvalsh(T)[::-1][:keep_out]
    rng = np.random.default_rng(0)
    S = np.zeros((c, keep_out))
    for j in range(keep_out):
        x = rng.standard_normal(c)
        for _ in range(2):
            x = band_lu_solve(A, th[j], b, [x])[0]
            x -= S[:, :j] @ (S[:, :j].T @ x) if False else 0.0
            x /= np.linalg.norm(x)
        S[:, j] = x
    S = np.stack([apply_arrow_back(refl, kp + b, S[:, j]) if kp > 0 else S[:, j]
                  for j in range(keep_out)], axis=1)
    return th, S, offmax, A


def test_random():
    rng = np.random.default_rng(1)
    b, kp_blocks, nb = 8, 3, 12
    c = nb * b
    # a matrix with the Krylov-Schur structure
    theta = np.sort(rng.standard_normal(kp_blocks * b))[::-1] * 3
    hloc = {}
    H = np.zeros((c, c))
    kp = kp_blocks * b
    H[:kp, :kp] = np.diag(theta)
    for j in range(kp_blocks, nb):
        o = j * b
        D = rng.standard_normal((b, b))
        D = D + D.T
        H[o:o + b, o:o + b] = D
        if j == kp_blocks:
            BT = rng.standard_normal((kp, b))
            H[:kp, o:o + b] = BT
            H[o:o + b, :kp] = BT.T
            hloc[j] = np.vstack([BT, D])
        else:
            R = np.triu(rng.standard_normal((b, b)))
            H[o:o + b, o - b:o] = R
            H[o - b:o, o:o + b] = R.T
            hloc[j] = np.vstack([R.T, D])
    th, S, offmax, _ = band_rr(theta, hloc, kp_blocks, nb, b, 20)
    ev, EV = np.linalg.eigh(H)
    ev, EV = ev[::-1][:20], EV[:, ::-1][:, :20]
    print("theta err", np.abs(th - ev).max(), "chase off-tridiag", offmax)
    res = np.linalg.norm(H @ S - S * th[None, :], axis=0).max()
    print("residual", res, "orth", np.abs(S.T @ S - np.eye(20)).max())
    assert np.abs(th - ev).max() < 1e-10 and res < 1e-9


def test_first_cycle():
    rng = np.random.default_rng(2)
    b, nb = 8, 10
    c = nb * b
    hloc = {}
    H = np.zeros((c, c))
    for j in range(nb):
        o = j * b
        D = rng.standard_normal((b, b))
        D = D + D.T
        H[o:o + b, o:o + b] = D
        if j == 0:
            hloc[j] = D
        else:
            R = np.triu(rng.standard_normal((b, b)))
            H[o:o + b, o - b:o] = R
            H[o - b:o, o:o + b] = R.T
            hloc[j] = np.vstack([R.T, D])
    th, S, offmax, _ = band_rr(None, hloc, 0, nb, b, 16)
    ev = np.linalg.eigvalsh(H)[::-1][:16]
    res = np.linalg.norm(H @ S - S * th[None, :], axis=0).max()
    print("first cycle theta err", np.abs(th - ev).max(), "residual", res)
    assert np.abs(th - ev).max() < 1e-10 and res < 1e-9


if __name__ == "__main__":
    test_random()
    test_first_cycle()

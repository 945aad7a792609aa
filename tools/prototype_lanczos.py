"""Design prototype (NOT product, NOT oracle): numpy model of the GPU eigensolver.

Block Krylov-Schur / thick-restart block Lanczos on M = sum_k A_k A_k^T with explicit
Rayleigh-Ritz.  fp32 basis + fp32 SpMM (as on the GPU), fp64 small reductions.  Used to pick
block size, basis size and the residual tolerance before writing the HIP driver.
"""
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, ".")


def gram_apply(layers, layersT, X):
    W = None
    for A, AT in zip(layers, layersT):
        Z = (AT @ X).astype(np.float32)
        Y = (A @ Z).astype(np.float32)
        W = Y if W is None else W + Y
    return W


def cholqr(Z):
    for _ in range(2):
        G = Z.T.astype(np.float64) @ Z.astype(np.float64)
        G = 0.5 * (G + G.T)
        sh = 0.0
        while True:
            try:
                R = np.linalg.cholesky(G + sh * np.eye(G.shape[0]) * np.trace(G)).T
                break
            except np.linalg.LinAlgError:
                sh = max(sh * 10, 1e-12)
        Z = (Z.astype(np.float64) @ np.linalg.inv(R)).astype(np.float32)
    return Z


def block_ks(layers, d, b=None, maxcols=None, keep=None, tol=1e-6, maxcycles=200, seed=0,
             verbose=True):
    layersT = [A.T.tocsr() for A in layers]
    n = layers[0].shape[0]
    b = b or d
    maxcols = maxcols or 4 * b
    keep = keep or max(d + b // 2, 2 * d)
    rng = np.random.default_rng(seed)
    Q = cholqr(rng.standard_normal((n, b)).astype(np.float32))
    W = gram_apply(layers, layersT, Q)
    napps = b
    for cyc in range(maxcycles):
        while Q.shape[1] < maxcols:
            Wl = W[:, -b:]
            Z = Wl - Q @ (Q.T.astype(np.float64) @ Wl).astype(np.float32)
            Z = Z - Q @ (Q.T.astype(np.float64) @ Z).astype(np.float32)
            Qn = cholqr(Z)
            Q = np.hstack([Q, Qn])
            W = np.hstack([W, gram_apply(layers, layersT, Qn)])
            napps += b
        H = Q.T.astype(np.float64) @ W.astype(np.float64)
        H = 0.5 * (H + H.T)
        th, S = np.linalg.eigh(H)
        th, S = th[::-1], S[:, ::-1]
        X = (Q.astype(np.float64) @ S[:, :keep])
        MX = (W.astype(np.float64) @ S[:, :keep])
        R = MX - X * th[None, :keep]
        res = np.linalg.norm(R, axis=0) / th[0]
        if verbose:
            print(f"cycle {cyc} apps {napps} maxres[:d] {res[:d].max():.2e} "
                  f"res[d-1] {res[d-1]:.2e}")
        if res[:d].max() < tol:
            return th[:d], X[:, :d].astype(np.float32), napps, cyc
        # next block from the old basis, then truncate
        Wl = W[:, -b:]
        Z = Wl - Q @ (Q.T.astype(np.float64) @ Wl).astype(np.float32)
        Z = Z - Q @ (Q.T.astype(np.float64) @ Z).astype(np.float32)
        Q = np.hstack([X.astype(np.float32), None][:1])
        W = MX.astype(np.float32)
        Z = Z - Q @ (Q.T.astype(np.float64) @ Z).astype(np.float32)
        Qn = cholqr(Z)
        Q = np.hstack([Q, Qn])
        W = np.hstack([W, gram_apply(layers, layersT, Qn)])
        napps += b
    return th[:d], X[:, :d].astype(np.float32), napps, maxcycles


def embed_from_u(layers, U, theta):
    s = np.sqrt(theta)
    Y = np.stack([(A.T @ U) / np.sqrt(s)[None, :] for A in layers])
    return Y, s


if __name__ == "__main__":
    from node2vec2rank_amd import synthetic
    from oracle import n2v2r_oracle as orc
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    b = int(sys.argv[3]) if len(sys.argv) > 3 else d
    mc = int(sys.argv[4]) if len(sys.argv) > 4 else 4 * b
    tol = float(sys.argv[5]) if len(sys.argv) > 5 else 1e-6
    layers = synthetic.er_layers(n, 20, 2)
    t = time.time()
    th, U, napps, cyc = block_ks(layers, d, b=b, maxcols=mc, tol=tol)
    print("proto time", time.time() - t, "apps", napps)
    Yp, sp_ = embed_from_u(layers, U, th)
    t = time.time()
    Yr, sr, _ = orc.uase(layers, d, seed=42)
    print("svds time", time.time() - t)
    print("sigma rel err", np.abs(sp_ - sr).max() / sr[0])
    Ya = orc.align_signs(Yp, Yr)
    print("Y max abs err / max|Y|", np.abs(Ya - Yr).max() / np.abs(Yr).max())
    dims = [d // 8, d // 4, d // 2, d]
    for m in ("cosine", "euclidean"):
        for dim in dims:
            e = np.abs(orc.distances_fast(Ya[0, :, :dim], Ya[1, :, :dim], m)
                       - orc.distances_fast(Yr[0, :, :dim], Yr[1, :, :dim], m)).max()
            print(m, dim, "dist max abs err", e)

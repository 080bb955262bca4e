"""CPU oracle of the D = 3 path -- TEST INFRASTRUCTURE ONLY.

Only tests/ and __graft_entry__.smoke() use this module, as the checker of
libdgs.so's dgs_volume_* entry points; the product never imports it.

PARITY UNPINNED against the reference: the reference has no D = 3 path (its device
functions stop at D = 2, cuda_sampler/forward.cu:164-275 and backward.cu:108-416; its radius
is 0 at D = 3, forward.cu:52-61).  What this restates is the reference's per-pair arithmetic
carried to three dimensions (include/dgs_volume.h):
  * X_d = wrap(mean_d - sample_d), the per-axis torus wrap of forward.cu:149-157;
  * power = -0.5 * (c00 X0 X0 + c11 X1 X1 + c22 X2 X2) - (c01 X0 X1 + c02 X0 X2 + c12 X1 X2),
    in float32 in exactly this operation order (no contraction; the GPU does the same), a pair
    with power > 0 skipped as in forward.cu:166-171;
  * the four functions in index form, which at D = 2 are exactly the expressions of
    forward.cu:164-275 (tests/test_volume_oracle.py checks that);
  * every pair of every Gaussian (brute force: no culling), sums in float64.
The gradient formulas are checked against torch float64 autograd of the forward
(tests/test_volume_oracle.py).
"""
import itertools

import numpy as np

PAIRS = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]  # packed conic order
TRIPLES = [t for t in itertools.combinations_with_replacement(range(3), 3)]
NUNIQUE = [1, 3, 6, 10]


def pidx(i, j):
    return PAIRS.index((min(i, j), max(i, j)))


def umap(function):
    """unique component of every full output index (row-major over 3^function)"""
    if function == 0:
        return [0]
    if function == 1:
        return [0, 1, 2]
    if function == 2:
        return [pidx(i, j) for i in range(3) for j in range(3)]
    return [TRIPLES.index(tuple(sorted((i, j, k)))) for i in range(3) for j in range(3) for k in range(3)]


def _wrap(x):
    """forward.cu:149-157 on a float32 array"""
    x = x.copy()
    big = np.abs(x) > np.float32(1.0)
    pos = big & (x >= 0)
    neg = big & (x < 0)
    two = np.float32(2.0)
    x[pos] = np.fmod(x[pos], two) - two
    x[neg] = np.fmod(x[neg], two) + two
    return x


def _pairs(means, conics, s):
    """X [P, n, 3] (float32), power and G for the samples s [n, 3] against every Gaussian"""
    m = means[:, None, :].astype(np.float32)
    X = _wrap(m - s[None, :, :].astype(np.float32))
    c = [conics[:, q].astype(np.float32)[:, None] for q in range(6)]
    X0, X1, X2 = X[..., 0], X[..., 1], X[..., 2]
    qd = c[0] * X0 * X0 + c[3] * X1 * X1 + c[5] * X2 * X2
    qo = c[1] * X0 * X1 + c[2] * X0 * X2 + c[4] * X1 * X2
    power = np.float32(-0.5) * qd - qo
    live = power <= 0
    with np.errstate(over="ignore"):
        G = np.where(live, np.exp(np.minimum(power, np.float32(0.0))), np.float32(0.0))
    return X.astype(np.float64), G.astype(np.float64), live


def _amat(conics):
    A = np.zeros((conics.shape[0], 3, 3))
    for q, (i, j) in enumerate(PAIRS):
        A[:, i, j] = A[:, j, i] = conics[:, q]
    return A


def _terms(function, a, A):
    """unique-component terms t [P, n, KU] from a [P, n, 3] and A [P, 3, 3]"""
    if function == 0:
        return np.ones(a.shape[:-1] + (1,))
    if function == 1:
        return a.copy()
    if function == 2:
        return np.stack([a[..., i] * a[..., j] - A[:, i, j][:, None] for i, j in PAIRS], -1)
    return np.stack([A[:, i, j][:, None] * a[..., k] + A[:, i, k][:, None] * a[..., j]
                     + A[:, j, k][:, None] * a[..., i] - a[..., i] * a[..., j] * a[..., k]
                     for i, j, k in TRIPLES], -1)


def forward(function, means, values, conics, samples, chunk=512):
    """out [N, 3^function, C] (float64)"""
    P, N, C = means.shape[0], samples.shape[0], values.shape[1]
    K = 3 ** function
    out = np.zeros((N, K, C))
    if P == 0 or N == 0:
        return out
    A = _amat(conics.astype(np.float64))
    um = umap(function)
    v = values.astype(np.float64)
    for s0 in range(0, N, chunk):
        s = samples[s0:s0 + chunk]
        X, G, _ = _pairs(means, conics, s)
        a = np.einsum("pij,pnj->pni", A, X)
        t = _terms(function, a, A)  # [P, n, KU]
        uo = np.einsum("pn,pnu,pc->nuc", G, t, v)
        out[s0:s0 + chunk] = uo[:, um, :]
    return out


def backward(function, means, values, conics, samples, dL, chunk=512):
    """(dmeans [P, 3], dvalues [P, C], dconics [P, 6]) of sum(dL * out), float64"""
    P, N, C = means.shape[0], samples.shape[0], values.shape[1]
    K, KU = 3 ** function, NUNIQUE[function]
    dm, dv, dc = np.zeros((P, 3)), np.zeros((P, C)), np.zeros((P, 6))
    if P == 0 or N == 0:
        return dm, dv, dc
    A = _amat(conics.astype(np.float64))
    um = umap(function)
    v = values.astype(np.float64)
    dL = dL.reshape(N, K, C).astype(np.float64)
    hs = np.zeros((N, KU, C))
    for f in range(K):
        hs[:, um[f], :] += dL[:, f, :]
    for s0 in range(0, N, chunk):
        s = samples[s0:s0 + chunk]
        h = hs[s0:s0 + chunk]  # [n, KU, C]
        X, G, live = _pairs(means, conics, s)
        a = np.einsum("pij,pnj->pni", A, X)
        t = _terms(function, a, A)
        dv += np.einsum("pn,pnu,nuc->pc", G, t, h)
        hv = np.einsum("pc,nuc->pnu", v, h)  # [P, n, KU]
        phi = np.einsum("pnu,pnu->pn", hv, t)
        g = np.zeros(a.shape)
        e = np.zeros(a.shape[:-1] + (6,))
        if function == 1:
            g = hv.copy()
        elif function == 2:
            for u, (i, j) in enumerate(PAIRS):
                g[..., i] += hv[..., u] * a[..., j]
                g[..., j] += hv[..., u] * a[..., i]
                e[..., pidx(i, j)] -= hv[..., u]
        elif function == 3:
            for u, (i, j, k) in enumerate(TRIPLES):
                hu = hv[..., u]
                g[..., k] += hu * A[:, i, j][:, None]
                g[..., j] += hu * A[:, i, k][:, None]
                g[..., i] += hu * A[:, j, k][:, None]
                g[..., i] -= hu * a[..., j] * a[..., k]
                g[..., j] -= hu * a[..., i] * a[..., k]
                g[..., k] -= hu * a[..., i] * a[..., j]
                e[..., pidx(i, j)] += hu * a[..., k]
                e[..., pidx(i, k)] += hu * a[..., j]
                e[..., pidx(j, k)] += hu * a[..., i]
        Ag = np.einsum("pij,pnj->pni", A, g)
        dm += np.einsum("pn,pni->pi", G, Ag - a * phi[..., None])
        for q, (p_, r) in enumerate(PAIRS):
            dpow = -0.5 * X[..., p_] ** 2 if p_ == r else -X[..., p_] * X[..., r]
            da = g[..., p_] * X[..., p_] if p_ == r else g[..., p_] * X[..., r] + g[..., r] * X[..., p_]
            dc[:, q] += np.einsum("pn,pn->p", G, phi * dpow + da + e[..., q])
    return dm, dv, dc


def gaussians3(P, C=1, seed=0, scale=1.0):
    """Seeded D = 3 field like synthetic.gaussians, float32 numpy:
    means ~ U[-1, 1)^3, anisotropic rotated covariances of scale h = 2 / P^(1/3)."""
    rng = np.random.default_rng(seed)
    means = rng.uniform(-1.0, 1.0, (P, 3))
    h = 2.0 / max(P, 1) ** (1.0 / 3.0) * scale
    sig = h * (0.5 + rng.random((P, 3)))
    q, _ = np.linalg.qr(rng.normal(size=(P, 3, 3)))
    cov = np.einsum("pij,pj,pkj->pik", q, sig ** 2, q)
    inv = np.linalg.inv(cov)
    conics = np.stack([inv[:, i, j] for i, j in PAIRS], -1)
    covs = np.stack([cov[:, i, j] for i, j in PAIRS], -1)
    values = rng.normal(size=(P, C))
    f = np.float32
    return means.astype(f), values.astype(f), covs.astype(f), conics.astype(f)


def samples3(N, seed=4):
    return np.random.default_rng(seed).uniform(-1.0, 1.0, (N, 3)).astype(np.float32)

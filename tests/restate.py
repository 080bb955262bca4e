"""A second, independent restatement of the reference sampler used to PIN the C oracle.

TEST INFRASTRUCTURE ONLY.  The C oracle (oracle/oracle.c) restates the reference literally in
fp32; this module restates it again in a different form so that the two can check each other:

  * binning (radii, tiles touched, per-tile Gaussian lists, sample keys) in numpy float32,
    vectorised per axis: forward.cu:24-83, auxiliary.h:21-31, sampler_impl.cu:54-189;
  * the per-pair forward functions in torch float64 (forward.cu:168-275), so that
    torch.autograd gives the exact gradient the reference's hand-written backward
    (backward.cu:108-416) is meant to compute;
  * the one reference backward term that is NOT the autograd gradient -- D=1 third-derivative
    dL/dconics (backward.cu:322-325) -- transcribed literally in float64.

The reference ships no tests or golden vectors and cannot run here (CUDA only); these checks,
plus the known answers in test_oracle.py, are what "pinned" means for this oracle
("Parity").
"""
import numpy as np
import torch

TILE = np.float32(0.51)  # config.h:18 BLOCK_SIZE
F = {"gaussian": 0, "derivative": 1, "laplacian": 2, "third": 3}


def _sat_int(x):
    """float32 -> int32 as the CUDA cvt instructions do (saturating, NaN -> 0)."""
    x = np.asarray(x, np.float64)
    out = np.where(np.isnan(x), 0.0, np.clip(x, -2147483648.0, 2147483647.0))
    return np.trunc(out).astype(np.int64)


def radius(D, cov):
    """forward.cu:52-61 in float32 with the reference's double promotions."""
    cov = np.asarray(cov, np.float32)
    if D == 1:
        return (3.0 * np.sqrt(cov[:, 0]).astype(np.float64)).astype(np.float32)
    det = cov[:, 0] * cov[:, 2] - cov[:, 1] * cov[:, 1]
    mid = np.float32(0.5) * (cov[:, 0] + cov[:, 2])
    disc = mid * mid - det
    lam = (mid.astype(np.float64) + np.sqrt(np.maximum(1e-6, disc.astype(np.float64)))).astype(np.float32)
    r = (3.0 * np.sqrt(lam).astype(np.float64)).astype(np.float32)
    return np.where(det == 0, np.float32(0), r)


def rect(means, r, off):
    """auxiliary.h:21-31 (TORUS): floor/ceil of ((p - off) -+ r) / 0.51 per axis."""
    p = np.asarray(means, np.float32) - np.asarray(off, np.float32)[None, :]
    lo = (p - r[:, None]) / TILE
    hi = (p + r[:, None]) / TILE
    return _sat_int(np.floor(lo)), _sat_int(np.ceil(hi))


def sample_keys(samples, grid, off):
    """sampler_impl.cu:168-182: (int)((s - off) / 0.51) clamped to [0, grid] per axis."""
    s = np.asarray(samples, np.float32)
    t = _sat_int((s - np.asarray(off, np.float32)[None, :]) / TILE)
    t = np.minimum(np.maximum(t, 0), np.asarray(grid)[None, :])
    if s.shape[1] == 1:
        return t[:, 0]
    return t[:, 1] * grid[0] + t[:, 0]


def bin_gaussians(means, covs, samples, grid, off):
    """(radii, R, tile_lists, skeys).  grid/off as the oracle reports them."""
    means = np.asarray(means, np.float32)
    P, D = means.shape
    grid = np.asarray(grid, np.int64)[:D]
    r = radius(D, covs)
    rmin, rmax = rect(means, r, off)
    span = np.minimum(rmax - rmin, grid[None, :])
    touched = span[:, 0] if D == 1 else span[:, 0] * span[:, 1]
    if D == 2:  # det == 0 -> skipped before the rect (forward.cu:52-55)
        c = np.asarray(covs, np.float32)
        touched = np.where(c[:, 0] * c[:, 2] - c[:, 1] * c[:, 1] == 0, 0, touched)
    # D = 1 with zero variance: radius 0 but the tile still counts in R (no key is emitted)
    radii = np.where(touched > 0, r, np.float32(0))
    T = int(np.prod(grid))
    lists = [[] for _ in range(T)]
    for g in range(P):
        if not radii[g] > 0:
            continue
        axes = []
        for d in range(D):
            lo, hi = int(rmin[g, d]), int(rmax[g, d])
            if hi - lo >= grid[d]:
                lo, hi = 0, int(grid[d])
            x = np.arange(lo, hi)
            # sampler_impl.cu:88-89 with C's truncating %: x = -k*g wraps to g, not 0
            axes.append(np.where(x < 0, grid[d] + np.fmod(x, grid[d]), np.fmod(x, grid[d])))
        if D == 1:
            keys = axes[0]
        else:
            keys = (axes[1][:, None] * grid[0] + axes[0][None, :]).reshape(-1)
        for k in keys:
            if k < T:  # a y-wrap to gy lands past the T tiles and is never rendered
                lists[int(k)].append(g)
    return radii, int(touched.sum()), [np.asarray(sorted(set(l)), np.int64) for l in lists], \
        sample_keys(samples, grid, off)


def pairs(tile_lists, skeys):
    """(sid, gid) of every (sample, Gaussian) pair the reference evaluates."""
    sid, gid = [], []
    T = len(tile_lists)
    for i, t in enumerate(skeys):
        if 0 <= t < T and len(tile_lists[t]):
            sid.append(np.full(len(tile_lists[t]), i, np.int64))
            gid.append(tile_lists[t])
    if not sid:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    return np.concatenate(sid), np.concatenate(gid)


def wrap(X):
    """forward.cu:149-157: |x| > 1 -> fmod(x, 2) -+ 2 (sign of x)."""
    w = torch.where(X >= 0, torch.fmod(X, 2.0) - 2.0, torch.fmod(X, 2.0) + 2.0)
    return torch.where(X.abs() > 1.0, w, X)


def pair_forward(function, D, X, c, v):
    """forward.cu:168-275 per pair in float64: [npairs, K, C] contributions (0 where the
    exponent is > 0).  X [n, D], c [n, S], v [n, C]."""
    fn = F[function]
    if D == 1:
        x, c0 = X[:, 0], c[:, 0]
        x1 = c0 * x
        power = -0.5 * c0 * x * x
        keep = (power <= 0).to(X.dtype)
        G = torch.exp(torch.clamp(power, max=0.0)) * keep
        t = [torch.ones_like(x), x1, x1 * x1 - c0, 2.0 * c0 * x1 - x1 ** 3 + c0 * x1][fn][:, None]
        return (G[:, None] * t)[:, :, None] * v[:, None, :]
    x, y = X[:, 0], X[:, 1]
    c0, c1, c2 = c[:, 0], c[:, 1], c[:, 2]
    power = -0.5 * (c0 * x * x + c2 * y * y) - c1 * x * y
    keep = (power <= 0).to(X.dtype)
    G = torch.exp(torch.clamp(power, max=0.0)) * keep
    a1 = c0 * x + c1 * y
    a2 = c2 * y + c1 * x
    if fn == 0:
        t = torch.ones_like(x)[:, None]
    elif fn == 1:
        t = torch.stack([a1, a2], 1)
    elif fn == 2:
        xy = a1 * a2 - c1
        t = torch.stack([a1 * a1 - c0, xy, xy, a2 * a2 - c2], 1)
    else:
        xxx = 3.0 * c0 * a1 - a1 ** 3
        xxy = 2.0 * c1 * a1 - a1 * a1 * a2 + c0 * a2
        xyy = 2.0 * c1 * a2 - a1 * a2 * a2 + c2 * a1
        yyy = 3.0 * c2 * a2 - a2 ** 3
        t = torch.stack([xxx, xxy, xxy, xyy, xxy, xyy, xyy, yyy], 1)
    return (G[:, None] * t)[:, :, None] * v[:, None, :]


def forward(function, means, values, conics, samples, sid, gid, N):
    """Sum of pair_forward over the pair set: out [N, K, C] (float64, differentiable)."""
    D = means.shape[1]
    K = D ** F[function]
    C = values.shape[1]
    sid_t = torch.as_tensor(sid)
    gid_t = torch.as_tensor(gid)
    X = wrap(means[gid_t] - samples[sid_t])
    contrib = pair_forward(function, D, X, conics[gid_t], values[gid_t])
    out = torch.zeros(N, K, C, dtype=means.dtype)
    return out.index_add(0, sid_t, contrib)


def d1_third_dconics(means, values, conics, samples, dL, sid, gid, P):
    """backward.cu:322-325 transcribed literally (float64): the reference's D=1 third
    dL/dconics, which is not the derivative of the forward."""
    X = wrap(means[gid, 0] - samples[sid, 0])
    c0 = conics[gid, 0]
    x1 = c0 * X
    power = -0.5 * x1 * X
    keep = (power <= 0).to(X.dtype)
    G = torch.exp(torch.clamp(power, max=0.0)) * keep
    dLdG = (values[gid] * dL[sid, 0, :]).sum(1)
    dVdc = (2.0 * X * X - 2.0 * x1 * x1 * X - 0.5 * (2.0 * X * x1 - X) * X * X
            + 0.5 * (x1 * x1 - c0) * x1 * X * X) * dLdG * G
    return torch.zeros(P, dtype=X.dtype).index_add(0, gid, dVdc)[:, None]

"""Seeded synthetic Gaussian fields, generated on the CPU so that the
GPU path and the CPU oracle see identical bits.

    means     ~ U[-1, 1)^D                                   (seed + 0)
    sigma_d   ~ h * U[0.5, 1.5],  h = 2 / P^(1/D)             (seed + 1)
    theta     ~ U[0, pi)  (D = 2; anisotropic rotation)      (seed + 2)
    cov       = R diag(sigma^2) R^T, packed [xx, xy, yy] (D=2) / [xx] (D=1)
    conics    = exact inverse, packed [yy, -xy, xx] / det    (float64, then rounded)
    values    ~ N(0, 1) [P, C]                                (seed + 3)
    samples   ~ U[-1, 1)^D [N, D]                              (seed + 4)
    dL_dout   ~ N(0, 1) [N, K, C]                             (seed + 5)
"""
import math

import torch


def _gen(seed):
    g = torch.Generator()
    g.manual_seed(int(seed))
    return g


def gaussians(P, D=2, C=1, seed=0, scale=1.0, aniso=1.0):
    """Returns float32 CPU tensors (means, values, covariances, conics).  aniso > 1 (D = 2):
    per-Gaussian axis ratios sigma_0 / sigma_1 ~ U[1, aniso] (seed + 6) at the same area
    sigma_0 sigma_1 (the thin-Gaussian workload of bench.py --aniso)."""
    means = torch.rand(P, D, generator=_gen(seed), dtype=torch.float64) * 2.0 - 1.0
    h = 2.0 / (max(P, 1) ** (1.0 / D)) * scale
    sig = h * (0.5 + torch.rand(P, D, generator=_gen(seed + 1), dtype=torch.float64))
    if D == 2 and aniso > 1.0:
        ratio = 1.0 + (aniso - 1.0) * torch.rand(P, generator=_gen(seed + 6), dtype=torch.float64)
        sig = sig * torch.stack([ratio.sqrt(), 1.0 / ratio.sqrt()], -1)
    if D == 1:
        var = sig[:, 0] ** 2
        cov = var[:, None]
        con = (1.0 / var)[:, None]
    else:
        th = torch.rand(P, generator=_gen(seed + 2), dtype=torch.float64) * math.pi
        c, s = torch.cos(th), torch.sin(th)
        s0, s1 = sig[:, 0] ** 2, sig[:, 1] ** 2
        xx = c * c * s0 + s * s * s1
        xy = c * s * (s0 - s1)
        yy = s * s * s0 + c * c * s1
        det = xx * yy - xy * xy
        cov = torch.stack([xx, xy, yy], -1)
        con = torch.stack([yy / det, -xy / det, xx / det], -1)
    values = torch.randn(P, C, generator=_gen(seed + 3), dtype=torch.float64)
    return (means.float(), values.float(), cov.float(), con.float())


def samples(N, D=2, seed=4):
    return (torch.rand(N, D, generator=_gen(seed), dtype=torch.float64) * 2.0 - 1.0).float()


def strip_samples(N, D, rank, world, seed=4):
    """Rank `rank`'s query points of a spatially sharded run (config 4): uniform over strip
    `rank` of `world` equal strips of [-1, 1) along the last axis, so that the union over the
    ranks is uniform on [-1, 1)^D."""
    s = samples(N, D, seed)
    s[:, D - 1] = -1.0 + (2.0 / world) * (rank + 0.5 * (s[:, D - 1] + 1.0))
    return s


def grid_samples(n, D=2):
    """A regular n^D lattice on [-1, 1)^D (the physics-informed collocation grid)."""
    ax = torch.arange(n, dtype=torch.float64) * (2.0 / n) - 1.0
    if D == 1:
        return ax[:, None].float()
    yy, xx = torch.meshgrid(ax, ax, indexing="ij")
    return torch.stack([xx.reshape(-1), yy.reshape(-1)], -1).float()


def out_components(function, D):
    return D ** {"gaussian": 0, "derivative": 1, "laplacian": 2, "third": 3}[function]


def grad_out(N, K, C, seed=5):
    return torch.randn(N, K, C, generator=_gen(seed), dtype=torch.float64).float()


def gaussians3(P, C=1, seed=0, scale=1.0):
    """D = 3 field: means ~ U[-1, 1)^3, per-axis sigma ~ h U[0.5, 1.5] with
    h = 2 / P^(1/3), a random rotation (QR of a normal matrix); conics packed
    [c00 c01 c02 c11 c12 c22] (include/dgs_volume.h), covariances likewise.  float32 CPU."""
    g = _gen(seed)
    means = torch.rand(P, 3, generator=g, dtype=torch.float64) * 2.0 - 1.0
    h = 2.0 / (max(P, 1) ** (1.0 / 3.0)) * scale
    sig = h * (0.5 + torch.rand(P, 3, generator=_gen(seed + 1), dtype=torch.float64))
    q, _ = torch.linalg.qr(torch.randn(P, 3, 3, generator=_gen(seed + 2), dtype=torch.float64))
    cov = q @ torch.diag_embed(sig ** 2) @ q.transpose(1, 2)
    inv = torch.linalg.inv(cov)
    iu = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]
    conics = torch.stack([inv[:, i, j] for i, j in iu], -1)
    covs = torch.stack([cov[:, i, j] for i, j in iu], -1)
    values = torch.randn(P, C, generator=_gen(seed + 3), dtype=torch.float64)
    return means.float(), values.float(), covs.float(), conics.float()


def grid_samples3(n):
    """A regular n^3 lattice on [-1, 1)^3 (the "256^3 grid" of BASELINE config 5)."""
    ax = torch.arange(n, dtype=torch.float64) * (2.0 / n) - 1.0
    z, y, x = torch.meshgrid(ax, ax, ax, indexing="ij")
    return torch.stack([x.reshape(-1), y.reshape(-1), z.reshape(-1)], -1).float()

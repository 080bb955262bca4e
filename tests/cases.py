"""Hand-made input cases shared by the oracle tests, the golden-vector generator and the GPU
parity tests.  Each returns float32 CPU tensors (means, values, covariances, conics, samples).

They cover the edge cases SURVEY.md section 8c lists: torus wrap at +-1, a Gaussian whose
rect spans the whole grid (full range), det == 0 covariance (absent), a non-PD conic (the
`power > 0` skip), the radius floor (tiny Gaussian), the sample clamp to `grid` (aliasing,
sampler_impl.cu:169-177), D = 1 zero variance, and means far outside the sample domain
(rect indices that are negative multiples of the grid: C's `%` wraps them to `grid`).
"""
import math
import numpy as np
import torch

from diff_gaussian_sampling import synthetic as syn


def edge_gaussians():
    means = torch.tensor([[0.995, 0.0], [-0.999, 0.998], [0.1, -0.2], [0.3, 0.3],
                          [-0.5, 0.7], [0.0, -0.999], [0.25, 0.25], [0.6, -0.6]])
    covs = torch.tensor([[1e-3, 0.0, 1e-3], [2e-3, 5e-4, 1e-3], [0.25, 0.0, 0.25], [1.0, 1.0, 1.0],
                         [1e-3, 0.0, 1e-3], [1e-8, 0.0, 1e-8], [1e-3, 0.0, 2e-3], [1e-2, 0.0, 1e-2]])
    conics = torch.tensor([[1e3, 0.0, 1e3], [571.4286, -285.7143, 1142.8572], [4.0, 0.0, 4.0],
                           [1.0, 0.0, 1.0], [50.0, 80.0, 50.0], [1e8, 0.0, 1e8], [1e3, 0.0, 5e2],
                           [-10.0, 0.0, 100.0]])
    values = torch.tensor([[1.0], [-2.0], [0.5], [3.0], [1.5], [2.5], [-1.0], [0.75]])
    return means, values, covs, conics


def edge_case(n_random=3000):
    """Edge Gaussians over random samples plus samples placed on the wrap seams."""
    means, values, covs, conics = edge_gaussians()
    s = syn.samples(n_random, 2, seed=31)
    extra = torch.tensor([[-0.999, 0.0], [0.999, 0.998], [0.995, 0.0], [0.0, 0.999], [0.25, 0.25],
                          [0.3, 0.3], [-1.0, -1.0], [0.99999, 0.99999]])
    return means, values, covs, conics, torch.cat([s, extra])


def aliasing_domain():
    """An x-extent wide enough (> 32 units) that adding 1e-6f is absorbed, so the sample at
    the maximum lands in tile `grid` and aliases into the next row (sampler_impl.cu:169)."""
    f32 = np.float32
    inv = f32(1.0) / f32(0.51)
    for k in range(64, 400):
        d = f32(k) * f32(0.51)
        for cand in (d, np.nextafter(d, f32(np.inf)), np.nextafter(d, f32(0))):
            ext = f32(cand + f32(1e-6))
            g = int(np.ceil(f32(ext * inv)))
            t = int(f32(cand / f32(0.51)))
            if t >= g:
                return float(cand)
    return None


def aliasing_case(n=4000, P=600):
    d = aliasing_domain()
    g = torch.Generator().manual_seed(41)
    s = torch.rand(n, 2, generator=g) * torch.tensor([d, 1.0])
    s = torch.cat([s, torch.tensor([[0.0, 0.0], [d, 0.5], [d, 0.0], [d * 0.5, 1.0]])]).float()
    means = (torch.rand(P, 2, generator=g) * torch.tensor([d, 1.0])).float()
    sig = 0.05 + 0.05 * torch.rand(P, 1, generator=g)
    covs = torch.cat([sig ** 2, torch.zeros(P, 1), sig ** 2], 1).float()
    conics = torch.cat([1 / sig ** 2, torch.zeros(P, 1), 1 / sig ** 2], 1).float()
    values = torch.randn(P, 1, generator=g).float()
    return means, values, covs, conics, s


def d1_zero_variance_case(n=500):
    """D = 1 zero variance: the reference counts a tile (num_rendered) but emits no key."""
    means = torch.tensor([[0.3], [-0.2], [0.7]])
    covs = torch.tensor([[0.0], [1e-3], [4e-3]])
    conics = torch.tensor([[1e9], [1e3], [250.0]])
    values = torch.tensor([[1.0], [2.0], [-1.0]])
    return means, values, covs, conics, syn.samples(n, 1, seed=51)


def far_means_case(n=3000):
    """Means outside [-1, 1): rects start at negative multiples of the grid (C's `%` then
    gives key `grid`, i.e. the next row / past the end) and X wraps by more than one period."""
    g = torch.Generator().manual_seed(121)
    P = 64
    means = (torch.rand(P, 2, generator=g) * 8.0 - 5.0).float()
    means[:8, 0] = torch.tensor([-1.0 - 4 * 0.51, -1.0 - 8 * 0.51, -1.0 - 4 * 0.51 + 0.1, 3.3,
                                 -3.05, -5.1, 2.9, 1.02]).float()
    sig = 0.1 + 0.2 * torch.rand(P, 1, generator=g)
    covs = torch.cat([sig ** 2, torch.zeros(P, 1), 1.5 * sig ** 2], 1).float()
    conics = torch.cat([1 / sig ** 2, torch.zeros(P, 1), 1 / (1.5 * sig ** 2)], 1).float()
    values = torch.randn(P, 1, generator=g).float()
    return means, values, covs, conics, syn.samples(n, 2, seed=122)


def seam_case(D=2, P=400, n=4000, C=1, seed=131):
    """Gaussians hugging the domain edges (|m| within 0.02 of 1): their torus wraps onto the
    cells of the opposite edge, whose nominal extent reaches past the last sample (the tile
    grid spans 2.04 for samples spanning 2) -- the wrap shift must follow the samples."""
    g = torch.Generator().manual_seed(seed)
    side = torch.where(torch.rand(P, D, generator=g) < 0.5, -1.0, 1.0)
    means = (side * (1.0 - 0.02 * torch.rand(P, D, generator=g))).float()
    if D == 2:  # half of them only on one edge, free along the other axis
        free = torch.rand(P, generator=g) < 0.5
        means[free, 1] = (torch.rand(int(free.sum()), generator=g) * 2 - 1).float()
    sig = 0.004 + 0.01 * torch.rand(P, 1, generator=g)
    if D == 1:
        covs = (sig ** 2).float()
        conics = (1 / sig ** 2).float()
    else:
        covs = torch.cat([sig ** 2, 0.3 * sig ** 2, 1.2 * sig ** 2], 1).float()
        det = covs[:, 0] * covs[:, 2] - covs[:, 1] ** 2
        conics = torch.stack([covs[:, 2] / det, -covs[:, 1] / det, covs[:, 0] / det], 1).float()
    values = torch.randn(P, C, generator=g).float()
    return means, values, covs, conics, syn.samples(n, D, seed=seed + 1)


def thin_case(P=6000, n=40000, C=1, seed=151):
    """Thin rotated Gaussians (axis ratio up to 25, sigma_min down to 0.0008): cuts far longer
    than the fine cells in one direction and narrower than a sub-cell in the other -- the sub-cell
    lists' per-row slices (k_sub_lists) and the gather path's row ranges at their most anisotropic,
    a quarter of the means within 0.05 of a torus seam."""
    g = torch.Generator().manual_seed(seed)
    means = torch.rand(P, 2, generator=g, dtype=torch.float64) * 2 - 1
    edge = torch.rand(P, generator=g) < 0.25
    means[edge, 0] = torch.where(means[edge, 0] < 0, -1.0, 1.0) * (1 - 0.05 * torch.rand(int(edge.sum()), generator=g,
                                                                                          dtype=torch.float64))
    s_min = 0.0008 + 0.002 * torch.rand(P, generator=g, dtype=torch.float64)
    s_max = s_min * (1 + 24 * torch.rand(P, generator=g, dtype=torch.float64))
    th = torch.rand(P, generator=g, dtype=torch.float64) * math.pi
    c, sn = torch.cos(th), torch.sin(th)
    a, b = s_max ** 2, s_min ** 2
    xx, xy, yy = c * c * a + sn * sn * b, c * sn * (a - b), sn * sn * a + c * c * b
    det = xx * yy - xy * xy
    covs = torch.stack([xx, xy, yy], 1).float()
    conics = torch.stack([yy / det, -xy / det, xx / det], 1).float()
    values = torch.randn(P, C, generator=g).float()
    return means.float(), values, covs, conics, syn.samples(n, 2, seed=seed + 1)


def clustered_case(P=4000, n=30000, C=1, seed=161):
    """Strongly non-uniform densities: 70 % of the samples in a blob of sigma 0.03 and a third of
    the Gaussians around it (the fine cells are sized for the AVERAGE density, so the blob's cells
    hold thousands of samples: many forward sub units and long backward sample walks per cell),
    the rest uniform."""
    g = torch.Generator().manual_seed(seed)
    nb = int(0.7 * n)
    blob = torch.tensor([0.3, -0.2], dtype=torch.float64) + 0.03 * torch.randn(nb, 2, generator=g, dtype=torch.float64)
    rest = torch.rand(n - nb, 2, generator=g, dtype=torch.float64) * 2 - 1
    samples = torch.cat([blob, rest]).clamp(-1.0, 0.999).float()
    samples = samples[torch.randperm(n, generator=g)]
    means, values, covs, conics = syn.gaussians(P, 2, C, seed=seed + 1)
    k = P // 3
    means[:k] = (torch.tensor([0.3, -0.2]) + 0.05 * torch.randn(k, 2, generator=g)).float()
    return means, values, covs, conics, samples


def mixed_scales_case(P=3000, n=25000, C=1, seed=171):
    """Scales from 1e-4 to 0.2 (log-uniform) with axis ratios up to 5 and random rotations: tiny
    Gaussians under the radius floor, culled ones, and unculled ones whose cut exceeds half the
    period (full-tile lists) in one problem; one sample in eight duplicated 4 times (zero-width
    sub-cell boxes)."""
    g = torch.Generator().manual_seed(seed)
    means = torch.rand(P, 2, generator=g, dtype=torch.float64) * 2 - 1
    s_min = 10 ** (-4 + 2.7 * torch.rand(P, generator=g, dtype=torch.float64))
    s_max = s_min * (1 + 4 * torch.rand(P, generator=g, dtype=torch.float64))
    th = torch.rand(P, generator=g, dtype=torch.float64) * math.pi
    c, sn = torch.cos(th), torch.sin(th)
    a, b = s_max ** 2, s_min ** 2
    xx, xy, yy = c * c * a + sn * sn * b, c * sn * (a - b), sn * sn * a + c * c * b
    det = xx * yy - xy * xy
    covs = torch.stack([xx, xy, yy], 1).float()
    conics = torch.stack([yy / det, -xy / det, xx / det], 1).float()
    values = torch.randn(P, C, generator=g).float()
    samples = syn.samples(n, 2, seed=seed + 1)
    k = n // 8
    samples[n - 4 * k:] = samples[:k].repeat(4, 1)
    return means.float(), values, covs, conics, samples


def agg_problem(P=120, D=2, L=6, K=5, F=3, seed=0, spread=1.0, radius=(0.3, 1.2), centre=0.0):
    """aggregate_neighbors inputs (aggregate_neighbors.cu:323-475): means, conics, radii and the
    feature tensors.  Gaussians 0-2 have radius 0 (absent from every list); Gaussian 5 has a
    non-PD conic when D == 2 (power > 0 slots, index -1).  E = 2 D F + 1."""
    r = np.random.default_rng(seed)
    means = (centre + r.uniform(-1, 1, (P, D)) * spread).astype(np.float32)
    radii = r.uniform(radius[0], radius[1], P).astype(np.float32)
    radii[:min(3, P)] = 0.0
    if D == 2:
        sx, sy = r.uniform(0.05, 0.2, P), r.uniform(0.05, 0.2, P)
        conics = np.stack([1 / sx ** 2, r.uniform(-0.3, 0.3, P) / (sx * sy), 1 / sy ** 2], 1)
        if P > 5:
            conics[5] = [-3.0, 0.0, 4.0]
    else:
        conics = 1 / r.uniform(0.05, 0.2, (P, 1)) ** 2
    E = 2 * D * F + 1
    feats = dict(features=r.normal(size=(P, L)), transform=r.normal(size=(L, L)) / max(L, 1),
                 queries=r.normal(size=(P, K)), keys=r.normal(size=(P, K)),
                 frequencies=r.uniform(0.5, 3.0, F), distance_transform=r.normal(size=2 * E))
    return means, conics.astype(np.float32), radii, {k: v.astype(np.float32) for k, v in feats.items()}


AGG_FEATURES = ("features", "transform", "queries", "keys", "frequencies", "distance_transform")


def wide_domain_case(n=20000, P=3000, half=40.0, seed=141):
    """Query points over [-half, half)^2: ~157^2 tiles of one fine cell each, so 2 * ncells
    exceeds 2^16 and the binning sorts 32-bit (cell, flag) keys (the 16-bit path elsewhere)."""
    g = torch.Generator().manual_seed(seed)
    means = ((torch.rand(P, 2, generator=g) * 2.0 - 1.0) * half).float()
    sig = 0.2 + 0.4 * torch.rand(P, 1, generator=g)
    covs = torch.cat([sig ** 2, 0.1 * sig ** 2, 0.8 * sig ** 2], 1).float()
    det = covs[:, 0] * covs[:, 2] - covs[:, 1] ** 2
    conics = torch.stack([covs[:, 2] / det, -covs[:, 1] / det, covs[:, 0] / det], 1).float()
    values = torch.randn(P, 1, generator=g).float()
    samples = ((torch.rand(n, 2, generator=g) * 2.0 - 1.0) * half).float()
    return means, values, covs, conics, samples


def unculled_case(P=1500, n=12000, seed=191):
    """Gaussians the binning cannot cull (k_wide: one wave each, every non-empty cell of their
    tiles): a third with non-positive-definite conics (c1^2 > c0 c2: the reference's `power > 0`
    skip), a third positive definite but past kRho2Max (rho^2 in (0.9995, 0.9999): axis ratio
    ~90-200), a third with cuts wider than half the domain's period (sigma ~ 0.05)."""
    g = torch.Generator().manual_seed(seed)
    means = (torch.rand(P, 2, generator=g) * 2 - 1).float()
    k = torch.arange(P) % 3
    c0 = 40.0 + 80.0 * torch.rand(P, generator=g)
    c2 = 40.0 + 80.0 * torch.rand(P, generator=g)
    sgn = torch.where(torch.rand(P, generator=g) < 0.5, -1.0, 1.0)
    rho = torch.where(k == 0, 1.05 + 0.5 * torch.rand(P, generator=g),
                      torch.sqrt(0.9995 + 0.0004 * torch.rand(P, generator=g)))
    c1 = sgn * rho * torch.sqrt(c0 * c2)
    big = k == 2
    c0 = torch.where(big, 1.0 / (0.04 + 0.02 * torch.rand(P, generator=g)) ** 2, c0)
    c2 = torch.where(big, 1.0 / (0.04 + 0.02 * torch.rand(P, generator=g)) ** 2, c2)
    c1 = torch.where(big, 0.3 * torch.sqrt(c0 * c2) * sgn, c1)
    conics = torch.stack([c0, c1, c2], 1).float()
    # covariances: the inverse where it exists (positive definite), a round one of the conic's
    # scale otherwise (the reference reads covariances for the radius only)
    det = c0 * c2 - c1 * c1
    pd = det > 0
    covs = torch.where(pd[:, None], torch.stack([c2 / det, -c1 / det, c0 / det], 1),
                       torch.stack([1.0 / c0, torch.zeros(P), 1.0 / c2], 1)).float()
    values = torch.randn(P, 1, generator=g).float()
    return means, values, covs, conics, syn.samples(n, 2, seed=seed + 1)

"""GPU parity of the D = 3 path (libdgs.so dgs_volume_*) against the
brute-force oracle (oracle/volume.py: every pair of every Gaussian, float64 sums).  Parity
unpinned against the reference, which has no D = 3 path (forward.cu:164-275 stops at D = 2).

Tolerances as test_gpu_parity.py: forward |d| <= 1e-5 |ref| + 1e-6 max|ref|, gradients
|d| <= 1e-5 |ref| + 1e-6 max|ref| (the same bound)."""
import numpy as np
import pytest
import torch

from helpers import close

from oracle import volume as vo

pytestmark = pytest.mark.gpu

RTOL, ATOL_FWD, ATOL_BWD = 1e-5, 1e-6, 1e-6  # SURVEY 8c (backward: atol 1e-6 max|ref|)


def _field(P, C, seed):
    """sigma ~ 0.018 * U[0.5, 1.5]: cuts up to ~0.4, the culled path (test_volume_big_gaussians
    adds Gaussians of the every-sample path)"""
    return vo.gaussians3(P, C, seed=seed, scale=0.009 * max(P, 1) ** (1.0 / 3.0))


def _close(got, ref, atol_frac, what):
    close(got, ref, RTOL, atol_frac, what)


def _run(function, means, values, conics, samples, dL=None, debug=False):
    from diff_gaussian_sampling import _C
    dev = torch.device("cuda:0")
    m, v, c, s = (torch.from_numpy(x).to(dev) for x in (means, values, conics, samples))
    buf = _C.volume_preprocess(m, c, s, debug)
    out = _C.volume_forward(function, m, v, c, s, buf, debug)
    grads = None
    if dL is not None:
        grads = _C.volume_backward(function, m, v, c, s, buf, torch.from_numpy(dL).to(dev), debug)
        grads = tuple(g.cpu().numpy() for g in grads)
    torch.cuda.synchronize()
    return out.cpu().numpy(), grads


def _check(function, means, values, conics, samples, seed=5, debug=False):
    N, C, K = samples.shape[0], values.shape[1], 3 ** function
    dL = np.random.default_rng(seed).normal(size=(N, K, C)).astype(np.float32)
    out, (dm, dv, dc) = _run(function, means, values, conics, samples, dL, debug)
    ref = vo.forward(function, means, values, conics, samples)
    _close(out.reshape(N, K, C), ref, ATOL_FWD, f"fn{function} forward")
    rm, rv, rc = vo.backward(function, means, values, conics, samples, dL)
    _close(dm, rm, ATOL_BWD, f"fn{function} dmeans")
    _close(dv, rv, ATOL_BWD, f"fn{function} dvalues")
    _close(dc, rc, ATOL_BWD, f"fn{function} dconics")


@pytest.mark.parametrize("function", [0, 1, 2, 3])
@pytest.mark.parametrize("C", [1, 3])
def test_volume_parity(dgs, function, C):
    means, values, _, conics = _field(1000, C, function)
    samples = vo.samples3(2000, seed=11 + C)
    _check(function, means, values, conics, samples)


def test_volume_parity_wide_channels(dgs):
    """C = 9: two channel blocks of 8 (the backward's mean/conic sums from the first only)."""
    means, values, _, conics = _field(800, 9, 3)
    samples = vo.samples3(1500, seed=9)
    _check(2, means, values, conics, samples)


@pytest.mark.parametrize("function", [0, 3])
def test_volume_big_gaussians(dgs, function):
    """Gaussians outside the culled class meet every sample: wide ones (cut > 0.45), an
    ill-conditioned one, and one whose conic is not positive definite (pairs with power > 0
    skipped, forward.cu:166-171)."""
    means, values, _, conics = _field(600, 2, 7)
    conics[0] = [4.0, 0.0, 0.0, 4.0, 0.0, 4.0]  # sigma 0.5: wide
    conics[1] = [1e4, 0.0, 0.0, 1e-1, 0.0, 1e4]  # cond 1e5
    conics[2] = [30.0, 0.0, 0.0, -5.0, 0.0, 30.0]  # indefinite
    conics[3] = [2000.0, 1999.0, 0.0, 2000.0, 0.0, 50.0]  # nearly singular
    samples = vo.samples3(1200, seed=8)
    _check(function, means, values, conics, samples)


def test_volume_seams_and_images(dgs):
    """Means and samples at the faces of [-1, 1)^3 and beyond it: the displacements cross the
    wrap breakpoints (|x| = 1, the images x in [2k - E, 2k])."""
    rng = np.random.default_rng(2)
    means, values, _, conics = _field(400, 1, 2)
    means[:100, 0] = np.float32(0.999)
    means[100:200, 1] = np.float32(-0.999)
    means[200:220] = rng.uniform(2.5, 3.5, (20, 3)).astype(np.float32)  # far outside: images
    samples = vo.samples3(1500, seed=3)
    samples[:300, 0] = np.float32(-0.998)
    samples[300:400] = rng.uniform(-3.2, -2.8, (100, 3)).astype(np.float32)
    for f in (0, 1):
        _check(f, means, values, conics, samples, seed=f)


def test_volume_grid_lattice(dgs):
    """A regular lattice of query points (the "256^3 grid" of BASELINE config 5, at 24^3)."""
    ax = np.arange(24, dtype=np.float64) * (2.0 / 24) - 1.0
    g = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3).astype(np.float32)
    means, values, _, conics = _field(500, 1, 4)
    for f in (1, 2, 3):
        _check(f, means, values, conics, g, seed=f)


def test_volume_edge_sizes(dgs):
    means, values, _, conics = _field(50, 2, 1)
    samples = vo.samples3(40, seed=1)
    for P, N in ((0, 40), (50, 0), (1, 1), (50, 1)):
        _check(2, means[:P], values[:P], conics[:P], samples[:N])


def test_volume_debug_and_repeatable(dgs):
    means, values, _, conics = _field(700, 1, 6)
    samples = vo.samples3(900, seed=6)
    dL = np.random.default_rng(1).normal(size=(900, 27, 1)).astype(np.float32)
    a, ga = _run(3, means, values, conics, samples, dL, debug=True)
    b, gb = _run(3, means, values, conics, samples, dL)
    assert np.array_equal(a, b)
    for x, y in zip(ga, gb):
        assert np.array_equal(x, y)


def test_volume_stale_buffer_is_loud(dgs):
    """A binning of other sizes makes the kernels write NaN instead of reading out of range."""
    from diff_gaussian_sampling import _C
    dev = torch.device("cuda:0")
    means, values, _, conics = (torch.from_numpy(x).to(dev) for x in _field(100, 1, 1))
    s = torch.from_numpy(vo.samples3(200)).to(dev)
    buf = _C.volume_preprocess(means, conics, s[:100], False)
    out = _C.volume_forward(0, means, values, conics, s, buf, False)
    assert torch.isnan(out).all()


def test_volume_sampler_autograd(dgs):
    """VolumeSampler (GaussianSampler's shape) through autograd equals the oracle."""
    from diff_gaussian_sampling.volume import VolumeSampler
    dev = torch.device("cuda:0")
    means, values, covs, conics = _field(900, 2, 8)
    samples = vo.samples3(1100, seed=8)
    m, v, cv, c, s = (torch.from_numpy(x).to(dev) for x in (means, values, covs, conics, samples))
    for t in (m, v, c):
        t.requires_grad_(True)
    vs = VolumeSampler(False)
    vs.preprocess(m, v, cv, c, s)
    lap = vs.sample_gaussians_laplacian()
    assert lap.shape == (1100, 3, 3, 2)
    dL = torch.randn(lap.shape, generator=torch.Generator().manual_seed(0)).to(dev)
    (lap * dL).sum().backward()
    rm, rv, rc = vo.backward(2, means, values, conics, samples, dL.cpu().numpy())
    _close(lap.detach().cpu().numpy().reshape(1100, 9, 2), vo.forward(2, means, values, conics, samples),
           ATOL_FWD, "laplacian forward")
    _close(m.grad.cpu().numpy(), rm, ATOL_BWD, "dmeans")
    _close(v.grad.cpu().numpy(), rv, ATOL_BWD, "dvalues")
    _close(c.grad.cpu().numpy(), rc, ATOL_BWD, "dconics")


def test_volume_changed_inputs_are_loud(dgs):
    """Same sizes, different tensors (an in-place step, moved samples): the device-side check of
    every call writes NaN instead of mixing the binned means with the new ones."""
    from diff_gaussian_sampling import _C
    dev = torch.device("cuda:0")
    means, values, _, conics = (torch.from_numpy(x).to(dev) for x in _field(400, 1, 2))
    s = torch.from_numpy(vo.samples3(500, seed=2)).to(dev)
    buf = _C.volume_preprocess(means, conics, s, False)
    ok = _C.volume_forward(0, means, values, conics, s, buf, False)
    assert torch.isfinite(ok).all()
    for which in range(3):
        m2, c2, s2 = means.clone(), conics.clone(), s.clone()
        (m2, c2, s2)[which][7, 0] += 1e-3
        out = _C.volume_forward(0, m2, values, c2, s2, buf, False)
        assert torch.isnan(out).all(), which
        dm, dv, dc = _C.volume_backward(0, m2, values, c2, s2, buf, torch.ones_like(out), False)
        assert torch.isnan(dm).all() and torch.isnan(dc).all(), which
        with pytest.raises(RuntimeError, match="differ from the binned"):  # a count has no NaN
            _C.volume_count_pairs(m2, c2, s2, buf)
    assert _C.volume_count_pairs(means, conics, s, buf)[1] > 0
    again = _C.volume_forward(0, means, values, conics, s, buf, False)  # the binned tensors: fine again
    assert torch.equal(again, ok)


def test_volume_sampler_rebins_after_inplace_step(dgs):
    """VolumeSampler keeps its tensors by reference: after an in-place optimizer step the next
    call re-bins, and the result equals the oracle at the new parameters."""
    from diff_gaussian_sampling.volume import VolumeSampler
    dev = torch.device("cuda:0")
    means, values, covs, conics = _field(700, 1, 9)
    samples = vo.samples3(900, seed=9)
    m, v, cv, c, s = (torch.from_numpy(x).to(dev) for x in (means, values, covs, conics, samples))
    vs = VolumeSampler(False)
    vs.preprocess(m, v, cv, c, s)
    vs.sample_gaussians()
    with torch.no_grad():
        m[:, 0] += 0.013  # moves every Gaussian by about a cell
    out = vs.sample_gaussians_derivative()
    ref = vo.forward(1, m.cpu().numpy(), values, conics, samples)
    _close(out.cpu().numpy().reshape(900, 3, 1), ref, ATOL_FWD, "derivative after the in-place step")

"""The ctypes binding of the C ABI (tools/dgs_ctypes.py, shown in INTEGRATION.md) against the
compiled torch extension: same binning bytes, same outputs, same gradients."""
import os
import sys

import numpy as np
import pytest
import torch

from diff_gaussian_sampling import synthetic as syn
from helpers import FUNCS, FWD_NAME

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("function", FUNCS)
def test_ctypes_binding_matches_extension(dgs, function):
    import dgs_ctypes
    dev = "cuda:0"
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(2000, 2, 2, seed=141))
    samples = syn.samples(8000, 2, seed=142).to(dev)
    a = dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
    b = dgs_ctypes.preprocess_gaussians(means, values, covs, conics, samples, False)
    assert a[0] == b[0]
    for x, y in zip(a[3:], b[3:]):  # ranges, sample_ranges, radii
        assert torch.equal(x, y)
    fa = getattr(dgs._C, FWD_NAME[function])(means, values, conics, samples, *a[:5], False)
    fb = getattr(dgs_ctypes, FWD_NAME[function])(means, values, conics, samples, *b[:5], False)
    assert torch.equal(fa, fb)
    dL = torch.randn_like(fa)
    ga = getattr(dgs._C, FWD_NAME[function] + "_backward")(means, values, conics, samples, a[0], dL, *a[1:5], False)
    gb = getattr(dgs_ctypes, FWD_NAME[function] + "_backward")(means, values, conics, samples, b[0], dL, *b[1:5], False)
    for x, y in zip(ga, gb):  # atomics: order-dependent in the last bits
        np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=1e-5,
                                   atol=1e-6 * float(x.abs().max()))


def test_ctypes_aggregate_matches_extension(dgs):
    import dgs_ctypes
    from cases import AGG_FEATURES, agg_problem
    means, conics, radii, fe = agg_problem(P=800, D=2, L=16, K=16, F=4, seed=150)
    cu = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    a = dgs._C.preprocess_aggregate(cu(means), cu(conics), cu(radii), False)
    b = dgs_ctypes.preprocess_aggregate(cu(means), cu(conics), cu(radii), False)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    t = [cu(fe[k]) for k in AGG_FEATURES]
    fa = dgs._C.aggregate_neighbors(*t, *a, False)
    fb = dgs_ctypes.aggregate_neighbors(*t, *b, False)
    for x, y in zip(fa, fb):
        assert torch.equal(x, y)
    g = torch.randn_like(fa[3])
    ga = dgs._C.aggregate_neighbors_backward(*t, *a[:4], *fa[:3], a[4], g, False)
    gb = dgs_ctypes.aggregate_neighbors_backward(*t, *b[:4], *fb[:3], b[4], g, False)
    gc = dgs_ctypes.aggregate_neighbors_backward(*t, *b[:4], *fb[:3], b[4], g, False, transposed=False)
    # the two shared-array gradients (d/dfrequencies, d/ddistance_transform: a handful of
    # elements, each a float sum over EVERY slot) at test_gpu_aggregate's LIT_SHARED = 1e-4: the
    # atomic form's order moved one of them by 2.8e-5 relative on MI355X
    for x, y, z in zip(ga, gb, gc):
        rtol = 1e-4 if x.numel() <= 64 else 1e-5
        np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=rtol, atol=1e-6 * float(x.abs().max()))
        np.testing.assert_allclose(x.cpu().numpy(), z.cpu().numpy(), rtol=rtol, atol=1e-6 * float(x.abs().max()))


def test_ctypes_multi_matches_extension(dgs):
    """dgs_sample_{forward,backward}_multi through ctypes against the extension's fused call."""
    import dgs_ctypes
    dev = "cuda:0"
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(2000, 2, 1, seed=151))
    samples = syn.samples(8000, 2, seed=152).to(dev)
    a = dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
    codes = [3, 0, 2]
    fa = dgs._C.sample_gaussians_multi(codes, means, values, conics, samples, a[1], a[2], False)
    fb = dgs_ctypes.sample_gaussians_multi(codes, means, values, conics, samples, a[1], a[2], False)
    for x, y in zip(fa, fb):
        assert torch.equal(x, y)
    dLs = [torch.randn_like(x) for x in fa]
    ga = dgs._C.sample_gaussians_multi_backward(codes, means, values, conics, samples, dLs, a[1], a[2], False)
    gb = dgs_ctypes.sample_gaussians_multi_backward(codes, means, values, conics, samples, dLs, a[1], a[2], False)
    for x, y in zip(ga, gb):
        np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=1e-5,
                                   atol=1e-6 * float(x.abs().max()))

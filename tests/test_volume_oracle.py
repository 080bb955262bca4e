"""CPU checks of the D = 3 oracle (oracle/volume.py; SURVEY.md §8f row f4, beyond the
reference).  Its gradient formulas against torch float64 autograd of its own forward, its
index-form functions against the reference's D = 2 expressions (forward.cu:164-275) in the
plane X2 = 0, and closed-form values."""
import numpy as np
import pytest
import torch

from oracle import volume as vo


def _torch_forward(function, means, values, conics, samples):
    """The oracle's forward in torch float64 (autograd target): same wrap, power and terms."""
    X = means[:, None, :] - samples[None, :, :]
    with torch.no_grad():  # wrap: a per-pair constant shift (derivative 1, as in the reference)
        Xd = X.detach().numpy().astype(np.float32)
        shift = torch.from_numpy((vo._wrap(Xd) - Xd).astype(np.float64))
    X = X + shift
    A = torch.zeros(means.shape[0], 3, 3, dtype=torch.float64)
    for q, (i, j) in enumerate(vo.PAIRS):
        A[:, i, j] = conics[:, q]
        A[:, j, i] = conics[:, q]
    power = -0.5 * torch.einsum("pni,pij,pnj->pn", X, A, X)
    G = torch.exp(power) * (power <= 0)
    a = torch.einsum("pij,pnj->pni", A, X)
    if function == 0:
        t = torch.ones(a.shape[:-1] + (1,), dtype=torch.float64)
    elif function == 1:
        t = a
    elif function == 2:
        t = torch.stack([a[..., i] * a[..., j] - A[:, i, j][:, None] for i, j in vo.PAIRS], -1)
    else:
        t = torch.stack([A[:, i, j][:, None] * a[..., k] + A[:, i, k][:, None] * a[..., j]
                         + A[:, j, k][:, None] * a[..., i] - a[..., i] * a[..., j] * a[..., k]
                         for i, j, k in vo.TRIPLES], -1)
    uo = torch.einsum("pn,pnu,pc->nuc", G, t, values)
    return uo[:, vo.umap(function), :]


@pytest.mark.parametrize("function", [0, 1, 2, 3])
@pytest.mark.parametrize("C", [1, 2])
def test_volume_oracle_gradients_match_autograd(function, C):
    means, values, _, conics = vo.gaussians3(6, C, seed=function, scale=6.0)
    samples = vo.samples3(9, seed=10 + function)
    samples[0] = means[0]  # an exact hit
    samples[1] = means[1] + np.float32(1.95)  # across the seam (wrapped)
    samples[1] = np.where(samples[1] > 1, samples[1] - np.float32(4.0), samples[1])
    N, K = samples.shape[0], 3 ** function
    dL = np.random.default_rng(3).normal(size=(N, K, C))
    ref = vo.forward(function, means, values, conics, samples)
    m, v, c = (torch.tensor(x.astype(np.float64), requires_grad=True) for x in (means, values, conics))
    out = _torch_forward(function, m, v, c, torch.tensor(samples.astype(np.float64)))
    np.testing.assert_allclose(out.detach().numpy(), ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
    (out * torch.tensor(dL)).sum().backward()
    dm, dv, dc = vo.backward(function, means, values, conics, samples, dL)
    for name, got, want in (("means", dm, m.grad), ("values", dv, v.grad), ("conics", dc, c.grad)):
        want = want.numpy()
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * np.abs(want).max(), err_msg=name)


def test_volume_terms_reduce_to_the_reference_d2_expressions():
    """In the plane (X2 = 0, c02 = c12 = 0) the index-form terms are forward.cu's D = 2 ones."""
    rng = np.random.default_rng(0)
    a1, a2 = rng.normal(size=2)
    c0, c1, c2 = 2.0, 0.3, 1.5
    A = np.zeros((1, 3, 3))
    A[0, :2, :2] = [[c0, c1], [c1, c2]]
    a = np.array([[[a1, a2, 0.0]]])
    lap = vo._terms(2, a, A)[0, 0]
    assert np.allclose([lap[vo.pidx(0, 0)], lap[vo.pidx(0, 1)], lap[vo.pidx(1, 1)]],
                       [a1 * a1 - c0, a1 * a2 - c1, a2 * a2 - c2])  # forward.cu:214-217
    third = vo._terms(3, a, A)[0, 0]
    T = vo.TRIPLES.index
    dxxx = 3.0 * c0 * a1 - a1 ** 3  # forward.cu:245-248
    dxxy = 2.0 * c1 * a1 - a1 * a1 * a2 + c0 * a2
    dxyy = 2.0 * c1 * a2 - a1 * a2 * a2 + c2 * a1
    dyyy = 3.0 * c2 * a2 - a2 ** 3
    assert np.allclose([third[T((0, 0, 0))], third[T((0, 0, 1))], third[T((0, 1, 1))], third[T((1, 1, 1))]],
                       [dxxx, dxxy, dxyy, dyyy])
    der = vo._terms(1, a, A)[0, 0]
    assert np.allclose(der[:2], [a1, a2])  # forward.cu:190-191 (x1 + c1 X1 = a1)


def test_volume_closed_forms():
    """A Gaussian evaluated at its mean: value v, derivative 0, Hessian -A, third 0.  A sample
    exactly 2 away along x has X0 = fmod(2, 2) - 2 = -2 under the reference's wrap
    (forward.cu:149-157), not 0: value v exp(-0.5 c00 4)."""
    means = np.array([[0.2, -0.3, 0.5]], np.float32)
    conics = np.array([[4.0, 0.5, 0.0, 3.0, 0.25, 2.0]], np.float32)
    values = np.array([[1.5]], np.float32)
    s = np.array([[0.2, -0.3, 0.5], [0.2 - 2.0, -0.3, 0.5]], np.float32)
    f0 = vo.forward(0, means, values, conics, s)
    assert np.allclose(f0[:, 0, 0], [1.5, 1.5 * np.exp(-8.0)])
    assert np.allclose(vo.forward(1, means, values, conics, s[:1]), 0.0)
    hess = vo.forward(2, means, values, conics, s)[0, :, 0].reshape(3, 3)
    A = vo._amat(conics.astype(np.float64))[0]
    assert np.allclose(hess, -1.5 * A)
    assert np.allclose(vo.forward(3, means, values, conics, s[:1]), 0.0)


def test_volume_output_symmetry():
    means, values, _, conics = vo.gaussians3(20, 2, seed=1, scale=8.0)
    s = vo.samples3(5, seed=2)
    out = vo.forward(3, means, values, conics, s).reshape(5, 3, 3, 3, 2)
    assert np.allclose(out, out.transpose(0, 2, 1, 3, 4))
    assert np.allclose(out, out.transpose(0, 3, 2, 1, 4))

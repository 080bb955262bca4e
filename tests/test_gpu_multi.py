"""GPU parity of the fused multi-function entry point (sample_gaussians_multi).

The fused call evaluates several of the four functions in one traversal of the binned pairs.
Its forward outputs must equal the oracle's per-function outputs, and its gradients the sum of
the oracle's per-function gradients (the loss of a fused call is the sum of the functions'
losses), with the tolerances of test_gpu_parity.py.
"""
import itertools

import numpy as np
import pytest
import torch

from diff_gaussian_sampling import synthetic as syn
import cases
from helpers import close, margin_of, model_distances, order_bounds, record_margin

pytestmark = pytest.mark.gpu

RTOL, ATOL_FWD, ATOL_BWD = 1e-5, 1e-6, 1e-6  # SURVEY 8c (backward: atol 1e-6 max|ref|)
NAMES = ["gaussian", "derivative", "laplacian", "third"]
MULTI = [c for r in (2, 3, 4) for c in itertools.combinations(NAMES, r)]


def _run(dgs, functions, means, values, covs, conics, samples, dLs):
    dev = torch.device("cuda:0")
    m, v, cv, c, s = (t.to(dev) for t in (means, values, covs, conics, samples))
    R, gb, sb, rg, srg, _ = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
    codes = [dgs.FUNCTIONS[f] for f in functions]
    outs = dgs._C.sample_gaussians_multi(codes, m, v, c, s, gb, sb, False)
    grads = dgs._C.sample_gaussians_multi_backward(codes, m, v, c, s, [d.to(dev) for d in dLs],
                                                  gb, sb, False)
    torch.cuda.synchronize()
    return [o.cpu().numpy() for o in outs], [g.cpu().numpy() for g in grads]


def _check(dgs, oracle, functions, means, values, covs, conics, samples, seed=7, apriori=False):
    """apriori: the thin Gaussians' stated bound -- the 8c bound plus the a-priori exponent-order
    bound (helpers.order_bounds, test_gpu_parity.py)."""
    N, D, C = samples.shape[0], samples.shape[1], values.shape[1]
    dLs = [syn.grad_out(N, syn.out_components(f, D), C, seed=seed + i) for i, f in enumerate(functions)]
    outs, grads = _run(dgs, functions, means, values, covs, conics, samples, dLs)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    bounds = order_bounds(ob, functions, values, conics, dLs) if apriori else {}
    models = model_distances(oracle, functions, means, values, covs, conics, samples, dLs, bounds) if apriori else None
    ref_g = None
    for f, o, dL in zip(functions, outs, dLs):
        ref = ob.forward(f, values.numpy(), conics.numpy())
        if apriori:
            record_margin(f"multi {f} forward [gpu vs fmad, 8c + a-priori bound]",
                          margin_of(o.reshape(N, -1, C), models["fmad"][0][f], RTOL, ATOL_FWD, bounds[f"{f} forward"]),
                          RTOL, ATOL_FWD, int(ref.size))
        close(o.reshape(N, -1, C), ref, RTOL, ATOL_FWD, f"multi {functions} {f} forward", bounds.get(f"{f} forward"))
        g = ob.backward(f, values.numpy(), conics.numpy(), dL.numpy(), exact=True)
        ref_g = list(g) if ref_g is None else [a + b for a, b in zip(ref_g, g)]
    for i, (name, got, ref) in enumerate(zip(("means", "values", "conics"), grads, ref_g)):
        if apriori:
            record_margin(f"multi d{name} [gpu vs fmad, 8c + a-priori bound]",
                          margin_of(got, models["fmad"][1][i], RTOL, ATOL_BWD, bounds[f"d{name}"]), RTOL, ATOL_BWD,
                          int(ref.size))
        close(got, ref, RTOL, ATOL_BWD, f"multi {functions} dL/d{name}", bounds.get(f"d{name}"))


@pytest.mark.parametrize("functions", MULTI, ids=lambda f: "+".join(x[:3] for x in f))
def test_multi_synthetic(dgs, oracle, functions):
    means, values, covs, conics = syn.gaussians(1000, 2, 1, seed=11)
    samples = syn.samples(4000, 2, seed=12)
    _check(dgs, oracle, functions, means, values, covs, conics, samples)


@pytest.mark.parametrize("functions", [tuple(NAMES), ("gaussian", "laplacian")])
def test_multi_edge_and_seam(dgs, oracle, functions):
    """Torus wrap, full-range, det == 0 and non-PD conics (the reference-literal pair path of
    the fused kernels), and seam Gaussians (constant-shift wraps)."""
    _check(dgs, oracle, functions, *cases.edge_case(), seed=31)
    _check(dgs, oracle, functions, *cases.seam_case(D=2, C=1), seed=41)


@pytest.mark.parametrize("functions", [tuple(NAMES)])
def test_multi_thin_anisotropic(dgs, oracle, functions):
    """Thin rotated Gaussians (cases.thin_case): the fused moment-form backward and the fused
    forward next to the reference-literal path of the ill-conditioned conics."""
    _check(dgs, oracle, functions, *cases.thin_case(P=3000, n=20000), seed=51, apriori=True)


def test_multi_order_and_fallback(dgs, oracle):
    """Outputs come back in the order asked; C > 1 (no fused kernel) runs the per-function
    kernels in turn and adds their gradients."""
    means, values, covs, conics = syn.gaussians(600, 2, 3, seed=5)
    samples = syn.samples(3000, 2, seed=6)
    _check(dgs, oracle, ("third", "gaussian"), means, values, covs, conics, samples)
    means, values, covs, conics = syn.gaussians(600, 2, 1, seed=5)
    _check(dgs, oracle, ("laplacian", "derivative", "gaussian"), means, values, covs, conics, samples)


def test_multi_autograd_matches_separate_calls(dgs):
    """GaussianSampler.sample_gaussians_multi through autograd equals the per-function calls
    (some outputs unused: their gradient is None)."""
    dev = torch.device("cuda:0")
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(2000, 2, 1, seed=3))
    samples = syn.samples(8000, 2, seed=4).to(dev)
    w = [torch.randn(8000, *(2,) * k, 1, generator=torch.Generator().manual_seed(k)).to(dev) for k in range(4)]

    def grads(fused):
        ps = [t.clone().requires_grad_(True) for t in (means, values, conics)]
        s = dgs.GaussianSampler(False)
        s.preprocess(ps[0], ps[1], covs, ps[2], samples)
        if fused:
            outs = s.sample_gaussians_multi("gaussian", "derivative", "laplacian", "third")
        else:
            outs = (s.sample_gaussians(), s.sample_gaussians_derivative(), s.sample_gaussians_laplacian(),
                    s.sample_gaussians_third_derivative())
        loss = (outs[0] * w[0]).sum() + (outs[2] * w[2]).sum() + (outs[3] * w[3]).sum()  # derivative unused
        loss.backward()
        return [o.detach().cpu().numpy() for o in outs], [p.grad.cpu().numpy() for p in ps]

    fo, fg = grads(True)
    so, sg = grads(False)
    for a, b in zip(fo, so):
        close(a, b, RTOL, ATOL_FWD, "fused vs separate forward")
    for a, b in zip(fg, sg):
        close(a, b, RTOL, ATOL_BWD, "fused vs separate gradient")


def test_multi_errors(dgs):
    dev = torch.device("cuda:0")
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(50, 2, 1, seed=1))
    samples = syn.samples(100, 2, seed=2).to(dev)
    R, gb, sb, rg, srg, _ = dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
    with pytest.raises(RuntimeError):
        dgs._C.sample_gaussians_multi([0, 0], means, values, conics, samples, gb, sb, False)
    with pytest.raises(RuntimeError):
        dgs._C.sample_gaussians_multi([4], means, values, conics, samples, gb, sb, False)
    with pytest.raises(RuntimeError):
        dgs._C.sample_gaussians_multi([], means, values, conics, samples, gb, sb, False)

"""The oracle's FMA contraction models (oracle/oracle.c header, oracle/Makefile) on the CPU.

The reference is compiled by nvcc with its default --fmad=true (setup.py:30 sets no
--fmad=false), so its a*b + c sites may be fused (forward.cu:55,59,177,182,199,223,252;
backward.cu:122,141,147-148, ...).  "fmad" / "fmad_alt" model that (the two fusing choices at
a*b + c*d); "nocontract" is the model the GPU path reproduces bit for bit in its integer outputs.
These tests pin what the models say (the numbers behind DESIGN.md 6 and
profiles/r05_contraction.json):
  * the contracting builds really contract (their outputs differ from the unfused ones);
  * no golden / parity case changes a binning decision: det == 0, presence, num_rendered, ranges
    are identical in every model -- only radii move, by ulps;
  * outside thin Gaussians the models' float outputs stay well inside the 8c bound;
  * for thin Gaussians (rho^2 >= 0.82) they do not: the spread exceeds the bound, which is why
    tests/test_gpu_parity.py states the 8c bound plus the a-priori exponent-order bound there
    (oracle.c orc_forward_bound / orc_backward_bound) -- and the models fall inside THAT bound.
"""
import os

import numpy as np
import pytest

import cases
from diff_gaussian_sampling import synthetic as syn
from helpers import margin_of

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MODELS = ("fmad", "fmad_alt")


def _golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    return z["means"], z["values"], z["covariances"], z["conics"], z["samples"]


def test_models_load_and_identify(oracle):
    assert oracle._load("nocontract").orc_fmad_model() == 0
    assert oracle._load("fmad").orc_fmad_model() == 1
    assert oracle._load("fmad_alt").orc_fmad_model() == 2


@pytest.mark.parametrize("name", ["d2_c1_1k_4k", "d2_c16_200_800", "edge", "far_means", "seam_d2", "aliasing",
                                  "d1_c2_256_1k", "seam_d1", "d1_zero_variance"])
def test_binning_decisions_model_independent(oracle, name):
    means, values, covs, conics, samples = _golden(name)
    b0 = oracle.OracleBins(means, covs, samples)
    r0, s0 = b0.ranges()
    for m in MODELS:
        b = oracle.OracleBins(means, covs, samples, model=m)
        r, s = b.ranges()
        assert b.num_rendered == b0.num_rendered
        assert np.array_equal(r, r0) and np.array_equal(s, s0)
        assert np.array_equal(b.radii > 0, b0.radii > 0)
        # radii move by a few ulps (forward.cu:55,59 fused; the mid^2 - det cancellation of
        # near-isotropic covariances amplifies it, up to ~10 ulps), never by more than 1e-5
        d = np.abs(b.radii.astype(np.float64) - b0.radii.astype(np.float64))
        assert np.all(d <= 1e-5 * np.abs(b0.radii))


def test_contracting_builds_contract(oracle):
    means, values, covs, conics, samples = _golden("d2_c1_1k_4k")
    outs = {m: oracle.OracleBins(means, covs, samples, model=m).forward("gaussian", values, conics)
            for m in ("nocontract",) + MODELS}
    assert not np.array_equal(outs["fmad"], outs["nocontract"])
    assert not np.array_equal(outs["fmad_alt"], outs["fmad"])
    # the golden fixtures are the unfused model's outputs, bit for bit
    z = np.load(os.path.join(GOLDEN, "d2_c1_1k_4k.npz"))
    assert np.array_equal(outs["nocontract"].reshape(z["gaussian_out"].shape), z["gaussian_out"])


@pytest.mark.parametrize("function", ["gaussian", "derivative", "laplacian", "third"])
@pytest.mark.parametrize("name", ["d2_c1_1k_4k", "d2_c16_200_800", "edge", "seam_d2", "d1_c2_256_1k"])
def test_models_within_bound_off_thin(oracle, name, function):
    means, values, covs, conics, samples = _golden(name)
    N, D, C = samples.shape[0], means.shape[1], values.shape[1]
    dL = syn.grad_out(N, D ** ["gaussian", "derivative", "laplacian", "third"].index(function), C, seed=5).numpy()
    b0 = oracle.OracleBins(means, covs, samples)
    f0 = b0.forward(function, values, conics)
    g0 = b0.backward(function, values, conics, dL, exact=True)
    for m in MODELS:
        b = oracle.OracleBins(means, covs, samples, model=m)
        assert margin_of(b.forward(function, values, conics), f0, 1e-5, 1e-6) < 0.3
        for a, r in zip(b.backward(function, values, conics, dL, exact=True), g0):
            assert margin_of(a, r, 1e-5, 1e-6) < 0.3


def test_thin_spread_exceeds_bound(oracle):
    """cases.thin_case (axis ratios up to 25): the fused and unfused reference differ by more than
    the 8c bound -- the finding behind the thin stated bound (profiles/r05_contraction.json)."""
    means, values, covs, conics, samples = (t.numpy() for t in cases.thin_case())
    b0 = oracle.OracleBins(means, covs, samples)
    sub = np.nonzero(b0.sample_keys() < b0.T)[0][:8000].astype(np.int32)
    f0 = b0.forward("gaussian", values, conics, subset=sub)[sub]
    worst = 0.0
    for m in MODELS:
        b = oracle.OracleBins(means, covs, samples, model=m)
        worst = max(worst, margin_of(b.forward("gaussian", values, conics, subset=sub)[sub], f0, 1e-5, 1e-6))
    assert worst > 1.0, worst


@pytest.mark.parametrize("function", ["gaussian", "third"])
def test_thin_models_within_apriori_bound(oracle, function):
    """The a-priori exponent-order bound (the thin stated bound of test_gpu_parity.py, computed
    from the reference's expression alone) holds the reference's own contraction models: every
    fmad / fmad_alt output and exact-sum gradient is within 1e-5 |ref| + 1e-6 max|ref| + B of the
    unfused model on cases.thin_case, where they are 1-7x the plain 8c bound apart."""
    means, values, covs, conics, samples = (t.numpy() for t in cases.thin_case())
    N = samples.shape[0]
    K = 1 if function == "gaussian" else 8
    dL = syn.grad_out(N, K, 1, seed=5).numpy()
    b0 = oracle.OracleBins(means, covs, samples)
    sub = np.nonzero(b0.sample_keys() < b0.T)[0][:6000].astype(np.int32)
    f0 = b0.forward(function, values, conics, subset=sub)[sub]
    g0 = b0.backward(function, values, conics, dL, subset=sub, exact=True)
    fb = b0.order_bound(function, values, conics, subset=sub)[sub]
    gb = b0.order_bound(function, values, conics, dL, subset=sub)
    plain = 0.0
    for m in MODELS:
        b = oracle.OracleBins(means, covs, samples, model=m)
        f = b.forward(function, values, conics, subset=sub)[sub]
        plain = max(plain, margin_of(f, f0, 1e-5, 1e-6))
        assert margin_of(f, f0, 1e-5, 1e-6, fb) < 0.5, m
        for a, r, bb in zip(b.backward(function, values, conics, dL, subset=sub, exact=True), g0, gb):
            plain = max(plain, margin_of(a, r, 1e-5, 1e-6))
            assert margin_of(a, r, 1e-5, 1e-6, bb) < 0.5, m
    assert plain > 1.0, plain  # (the bound is needed: the plain 8c bound does not hold them)


def test_det_zero_decisions(oracle):
    """forward.cu:55-56 `det == 0`: the edge case's singular covariance is absent in every model,
    and exact singular products stay singular whichever product is fused."""
    means, values, covs, conics, samples = _golden("edge")
    for m in ("nocontract",) + MODELS:
        b = oracle.OracleBins(means, covs, samples, model=m)
        assert b.radii[3] == 0.0  # cov [1, 1, 1]: det == 0

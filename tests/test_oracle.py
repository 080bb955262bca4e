"""CPU tests pinning the oracle (oracle/oracle.c) -- no GPU needed.

The reference cannot run here and ships no golden vectors, so the oracle is
pinned by:
  1. an independent numpy restatement of the binning (tests/restate.py): radii, num_rendered,
     every tile's Gaussian list and every sample key must be bit-identical;
  2. torch float64 restatement of the forward functions (forward.cu:168-275): the oracle's
     fp32 forward must agree to fp32 rounding;
  3. torch.autograd of that float64 forward: the oracle's literal backward formulas
     (backward.cu:108-416) must agree to fp32 rounding -- except D=1 third dL/dconics
     (backward.cu:322-325), which is not the derivative and is checked against a literal
     float64 transcription instead;
  4. closed-form known answers (single Gaussian at the sample, torus wrap, grid size, the
     sample-clamp aliasing).
"""
import numpy as np
import pytest
import torch

import cases
import restate
from diff_gaussian_sampling import synthetic as syn
from helpers import FUNCS, close

# fp32 oracle vs float64 restatement: observed worst error is ~1e-6 of the largest element
# (fp32 sums over ~1e2-1e3 live terms with cancellation); the bound leaves 5x headroom.
RTOL = 1e-4
ATOL = 5e-6

BIN_CASES = {
    "synthetic_d2": lambda: syn.gaussians(1000, 2, 1, seed=11) + (syn.samples(4000, 2, seed=12),),
    "synthetic_d2_large_sigma": lambda: syn.gaussians(300, 2, 1, seed=13, scale=6.0) + (syn.samples(2000, 2, seed=14),),
    "synthetic_d1": lambda: syn.gaussians(300, 1, 2, seed=15) + (syn.samples(3000, 1, seed=16),),
    "edge": cases.edge_case,
    "aliasing": cases.aliasing_case,
    "d1_zero_variance": cases.d1_zero_variance_case,
    "far_means": cases.far_means_case,
    "seam_d1": lambda: cases.seam_case(D=1),
    "seam_d2": lambda: cases.seam_case(D=2),
}


def _np(*ts):
    return [t.numpy() for t in ts]


@pytest.mark.parametrize("case", list(BIN_CASES))
def test_binning_matches_numpy_restatement(oracle, case):
    means, values, covs, conics, samples = BIN_CASES[case]()
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    radii, R, lists, skeys = restate.bin_gaussians(means.numpy(), covs.numpy(), samples.numpy(),
                                                   ob.grid, ob.offset)
    assert np.array_equal(ob.radii, radii), "radii"
    assert ob.num_rendered == R, "num_rendered"
    assert np.array_equal(ob.sample_keys(), skeys), "sample keys"
    assert ob.T == len(lists)
    for t in range(ob.T):
        assert np.array_equal(ob.tile_gaussians(t), lists[t]), f"tile {t} Gaussian list"
    # reference-layout ranges: [start, end) into the sorted lists, (0, 0) when empty
    rg, srg = ob.ranges()
    start = 0
    for t in range(ob.T):
        n = len(lists[t])
        exp = (start, start + n) if n else (0, 0)
        assert tuple(rg[t]) == exp, f"ranges[{t}]"
        start += n
    counts = np.bincount(skeys[skeys < ob.T], minlength=ob.T)
    start = 0
    for t in range(ob.T):
        exp = (start, start + counts[t]) if counts[t] else (0, 0)
        assert tuple(srg[t]) == exp, f"sample_ranges[{t}]"
        start += counts[t]


def _pairs(ob):
    lists = [ob.tile_gaussians(t).astype(np.int64) for t in range(ob.T)]
    return restate.pairs(lists, ob.sample_keys())


AD_CASES = [(2, 400, 1500, 1, 11), (2, 300, 1200, 3, 12), (1, 120, 1500, 2, 13)]


@pytest.mark.parametrize("function", FUNCS)
@pytest.mark.parametrize("D,P,N,C,seed", AD_CASES)
def test_forward_and_backward_vs_autograd(oracle, function, D, P, N, C, seed):
    means, values, covs, conics = syn.gaussians(P, D, C, seed=seed)
    samples = syn.samples(N, D, seed=seed + 100)
    K = syn.out_components(function, D)
    dL = syn.grad_out(N, K, C, seed=seed + 200)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    sid, gid = _pairs(ob)
    assert len(sid) > 0
    m, v, c = (t.double().requires_grad_(True) for t in (means, values, conics))
    ref = restate.forward(function, m, v, c, samples.double(), sid, gid, N)
    got = ob.forward(function, values.numpy(), conics.numpy())
    close(got, ref.detach().numpy(), RTOL, ATOL, f"{function} D={D} forward")

    gm, gv, gc = torch.autograd.grad(ref, (m, v, c), dL.double().reshape(ref.shape))
    dm, dv, dc = ob.backward(function, values.numpy(), conics.numpy(), dL.numpy())
    close(dm, gm.numpy(), RTOL, ATOL, f"{function} D={D} dL/dmeans")
    close(dv, gv.numpy(), RTOL, ATOL, f"{function} D={D} dL/dvalues")
    if D == 1 and function == "third":
        lit = restate.d1_third_dconics(means.double(), values.double(), conics.double(),
                                       samples.double(), dL.double(), torch.as_tensor(sid),
                                       torch.as_tensor(gid), P)
        close(dc, lit.numpy(), RTOL, ATOL, "D=1 third dL/dconics (literal backward.cu:322-325)")
        # ... and it really is not the autograd gradient (the documented reference defect)
        assert np.max(np.abs(lit.numpy() - gc.numpy())) > 1e-2 * np.max(np.abs(gc.numpy()))
    else:
        close(dc, gc.numpy(), RTOL, ATOL, f"{function} D={D} dL/dconics")


@pytest.mark.parametrize("function", FUNCS)
def test_edge_case_forward_vs_restatement(oracle, function):
    """Non-PD conic (power > 0 skipped), wrap seams, full-range Gaussian, det == 0."""
    means, values, covs, conics, samples = cases.edge_case(n_random=1000)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    sid, gid = _pairs(ob)
    ref = restate.forward(function, means.double(), values.double(), conics.double(),
                          samples.double(), sid, gid, samples.shape[0])
    close(ob.forward(function, values.numpy(), conics.numpy()), ref.numpy(), RTOL, ATOL,
          f"edge {function}")


def _single(mean, sample, conic, cov, value=1.7):
    means = np.asarray([mean], np.float32)
    # a second far sample fixes the grid so that the first sample's tile contains the mean
    samples = np.asarray([sample, [-1.0, -1.0], [0.999, 0.999]], np.float32)
    return means, np.asarray([[value]], np.float32), np.asarray([cov], np.float32), \
        np.asarray([conic], np.float32), samples


def test_known_answer_gaussian_at_sample(oracle):
    """A Gaussian centred on the sample: value v, derivative 0, Hessian -v*A, third 0."""
    means, values, covs, conics, samples = _single([0.2, -0.3], [0.2, -0.3], [30.0, 5.0, 20.0],
                                                   [0.0345, -0.0086, 0.0517])
    ob = oracle.OracleBins(means, covs, samples)
    v = float(values[0, 0])
    assert ob.forward("gaussian", values, conics)[0, 0, 0] == np.float32(v)
    assert np.all(ob.forward("derivative", values, conics)[0, :, 0] == 0.0)
    lap = ob.forward("laplacian", values, conics)[0, :, 0]
    assert np.allclose(lap, -v * np.array([30.0, 5.0, 5.0, 20.0]), rtol=1e-6)
    assert np.all(ob.forward("third", values, conics)[0, :, 0] == 0.0)


def test_known_answer_torus_wrap(oracle):
    """Mean at x = 0.95, sample at x = -0.95: X = 1.9 wraps to fmod(1.9, 2) - 2 = -0.1."""
    means, values, covs, conics, samples = _single([0.95, 0.0], [-0.95, 0.0], [100.0, 0.0, 100.0],
                                                   [0.01, 0.0, 0.01])
    ob = oracle.OracleBins(means, covs, samples)
    assert ob.sample_keys()[0] in [t for t in range(ob.T) if 0 in ob.tile_gaussians(t)]
    x = np.float32(np.float32(0.95) - np.float32(-0.95))
    xw = np.float32(np.fmod(np.float64(x), 2.0) - 2.0)
    expect = 1.7 * np.exp(-0.5 * 100.0 * float(xw) ** 2)
    got = ob.forward("gaussian", values, conics)[0, 0, 0]
    assert abs(got - expect) <= 1e-6 * expect
    d = ob.forward("derivative", values, conics)[0, :, 0]
    assert abs(d[0] - expect * 100.0 * float(xw)) <= 1e-5 * abs(d[0])


def test_known_answer_tile_grid(oracle):
    """Samples spanning [-1, 1]: ceil((2 + 1e-6) / 0.51) = 4 tiles per axis, offset -1."""
    s = np.asarray([[-1.0, -1.0], [1.0, 1.0], [0.0, 0.5]], np.float32)
    grid, off = oracle.tile_grid(s)
    assert list(grid) == [4, 4] and list(off) == [-1.0, -1.0]
    grid1, _ = oracle.tile_grid(np.asarray([[0.0], [0.509]], np.float32))
    assert list(grid1) == [1]


def test_known_answer_sample_clamp_aliasing(oracle):
    """A sample at the x maximum of an aliasing domain gets x-tile == grid, i.e. the key of
    tile 0 in the next row (sampler_impl.cu:169-177)."""
    means, values, covs, conics, s = cases.aliasing_case(n=100, P=10)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), s.numpy())
    gx = int(ob.grid[0])
    keys = ob.sample_keys()
    # appended samples: [d, 0.5] has y-tile 0 -> key gx (row 1, tile 0); [d, 0.0] likewise
    assert keys[-3] == gx and keys[-2] == gx


def test_known_answer_full_range_and_absent(oracle):
    """det == 0 -> radius 0 and no tiles; a rect wider than the grid covers every tile once."""
    means = np.asarray([[0.0, 0.0], [0.1, 0.1]], np.float32)
    covs = np.asarray([[1.0, 1.0, 1.0], [4.0, 0.0, 4.0]], np.float32)
    samples = np.asarray([[-1.0, -1.0], [1.0, 1.0]], np.float32)
    ob = oracle.OracleBins(means, covs, samples)
    assert ob.radii[0] == 0.0 and ob.radii[1] > 0
    assert ob.num_rendered == ob.T
    for t in range(ob.T):
        assert list(ob.tile_gaussians(t)) == [1]


@pytest.mark.parametrize("case", ["synthetic", "seam"])
def test_torch_eager_baseline_matches_oracle(oracle, case):
    """oracle/torch_eager.py (bench.py's PyTorch-eager CPU baseline) computes what the C oracle
    computes: gaussian forward and its gradients over the reference's tile pair set."""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import torch_eager as te
    if case == "synthetic":
        means, values, covs, conics = syn.gaussians(800, 2, 2, seed=3)
        samples = syn.samples(3000, 2, seed=4)
    else:
        means, values, covs, conics, samples = cases.seam_case(D=2, C=2)
    N = samples.shape[0]
    dL = syn.grad_out(N, 1, values.shape[1], seed=6)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    sub = np.arange(N, dtype=np.int32)
    out, grads = te.gaussian_fwd_bwd(ob, means.numpy(), values.numpy(), conics.numpy(), samples.numpy(),
                                     dL.numpy(), sub)
    ref = ob.forward("gaussian", values.numpy(), conics.numpy(), subset=sub).reshape(out.shape)
    close(out.numpy(), ref, 1e-5, 1e-6, "torch eager forward")
    for g, r, name in zip(grads, ob.backward("gaussian", values.numpy(), conics.numpy(), dL.numpy(), subset=sub),
                          ("means", "values", "conics")):
        close(g.numpy(), r, 1e-4, 1e-5, f"torch eager d/d{name}")

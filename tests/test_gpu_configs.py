"""GPU parity at the BASELINE.json configurations that the small-case tests do not reach.

* config 2 -- 100k Gaussians x 256k query points, C = 16 (the lane-per-sample forward and the
  reference-literal backward terms), all four functions;
* config 5 -- aggregate_neighbors on the headline's 1M Gaussians (K = L = 16, F = 4), and the
  derivative / laplacian / third functions on a 4096^2 lattice of query points (SURVEY 8d's 2-D
  restatement of the "256^3 grid");
* config 4 on one GPU -- "fake shards": contiguous sample shards binned with the GLOBAL tile grid
  through preprocess_gaussians_bounded (the entry point every multi-GPU rank and bench.py use),
  outputs concatenated and gradients summed, against the oracle over all samples.

The CPU oracle cannot evaluate these sizes whole, so each check is a bounded subset: the forward
on a few thousand query points, the backward with dL/dout non-zero only on them (the gradients
then depend on those points alone), the neighbour lists row by row (oracle/oracle_agg.c's
row-restricted scan).  Tolerances are those of test_gpu_parity.py / test_gpu_aggregate.py.
"""
import numpy as np
import pytest
import torch

from diff_gaussian_sampling import synthetic as syn
from cases import AGG_FEATURES
from helpers import FUNCS, FWD_NAME, close

pytestmark = pytest.mark.gpu

RTOL = 1e-5
ATOL_FWD = 1e-6
ATOL_BWD = 1e-6  # rtol 1e-5 + atol 1e-6 max|ref|


def _subset(N, n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randperm(N, generator=g)[:n].sort().values.numpy().astype(np.int32)


def _check_subset(dgs, oracle, function, means, values, covs, conics, samples, subset, seed):
    """preprocess + forward + backward on the GPU (whole problem), checked on `subset`."""
    N, C = samples.shape[0], values.shape[1]
    K = syn.out_components(function, means.shape[1])
    dL = torch.zeros(N, K, C)
    dL[subset] = syn.grad_out(len(subset), K, C, seed=seed)
    dev = torch.device("cuda:0")
    m, v, cv, c, s = (t.to(dev) for t in (means, values, covs, conics, samples))
    R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
    out = getattr(dgs._C, FWD_NAME[function])(m, v, c, s, R, gb, sb, rg, srg, False)
    grads = getattr(dgs._C, FWD_NAME[function] + "_backward")(
        m, v, c, s, R, dL.to(dev).reshape(out.shape), gb, sb, rg, srg, False)
    got = out.reshape(N, K, C)[torch.from_numpy(subset).long().to(dev)].cpu().numpy()
    grads = [gg.cpu().numpy() for gg in grads]
    radii = radii.cpu().numpy()
    del out, gb, sb
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    assert R == ob.num_rendered, (R, ob.num_rendered)
    assert np.array_equal(radii, ob.radii), "radii"
    ref = ob.forward(function, values.numpy(), conics.numpy(), subset=subset)[subset]
    close(got, ref, RTOL, ATOL_FWD, f"{function} forward")
    dm, dv, dc = ob.backward(function, values.numpy(), conics.numpy(), dL.numpy(), subset=subset, exact=True)
    close(grads[0], dm, RTOL, ATOL_BWD, f"{function} dL/dmeans")
    close(grads[1], dv, RTOL, ATOL_BWD, f"{function} dL/dvalues")
    close(grads[2], dc, RTOL, ATOL_BWD, f"{function} dL/dconics")


@pytest.mark.parametrize("function", FUNCS)
def test_parity_config2_c16(dgs, oracle, function):
    """BASELINE config 2: 100k Gaussians x 256k query points, C = 16 (deg-3 SH -> 16 channels)."""
    P, N, C = 100_000, 256_000, 16
    means, values, covs, conics = syn.gaussians(P, 2, C, seed=0)
    samples = syn.samples(N, 2, seed=4)
    _check_subset(dgs, oracle, function, means, values, covs, conics, samples,
                  _subset(N, 1500, 201), seed=202)


@pytest.mark.slow
@pytest.mark.parametrize("function", ["derivative", "laplacian", "third"])
def test_parity_config5_grid_4096(dgs, oracle, function):
    """BASELINE config 5, sampling half: the headline's 1M Gaussians on a 4096^2 lattice
    (16.8M query points; samples on exact lattice positions hit tile and cell edges)."""
    P = 1_000_000
    means, values, covs, conics = syn.gaussians(P, 2, 1, seed=0)
    samples = syn.grid_samples(4096, 2)
    _check_subset(dgs, oracle, function, means, values, covs, conics, samples,
                  _subset(samples.shape[0], 1000, 211), seed=212)


@pytest.mark.slow
def test_aggregate_config5_subset(dgs, oracle):
    """BASELINE config 5, aggregation half: preprocess_aggregate / aggregate_neighbors /
    backward at P = 1M, K = L = 16, F = 4 on the headline Gaussians (radii from their binning).
    300 rows: their lists bit-exact against the oracle's row scan, their outputs, and the
    gradients of a loss whose dL is non-zero on those rows only."""
    P, L, K, F, D = 1_000_000, 16, 16, 4, 2
    E = 2 * D * F + 1
    means, values, covs, conics = syn.gaussians(P, D, 1, seed=0)
    dev = torch.device("cuda:0")
    m, v, cv, c = (t.to(dev) for t in (means, values, covs, conics))
    s = syn.samples(2_000_000, D, seed=4).to(dev)
    radii = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)[5]
    del s
    g = torch.Generator().manual_seed(221)
    fe = [torch.randn(P, L, generator=g), torch.randn(L, L, generator=g) / L,
          torch.randn(P, K, generator=g), torch.randn(P, K, generator=g),
          torch.rand(F, generator=g) * 2.5 + 0.5, torch.randn(2 * E, generator=g)]
    rows = _subset(P, 300, 222)
    idx, rg, X, dn, inv = dgs._C.preprocess_aggregate(m, c, radii, False)
    r_idx, r_rg, r_X, r_dn, r_inv = oracle.agg_preprocess_rows(
        means.numpy(), conics.numpy(), radii.cpu().numpy(), rows)
    rg_h = rg.cpu().numpy()
    starts = np.where(rows == 0, 0, rg_h[np.maximum(rows - 1, 0)])
    ends = rg_h[rows]
    assert np.array_equal(ends - starts, np.diff(np.concatenate([[0], r_rg]))), "row lengths"
    sel = torch.from_numpy(np.concatenate([np.arange(a, b) for a, b in zip(starts, ends)])).long().to(dev)
    assert np.array_equal(idx[sel].cpu().numpy(), r_idx), "indices"
    assert np.array_equal(X[sel].cpu().numpy().reshape(r_X.shape), r_X), "dists"
    close(dn[sel].cpu().numpy(), r_dn, 1e-6, 0.0, "densities")
    close(inv[torch.from_numpy(rows).long().to(dev)].cpu().numpy(), r_inv, 1e-5, 0.0, "inv_total")
    fd = [t.to(dev) for t in fe]
    w, e, f, out = dgs._C.aggregate_neighbors(*fd, idx, rg, X, dn, inv, False)
    args = [t.numpy() for t in fe]
    w_r, e_r, f_r, out_lit = oracle.agg_forward_rows(*args, rows, r_idx, r_rg, r_X, r_dn, r_inv)
    # neighbor_features / gradients: exact accumulation of the reference's per-slot float terms
    # (its own float order is ~1e-5 away from it at ~1100 slots per row; tests/test_gpu_aggregate.py)
    out_r = oracle.agg_forward_rows(*args, rows, r_idx, r_rg, r_X, r_dn, r_inv, exact=True)[3]
    close(w[sel].cpu().numpy(), w_r, 1e-5, 1e-6, "weights")
    close(e[sel].cpu().numpy(), e_r, 1e-5, 1e-6, "embeddings")
    close(f[sel].cpu().numpy(), f_r, 1e-5, 1e-6, "factors")
    rws = torch.from_numpy(rows).long().to(dev)
    close(out[rws].cpu().numpy(), out_r, 1e-5, 1e-6, "neighbor_features")
    # and against the reference's own (literal) float order at the stated looser bound
    # (test_gpu_aggregate.py LIT_RTOL / LIT_ATOL)
    close(out[rws].cpu().numpy(), out_lit, 3e-5, 3e-6, "neighbor_features vs the literal order")
    dL_rows = np.random.default_rng(223).normal(size=(len(rows), L)).astype(np.float32)
    dL = torch.zeros(P, L, device=dev)
    dL[rws] = torch.from_numpy(dL_rows).to(dev)
    got = dgs._C.aggregate_neighbors_backward(*fd, idx, rg, X, dn, w, e, f, inv, dL, False)
    ref = oracle.agg_backward_rows(*args, rows, r_idx, r_rg, r_X, r_dn, w_r, e_r, f_r, r_inv, dL_rows,
                                   exact=True)
    for name, a, b in zip(AGG_FEATURES, got, ref):
        close(a.cpu().numpy().reshape(b.shape), b, 1e-5, 1e-5, f"d/d{name}")
    lit = oracle.agg_backward_rows(*args, rows, r_idx, r_rg, r_X, r_dn, w_r, e_r, f_r, r_inv, dL_rows)
    for name, a, b in zip(AGG_FEATURES, got, lit):  # (all-slot sums: 1e-4, test_gpu_aggregate.py LIT_SHARED)
        tol = 1e-4 if name in ("frequencies", "distance_transform") else 3e-5
        close(a.cpu().numpy().reshape(b.shape), b, tol, tol, f"d/d{name} vs the literal order")


@pytest.mark.parametrize("function,C", [("gaussian", 1), ("derivative", 1), ("laplacian", 3)])
@pytest.mark.parametrize("shards", [2, 4])
def test_fake_shards_bounded_preprocess(dgs, oracle, function, C, shards):
    """One GPU, `shards` contiguous sample shards, each binned by preprocess_gaussians_bounded
    with the global grid: concatenated outputs and summed gradients equal the oracle over all
    samples (the single-GPU reference result); every shard reports the same num_rendered."""
    P, N, D = 20_000, 60_001, 2
    means, values, covs, conics = syn.gaussians(P, D, C, seed=231)
    samples = syn.samples(N, D, seed=232)
    samples = samples[torch.argsort(samples[:, 1])]  # every shard's own bounds differ from the global ones
    K = syn.out_components(function, D)
    dL = syn.grad_out(N, K, C, seed=233)
    dev = torch.device("cuda:0")
    m, v, cv, c, s, w = (t.to(dev) for t in (means, values, covs, conics, samples, dL))
    grid, off = dgs._C.tile_grid(s)
    outs, gsum = [], None
    for idx in torch.tensor_split(torch.arange(N), shards):
        sh = s[idx.to(dev)]
        R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians_bounded(m, v, cv, c, sh, list(grid), list(off), False)
        o = getattr(dgs._C, FWD_NAME[function])(m, v, c, sh, R, gb, sb, rg, srg, False)
        gr = getattr(dgs._C, FWD_NAME[function] + "_backward")(
            m, v, c, sh, R, w[idx.to(dev)].reshape(o.shape).contiguous(), gb, sb, rg, srg, False)
        outs.append(o.cpu())
        gsum = [g.clone() for g in gr] if gsum is None else [a + b for a, b in zip(gsum, gr)]
        ob_R = R
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    assert list(grid) == list(ob.grid) and np.array_equal(np.float32(off), ob.offset)
    assert ob_R == ob.num_rendered
    out = torch.cat(outs).numpy().reshape(N, K, C)
    close(out, ob.forward(function, values.numpy(), conics.numpy()), RTOL, ATOL_FWD, f"{function} sharded forward")
    dm, dv, dc = ob.backward(function, values.numpy(), conics.numpy(), dL.numpy(), exact=True)
    close(gsum[0].cpu().numpy(), dm, RTOL, ATOL_BWD, "sharded dL/dmeans")
    close(gsum[1].cpu().numpy(), dv, RTOL, ATOL_BWD, "sharded dL/dvalues")
    close(gsum[2].cpu().numpy(), dc, RTOL, ATOL_BWD, "sharded dL/dconics")

"""CPU tests pinning the aggregate_neighbors oracle (oracle/oracle_agg.c).

  * the neighbour predicate and slot order (aggregate_neighbors.cu:18-127) against an
    independent numpy restatement, plus known answers: the asymmetric torus wrap (only a
    positive dx wraps), the radius skip, self-inclusion, index -1 for power > 0;
  * the forward (129-208) against a torch float64 restatement, and the backward (210-321)
    against torch.autograd of it, with indices / dists / densities held fixed (the reference
    passes no gradient through them).
"""
import math

import numpy as np
import pytest
import torch

from cases import agg_problem
from helpers import close


def _problem(**kw):
    return agg_problem(**kw)


def np_neighbours(means, radii):
    """findCollisions restated with numpy (float32, CUDA's double-promoted min/fmod)."""
    P, D = means.shape
    rad = (radii.astype(np.float64) * 0.2).astype(np.float32)
    lists = []
    for i in range(P):
        if rad[i] < 1e-6:
            lists.append([])
            continue
        dx = (means - means[i]).astype(np.float32)  # other - my
        w = np.abs(2.0 - np.fmod(np.abs(dx).astype(np.float64), 2.0))
        dxw = np.minimum(dx.astype(np.float64), w).astype(np.float32)
        dist = np.zeros(P, np.float32)
        for d in range(D):
            dist = (dist + dxw[:, d] * dxw[:, d]).astype(np.float32)
        R = (rad[i] + rad).astype(np.float32)
        ok = ~(dist > R * R) & (rad >= 1e-6)
        lists.append(list(np.nonzero(ok)[0]))
    return lists


@pytest.mark.parametrize("D", [1, 2])
def test_neighbour_lists_match_numpy(oracle, D):
    means, conics, radii, _ = _problem(D=D, seed=D)
    idx, ranges, dists, dens, inv = oracle.agg_preprocess(means, conics, radii)
    lists = np_neighbours(means, radii)
    assert list(np.diff(np.r_[0, ranges])) == [len(l) for l in lists]
    for i, l in enumerate(lists):
        s, e = (0 if i == 0 else ranges[i - 1]), ranges[i]
        slot_ids = idx[s:e]
        valid = slot_ids >= 0
        assert np.array_equal(np.asarray(l)[valid], slot_ids[valid]), i  # ascending j, -1 skips
        assert np.all(dens[s:e][~valid] == 0)


def test_known_answers_asymmetric_wrap_and_skips(oracle):
    means = np.array([[-0.99, 0.0], [0.99, 0.0], [0.0, 0.5], [0.0, 0.52]], np.float32)
    radii = np.array([0.5, 0.5, 0.0, 0.5], np.float32)  # 0.2 r = 0.1; Gaussian 2 absent
    conics = np.tile(np.array([100.0, 0.0, 100.0], np.float32), (4, 1))
    idx, ranges, dists, dens, inv = oracle.agg_preprocess(means, conics, radii)
    rows = [idx[(0 if i == 0 else ranges[i - 1]):ranges[i]].tolist() for i in range(4)]
    assert rows[0] == [0, 1]  # 0 -> 1: dx = +1.98 wraps to 0.02 (and self)
    assert rows[1] == [1]     # 1 -> 0: dx = -1.98 does not wrap
    assert rows[2] == []      # radius-0 row
    assert rows[3] == [3]     # 2 is absent from every list; 3 alone
    # row 0's slot for Gaussian 1: X = 1.98 wrapped to -0.02, scaled by 1/(0.333 r + 1e-6)
    x = np.float32(np.float32(0.99) - np.float32(-0.99))
    xw = np.float32(math.fmod(float(x), 2.0) - 2.0)
    inv_r = np.float32(1.0 / (float(np.float32(0.5 * 0.333)) + 1e-6))
    assert dists[1, 0] == np.float32(xw * inv_r)
    assert abs(dens[1] - np.exp(-0.5 * 100.0 * float(xw) ** 2)) < 1e-6
    # radius-0 row: total 0 -> inv_total = 1 / 1e-6
    assert inv[2] == np.float32(1.0 / 1e-6)


def torch_forward(D, f, T, q, k, fr, dt, idx, ranges, X, dens, inv):
    """aggregateNeighbors in float64 torch (differentiable in f, T, q, k, fr, dt)."""
    P, L = f.shape
    E = dt.numel() // 2
    F, stride = (E - 1) // D // 2, (E - 1) // D
    rows = torch.repeat_interleave(torch.arange(P), torch.diff(torch.cat([torch.zeros(1, dtype=torch.long), ranges])))
    keep = idx >= 0
    rows, j, Xs, dn = rows[keep], idx[keep], X[keep], dens[keep]
    w = (q[rows] * k[j]).sum(1)
    emb = dt[E - 1] * torch.ones_like(w)
    fac = dt[2 * E - 1] * torch.ones_like(w)
    for d in range(D):
        for e in range(F):
            a = fr[e] * math.pi * Xs[:, d]
            emb = emb + dt[d * stride + 2 * e] * torch.sin(a) + dt[d * stride + 2 * e + 1] * torch.cos(a)
            fac = fac + dt[E + d * stride + 2 * e] * torch.sin(a) + dt[E + d * stride + 2 * e + 1] * torch.cos(a)
    dw = inv[rows] * dn * w
    embedded = (dw * emb)[:, None] + (dw * fac)[:, None] * f[j]
    A = torch.zeros(P, L, dtype=f.dtype).index_add(0, rows, embedded)
    return A @ T, w, emb, fac, keep


@pytest.mark.parametrize("D", [1, 2])
def test_forward_and_backward_vs_autograd(oracle, D):
    means, conics, radii, fe = _problem(D=D, seed=10 + D)
    idx, ranges, dists, dens, inv = oracle.agg_preprocess(means, conics, radii)
    args = [fe[k] for k in ("features", "transform", "queries", "keys", "frequencies", "distance_transform")]
    w, emb, fac, out = oracle.agg_forward(*args, idx, ranges, dists, dens, inv)
    t = [torch.tensor(a, dtype=torch.float64, requires_grad=True) for a in args]
    ref, tw, temb, tfac, keep = torch_forward(D, *t, torch.tensor(idx), torch.tensor(ranges),
                                              torch.tensor(dists, dtype=torch.float64),
                                              torch.tensor(dens, dtype=torch.float64),
                                              torch.tensor(inv, dtype=torch.float64))
    close(out, ref.detach().numpy(), 1e-4, 1e-5, "aggregate forward")
    close(w[keep.numpy()], tw.detach().numpy(), 1e-5, 1e-6, "weights")
    close(emb[keep.numpy()], temb.detach().numpy(), 1e-5, 1e-6, "embeddings")
    close(fac[keep.numpy()], tfac.detach().numpy(), 1e-5, 1e-6, "factors")
    assert np.all(w[~keep.numpy()] == 0)
    g = np.random.default_rng(5).normal(size=out.shape).astype(np.float32)
    grads = torch.autograd.grad(ref, t, torch.tensor(g, dtype=torch.float64))
    got = oracle.agg_backward(*args, idx, ranges, dists, dens, w, emb, fac, inv, g)
    for name, a, b in zip(("features", "transform", "queries", "keys", "frequencies", "distance_transform"),
                          got, grads):
        close(a, b.numpy(), 1e-4, 2e-5, f"d/d{name}")
    # the exact-accumulation twins (the GPU tests' reference): same formula, only the float
    # summation rounding removed, so they sit much closer to the fp64 autograd
    out64 = oracle.agg_forward(*args, idx, ranges, dists, dens, inv, exact=True)[3]
    assert out64.dtype == np.float64
    close(out64, ref.detach().numpy(), 1e-5, 1e-6, "aggregate forward (exact accumulation)")
    got64 = oracle.agg_backward(*args, idx, ranges, dists, dens, w, emb, fac, inv, g, exact=True)
    for name, a, b in zip(("features", "transform", "queries", "keys", "frequencies", "distance_transform"),
                          got64, grads):
        close(a, b.numpy(), 1e-5, 1e-6, f"d/d{name} (exact accumulation)")


@pytest.mark.parametrize("D", [1, 2])
def test_row_restricted_oracle_equals_full(oracle, D):
    """The row-restricted scan and its forward/backward (the config-5 GPU subset check) equal the
    full oracle: the same slots, outputs, and the gradients of a loss with dL on those rows only."""
    m, c, r, fe = _problem(P=150, D=D, seed=31)
    full = oracle.agg_preprocess(m, c, r)
    rows = np.array([0, 3, 5, 77, 149], np.int32)
    sub = oracle.agg_preprocess_rows(m, c, r, rows)
    rg = full[1]
    sl = np.concatenate([np.arange(0 if i == 0 else rg[i - 1], rg[i]) for i in rows])
    assert np.array_equal(full[0][sl], sub[0]) and np.array_equal(full[2][sl], sub[2])
    assert np.array_equal(full[3][sl], sub[3]) and np.array_equal(full[4][rows], sub[4])
    args = [fe[k] for k in ("features", "transform", "queries", "keys", "frequencies", "distance_transform")]
    w, e, f, out = oracle.agg_forward(*args, *full)
    ws, es, fs, outs = oracle.agg_forward_rows(*args, rows, *sub)
    assert np.array_equal(w[sl], ws) and np.array_equal(out[rows], outs)
    g = np.zeros_like(out)
    g[rows] = np.random.default_rng(32).normal(size=(len(rows), out.shape[1])).astype(np.float32)
    ref = oracle.agg_backward(*args, *full[:4], w, e, f, full[4], g)
    got = oracle.agg_backward_rows(*args, rows, *sub[:4], ws, es, fs, sub[4], g[rows])
    for a, b in zip(got, ref):
        close(a, b, 1e-6, 1e-7, "row-restricted gradient")


def test_torch_eager_aggregate_matches_oracle(oracle):
    """bench.py's PyTorch-eager CPU baseline for aggregate_neighbors (oracle/torch_eager.py) is the
    same math: forward and autograd gradients equal the oracle's exact accumulation."""
    import numpy as np
    from cases import AGG_FEATURES, agg_problem
    from oracle import torch_eager as te
    means, conics, radii, fe = agg_problem(P=500, D=2, L=16, K=16, F=4, seed=9)
    idx, rg, X, dn, inv = oracle.agg_preprocess(means, conics, radii)
    args = [fe[k] for k in AGG_FEATURES]
    w, e, f, out = oracle.agg_forward(*args, idx, rg, X, dn, inv, exact=True)
    g = np.random.default_rng(2).normal(size=out.shape).astype(np.float32)
    ref = oracle.agg_backward(*args, idx, rg, X, dn, w, e, f, inv, g, exact=True)
    o2, grads = te.aggregate_fwd_bwd(*args, idx, rg, X, dn, inv, g, rows=500)
    np.testing.assert_allclose(o2.numpy(), out, rtol=1e-4, atol=1e-5 * np.abs(out).max())
    for name, a, b in zip(AGG_FEATURES, grads, ref):
        np.testing.assert_allclose(a.numpy().reshape(b.shape), b, rtol=1e-4, atol=1e-5 * np.abs(b).max(), err_msg=name)

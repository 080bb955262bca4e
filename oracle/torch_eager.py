"""PyTorch-eager CPU evaluation of the gaussian function, forward + backward, on the host cores.

TEST INFRASTRUCTURE ONLY, like the rest of oracle/: bench.py's cpu_baseline leg imports it to
time "a PyTorch-eager CPU evaluation of the same math on the host cores" (BASELINE.json
north_star) next to the GPU; the product package never does.

The math is the reference's, vectorised: for every query point, every Gaussian of its tile
(the reference's pair set, taken from the C oracle's binning, sample_points.cu:38-98 and
sampler_impl.cu:216-330), X = mean - sample with the period-2 wrap of forward.cu:149-157,
power = -0.5 (c0 X0^2 + c2 X1^2) - c1 X0 X1 (forward.cu:225-235), G = exp(power) unless
power > 0, out = sum v G; the backward is torch autograd of that forward (the reference's
backward.cu gradients for the gaussian function equal it, tests/test_oracle.py).
Tiles are evaluated in chunks of query points so the [points x Gaussians] temporaries stay
bounded; each chunk's loss is back-propagated at once.
"""
import numpy as np
import torch


def _wrap(X):
    ax = X.abs()
    r = torch.where(ax < 2.0, ax, torch.fmod(ax, 2.0)) - 2.0
    return torch.where(ax > 1.0, torch.where(X >= 0, r, -r), X)


def gaussian_fwd_bwd(ob, means, values, conics, samples, dL, subset, chunk=256):
    """Forward + backward of the gaussian function (D = 2) for the query points `subset`.
    Returns (out[len(subset), C], (dmeans, dvalues, dconics)) -- partial gradients over them."""
    m = torch.from_numpy(np.ascontiguousarray(means, np.float32)).requires_grad_(True)
    v = torch.from_numpy(np.ascontiguousarray(values, np.float32)).requires_grad_(True)
    c = torch.from_numpy(np.ascontiguousarray(conics, np.float32)).requires_grad_(True)
    s = torch.from_numpy(np.ascontiguousarray(samples, np.float32))
    g_out = torch.from_numpy(np.ascontiguousarray(dL, np.float32)).reshape(samples.shape[0], -1)
    keys = ob.sample_keys()
    subset = np.asarray(subset)
    out = torch.zeros(len(subset), values.shape[1])
    for t in np.unique(keys[subset]):
        if t < 0 or t >= ob.T:  # never rendered (sampler_impl.cu:177-182): output stays 0
            continue
        rows = np.nonzero(keys[subset] == t)[0]
        gid = torch.from_numpy(ob.tile_gaussians(int(t)).astype(np.int64))
        if gid.numel() == 0:
            continue
        for a in range(0, len(rows), chunk):
            r = rows[a:a + chunk]
            sid = torch.from_numpy(subset[r].astype(np.int64))
            X = _wrap(m[gid][None, :, :] - s[sid][:, None, :])          # [S, G, 2]
            cg = c[gid]
            power = (-0.5 * (cg[None, :, 0] * X[..., 0] * X[..., 0] + cg[None, :, 2] * X[..., 1] * X[..., 1])
                     - cg[None, :, 1] * X[..., 0] * X[..., 1])
            G = torch.where(power > 0, torch.zeros_like(power), torch.exp(power))
            o = G @ v[gid]                                               # [S, C]
            (o * g_out[sid]).sum().backward()
            out[torch.from_numpy(r.astype(np.int64))] = o.detach()
    return out, (m.grad, v.grad, c.grad)


def aggregate_fwd_bwd(features, transform, queries, keys, frequencies, distance_transform, indices,
                      ranges, dists, densities, inv_total, dL, rows):
    """PyTorch-eager CPU evaluation of aggregate_neighbors (aggregate_neighbors.cu:129-208) for
    the first `rows` rows of the given neighbour lists, forward + autograd backward (the
    reference's aggregateNeighborsBackward gradients equal autograd of this forward,
    tests/test_oracle_agg.py).  Vectorised over the rows' slots:
      weight = q_i . k_j,  emb / fac = sum_{d,e} dt[.] sin / cos(f_e pi X_d) + bias,
      dw = inv_total_i density_s weight,  out_i = T^T sum_s (dw emb 1 + dw fac feat_j).
    Returns (out[rows, L], the six gradients)."""
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    feat, T, q, k = (t(a).float().requires_grad_(True) for a in (features, transform, queries, keys))
    fr, dt = (t(a).float().requires_grad_(True) for a in (frequencies, distance_transform))
    rg = np.asarray(ranges)
    nslot = int(rg[rows - 1])
    idx = t(np.asarray(indices)[:nslot]).long()
    X = t(np.asarray(dists)[:nslot]).float().reshape(nslot, -1)
    dens = t(np.asarray(densities)[:nslot]).float()
    row_of = torch.repeat_interleave(torch.arange(rows), t(np.diff(np.concatenate([[0], rg[:rows]]))).long())
    valid = idx >= 0
    j = torch.where(valid, idx, torch.zeros_like(idx))
    D, L = X.shape[1], feat.shape[1]
    E = dt.shape[0] // 2
    F = (E - 1) // D // 2
    stride = (E - 1) // D
    weight = (q[row_of] * k[j]).sum(1)
    arg = fr[:F][None, None, :] * np.pi * X[:, :, None]           # [s, d, e]
    sn, cs = torch.sin(arg), torch.cos(arg)
    a_idx = torch.arange(D)[:, None] * stride + 2 * torch.arange(F)[None, :]
    emb = (dt[a_idx] * sn + dt[a_idx + 1] * cs).sum((1, 2)) + dt[E - 1]
    fac = (dt[E + a_idx] * sn + dt[E + a_idx + 1] * cs).sum((1, 2)) + dt[2 * E - 1]
    dw = t(np.asarray(inv_total)).float()[row_of] * dens * weight
    dw = torch.where(valid, dw, torch.zeros_like(dw))
    embedded = (dw * emb)[:, None] + (dw * fac)[:, None] * feat[j]   # [s, L]
    summed = torch.zeros(rows, L).index_add(0, row_of, embedded)
    out = summed @ T
    out.backward(t(np.asarray(dL)[:rows]).float())
    return out.detach(), tuple(x.grad for x in (feat, T, q, k, fr, dt))

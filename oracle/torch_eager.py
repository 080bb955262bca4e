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

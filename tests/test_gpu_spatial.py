"""Spatial sharding and BASELINE config 4 on the HIP path, against the oracle.

* config 4 on one GPU: 1M Gaussians, 8 strip shards of 1M query points each (the 1M x 8M union,
  uniform), each shard binned with the GLOBAL grid through preprocess_gaussians_sharded with the
  rank's held rows (distributed.SupportExchange) and its own sample area.  Every shard's partial
  gradient is exactly 0 outside the rows its strip touches (what makes the sparse owner reduce
  exact); the owners' sums and the outputs equal the oracle on a 1,500-point subset (dL/dout
  non-zero only there, reference file:line sample_points.cu:70-74, forward.cu:149-157).
* 2 ranks over gloo, both on cuda:0 (a 1-GPU box; RCCL refuses two ranks per device):
  SpatialShardedGaussianSampler over the real _C against the oracle, and three Adam steps with
  push() against the single-process loop on the same GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from diff_gaussian_sampling import synthetic as syn
from helpers import FWD_NAME, close

pytestmark = pytest.mark.gpu

RTOL, ATOL_FWD, ATOL_BWD = 1e-5, 1e-6, 1e-6  # SURVEY 8c (backward: atol 1e-6 max|ref|)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("function", ["gaussian", "laplacian"])
def test_config4_strip_shards_one_gpu(dgs, oracle, function):
    import diff_gaussian_sampling.distributed as dd
    P, Nr, W, D, C = 1_000_000, 1_000_000, 8, 2, 1
    K = syn.out_components(function, D)
    means, values, covs, conics = syn.gaussians(P, D, C, seed=0)
    shards = [syn.strip_samples(Nr, D, r, W, seed=4 + 1000 * r) for r in range(W)]
    allpts = torch.cat(shards)
    sub = torch.randperm(W * Nr, generator=torch.Generator().manual_seed(241))[:1500].sort().values
    dL = torch.zeros(W * Nr, K, C)
    dL[sub] = syn.grad_out(len(sub), K, C, seed=242)
    dev = torch.device("cuda:0")
    m, v, cv, c = (t.to(dev) for t in (means, values, covs, conics))
    grid, off = dgs._C.tile_grid(allpts.to(dev))
    ext = torch.stack([torch.stack([s[:, 1].min(), s[:, 1].max()]) for s in shards]).double()
    mask, owner = dd.exchange_sets(m, c, ext)
    touch = [((mask >> r) & 1).bool() for r in range(W)]
    owner_h = owner.cpu()
    # the owner touches its row whenever the row touches any strip
    anyt = torch.stack(touch).any(0)
    assert bool(torch.stack(touch)[owner, torch.arange(P, device=dev)][anyt].all())
    out = torch.empty(W * Nr, K, C)
    gsum = None
    wcand = []
    for r, s in enumerate(shards):
        held = touch[r] | (owner == r)
        sd = s.to(dev)
        lo, hi = s.min(0).values, s.max(0).values
        area = float((hi - lo).prod())
        R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians_sharded(
            m, v, cv, c, sd, list(grid), list(off), held, area, False)
        o = getattr(dgs._C, FWD_NAME[function])(m, v, c, sd, R, gb, sb, rg, srg, False)
        out[r * Nr:(r + 1) * Nr] = o.reshape(Nr, K, C).cpu()
        gr = getattr(dgs._C, FWD_NAME[function] + "_backward")(
            m, v, c, sd, R, dL[r * Nr:(r + 1) * Nr].to(dev).reshape(o.shape).contiguous(), gb, sb, rg, srg, False)
        nt = ~touch[r]
        for g in gr:  # the sparse reduce is exact: nothing outside the touched rows
            assert int((g[nt] != 0).sum()) == 0
        gsum = [g.clone() for g in gr] if gsum is None else [a + b for a, b in zip(gsum, gr)]
        wcand.append(dgs._C.count_pairs(m, c, sd, gb, sb, -104.0)[0] / Nr)
        del gb, sb, o
    # cells sized for each strip's own density: no more candidates per point than the 1-GPU headline
    assert max(wcand) < 1254, wcand
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), allpts.numpy())
    assert list(grid) == list(ob.grid) and np.array_equal(np.float32(off), ob.offset)
    sn = sub.numpy().astype(np.int32)
    ref = ob.forward(function, values.numpy(), conics.numpy(), subset=sn)[sn]
    close(out[sub].numpy().reshape(ref.shape), ref, RTOL, ATOL_FWD, f"{function} config-4 forward")
    dm, dv, dc = ob.backward(function, values.numpy(), conics.numpy(), dL.numpy(), subset=sn, exact=True)
    close(gsum[0].cpu().numpy(), dm, RTOL, ATOL_BWD, "config-4 owner-summed dL/dmeans")
    close(gsum[1].cpu().numpy(), dv, RTOL, ATOL_BWD, "config-4 owner-summed dL/dvalues")
    close(gsum[2].cpu().numpy(), dc, RTOL, ATOL_BWD, "config-4 owner-summed dL/dconics")


def _problem():
    means, values, covs, conics = syn.gaussians(40000, 2, 1, seed=251)
    samples = syn.samples(60000, 2, seed=252)
    sub = torch.randperm(60000, generator=torch.Generator().manual_seed(253))[:3000].sort().values
    w = torch.zeros(60000, 2, 1)
    w[sub] = syn.grad_out(len(sub), 2, 1, seed=254)
    return means, values, covs, conics, samples, w, sub


def _cov_of(conics):
    c = conics.detach().double()
    det = c[:, 0] * c[:, 2] - c[:, 1] ** 2
    return torch.stack([c[:, 2] / det, -c[:, 1] / det, c[:, 0] / det], 1).float()


ADAM_STEPS, ADAM_LR = 3, 1e-3


def _loop(sampler, m, v, c, samples, w, steps, push):
    opt = torch.optim.Adam([m, v, c], lr=ADAM_LR)
    outs = []
    for _ in range(steps):
        sampler.preprocess(m, v, _cov_of(c), c, samples)
        opt.zero_grad()
        out = sampler.sample_gaussians_derivative()
        outs.append(out.detach().cpu())
        (out * w).sum().backward()
        if not outs[1:]:
            first = tuple(t.grad.detach().cpu().clone() for t in (m, v, c))
        opt.step()
        if push:
            sampler.push([m, v, c])
    return outs, first


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import diff_gaussian_sampling.distributed as dd
        means, values, covs, conics, samples, w, sub = _problem()
        order = torch.argsort(samples[:, 1])
        shard = torch.tensor_split(order, world)[rank].sort().values
        dev = torch.device("cuda:0")
        m, v, c = (t.to(dev).requires_grad_(True) for t in (means, values, conics))
        sampler = dd.SpatialShardedGaussianSampler(debug=True)
        outs, first = _loop(sampler, m, v, c, samples[shard].to(dev), w[shard].to(dev), ADAM_STEPS, True)
        x = sampler.xchg
        np.savez(os.path.join(outdir, f"g{rank}.npz"), shard=shard.numpy(), out0=outs[0].numpy(),
                 gm=first[0].numpy(), gv=first[1].numpy(), gc=first[2].numpy(),
                 m=m.detach().cpu().numpy(), v=v.detach().cpu().numpy(), c=c.detach().cpu().numpy(),
                 owned=x.owned.cpu().numpy(), held=x.held.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_spatial_sampler_two_ranks_real_C(dgs, oracle, tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    import diff_gaussian_sampling.distributed as dd
    means, values, covs, conics, samples, w, sub = _problem()
    ranks = [np.load(tmp_path / f"g{r}.npz") for r in range(world)]
    grid, off = dd.global_tile_grid(samples)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy(), grid, off)
    sn = sub.numpy().astype(np.int32)
    ref = ob.forward("derivative", values.numpy(), conics.numpy(), subset=sn)
    got = np.zeros_like(ref)
    for r in ranks:
        got[r["shard"]] = r["out0"].reshape(len(r["shard"]), 2, 1)
    close(got[sn], ref[sn], RTOL, ATOL_FWD, "2-rank spatial forward")
    dm, dv, dc = ob.backward("derivative", values.numpy(), conics.numpy(), w.numpy(), subset=sn, exact=True)
    assert np.array_equal(ranks[0]["owned"], ~ranks[1]["owned"])
    for r in ranks:  # the first step's gradient: global sums on the owned rows, 0 elsewhere
        mine = r["owned"]
        for k, exp in (("gm", dm), ("gv", dv), ("gc", dc)):
            close(r[k][mine], exp[mine], RTOL, ATOL_BWD, f"2-rank owned {k}")
            assert np.all(r[k][~mine] == 0)
    # the same 3 Adam steps in one process over all the points, on the same GPU
    dev = torch.device("cuda:0")
    m, v, c = (t.to(dev).requires_grad_(True) for t in (means, values, conics))
    _loop(dd.ShardedGaussianSampler(), m, v, c, samples.to(dev), w.to(dev), ADAM_STEPS, False)
    refp = {"m": m.detach().cpu().numpy(), "v": v.detach().cpu().numpy(), "c": c.detach().cpu().numpy()}
    assert not np.allclose(refp["m"], means.numpy())
    # Adam divides each step by the gradient's running RMS, so where the exact gradient is at the
    # float noise of two summation orders (|g| within the parity bound of 0) the two runs' updates
    # may differ by up to the step size itself; there the check is that bound, elsewhere 2e-5
    # (the first step's full gradient: the owned rows of the two ranks)
    full = {k: sum(r[gk] for r in ranks) for k, gk in (("m", "gm"), ("v", "gv"), ("c", "gc"))}
    for r in ranks:
        h = r["held"]
        for k in ("m", "v", "c"):
            g = np.abs(full[k]).reshape(refp[k].shape)
            noise = g <= 10 * ATOL_BWD * g.max()
            a, b = r[k][h], refp[k][h]
            nz = noise[h]
            np.testing.assert_allclose(a[~nz], b[~nz], rtol=2e-5, atol=1e-6 * np.abs(refp[k]).max())
            assert np.all(np.abs(a[nz] - b[nz]) <= 2 * ADAM_LR * ADAM_STEPS), k


def test_padded_push_and_reduce_without_host_sync(dgs):
    """the sync-free push and the padded reduce issue no host synchronisation.
    One process plays rank 0 of 2 strips with a device-copy stand-in for the all-to-all (no
    process group), and the push + reduce run under torch.cuda.set_sync_debug_mode("error"): any
    blocking H2D copy, .item() or output-size readback inside them raises."""
    import diff_gaussian_sampling.distributed as dd
    dev = torch.device("cuda:0")
    P, D, C = 4000, 2, 1
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, D, C, seed=7))
    ext = torch.tensor([[-1.0, 0.0], [0.0, 1.0]], dtype=torch.float64)
    xchg = dd.SupportExchange(means, conics, ext, rank=0)
    assert xchg.world == 2 and xchg._padded_ok

    def a2a(out, inp, out_splits, in_splits):  # (what rank 1 would send: shape-correct, device only)
        n = min(out.numel(), inp.numel())
        out.view(-1)[n:].zero_()
        if n:
            out.view(-1)[:n].copy_(inp.reshape(-1)[:n])

    xchg._a2a = a2a
    moved = means.clone()
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        sent = xchg.push([moved, values], moved, conics, sync=False)
        G = torch.randn(P, 6, device=dev)
        xchg.reduce(G)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    assert xchg.padded is not None and sent.is_cuda
    assert torch.isfinite(G).all()
    assert bool((G[~xchg.owned] == 0).all())

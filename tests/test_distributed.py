"""Query-point sharding over torch.distributed, world_size 2 on CPU with gloo.

Each rank runs diff_gaussian_sampling.distributed.ShardedGaussianSampler on its contiguous
shard of the samples with an oracle-backed `_C` (tests/oracle_stub.py).  The shards' outputs,
concatenated, and the all-reduced gradients must equal a single-process run over all samples
with the same (global) tile grid -- i.e. the global-grid all-reduce (MIN/MAX) and the packed
gradient all-reduce are exactly what makes sharding transparent.  The GPU bench uses the same
code with the nccl (RCCL) backend.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem():
    from diff_gaussian_sampling import synthetic as syn
    means, values, covs, conics = syn.gaussians(600, 2, 2, seed=301)
    samples = syn.samples(3001, 2, seed=302)
    # sort by x so that every shard's own bounding box differs from the global one
    samples = samples[torch.argsort(samples[:, 0])]
    w = syn.grad_out(3001, 2, 2, seed=303).reshape(3001, 2, 2)
    return means, values, covs, conics, samples, w


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import diff_gaussian_sampling.distributed as dd
        from oracle_stub import OracleC
        dd._C = OracleC()
        means, values, covs, conics, samples, w = _problem()
        shard = torch.tensor_split(torch.arange(samples.shape[0]), world)[rank]
        m, v, c = (t.clone().requires_grad_(True) for t in (means, values, conics))
        sampler = dd.ShardedGaussianSampler(False)
        sampler.preprocess(m, v, covs, c, samples[shard])
        out = sampler.sample_gaussians_derivative()
        (out * w[shard]).sum().backward()
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), out=out.detach().numpy(),
                 shard=shard.numpy(), gm=m.grad.numpy(), gv=v.grad.numpy(), gc=c.grad.numpy(),
                 grid=np.asarray(sampler.grid), offset=np.asarray(sampler.offset, np.float32))
    finally:
        dist.destroy_process_group()


def test_sharded_sampler_matches_single_process(tmp_path, oracle):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    means, values, covs, conics, samples, w = _problem()
    ranks = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    # every rank derived the same global grid
    for r in ranks[1:]:
        assert np.array_equal(r["grid"], ranks[0]["grid"])
        assert np.array_equal(r["offset"], ranks[0]["offset"])
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy(), ranks[0]["grid"],
                           ranks[0]["offset"])
    ref = ob.forward("derivative", values.numpy(), conics.numpy())
    got = np.zeros_like(ref)
    for r in ranks:
        got[r["shard"]] = r["out"].reshape(len(r["shard"]), 2, 2)
    assert np.array_equal(got, ref)
    dm, dv, dc = ob.backward("derivative", values.numpy(), conics.numpy(), w.numpy())
    for r in ranks:  # all-reduced: every rank holds the full gradient
        for k, exp in (("gm", dm), ("gv", dv), ("gc", dc)):
            np.testing.assert_allclose(r[k], exp, rtol=1e-5, atol=1e-5 * np.abs(exp).max())


def test_global_grid_differs_from_shard_grid(oracle):
    """Sanity: the shards' own grids differ from the global one on this problem, so the test
    above would fail without global_tile_grid's all-reduce."""
    _, _, _, _, samples, _ = _problem()
    g_all, o_all = oracle.tile_grid(samples.numpy())
    g0, o0 = oracle.tile_grid(samples[:1500].numpy())
    assert not (np.array_equal(g_all, g0) and np.array_equal(o_all, o0))


def test_allreduce_grads_single_process_passthrough():
    from diff_gaussian_sampling.distributed import allreduce_grads
    g = (torch.ones(3, 2), torch.ones(3, 1), torch.ones(3, 3))
    assert allreduce_grads(g) is g


def _chunk_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from diff_gaussian_sampling.distributed import allreduce_grads
        g = torch.Generator().manual_seed(400 + rank)
        P = 1001  # (not a multiple of the block counts)
        grads = (torch.randn(P, 2, generator=g), torch.randn(P, 3, generator=g), torch.randn(P, 3, generator=g))
        res = {}
        for chunks in (1, 2, 4, 7):
            out = allreduce_grads(tuple(t.clone() for t in grads), chunks=chunks)
            res[f"c{chunks}"] = np.concatenate([o.reshape(P, -1).numpy() for o in out], 1)
        np.savez(os.path.join(outdir, f"chunk{rank}.npz"), **res,
                 mine=np.concatenate([t.numpy() for t in grads], 1))
    finally:
        dist.destroy_process_group()


def test_chunked_allreduce_equals_unchunked(tmp_path):
    """allreduce_grads in 2, 4, 7 pipelined row blocks equals the one-collective sum bit for bit
    at world 2 (and is the sum of both ranks' partial gradients)."""
    port = _free_port()
    mp.start_processes(_chunk_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="fork")
    r = [np.load(tmp_path / f"chunk{k}.npz") for k in range(2)]
    want = r[0]["mine"] + r[1]["mine"]
    for k in range(2):
        for c in ("c2", "c4", "c7"):
            assert np.array_equal(r[k][c], r[k]["c1"]), (k, c)
        assert np.array_equal(r[k]["c1"], want)


def _spatial_problem():
    """Gaussians small against the strips (h = 2 / sqrt(P) = 0.01, cut half-widths ~0.2), so
    most of them reach one rank only; the uniform points wrap across y = +-1 (rank 0 <-> W-1)."""
    from diff_gaussian_sampling import synthetic as syn
    means, values, covs, conics = syn.gaussians(40000, 2, 2, seed=321)
    samples = syn.samples(6001, 2, seed=322)
    w = syn.grad_out(6001, 2, 2, seed=323).reshape(6001, 2, 2)
    return means, values, covs, conics, samples, w


def _spatial_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import diff_gaussian_sampling.distributed as dd
        from oracle_stub import OracleC
        dd._C = OracleC()
        means, values, covs, conics, samples, w = _spatial_problem()
        order = torch.argsort(samples[:, 1])  # spatial strips along y
        shard = torch.tensor_split(order, world)[rank].sort().values
        m, v, c = (t.clone().requires_grad_(True) for t in (means, values, conics))
        sampler = dd.SpatialShardedGaussianSampler(debug=True)
        sampler.preprocess(m, v, covs, c, samples[shard])
        out = sampler.sample_gaussians_derivative()
        (out * w[shard]).sum().backward()
        x = sampler.xchg
        mask, _ = dd.exchange_sets(means, conics, x.extents)
        np.savez(os.path.join(outdir, f"srank{rank}.npz"), out=out.detach().numpy(),
                 shard=shard.numpy(), gm=m.grad.numpy(), gv=v.grad.numpy(), gc=c.grad.numpy(),
                 touch=np.stack([((mask >> r) & 1).bool().numpy() for r in range(world)], 1),
                 owner=x.owner.numpy(), held=x.held.numpy(), moved=x.rows_moved())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_spatial_shards_support_exchange(tmp_path, oracle, world):
    """SpatialShardedGaussianSampler: strips of the points along y, each rank binning
    only the Gaussians it holds.  Outputs equal the single-process oracle bit for bit; after the
    backward every rank holds the single-process gradient on the rows it owns and exactly 0
    elsewhere; every row has one owner, a rank it touches when it touches any; fewer rows move
    than are touched."""
    mp.spawn(_spatial_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    means, values, covs, conics, samples, w = _spatial_problem()
    ranks = [np.load(tmp_path / f"srank{r}.npz") for r in range(world)]
    from diff_gaussian_sampling.distributed import global_tile_grid
    grid, off = global_tile_grid(samples)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy(), grid, off)
    ref = ob.forward("derivative", values.numpy(), conics.numpy())
    got = np.zeros_like(ref)
    for r in ranks:
        got[r["shard"]] = r["out"].reshape(len(r["shard"]), 2, 2)
    assert np.array_equal(got, ref)
    dm, dv, dc = ob.backward("derivative", values.numpy(), conics.numpy(), w.numpy())
    P = means.shape[0]
    owner = ranks[0]["owner"]
    touch = ranks[0]["touch"]
    assert np.all(touch[np.arange(P), owner] | ~touch.any(1))  # the owner touches the row
    for ri, r in enumerate(ranks):
        assert np.array_equal(r["owner"], owner) and np.array_equal(r["touch"], touch)
        mine = owner == ri
        t = touch[:, ri]
        assert 0 < t.sum() < P  # strips: not every Gaussian reaches every rank
        assert np.array_equal(r["held"], t | mine)
        for k, exp in (("gm", dm), ("gv", dv), ("gc", dc)):
            np.testing.assert_allclose(r[k][mine], exp[mine], rtol=1e-5, atol=1e-5 * np.abs(exp).max())
            assert np.all(r[k][~mine] == 0)
        assert r["moved"] < 0.5 * t.sum()


def _cov_of(conics):
    """D = 2 covariances [xx, xy, yy] of packed conics [c0, c1, c2] (exact 2x2 inverse)."""
    c = conics.detach().double()
    det = c[:, 0] * c[:, 2] - c[:, 1] ** 2
    return torch.stack([c[:, 2] / det, -c[:, 1] / det, c[:, 0] / det], 1).float()


ADAM_STEPS, ADAM_LR = 3, 1e-3


def _adam_worker(rank, world, port, outdir, mode="sync"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import diff_gaussian_sampling.distributed as dd
        from oracle_stub import OracleC
        dd._C = OracleC()
        if mode == "overflow":  # capacities far below the counts: every padded push overflows
            dd.SupportExchange.cap_of = staticmethod(lambda n: max(n // 8, 1) if n else 0)
        means, values, covs, conics, samples, w = _spatial_problem()
        order = torch.argsort(samples[:, 1])
        shard = torch.tensor_split(order, world)[rank].sort().values
        m, v, c = (t.clone().requires_grad_(True) for t in (means, values, conics))
        opt = torch.optim.Adam([m, v, c], lr=ADAM_LR)
        sampler = dd.SpatialShardedGaussianSampler()
        moved = []
        for _ in range(ADAM_STEPS):
            sampler.preprocess(m, v, _cov_of(c), c, samples[shard])
            opt.zero_grad()
            (sampler.sample_gaussians_derivative() * w[shard]).sum().backward()
            opt.step()
            moved.append(int(sampler.xchg.push([m, v, c], m, c, sync=mode == "sync")))
        # (the next step's preprocess -- where a padded push's overflow is answered by an exact one)
        sampler.preprocess(m, v, _cov_of(c), c, samples[shard])
        np.savez(os.path.join(outdir, f"adam{rank}.npz"), m=m.detach().numpy(), v=v.detach().numpy(),
                 c=c.detach().numpy(), owned=sampler.xchg.owned.numpy(), held=sampler.xchg.held.numpy(),
                 moved=np.asarray(moved))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sync", "padded", "overflow"])
def test_spatial_shards_adam_matches_single_process(tmp_path, oracle, mode):
    """Three Adam steps of a 2-rank spatially sharded run (owner-side reduce, optimizer over the
    full tensors, push of the owners' rows) against the same loop in one process over all the
    points: every rank's held rows -- the owned and the pushed ones, i.e. every row its strip
    reads -- equal the single-process parameters.  mode: the exact push (host-known counts), the
    sync-free padded push (capacities from the last exact exchange, device-side counts), and the
    padded push with capacities too small (its overflow is answered by an exact push at the next
    preprocess)."""
    import diff_gaussian_sampling.distributed as dd
    from oracle_stub import OracleC
    world = 2
    mp.spawn(_adam_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world, join=True)
    means, values, covs, conics, samples, w = _spatial_problem()
    saved = dd._C
    dd._C = OracleC()
    try:
        m, v, c = (t.clone().requires_grad_(True) for t in (means, values, conics))
        opt = torch.optim.Adam([m, v, c], lr=ADAM_LR)
        sampler = dd.ShardedGaussianSampler()
        for _ in range(ADAM_STEPS):
            sampler.preprocess(m, v, _cov_of(c), c, samples)
            opt.zero_grad()
            (sampler.sample_gaussians_derivative() * w).sum().backward()
            opt.step()
    finally:
        dd._C = saved
    ref = {"m": m.detach().numpy(), "v": v.detach().numpy(), "c": c.detach().numpy()}
    ranks = [np.load(tmp_path / f"adam{r}.npz") for r in range(world)]
    assert np.array_equal(ranks[0]["owned"], ~ranks[1]["owned"])
    for r in ranks:
        h = r["held"]
        assert 0 < h.sum() < len(h) and np.all(r["moved"] > 0)
        for k in ("m", "v", "c"):
            np.testing.assert_allclose(r[k][h], ref[k][h], rtol=2e-5, atol=1e-6 * np.abs(ref[k]).max())
        assert not np.allclose(ref["m"], means.numpy())  # the steps moved the parameters


def test_support_halfwidth_bounds_the_live_pairs(oracle):
    """The y-extent sqrt(210 (A^-1)_yy) of the cut bounds every pair with a non-zero exponent:
    count live pairs (power >= -104) whose |dy| (after the torus wrap) exceeds it -- none."""
    from diff_gaussian_sampling import synthetic as syn
    from diff_gaussian_sampling.distributed import support_halfwidth
    means, values, covs, conics = syn.gaussians(300, 2, 1, seed=311)
    samples = syn.samples(4000, 2, seed=312)
    e = support_halfwidth(means, conics).numpy()
    X = means.numpy()[:, None, :].astype(np.float64) - samples.numpy()[None, :, :]
    X = np.where(np.abs(X) > 1, np.fmod(X, 2.0) - 2.0 * np.sign(X), X)
    c = conics.numpy().astype(np.float64)
    q = c[:, None, 0] * X[..., 0] ** 2 + 2 * c[:, None, 1] * X[..., 0] * X[..., 1] + c[:, None, 2] * X[..., 1] ** 2
    live = -0.5 * q >= -104.0
    assert live.any()
    assert not np.any(live & (np.abs(X[..., 1]) > e[:, None]))


def _strip_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import diff_gaussian_sampling.distributed as dd
        from oracle_stub import OracleC
        dd._C = OracleC()
        means, values, covs, conics, samples, w = _spatial_problem()
        order = torch.argsort(samples[:, 1])
        shard = torch.tensor_split(order, world)[rank].sort().values
        m, v, c = (t.clone().requires_grad_(True) for t in (means, values, conics))
        sampler = dd.SpatialShardedGaussianSampler()
        sampler.preprocess(m, v, covs, c, samples[shard])
        moved = samples[shard].clone()
        if rank == 1:  # only this rank's points leave its strip
            moved[:, 1] -= 0.05
        try:
            sampler.preprocess(m, v, covs, c, moved)
            raised = False
        except ValueError:
            raised = True
        # a collective after the call: a rank that had not raised would be the only one here
        flag = torch.tensor([int(raised)])
        dist.all_reduce(flag)
        np.savez(os.path.join(outdir, f"strip{rank}.npz"), raised=raised, total=int(flag))
    finally:
        dist.destroy_process_group()


def test_spatial_strip_violation_raises_on_every_rank(tmp_path):
    """A later preprocess whose points leave one rank's strip raises ValueError on EVERY rank
    (the check is folded into the grid all-reduce), so no rank waits alone in the backward's
    all-to-all."""
    world = 2
    mp.spawn(_strip_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        z = np.load(tmp_path / f"strip{r}.npz")
        assert bool(z["raised"]) and int(z["total"]) == world

"""Query-point sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Each rank holds all P Gaussians (replicated) and its own shard of the query points.  The
reference derives the tile grid from the samples it is given (sample_points.cu:70-74), so a
shard must use the GLOBAL grid -- the min/max over all shards -- or its tile membership, and
therefore its results, would differ from the single-GPU run.  `global_tile_grid` obtains it
with two tiny all-reduces (MIN and MAX of D floats) and then applies the reference formula.

The forward needs no communication (a query point's value depends only on the Gaussians);
the backward's per-Gaussian gradients are partial sums over each rank's points.

* ShardedGaussianSampler: any split of the points; ONE all-reduce of the packed
  [dmeans | dvalues | dconics] buffer (P (D + C + S) floats: 24 MB at 1M Gaussians, C = 1).
* SpatialShardedGaussianSampler: ranks own spatial strips of the points.  A
  Gaussian's partial gradient can be non-zero only on the ranks whose points lie within its
  exact-zero cut (X^T A X <= 210, the binning's culling bound; with the torus images 2k), so
  the sum needs only those ranks: SupportExchange sends each such row to the Gaussian's owner
  (an all-to-all whose splits every rank derives from the replicated means and conics, no
  count exchange) and returns the sums to the contributing ranks.  With strips, only the
  Gaussians near a strip boundary travel (~1 MB per rank at config 4 against 24 MB).
"""
import math

import torch
import torch.distributed as dist

from . import _C, call_debug

_FWD = {"gaussian": "sample_gaussians", "derivative": "sample_gaussians_derivative",
        "laplacian": "sample_gaussians_laplacian", "third": "sample_gaussians_third_derivative"}


def _world(group=None):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def global_tile_grid(samples, group=None):
    """(grid, offset) of the union of every rank's `samples` (reference formula, torch ops)."""
    mn = samples.min(0).values.clone()
    mx = samples.max(0).values.clone()
    if _world(group) > 1:
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    grid = torch.ceil((mx - mn + 1e-6) / 0.51).to(torch.int32)
    return [int(g) for g in grid.cpu()], [float(o) for o in mn.cpu()]


def allreduce_grads(grads, group=None):
    """Sums (dmeans, dvalues, dconics) over ranks with one collective on a packed buffer."""
    if _world(group) == 1:
        return grads
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    out, o = [], 0
    for g in grads:
        out.append(flat[o:o + g.numel()].view_as(g))
        o += g.numel()
    return tuple(out)


class _ShardedSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, function, group, means, values, conics, samples, num_rendered, binning,
                sample_binning, ranges, sample_ranges, debug):
        fwd = getattr(_C, _FWD[function])
        out = call_debug(fwd, debug, "shard_fw", means, values, conics, samples, num_rendered,
                         binning, sample_binning, ranges, sample_ranges, debug)
        ctx.function, ctx.group, ctx.debug, ctx.num_rendered = function, group, debug, num_rendered
        ctx.save_for_backward(means, values, conics, samples, binning, sample_binning, ranges,
                              sample_ranges)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        means, values, conics, samples, binning, sample_binning, ranges, sample_ranges = ctx.saved_tensors
        bwd = getattr(_C, _FWD[ctx.function] + "_backward")
        grads = call_debug(bwd, ctx.debug, "shard_bw", means, values, conics, samples,
                           ctx.num_rendered, grad_out.contiguous(), binning, sample_binning,
                           ranges, sample_ranges, ctx.debug)
        gm, gv, gc = allreduce_grads(grads, ctx.group)
        return (None, None, gm, gv, gc) + (None,) * 7


class ShardedGaussianSampler:
    """GaussianSampler over a process group: this rank's `samples` are its shard; gradients
    flowing back to (means, values, conics) are the sums over all shards."""

    def __init__(self, debug=False, group=None):
        self.debug = debug
        self.group = group

    def preprocess(self, means, values, covariances, conics, samples):
        grid, offset = global_tile_grid(samples, self.group)
        (self.num_rendered, self.binning_buffer, self.sample_binning_buffer, self.ranges,
         self.sample_ranges, self.radii) = call_debug(
            _C.preprocess_gaussians_bounded, self.debug, "shard_preprocess", means, values,
            covariances, conics, samples, grid, offset, self.debug)
        self.grid, self.offset = grid, offset
        self.means, self.values, self.conics, self.samples = means, values, conics, samples

    def _sample(self, function):
        return _ShardedSample.apply(function, self.group, self.means, self.values, self.conics,
                                    self.samples, self.num_rendered, self.binning_buffer,
                                    self.sample_binning_buffer, self.ranges, self.sample_ranges,
                                    self.debug)

    def sample_gaussians(self):
        return self._sample("gaussian")

    def sample_gaussians_derivative(self):
        return self._sample("derivative")

    def sample_gaussians_laplacian(self):
        return self._sample("laplacian")

    def sample_gaussians_third_derivative(self):
        return self._sample("third")


# ------------------------------------------------------------------------ spatial shards (f3)
Q_CUT = 210.0  # X^T A X above this gives expf(-q / 2) == +0 in fp32 (dgs_internal.h kQCut)


def support_halfwidth(means, conics):
    """Half-width along the sharding axis (y at D = 2, x at D = 1) of every Gaussian's
    exact-zero cut {X : X^T A X <= Q_CUT}: sqrt(Q_CUT * (A^-1)_axis).  inf for conics that are not
    positive definite (their pairs are bounded by no ellipse).  float64, widened by 1e-5."""
    D = means.shape[1]
    c = conics.detach().double()
    if D == 2:
        c0, c1, c2 = c[:, 0], c[:, 1], c[:, 2]
        det = c0 * c2 - c1 * c1
        pd = (c0 > 0) & (det > 0) & torch.isfinite(det) & torch.isfinite(c0) & torch.isfinite(c2)
        e = torch.sqrt(Q_CUT * c0 / torch.where(pd, det, torch.ones_like(det)))
    else:
        c0 = c[:, 0]
        pd = (c0 > 0) & torch.isfinite(c0)
        e = torch.sqrt(Q_CUT / torch.where(pd, c0, torch.ones_like(c0)))
    e = e * (1.0 + 1e-5) + 1e-6
    return torch.where(pd, e, torch.full_like(e, math.inf))


class SupportExchange:
    """Sparse sum of per-Gaussian partial gradients over the ranks that can touch them.

    `extents` [W, 2]: every rank's point range [lo, hi] along the sharding axis (all-gathered).
    Rank r's partial for Gaussian g can be non-zero only if some point of r lies within the
    cut of g or of one of its torus images m + 2k (forward.cu:149-157 wraps X with period 2):
    touch[g, r].  owner[g] = the rank whose range is nearest to the mean (first on ties).
    The sets are computed identically on every rank from replicated inputs, so the all-to-all
    splits need no exchange of counts."""

    def __init__(self, means, conics, extents, rank, group=None):
        D = means.shape[1]
        dev = means.device
        ext = extents.detach().double().cpu()
        W = ext.shape[0]
        self.rank, self.world, self.group = rank, W, group
        if means.is_cuda and W <= 32:
            # native (dgs_exchange_sets): bit r of mask[g] = rank r can touch g; owner[g]
            mask, owner = _C.exchange_sets(means.detach(), conics.detach(), [float(v) for v in ext.reshape(-1)])
            mask, owner = mask.long(), owner.long()
            touch_me = ((mask >> rank) & 1).bool()
            self._mask = mask
            self.touch = None
        else:  # host tensors (the CPU tests): a P x W matrix in torch ops
            y = means.detach()[:, D - 1].double()
            e = support_halfwidth(means, conics)
            lo, hi = ext[:, 0].to(dev), ext[:, 1].to(dev)
            span = float(ext[:, 1].max() - ext[:, 0].min()) if W else 0.0
            kmax = int(math.ceil(span / 2.0)) + 1
            touch = torch.zeros(y.numel(), W, dtype=torch.bool, device=dev)
            for k in range(-kmax, kmax + 1):
                a, b = y + 2.0 * k - e, y + 2.0 * k + e
                touch |= (a[:, None] <= hi[None, :]) & (b[:, None] >= lo[None, :])
            dist_r = torch.clamp(torch.maximum(lo[None, :] - y[:, None], y[:, None] - hi[None, :]), min=0.0)
            owner = torch.argmin(dist_r, dim=1)  # first minimum: deterministic
            touch_me = touch[:, rank]
            self._mask = None
            self.touch = touch
        self.owner = owner
        # rows this rank sends, grouped by owner (ascending id within a group), and the rows it
        # receives, grouped by source rank: two nonzero passes, one host read of the counts
        snd = torch.nonzero(touch_me & (owner != rank)).flatten()
        so = owner[snd]
        self.send_cat = snd[torch.argsort(so, stable=True)]
        mine = torch.nonzero(owner == rank).flatten()
        if self._mask is not None:
            tm = ((self._mask[mine][:, None] >> torch.arange(W, device=dev)) & 1).bool()
        else:
            tm = self.touch[mine].clone()
        tm[:, rank] = False
        rg = torch.nonzero(tm.t())  # (source rank, position in `mine`), rank-major
        self.recv_cat = mine[rg[:, 1]]
        counts = torch.stack([torch.bincount(so, minlength=W), torch.bincount(rg[:, 0], minlength=W)]).cpu()
        self.send_splits = [int(x) for x in counts[0]]
        self.recv_splits = [int(x) for x in counts[1]]
        self.send_idx = list(torch.split(self.send_cat, self.send_splits))
        self.recv_idx = list(torch.split(self.recv_cat, self.recv_splits))

    def touches(self, r):
        """Bool [P]: the Gaussians whose partial gradient can be non-zero on rank r."""
        if self.touch is not None:
            return self.touch[:, r]
        return ((self._mask >> r) & 1).bool()

    def rows_moved(self):
        """Gaussian rows this rank sends per step (each way)."""
        return sum(self.send_splits)

    def _a2a(self, out, inp, out_splits, in_splits):
        if inp.is_cuda and dist.get_backend(self.group) == "gloo":  # gloo: host staging
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def exchange(self, G):
        """G [P, F] float32, this rank's partial sums (modified in place): afterwards every row
        this rank can touch holds the sum over all ranks."""
        if self.world == 1:
            return G
        F = G.shape[1]
        # 1. partials to the owners, added in rank order (deterministic: no duplicates per add)
        send = G.index_select(0, self.send_cat).contiguous()
        recv = torch.empty((sum(self.recv_splits), F), dtype=G.dtype, device=G.device)
        self._a2a(recv, send, self.recv_splits, self.send_splits)
        o = 0
        for r in range(self.world):
            n = self.recv_splits[r]
            if n:
                G.index_add_(0, self.recv_idx[r], recv[o:o + n])
            o += n
        # 2. the owners' sums back to every contributing rank
        back = G.index_select(0, self.recv_cat).contiguous()
        got = torch.empty((sum(self.send_splits), F), dtype=G.dtype, device=G.device)
        self._a2a(got, back, self.send_splits, self.recv_splits)
        G.index_copy_(0, self.send_cat, got)
        return G


def shard_extents(samples, group=None):
    """[W, 2] point range [min, max] of every rank along the sharding axis (all-gather)."""
    D = samples.shape[1]
    ax = samples.detach()[:, D - 1]
    mine = torch.stack([ax.min(), ax.max()]) if ax.numel() else torch.tensor(
        [math.inf, -math.inf], device=samples.device)
    W = _world(group)
    if W == 1:
        return mine[None, :]
    out = [torch.empty_like(mine) for _ in range(W)]
    dist.all_gather(out, mine.contiguous(), group=group)
    return torch.stack(out)


def pack_grads(grads):
    """(dmeans [P,D], dvalues [P,C], dconics [P,S]) -> one [P, D + C + S] buffer."""
    return torch.cat([g.reshape(g.shape[0], -1) for g in grads], dim=1)


def unpack_grads(G, like):
    out, o = [], 0
    for g in like:
        k = g.reshape(g.shape[0], -1).shape[1]
        out.append(G[:, o:o + k].reshape(g.shape))
        o += k
    return tuple(out)


class _SpatialSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, function, xchg, means, values, conics, samples, num_rendered, binning,
                sample_binning, ranges, sample_ranges, debug):
        fwd = getattr(_C, _FWD[function])
        out = call_debug(fwd, debug, "spatial_fw", means, values, conics, samples, num_rendered,
                         binning, sample_binning, ranges, sample_ranges, debug)
        ctx.function, ctx.xchg, ctx.debug, ctx.num_rendered = function, xchg, debug, num_rendered
        ctx.save_for_backward(means, values, conics, samples, binning, sample_binning, ranges,
                              sample_ranges)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        means, values, conics, samples, binning, sample_binning, ranges, sample_ranges = ctx.saved_tensors
        bwd = getattr(_C, _FWD[ctx.function] + "_backward")
        grads = call_debug(bwd, ctx.debug, "spatial_bw", means, values, conics, samples,
                           ctx.num_rendered, grad_out.contiguous(), binning, sample_binning,
                           ranges, sample_ranges, ctx.debug)
        G = ctx.xchg.exchange(pack_grads(grads))
        gm, gv, gc = unpack_grads(G, grads)
        return (None, None, gm, gv, gc) + (None,) * 7


class SpatialShardedGaussianSampler(ShardedGaussianSampler):
    """ShardedGaussianSampler for ranks that own spatial strips of the query points (SURVEY 8f
    row f3): the same global grid and per-rank binning, and the gradients summed by
    SupportExchange instead of a dense all-reduce.  After backward, every Gaussian that can touch
    this rank's points carries the sum over all ranks; the other rows are this rank's partials,
    exactly zero (no point of this rank is within their cut)."""

    def preprocess(self, means, values, covariances, conics, samples):
        super().preprocess(means, values, covariances, conics, samples)
        rank = dist.get_rank(self.group) if _world(self.group) > 1 else 0
        self.xchg = SupportExchange(means, conics, shard_extents(samples, self.group), rank, self.group)

    def _sample(self, function):
        return _SpatialSample.apply(function, self.xchg, self.means, self.values, self.conics,
                                    self.samples, self.num_rendered, self.binning_buffer,
                                    self.sample_binning_buffer, self.ranges, self.sample_ranges,
                                    self.debug)

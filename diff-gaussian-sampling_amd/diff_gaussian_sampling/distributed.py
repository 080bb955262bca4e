"""Query-point sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Each rank holds all P Gaussians (replicated) and its own shard of the query points.  The
reference derives the tile grid from the samples it is given (sample_points.cu:70-74), so a
shard must use the GLOBAL grid -- the min/max over all shards -- or its tile membership, and
therefore its results, would differ from the single-GPU run.  `global_tile_grid` obtains it
with two tiny all-reduces (MIN and MAX of D floats) and then applies the reference formula.

The forward needs no communication (a query point's value depends only on the Gaussians);
the backward's per-Gaussian gradients are partial sums over each rank's points and are summed
with ONE all-reduce of the packed [dmeans | dvalues | dconics] buffer.
"""
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

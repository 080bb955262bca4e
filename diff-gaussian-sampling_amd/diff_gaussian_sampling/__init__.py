"""diff_gaussian_sampling -- MI355X-native drop-in for kr4b/diff-gaussian-sampling.

Same public surface as the reference package (diff_gaussian_sampling/__init__.py:1-317):
the functional entry points, `call_debug`, the autograd Functions and `GaussianSampler`,
with the same argument order, return arity and debug behaviour.  The compute is the HIP
library libdgs.so behind `diff_gaussian_sampling._C` (csrc/torch_ext.cpp); there is no CPU
fallback -- importing this package without the built extension raises ImportError.
"""
import torch

try:
    from . import _C
except ImportError as exc:  # pragma: no cover - exercised on an unbuilt tree
    raise ImportError(
        "diff_gaussian_sampling._C is not built; run `python diff-gaussian-sampling_amd/build.py` "
        "(hipcc, gfx950) first") from exc

__all__ = [
    "sample_gaussians", "sample_gaussians_derivative", "sample_gaussians_laplacian",
    "sample_gaussians_third_derivative", "aggregate_neighbors", "preprocess_gaussians",
    "preprocess_aggregate", "call_debug", "cpu_deep_copy_tuple", "GaussianSampler",
    "sample_gaussians_multi", "FUNCTIONS", "preprocess_gaussians_capturable", "capacity_from",
    "BinningStatusMonitor", "BinningOverflow",
]

# Function names of the fused entry point (codes of dgs_function, include/dgs.h).
FUNCTIONS = {"gaussian": 0, "derivative": 1, "laplacian": 2, "third": 3}


def cpu_deep_copy_tuple(input_tuple):
    """CPU clones of the tensor members of a tuple (py:17-19)."""
    return tuple(x.cpu().clone() if isinstance(x, torch.Tensor) else x for x in input_tuple)


# The first parameter is named `debug` in the reference but receives `means` (py:21-31).
def sample_gaussians(debug, *args):
    return _SampleGaussians.apply(debug, *args)


def sample_gaussians_derivative(debug, *args):
    return _SampleGaussiansDerivative.apply(debug, *args)


def sample_gaussians_laplacian(debug, *args):
    return _SampleGaussiansLaplacian.apply(debug, *args)


def sample_gaussians_third_derivative(debug, *args):
    return _SampleGaussiansThirdDerivative.apply(debug, *args)


def aggregate_neighbors(features, transform, queries, keys, frequencies, distance_transform,
                        indices, ranges, dists, densities, inv_total_densities, debug):
    return _AggregateNeighbors.apply(features, transform, queries, keys, frequencies,
                                     distance_transform, indices, ranges, dists, densities,
                                     inv_total_densities, debug)


def sample_gaussians_multi(functions, means, values, conics, samples, num_rendered,
                           binning_buffer, sample_binning_buffer, ranges, sample_ranges, debug):
    """Several sampling functions over one binning in one traversal of the pairs (not on the
    reference API).  `functions` is a sequence of names from FUNCTIONS
    ("gaussian", "derivative", "laplacian", "third"), each at most once; returns their
    outputs in that order, equal to the per-function calls within the parity tolerance.
    Gradients flow to (means, values, conics) as the sum over the returned outputs' losses.
    Several functions at D = 2, C = 1 share the traversal; otherwise the per-function kernels
    run in turn."""
    codes = tuple(FUNCTIONS[f] if isinstance(f, str) else int(f) for f in functions)
    return _SampleGaussiansMulti.apply(codes, means, values, conics, samples, num_rendered,
                                       binning_buffer, sample_binning_buffer, ranges,
                                       sample_ranges, debug)


def call_debug(func, debug, name, *args):
    """Runs func(*args); with debug, a CPU snapshot of the arguments is written to
    snapshot_<name>.dump when it raises, and the exception is re-raised (py:38-50)."""
    if not debug:
        return func(*args)
    snapshot = cpu_deep_copy_tuple(args)  # copied before the call can corrupt them
    try:
        return func(*args)
    except Exception:
        torch.save(snapshot, "snapshot_{}.dump".format(name))
        print("\nAn error occured in {}. Please forward snapshot_{}.dump for debugging.".format(name, name))
        raise


def warmup():
    """Loads every code object of the native library onto the current GPU (dgs_warmup): the
    one-time cost the first call of each kind would otherwise pay.  Optional; call once at
    start-up (after torch.cuda.set_device)."""
    _C.warmup()


def preprocess_gaussians(means, values, covariances, conics, samples, debug):
    """Tile binning (py:52-65).  Returns (num_rendered, binning_buffer, sample_binning_buffer,
    ranges, sample_ranges, radii)."""
    args = (means, values, covariances, conics, samples, debug)
    return call_debug(_C.preprocess_gaussians, debug, "preprocess", *args)


def preprocess_gaussians_capturable(means, values, covariances, conics, samples, grid, offset, capacity,
                                    debug=False, status=None, samples_binned=None):
    """The graph-capturable binning (not on the reference API): no host
    synchronisation, so a training step -- re-binning after the optimizer moved the means, then the
    sample calls and the backward -- can be captured whole with torch.cuda.graph and replayed.

    grid / offset: the tile grid of the samples (sample_points.cu:70-74; e.g. `_C.tile_grid(samples)`
    or a first eager binning's), fixed for the captured step.  capacity = [E, Es, R]: list sizes,
    e.g. `capacity_from(binning_buffer, sample_binning_buffer)` of an eager binning.  Returns
    (num_rendered, binning_buffer, sample_binning_buffer, ranges, sample_ranges, radii, status)
    with num_rendered (int64[1]) and status (int32[1]) ON THE DEVICE.  status != 0: the
    capacities were too small (bits 1, 2, 4) or the samples' grid changed (bit 8); the step's
    outputs are then invalid (zeros) -- re-bin eagerly and re-capture with larger capacities.
    status: None (a fresh word, overwritten per call) or a caller's int32[1] device tensor the
    binning ORs its bits into (sticky across replays: BinningStatusMonitor.status).
    samples_binned: None, or the sample_binning_buffer of an eager binning of these samples (on
    this grid).  The captured binning then copies that binning's sample side at every replay
    instead of sorting the samples again (~0.15 ms at 2M points); the caller guarantees that the
    samples hold the same values at every replay (fixed collocation points) and keeps the buffer
    alive as long as the graph.  Status bit 8 is then not computed.
    The sample calls take num_rendered only for signature parity (pass any int)."""
    args = (means, values, covariances, conics, samples, [int(g) for g in grid], [float(o) for o in offset],
            [int(c) for c in capacity], debug, status, samples_binned)
    return call_debug(_C.preprocess_gaussians_capturable, debug, "preprocess_capturable", *args)


class BinningOverflow(RuntimeError):
    """A captured step's capturable binning reported a non-zero status (BinningStatusMonitor)."""


class BinningStatusMonitor:
    """Watches the sticky status of a captured PIGS step without a host sync inside the step.

    `status` (int32[1], allocated here, outside any capture) is passed to
    preprocess_gaussians_capturable(..., status=monitor.status), which ORs every replay's overflow
    bits into it.  `record()` goes INSIDE the captured step, after the binning: an async copy of
    the word into pinned host memory (a graph node).  `check()` goes after each `graph.replay()`:
    it waits for the PREVIOUS replay only (the GPU keeps running the one just launched) and raises
    BinningOverflow when that replay -- or any before it -- overflowed.  A step whose binning
    overflowed has zero outputs and gradients (dgs.h), so the loop learns of it one step later at
    most; `reset()` clears the word after an eager re-binning and re-capture."""

    def __init__(self, device=None):
        device = torch.device("cuda") if device is None else torch.device(device)
        self.status = torch.zeros(1, dtype=torch.int32, device=device)
        self._host = torch.zeros(1, dtype=torch.int32).pin_memory()
        self._prev = None
        self.replays = 0

    def record(self):
        """Inside the captured step (after the binning): the status word -> pinned memory."""
        self._host.copy_(self.status, non_blocking=True)

    def check(self):
        """After each replay: raises BinningOverflow if an earlier replay's binning overflowed."""
        prev, self._prev = self._prev, torch.cuda.Event()
        self._prev.record()
        self.replays += 1
        if prev is not None:
            prev.synchronize()  # (the previous replay; the current one keeps the GPU busy)
            st = int(self._host[0])
            if st != 0:
                raise BinningOverflow(f"capturable binning status {st} by replay {self.replays - 1}: "
                                      "re-bin eagerly, widen the capacities and re-capture")

    def reset(self):
        """Clears the sticky word (after an eager re-binning and re-capture)."""
        torch.cuda.synchronize(self.status.device)
        self.status.zero_()
        self._host.zero_()
        self._prev = None


def capacity_from(binning_buffer, sample_binning_buffer, slack=0.125):
    """[E, Es, R] of an eager binning (dgs_binning_info) widened by `slack`: capacities for
    preprocess_gaussians_capturable."""
    R, E, _, _, _, Es = _C.binning_info(binning_buffer, sample_binning_buffer)
    grow = lambda x: int(x + x * slack + 1024)  # noqa: E731
    return [grow(E), grow(Es), grow(R)]


def preprocess_aggregate(means, conics, radii, debug):
    """Neighbour lists for aggregate_neighbors (py:67-77)."""
    args = (means, conics, radii, debug)
    return call_debug(_C.preprocess_aggregate, debug, "preprocess_agg", *args)


def call_forward(ctx, func, name, *args):
    (means, values, conics, samples, num_rendered, binning_buffer, sample_binning_buffer,
     ranges, sample_ranges, debug) = args
    out = call_debug(func, debug, name, *args)
    ctx.debug = debug
    ctx.num_rendered = num_rendered
    ctx.save_for_backward(means, values, conics, samples, binning_buffer, sample_binning_buffer,
                          ranges, sample_ranges)
    return out


def call_backward(ctx, func, grad_out, name):
    (means, values, conics, samples, binning_buffer, sample_binning_buffer, ranges,
     sample_ranges) = ctx.saved_tensors
    args = (means, values, conics, samples, ctx.num_rendered, grad_out, binning_buffer,
            sample_binning_buffer, ranges, sample_ranges, ctx.debug)
    grad_means, grad_values, grad_conics = call_debug(func, ctx.debug, name, *args)
    # gradients for (means, values, conics); None for the remaining inputs (py:114-126)
    return (grad_means, grad_values, grad_conics) + (None,) * 8


class _SampleGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *args):
        return call_forward(ctx, _C.sample_gaussians, "fw", *args)

    @staticmethod
    def backward(ctx, grad_out):
        return call_backward(ctx, _C.sample_gaussians_backward, grad_out, "bw")


class _SampleGaussiansDerivative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *args):
        return call_forward(ctx, _C.sample_gaussians_derivative, "der_fw", *args)

    @staticmethod
    def backward(ctx, grad_out):
        return call_backward(ctx, _C.sample_gaussians_derivative_backward, grad_out, "der_bw")


class _SampleGaussiansLaplacian(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *args):
        return call_forward(ctx, _C.sample_gaussians_laplacian, "lap_fw", *args)

    @staticmethod
    def backward(ctx, grad_out):
        return call_backward(ctx, _C.sample_gaussians_laplacian_backward, grad_out, "lap_bw")


class _SampleGaussiansMulti(torch.autograd.Function):
    @staticmethod
    def forward(ctx, codes, means, values, conics, samples, num_rendered, binning_buffer,
                sample_binning_buffer, ranges, sample_ranges, debug):
        outs = call_debug(_C.sample_gaussians_multi, debug, "multi_fw", list(codes), means, values,
                          conics, samples, binning_buffer, sample_binning_buffer, debug)
        ctx.codes, ctx.debug = codes, debug
        ctx.save_for_backward(means, values, conics, samples, binning_buffer, sample_binning_buffer)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        means, values, conics, samples, binning_buffer, sample_binning_buffer = ctx.saved_tensors
        live = [(c, g.contiguous()) for c, g in zip(ctx.codes, grads) if g is not None]
        if not live:
            return (None,) * 11
        gm, gv, gc = call_debug(_C.sample_gaussians_multi_backward, ctx.debug, "multi_bw",
                                [c for c, _ in live], means, values, conics, samples,
                                [g for _, g in live], binning_buffer, sample_binning_buffer, ctx.debug)
        return (None, gm, gv, gc) + (None,) * 7


class _SampleGaussiansThirdDerivative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *args):
        return call_forward(ctx, _C.sample_gaussians_third_derivative, "3_fw", *args)

    @staticmethod
    def backward(ctx, grad_out):
        return call_backward(ctx, _C.sample_gaussians_third_derivative_backward, grad_out, "3_bw")


class _AggregateNeighbors(torch.autograd.Function):
    """py:165-212: tensors are kept as ctx attributes, as in the reference."""

    @staticmethod
    def forward(ctx, features, transform, queries, keys, frequencies, distance_transform,
                indices, ranges, dists, densities, inv_total_densities, debug):
        ctx.features, ctx.transform, ctx.queries, ctx.keys = features, transform, queries, keys
        ctx.frequencies, ctx.distance_transform = frequencies, distance_transform
        ctx.indices, ctx.ranges, ctx.dists, ctx.densities = indices, ranges, dists, densities
        ctx.inv_total_densities, ctx.debug = inv_total_densities, debug
        args = (features, transform, queries, keys, frequencies, distance_transform, indices,
                ranges, dists, densities, inv_total_densities, debug)
        weights, embeddings, factors, neighbor_features = call_debug(
            _C.aggregate_neighbors, debug, "aggregate", *args)
        if torch.isnan(neighbor_features.mean()):
            # The reference prints conics[i] here, a name undefined in that scope (py:188);
            # the diagnostic is kept without it.
            for i in range(neighbor_features.shape[0]):
                if torch.isnan(neighbor_features[i].mean()):
                    print(i, neighbor_features[i])
        ctx.weights, ctx.embeddings, ctx.factors = weights, embeddings, factors
        return neighbor_features

    @staticmethod
    def backward(ctx, grad_out):
        grads = call_debug(
            _C.aggregate_neighbors_backward, ctx.debug, "aggregate_bw",
            ctx.features, ctx.transform, ctx.queries, ctx.keys, ctx.frequencies,
            ctx.distance_transform, ctx.indices, ctx.ranges, ctx.dists, ctx.densities,
            ctx.weights, ctx.embeddings, ctx.factors, ctx.inv_total_densities, grad_out, ctx.debug)
        return tuple(grads) + (None,) * 6


class GaussianSampler:
    """Per-step state holder (py:214-317): preprocess once, then sample/aggregate."""

    def __init__(self, debug):
        self.debug = debug

    def preprocess(self, means, values, covariances, conics, samples):
        (self.num_rendered, self.binning_buffer, self.sample_binning_buffer, self.ranges,
         self.sample_ranges, self.radii) = preprocess_gaussians(
            means, values, covariances, conics, samples, self.debug)
        self.means, self.values, self.conics, self.samples = means, values, conics, samples

    def _args(self):
        return (self.means, self.values, self.conics, self.samples, self.num_rendered,
                self.binning_buffer, self.sample_binning_buffer, self.ranges,
                self.sample_ranges, self.debug)

    def sample_gaussians(self):
        return sample_gaussians(*self._args())

    def sample_gaussians_derivative(self):
        return sample_gaussians_derivative(*self._args())

    def sample_gaussians_laplacian(self):
        return sample_gaussians_laplacian(*self._args())

    def sample_gaussians_third_derivative(self):
        return sample_gaussians_third_derivative(*self._args())

    def sample_gaussians_multi(self, *functions):
        """Outputs of several functions ("gaussian", "derivative", "laplacian", "third") in
        one traversal of the binned pairs (see sample_gaussians_multi)."""
        return sample_gaussians_multi(functions, *self._args())

    def preprocess_aggregate(self):
        (self.indices, self.ranges_agg, self.dists, self.densities,
         self.inv_total_densities) = preprocess_aggregate(self.means, self.conics, self.radii,
                                                          self.debug)
        # the reference overwrites self.ranges with the aggregate CSR ranges (py:294-298)
        self.ranges = self.ranges_agg

    def aggregate_neighbors(self, features, transform, queries, keys, frequencies, distance_transform):
        return aggregate_neighbors(features, transform, queries, keys, frequencies,
                                   distance_transform, self.indices, self.ranges, self.dists,
                                   self.densities, self.inv_total_densities, self.debug)

"""Host-logic ("plumbing") scenario for the Python layer, run against a recording stub `_C`.

TEST INFRASTRUCTURE ONLY.  tests/golden/make_golden.py runs `scenario` against the
reference's own Python layer (diff_gaussian_sampling/__init__.py, compiled from its source
text with this stub as its `_C`) and stores the trace in tests/golden/api_trace.json;
tests/test_plumbing.py runs the same scenario against this repository's package and requires
an identical trace.  The trace records, for every `_C` call, the function name and what each
argument was (which input tensor, which earlier `_C` output, or the scalar), plus which `_C`
output each .grad ended up being -- i.e. argument order, ctx save/restore, return arity and
the GaussianSampler state flow, including the reference's quirks (first parameter named
`debug`, `preprocess_aggregate` overwriting `ranges`).
"""
import inspect
import os
import tempfile

import torch

PUBLIC = ["sample_gaussians", "sample_gaussians_derivative", "sample_gaussians_laplacian",
          "sample_gaussians_third_derivative", "aggregate_neighbors", "preprocess_gaussians",
          "preprocess_aggregate", "call_debug", "cpu_deep_copy_tuple"]
SAMPLER_METHODS = ["__init__", "preprocess", "sample_gaussians", "sample_gaussians_derivative",
                   "sample_gaussians_laplacian", "sample_gaussians_third_derivative",
                   "preprocess_aggregate", "aggregate_neighbors"]
FWD = ["sample_gaussians", "sample_gaussians_derivative", "sample_gaussians_laplacian",
       "sample_gaussians_third_derivative"]


class RecordingC:
    """Stands in for the `_C` extension: records calls, returns tagged dummy tensors."""

    def __init__(self):
        self.trace = []
        self.tags = {}
        self.keep = []  # tagged tensors stay alive so that their id() is never reused
        self.fail_next = False

    def tag(self, t, name):
        self.tags[id(t)] = name
        self.keep.append(t)
        return t

    def describe(self, a):
        if isinstance(a, torch.Tensor):
            if id(a) in self.tags:
                return self.tags[id(a)]
            return "tensor%s:%s" % (list(a.shape), str(a.dtype).replace("torch.", ""))
        return repr(a)

    def _record(self, name, args):
        self.trace.append([name] + [self.describe(a) for a in args])
        if self.fail_next:
            self.fail_next = False
            raise RuntimeError("injected failure in " + name)

    def _out(self, name, i, t):
        return self.tag(t, "%s#%d" % (name, i))

    # --- the 12 entry points of ext.cpp:20-31
    def preprocess_gaussians(self, means, values, covariances, conics, samples, debug):
        self._record("preprocess_gaussians", (means, values, covariances, conics, samples, debug))
        P = means.shape[0]
        bufs = [self._out("preprocess_gaussians", i, torch.zeros(16, dtype=torch.uint8)) for i in range(1, 5)]
        return (7,) + tuple(bufs) + (self._out("preprocess_gaussians", 5, torch.ones(P)),)

    def _fwd(self, name, k, means, values, conics, samples, R, gb, sb, rg, srg, debug):
        self._record(name, (means, values, conics, samples, R, gb, sb, rg, srg, debug))
        N, D, C = samples.shape[0], means.shape[1], values.shape[1]
        return self._out(name, 0, torch.zeros((N,) + (D,) * k + (C,)))

    def _bwd(self, name, means, values, conics, samples, R, dL, gb, sb, rg, srg, debug):
        self._record(name, (means, values, conics, samples, R, dL, gb, sb, rg, srg, debug))
        return tuple(self._grad(t, i) for i, t in enumerate((means, values, conics)))

    def _grad(self, like, i):
        """A gradient output filled with a constant unique to (call, position)."""
        return torch.full_like(like, float(100 * len(self.trace) + i + 1))

    def sample_gaussians(self, *a):
        return self._fwd("sample_gaussians", 0, *a)

    def sample_gaussians_derivative(self, *a):
        return self._fwd("sample_gaussians_derivative", 1, *a)

    def sample_gaussians_laplacian(self, *a):
        return self._fwd("sample_gaussians_laplacian", 2, *a)

    def sample_gaussians_third_derivative(self, *a):
        return self._fwd("sample_gaussians_third_derivative", 3, *a)

    def sample_gaussians_backward(self, *a):
        return self._bwd("sample_gaussians_backward", *a)

    def sample_gaussians_derivative_backward(self, *a):
        return self._bwd("sample_gaussians_derivative_backward", *a)

    def sample_gaussians_laplacian_backward(self, *a):
        return self._bwd("sample_gaussians_laplacian_backward", *a)

    def sample_gaussians_third_derivative_backward(self, *a):
        return self._bwd("sample_gaussians_third_derivative_backward", *a)

    def preprocess_aggregate(self, means, conics, radii, debug):
        self._record("preprocess_aggregate", (means, conics, radii, debug))
        P, D = means.shape
        n = 3 * P
        outs = (torch.zeros(n, dtype=torch.int64), torch.arange(1, P + 1, dtype=torch.int64) * 3,
                torch.zeros(n, D), torch.ones(n), torch.ones(P))
        return tuple(self._out("preprocess_aggregate", i, t) for i, t in enumerate(outs))

    def aggregate_neighbors(self, features, transform, queries, keys, frequencies,
                            distance_transform, indices, ranges, dists, densities, inv_total, debug):
        self._record("aggregate_neighbors", (features, transform, queries, keys, frequencies,
                                             distance_transform, indices, ranges, dists,
                                             densities, inv_total, debug))
        n = indices.shape[0]
        outs = (torch.ones(n), torch.ones(n), torch.ones(n), torch.zeros_like(features))
        return tuple(self._out("aggregate_neighbors", i, t) for i, t in enumerate(outs))

    def aggregate_neighbors_backward(self, *a):
        self._record("aggregate_neighbors_backward", a)
        return tuple(self._grad(t, i) for i, t in enumerate(a[:6]))


def _signature(obj):
    try:
        return str(inspect.signature(obj))
    except (TypeError, ValueError):
        return None


def scenario(pkg, stub):
    """Drives the package through every public path; returns the JSON-able trace."""
    res = {"public": {n: _signature(getattr(pkg, n, None)) for n in PUBLIC},
           "sampler": {m: _signature(getattr(pkg.GaussianSampler, m, None)) for m in SAMPLER_METHODS}}
    P, N, C = 5, 9, 2
    means = stub.tag(torch.rand(P, 2).requires_grad_(True), "means")
    values = stub.tag(torch.rand(P, C).requires_grad_(True), "values")
    covs = stub.tag(torch.rand(P, 3), "covariances")
    conics = stub.tag(torch.rand(P, 3).requires_grad_(True), "conics")
    samples = stub.tag(torch.rand(N, 2), "samples")
    grads = []

    def grab(*ts):
        g = [None if t.grad is None else [list(t.grad.shape)] + sorted(set(t.grad.reshape(-1).tolist()))
             for t in ts]
        for t in ts:
            t.grad = None
        return g

    s = pkg.GaussianSampler(False)
    s.preprocess(means, values, covs, conics, samples)
    for name in FWD:
        out = getattr(s, name)()
        res.setdefault("out_shapes", []).append(list(out.shape))
        out.backward(torch.ones_like(out))
        grads.append(grab(means, values, conics))
    # functional path, first parameter named `debug` but receiving means (py:21-31)
    out = pkg.sample_gaussians(means, values, conics, samples, s.num_rendered, s.binning_buffer,
                               s.sample_binning_buffer, s.ranges, s.sample_ranges, False)
    out.sum().backward()
    grads.append(grab(means, values, conics))
    # aggregate path; preprocess_aggregate overwrites the sampler's ranges (py:294-298)
    s.preprocess_aggregate()
    L, K, F = 4, 3, 2
    feats = stub.tag(torch.rand(P, L).requires_grad_(True), "features")
    transform = stub.tag(torch.rand(L, L).requires_grad_(True), "transform")
    queries = stub.tag(torch.rand(P, K).requires_grad_(True), "queries")
    keys = stub.tag(torch.rand(P, K).requires_grad_(True), "keys")
    freqs = stub.tag(torch.rand(F).requires_grad_(True), "frequencies")
    dt = stub.tag(torch.rand(2 * (2 * F * 2 + 1)).requires_grad_(True), "distance_transform")
    out = s.aggregate_neighbors(feats, transform, queries, keys, freqs, dt)
    out.sum().backward()
    grads.append(grab(feats, transform, queries, keys, freqs, dt))
    out = s.sample_gaussians()  # now with the aggregate ranges, as the reference does
    out.sum().backward()
    grads.append(grab(means, values, conics))
    # debug mode: snapshot written on failure, exception re-raised (py:38-50)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            d = pkg.GaussianSampler(True)
            stub.fail_next = True
            try:
                d.preprocess(means, values, covs, conics, samples)
                res["debug_raised"] = False
            except RuntimeError:
                res["debug_raised"] = True
            res["debug_files"] = sorted(os.listdir(tmp))
            snap = torch.load(os.path.join(tmp, "snapshot_preprocess.dump"), weights_only=True)
            res["debug_snapshot"] = [stub.describe(x) if not isinstance(x, torch.Tensor)
                                     else "tensor%s" % list(x.shape) for x in snap]
        finally:
            os.chdir(cwd)
    res["trace"] = stub.trace
    res["grads"] = grads
    return res

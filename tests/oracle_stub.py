"""An oracle-backed stand-in for `diff_gaussian_sampling._C` on CPU tensors.

TEST INFRASTRUCTURE ONLY: lets the host-side logic (autograd Functions, the sharded sampler
and its collectives) run on a machine without a GPU, against the oracle.  The product never
sees this module; tests patch it in explicitly.
"""
import numpy as np
import torch

from oracle import oracle as orc

_FWD = {"sample_gaussians": "gaussian", "sample_gaussians_derivative": "derivative",
        "sample_gaussians_laplacian": "laplacian", "sample_gaussians_third_derivative": "third"}


class OracleC:
    def __init__(self):
        self._bins = {}

    def _np(self, t):
        return t.detach().cpu().numpy()

    def preprocess_gaussians_bounded(self, means, values, covariances, conics, samples, grid,
                                     offset, debug):
        ob = orc.OracleBins(self._np(means), self._np(covariances), self._np(samples), grid, offset)
        gb = torch.zeros(16, dtype=torch.uint8)
        sb = torch.zeros(16, dtype=torch.uint8)
        self._bins[gb.data_ptr()] = (ob, gb)
        rg, srg = ob.ranges()
        pad = np.zeros(2, np.uint32)
        as_bytes = lambda r: torch.from_numpy(np.concatenate([r.reshape(-1), pad]).view(np.uint8).copy())
        return ob.num_rendered, gb, sb, as_bytes(rg), as_bytes(srg), torch.from_numpy(ob.radii.copy())

    def preprocess_gaussians_sharded(self, means, values, covariances, conics, samples, grid, offset,
                                     present, sample_area, debug):
        """`present` == 0 rows are left out as a det == 0 Gaussian is (zeroed covariance);
        `sample_area` only sizes the GPU's fine cells, so the oracle ignores it."""
        covs = covariances.detach().clone()
        if present is not None:
            covs[~present.bool().cpu()] = 0.0
        return self.preprocess_gaussians_bounded(means, values, covs, conics, samples, grid, offset, debug)

    def preprocess_gaussians(self, means, values, covariances, conics, samples, debug):
        return self.preprocess_gaussians_bounded(means, values, covariances, conics, samples,
                                                 None, None, debug)

    def __getattr__(self, name):
        base = name[:-len("_backward")] if name.endswith("_backward") else name
        if base not in _FWD:
            raise AttributeError(name)
        fn = _FWD[base]
        if name.endswith("_backward"):
            def bwd(means, values, conics, samples, R, dL, gb, sb, rg, srg, debug):
                ob = self._bins[gb.data_ptr()][0]
                grads = ob.backward(fn, self._np(values), self._np(conics), self._np(dL),
                                    means=self._np(means), samples=self._np(samples))
                return tuple(torch.from_numpy(g) for g in grads)
            return bwd

        def fwd(means, values, conics, samples, R, gb, sb, rg, srg, debug):
            ob = self._bins[gb.data_ptr()][0]
            out = ob.forward(fn, self._np(values), self._np(conics), means=self._np(means),
                             samples=self._np(samples))
            N, D = samples.shape
            return torch.from_numpy(out).reshape((N,) + (D,) * orc.FUNCTIONS[fn] + (values.shape[1],))
        return fwd

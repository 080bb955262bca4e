"""D = 3 Gaussian fields -- beyond the reference.

The reference stops at D = 2: its device functions have no D = 3 branch
(cuda_sampler/forward.cu:164-275, backward.cu:108-416), its radius is 0 there
(forward.cu:52-61) and its sample keys are uninitialised (sampler_impl.cu:177-182), so
`GaussianSampler` renders nothing at D = 3 and this package's reference API rejects it.
`VolumeSampler` carries the reference's per-pair arithmetic to three dimensions
(include/dgs_volume.h): the per-axis torus wrap of forward.cu:149-157, the
power with conics packed [c00 c01 c02 c11 c12 c22], and the four functions in index form
(gaussian v G, derivative v G a, laplacian v G (a a^T - A), third
v G (A_ij a_k + A_ik a_j + A_jk a_i - a_i a_j a_k)), summed over every Gaussian (no tile
truncation; only pairs whose contribution is exactly 0 in fp32 are skipped).

Outputs are [N, 3, ..., 3, C] (3^k components for the k-th derivative), gradients flow to
means [P, 3], values [P, C] and conics [P, 6] through autograd, as in the reference's
Functions (diff_gaussian_sampling/__init__.py:80-160 of the reference).
"""
import torch

from . import _C, call_debug

FUNCTION_CODES = {"gaussian": 0, "derivative": 1, "laplacian": 2, "third": 3}


def preprocess_volume(means, conics, samples, debug=False):
    """Cell binning of a D = 3 field; returns the opaque uint8 buffer."""
    return call_debug(_C.volume_preprocess, debug, "vol_preprocess", means, conics, samples, debug)


class _SampleVolume(torch.autograd.Function):
    @staticmethod
    def forward(ctx, function, means, values, conics, samples, binning, debug):
        out = call_debug(_C.volume_forward, debug, "vol_fw", function, means, values, conics, samples,
                         binning, debug)
        ctx.function, ctx.debug = function, debug
        ctx.save_for_backward(means, values, conics, samples, binning)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        means, values, conics, samples, binning = ctx.saved_tensors
        gm, gv, gc = call_debug(_C.volume_backward, ctx.debug, "vol_bw", ctx.function, means, values,
                                conics, samples, binning, grad_out.contiguous(), ctx.debug)
        return None, gm, gv, gc, None, None, None


def sample_volume(function, means, values, conics, samples, binning, debug=False):
    """One of the four functions ("gaussian", "derivative", "laplacian", "third" or 0..3) of a
    D = 3 field at `samples`, through the binning of preprocess_volume."""
    code = FUNCTION_CODES[function] if isinstance(function, str) else int(function)
    return _SampleVolume.apply(code, means, values, conics, samples, binning, debug)


class VolumeSampler:
    """GaussianSampler's shape for D = 3: preprocess once per (means, conics, samples), then
    sample any of the four functions.  covariances are accepted for signature parity with
    GaussianSampler.preprocess (reference py:214-230) and unused, as the cut is derived from
    the conics.  The tensors are kept by reference: when means, conics or samples were changed
    in place since preprocess (an optimizer step), the next sampling call re-bins them first.
    (The functional `sample_volume` with a stale binning writes NaN instead: every call compares
    its tensors with the binned ones on the device, include/dgs_volume.h.)"""

    def __init__(self, debug=False):
        self.debug = debug

    def preprocess(self, means, values, covariances, conics, samples):
        self.binning = preprocess_volume(means, conics, samples, self.debug)
        self.means, self.values, self.conics, self.samples = means, values, conics, samples
        self._versions = self._now()
        self._fresh = True

    def _now(self):
        ts = (self.means, self.conics, self.samples)
        if any(t.is_inference() for t in ts):  # no version counter: unknown
            return None
        return tuple(t._version for t in ts)

    def _run(self, code):
        now = self._now()
        # changed in place since the binning (or, for inference tensors, possibly changed: every
        # call after the first re-bins) -> re-bin
        if (now is None and not self._fresh) or now != self._versions:
            self.binning = preprocess_volume(self.means, self.conics, self.samples, self.debug)
            self._versions = self._now()
        self._fresh = False
        return sample_volume(code, self.means, self.values, self.conics, self.samples, self.binning,
                             self.debug)

    def sample_gaussians(self):
        return self._run(0)

    def sample_gaussians_derivative(self):
        return self._run(1)

    def sample_gaussians_laplacian(self):
        return self._run(2)

    def sample_gaussians_third_derivative(self):
        return self._run(3)

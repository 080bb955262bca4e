"""Shared helpers for the parity tests (GPU path vs the CPU oracle)."""
import numpy as np
import torch

FUNCS = ["gaussian", "derivative", "laplacian", "third"]
FWD_NAME = {"gaussian": "sample_gaussians", "derivative": "sample_gaussians_derivative",
            "laplacian": "sample_gaussians_laplacian", "third": "sample_gaussians_third_derivative"}


def close(got, ref, rtol, atol_frac, what=""):
    """|got - ref| <= rtol * |ref| + atol_frac * max|ref| elementwise (tolerance of SURVEY 8c)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = float(np.max(np.abs(ref))) if ref.size else 0.0
    err = np.abs(got - ref)
    bound = rtol * np.abs(ref) + atol_frac * scale + 1e-30
    bad = err > bound
    if bad.any():
        i = np.unravel_index(np.argmax(err / bound), err.shape)
        raise AssertionError(
            f"{what}: {bad.sum()} / {bad.size} elements out of tolerance; worst at {i}: got {got[i]!r} "
            f"ref {ref[i]!r} (scale {scale:.3e}, rtol {rtol}, atol_frac {atol_frac})")


def gpu_run(C_mod, function, means, values, covs, conics, samples, dL=None, debug=False):
    """preprocess + forward (+ backward) through diff_gaussian_sampling._C on cuda:0."""
    dev = torch.device("cuda:0")
    m, v, cv, c, s = (t.to(dev) for t in (means, values, covs, conics, samples))
    R, gb, sb, rg, srg, radii = C_mod.preprocess_gaussians(m, v, cv, c, s, debug)
    out = getattr(C_mod, FWD_NAME[function])(m, v, c, s, R, gb, sb, rg, srg, debug)
    res = {"R": R, "radii": radii.cpu().numpy(), "ranges": rg.cpu().numpy(),
           "sample_ranges": srg.cpu().numpy(), "out": out.cpu().numpy(), "gb": gb, "sb": sb}
    if dL is not None:
        grads = getattr(C_mod, FWD_NAME[function] + "_backward")(
            m, v, c, s, R, dL.to(dev).reshape(out.shape), gb, sb, rg, srg, debug)
        res["grads"] = [g.cpu().numpy() for g in grads]
    return res


def ref_ranges_bytes(orc_bins):
    """The oracle's ranges in the reference's byte layout (uint2[T] + 8 zero bytes)."""
    r, s = orc_bins.ranges()
    pad = np.zeros(2, np.uint32)
    return (np.concatenate([r.reshape(-1), pad]).view(np.uint8),
            np.concatenate([s.reshape(-1), pad]).view(np.uint8))

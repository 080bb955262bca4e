"""Shared helpers for the parity tests (GPU path vs the CPU oracle)."""
import json
import os

import numpy as np
import torch

FUNCS = ["gaussian", "derivative", "laplacian", "third"]
FWD_NAME = {"gaussian": "sample_gaussians", "derivative": "sample_gaussians_derivative",
            "laplacian": "sample_gaussians_laplacian", "third": "sample_gaussians_third_derivative"}


def record_margin(what, margin, rtol, atol_frac, n):
    """Appends one JSON line per check to $DGS_MARGINS (tools/margins_summary.py folds them into
    profiles/rNN_margins.json): the margin is max |got - ref| / bound, < 1 passes."""
    path = os.environ.get("DGS_MARGINS")
    if not path:
        return
    test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" (")[0]
    with open(path, "a") as f:
        f.write(json.dumps({"test": test, "what": what, "margin": margin, "rtol": rtol,
                            "atol_frac": atol_frac, "n": n}) + "\n")


def close(got, ref, rtol, atol_frac, what=""):
    """|got - ref| <= rtol * |ref| + atol_frac * max|ref| elementwise.

    SURVEY 8c: forward rtol 1e-5 + atol 1e-6 max|ref|; backward (atomic, nondeterministic order in
    the reference) rtol 1e-5 + atol 1e-6 max|ref| -- the same bound, see ATOL_BWD in the tests."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = float(np.max(np.abs(ref))) if ref.size else 0.0
    err = np.abs(got - ref)
    bound = rtol * np.abs(ref) + atol_frac * scale + 1e-30
    record_margin(what, float(np.max(err / bound)) if err.size else 0.0, rtol, atol_frac, int(err.size))
    bad = err > bound
    if bad.any():
        i = np.unravel_index(np.argmax(err / bound), err.shape)
        raise AssertionError(
            f"{what}: {bad.sum()} / {bad.size} elements out of tolerance; worst at {i}: got {got[i]!r} "
            f"ref {ref[i]!r} (scale {scale:.3e}, rtol {rtol}, atol_frac {atol_frac})")


def margin_of(got, ref, rtol, atol_frac):
    """max |got - ref| / (rtol |ref| + atol_frac max|ref|) (< 1: within the tolerance)."""
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    if not ref.size:
        return 0.0
    b = rtol * np.abs(ref) + atol_frac * float(np.max(np.abs(ref))) + 1e-30
    return float(np.max(np.abs(got - ref) / b))


def close_grad(got, exact, literal, rtol, atol_frac, what=""):
    """A gradient against the oracle's exact sum of the reference's float per-pair terms
    (OracleBins.backward(exact=True)) at the given tolerance.  The reference adds those terms with
    float atomics in no fixed order; `literal` is one such order (the oracle's serial float sums),
    whose distance from the exact sum -- the reference's own run-to-run spread -- is recorded next
    to the GPU's (profiles/r04_margins.json) as the evidence for a case's stated bound."""
    record_margin(what + " [reference serial order vs exact]", margin_of(literal, exact, rtol, atol_frac), rtol,
                   atol_frac, int(np.size(exact)))
    close(got, exact, rtol, atol_frac, what)


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


# Thin Gaussians' stated bound (tests/test_gpu_parity.py module docstring): the GPU within
# THIN_SPREAD_FACTOR times the larger distance of the two FMA-contraction models of the reference
# (oracle "fmad" / "fmad_alt", i.e. nvcc's default --fmad=true) from the unfused model, per
# tensor, never tighter than the 8c bound.  The fast path's exponent (pre-scaled k, its own FMA
# order) is one more operation order of the same cancellation-amplified sum: profiles/
# r05_margins.json records it at 1-2.6x the models' spread on cases.thin_case.
THIN_SPREAD_FACTOR = 3.0


def model_spread(oracle, functions, means, values, covs, conics, samples, dLs, subset=None, rtol=1e-5, atol=1e-6):
    """Margins (units of the 8c bound) of the contraction models' forward outputs (per function)
    and exact-sum gradients (summed over `functions`) from the unfused model's, each recorded as
    "[reference <model> vs no-contract]"; returns {output name: the larger of the two models}."""
    refs = {}
    for model in ("nocontract", "fmad", "fmad_alt"):
        ob = oracle.OracleBins(np.asarray(means), np.asarray(covs), np.asarray(samples), model=model)
        outs, grads = {}, None
        for f, dL in zip(functions, dLs):
            o = ob.forward(f, np.asarray(values), np.asarray(conics), subset=subset)
            outs[f] = o if subset is None else o[subset]
            g = ob.backward(f, np.asarray(values), np.asarray(conics), np.asarray(dL), subset=subset, exact=True)
            grads = list(g) if grads is None else [a + b for a, b in zip(grads, g)]
        refs[model] = (outs, grads)
    worst = {}
    for model in ("fmad", "fmad_alt"):
        pairs = [(f"{f} forward", refs[model][0][f], refs["nocontract"][0][f]) for f in functions]
        pairs += list(zip(("dmeans", "dvalues", "dconics"), refs[model][1], refs["nocontract"][1]))
        for name, a, b in pairs:
            mg = margin_of(a, b, rtol, atol)
            record_margin(f"{name} [reference {model} vs no-contract]", mg, rtol, atol, int(np.size(b)))
            worst[name] = max(worst.get(name, 0.0), mg)
    return worst


def spread_scale(worst, factor=THIN_SPREAD_FACTOR):
    return {k: max(1.0, factor * v) for k, v in worst.items()}

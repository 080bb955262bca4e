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


def close(got, ref, rtol, atol_frac, what="", extra=None):
    """|got - ref| <= rtol * |ref| + atol_frac * max|ref| (+ extra) elementwise.

    SURVEY 8c: forward rtol 1e-5 + atol 1e-6 max|ref|; backward (atomic, nondeterministic order in
    the reference) rtol 1e-5 + atol 1e-6 max|ref| -- the same bound, see ATOL_BWD in the tests.
    extra: an additive per-element bound (the a-priori exponent-order bound of thin Gaussians,
    OracleBins.order_bound)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = float(np.max(np.abs(ref))) if ref.size else 0.0
    err = np.abs(got - ref)
    bound = rtol * np.abs(ref) + atol_frac * scale + 1e-30
    if extra is not None:
        bound = bound + np.asarray(extra, np.float64).reshape(bound.shape)
    record_margin(what, float(np.max(err / bound)) if err.size else 0.0, rtol, atol_frac, int(err.size))
    bad = err > bound
    if bad.any():
        i = np.unravel_index(np.argmax(err / bound), err.shape)
        raise AssertionError(
            f"{what}: {bad.sum()} / {bad.size} elements out of tolerance; worst at {i}: got {got[i]!r} "
            f"ref {ref[i]!r} (scale {scale:.3e}, rtol {rtol}, atol_frac {atol_frac})")


def margin_of(got, ref, rtol, atol_frac, extra=None):
    """max |got - ref| / (rtol |ref| + atol_frac max|ref| [+ extra]) (< 1: within the tolerance)."""
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    if not ref.size:
        return 0.0
    b = rtol * np.abs(ref) + atol_frac * float(np.max(np.abs(ref))) + 1e-30
    if extra is not None:
        b = b + np.asarray(extra, np.float64).reshape(-1)
    return float(np.max(np.abs(got - ref) / b))


def close_grad(got, exact, literal, rtol, atol_frac, what="", extra=None):
    """A gradient against the oracle's exact sum of the reference's float per-pair terms
    (OracleBins.backward(exact=True)) at the given tolerance.  The reference adds those terms with
    float atomics in no fixed order; `literal` is one such order (the oracle's serial float sums),
    whose distance from the exact sum -- the reference's own run-to-run spread -- is recorded next
    to the GPU's (profiles/r04_margins.json) as the evidence for a case's stated bound."""
    record_margin(what + " [reference serial order vs exact]", margin_of(literal, exact, rtol, atol_frac, extra), rtol,
                   atol_frac, int(np.size(exact)))
    close(got, exact, rtol, atol_frac, what, extra)


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


# Thin Gaussians' stated bound (tests/test_gpu_parity.py module docstring): the 8c
# bound PLUS the a-priori bound of the exponent's evaluation order, B = sum over an element's pairs
# of |term| (exp(gamma_6 M) - 1), M = 0.5|c0 X0^2| + |c1 X0 X1| + 0.5|c2 X1^2| (oracle.c
# orc_forward_bound / orc_backward_bound).  B depends only on the reference's expression
# (forward.cu:177) and the inputs -- no GPU result and no tunable factor went into it.  The
# reference's own contraction models (nvcc --fmad=true, oracle "fmad" / "fmad_alt") are checked
# against the same bound on the CPU (tests/test_contraction.py).


def model_distances(oracle, functions, means, values, covs, conics, samples, dLs, bounds, subset=None,
                    rtol=1e-5, atol=1e-6):
    """Records the contraction models' forward outputs (per function) and exact-sum gradients
    (summed over `functions`) against the unfused model's, in units of the plain 8c bound and of
    the stated one (8c + the a-priori bound `bounds` {output name: B}); returns the models'
    outputs {model: (outs {function: array}, grads [dm, dv, dc])} for the GPU's own distances."""
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
    for model in ("fmad", "fmad_alt"):
        pairs = [(f"{f} forward", refs[model][0][f], refs["nocontract"][0][f]) for f in functions]
        pairs += list(zip(("dmeans", "dvalues", "dconics"), refs[model][1], refs["nocontract"][1]))
        for name, a, b in pairs:
            record_margin(f"{name} [reference {model} vs no-contract, plain 8c bound]", margin_of(a, b, rtol, atol),
                          rtol, atol, int(np.size(b)))
            record_margin(f"{name} [reference {model} vs no-contract, 8c + a-priori bound]",
                          margin_of(a, b, rtol, atol, bounds.get(name)), rtol, atol, int(np.size(b)))
    return refs


def order_bounds(ob, functions, values, conics, dLs, subset=None):
    """{output name: the a-priori exponent-order bound} of a case (forward per function, the
    gradients summed over `functions`), from the unfused oracle bins `ob`."""
    out, grads = {}, None
    for f, dL in zip(functions, dLs):
        b = ob.order_bound(f, np.asarray(values), np.asarray(conics), subset=subset)
        out[f"{f} forward"] = b if subset is None else b[subset]
        g = ob.order_bound(f, np.asarray(values), np.asarray(conics), np.asarray(dL), subset=subset)
        grads = list(g) if grads is None else [a + c for a, c in zip(grads, g)]
    out.update(dict(zip(("dmeans", "dvalues", "dconics"), grads)))
    return out

"""Parity margins of neighbour aggregation: max over elements of |x - ref| / (RTOL |ref| + ATOL
max|ref|) at the north star's tolerances (forward 1e-5 / 1e-6, gradients 1e-5 / 1e-5; < 1
passes), for the GPU against the C oracle and against the oracle's exact-accumulation twin
(exact=True), and for the oracle itself against that twin (how much of the GPU-oracle gap is
the reference's own float summation).

    python tools/agg_errstat.py
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "diff-gaussian-sampling_amd")):
    sys.path.insert(0, p)
import diff_gaussian_sampling as dgs  # noqa: E402
from cases import AGG_FEATURES, agg_problem  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def margin(got, ref, rtol, atol):
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    if ref.size == 0:
        return 0.0
    b = rtol * np.abs(ref) + atol * np.abs(ref).max() + 1e-30
    return float((np.abs(got - ref) / b).max())


def case(**kw):
    means, conics, radii, fe = agg_problem(**kw)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    idx_r, rg_r, X_r, dn_r, inv_r = orc.agg_preprocess(means, conics, radii)
    idx, rg, X, dn, inv = dgs._C.preprocess_aggregate(cu(means), cu(conics), cu(radii), False)
    args = [fe[k] for k in AGG_FEATURES]
    w_r, e_r, f_r, out_r = orc.agg_forward(*args, idx_r, rg_r, X_r, dn_r, inv_r)
    w, e, f, out = dgs._C.aggregate_neighbors(*[cu(a) for a in args], idx, rg, X, dn, inv, False)
    o64 = orc.agg_forward(*args, idx_r, rg_r, X_r, dn_r, inv_r, exact=True)[3]
    res = {"slots": int(idx_r.size),
           "out_gpu_vs_oracle": margin(out.cpu().numpy(), out_r, 1e-5, 1e-6),
           "out_gpu_vs_fp64": margin(out.cpu().numpy(), o64, 1e-5, 1e-6),
           "out_oracle_vs_fp64": margin(out_r, o64, 1e-5, 1e-6)}
    g = np.random.default_rng(5).normal(size=out_r.shape).astype(np.float32)
    ref = orc.agg_backward(*args, idx_r, rg_r, X_r, dn_r, w_r, e_r, f_r, inv_r, g)
    ref64 = orc.agg_backward(*args, idx_r, rg_r, X_r, dn_r, w_r, e_r, f_r, inv_r, g, exact=True)
    got = dgs._C.aggregate_neighbors_backward(*[cu(a) for a in args], idx, rg, X, dn, w, e, f, inv, cu(g), False)
    for name, a, b, b64 in zip(AGG_FEATURES, got, ref, ref64):
        a = a.cpu().numpy().reshape(b.shape)
        res["d" + name] = {"gpu_vs_oracle": margin(a, b, 1e-5, 1e-5), "gpu_vs_exact": margin(a, b64, 1e-5, 1e-5),
                           "oracle_vs_exact": margin(b, b64, 1e-5, 1e-5)}
    return res


if __name__ == "__main__":
    orc.build()
    out = {
        "config5_shape_d2": case(P=1500, D=2, L=16, K=16, F=4, seed=22),
        "config5_shape_d1": case(P=1500, D=1, L=16, K=16, F=4, seed=21),
        "long_rows": case(P=2000, D=2, L=16, K=16, F=4, seed=41, spread=0.3, radius=(0.6, 1.0)),
        "wide": case(P=500, D=2, L=64, K=64, F=2, seed=95),
        "autograd_case": case(P=700, D=2, L=16, K=16, F=4, seed=80),
    }
    print(json.dumps(out, indent=1))

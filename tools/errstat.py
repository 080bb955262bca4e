"""Parity margins of the gaussian path: for each check, max over elements of
|gpu - ref| / (RTOL |ref| + ATOL max|ref|) (the test tolerance; < 1 passes), on the headline
(1M x 2M, a 1500-sample subset as in test_parity_headline_size_subset) and a small dense case.
Run with PYTHONPATH pointing at a package variant (tools/variant.sh) to compare builds.

    python tools/errstat.py [--function gaussian]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
if not any("variants" in p for p in sys.path):
    sys.path.insert(0, os.path.join(REPO, "diff-gaussian-sampling_amd"))
import diff_gaussian_sampling as dgs  # noqa: E402
from diff_gaussian_sampling import synthetic as syn  # noqa: E402
from helpers import FWD_NAME  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def margin(got, ref, rtol, atol):
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    b = rtol * np.abs(ref) + atol * np.abs(ref).max() + 1e-30
    return float((np.abs(got - ref) / b).max())


def case(function, P, N, C, seed, nsub):
    means, values, covs, conics = syn.gaussians(P, 2, C, seed=seed)
    samples = syn.samples(N, 2, seed=seed + 4)
    K = syn.out_components(function, 2)
    sub = None
    dL = syn.grad_out(N, K, C, seed=seed + 5)
    if nsub:
        g = torch.Generator().manual_seed(seed + 7)
        sub = torch.randperm(N, generator=g)[:nsub].sort().values.numpy().astype(np.int32)
        d = torch.zeros_like(dL)
        d[sub] = dL[sub]
        dL = d
    dev = torch.device("cuda:0")
    m, v, cv, c, s = (t.to(dev) for t in (means, values, covs, conics, samples))
    R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
    out = getattr(dgs._C, FWD_NAME[function])(m, v, c, s, R, gb, sb, rg, srg, False)
    grads = getattr(dgs._C, FWD_NAME[function] + "_backward")(m, v, c, s, R, dL.to(dev).reshape(out.shape), gb, sb, rg, srg, False)
    ob = orc.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    ref = ob.forward(function, values.numpy(), conics.numpy(), subset=sub)
    got = out.cpu().numpy().reshape(ref.shape)
    if sub is not None:
        got, ref = got[sub], ref[sub]
    res = {"fwd": margin(got, ref, 1e-5, 1e-6)}
    dm, dv, dc = ob.backward(function, values.numpy(), conics.numpy(), dL.numpy(), subset=sub)
    for name, a, b in zip(("dmeans", "dvalues", "dconics"), grads, (dm, dv, dc)):
        res[name] = margin(a.cpu().numpy(), b, 1e-5, 1e-5)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--function", default="gaussian")
    a = ap.parse_args()
    orc.build()
    out = {"headline_subset": case(a.function, 1_000_000, 2_000_000, 1, 0, 1500),
           "small_dense": case(a.function, 20000, 60000, 1, 21, 0),
           "mid": case(a.function, 3000, 20000, 1, 11, 0)}
    print(json.dumps(out))

"""Times the fused multi-function call against the per-function calls at the headline size.

    python tools/multi_bench.py [--P 1000000] [--N 2000000] [--functions gaussian,laplacian,...]

Prints one JSON line: ms per fwd+bwd step of the fused call and of the separate calls (the
same outputs and gradients), both over the same binning (preprocess excluded).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("DGS_PKG_ROOT", os.path.join(REPO, "diff-gaussian-sampling_amd"))]  # variants: tools/variant.sh

import torch  # noqa: E402

import diff_gaussian_sampling as dgs  # noqa: E402
from diff_gaussian_sampling import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--N", type=int, default=2_000_000)
    ap.add_argument("--functions", default="gaussian,derivative,laplacian,third")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    fns = args.functions.split(",")
    dev = torch.device("cuda:0")
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(args.P, 2, 1, seed=0))
    samples = syn.samples(args.N, 2, seed=4).to(dev)
    for t in (means, values, conics):
        t.requires_grad_(True)
    s = dgs.GaussianSampler(False)
    s.preprocess(means, values, covs, conics, samples)
    w = {f: torch.randn(args.N, *(2,) * dgs.FUNCTIONS[f], 1, device=dev) for f in fns}
    single = {"gaussian": s.sample_gaussians, "derivative": s.sample_gaussians_derivative,
              "laplacian": s.sample_gaussians_laplacian, "third": s.sample_gaussians_third_derivative}

    def step(fused):
        for t in (means, values, conics):
            t.grad = None
        outs = s.sample_gaussians_multi(*fns) if fused else [single[f]() for f in fns]
        torch.autograd.backward(list(outs), [w[f] for f in fns])

    res = {"P": args.P, "N": args.N, "functions": fns}
    for fused in (True, False, True, False):
        for _ in range(2):
            step(fused)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(fused)
        torch.cuda.synchronize()
        res["fused_ms" if fused else "separate_ms"] = (time.perf_counter() - t0) * 1e3 / args.steps
    res["speedup"] = res["separate_ms"] / res["fused_ms"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""Render-kernel timing at the headline (1M Gaussians x 2M points, D = 2, C = 1, gaussian):
average forward / backward kernel time (HIP events on the launch stream) and ms per fwd+bwd
call pair.  Imports diff_gaussian_sampling from PYTHONPATH first (tools/variant.sh builds).

    python tools/kbench.py [--steps 30] [--warmup 3] [--function gaussian] [--C 1]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.append(os.path.join(REPO, "diff-gaussian-sampling_amd"))

import torch  # noqa: E402

import diff_gaussian_sampling as dgs  # noqa: E402
from diff_gaussian_sampling import synthetic as syn  # noqa: E402

FUNCS = ["gaussian", "derivative", "laplacian", "third"]
ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--N", type=int, default=2_000_000)
ap.add_argument("--C", type=int, default=1)
ap.add_argument("--function", default="gaussian", choices=FUNCS)
ap.add_argument("--prep", type=int, default=0, help="extra (warm) preprocess calls, for profiles")
ap.add_argument("--aniso", type=float, default=1.0, help="axis ratios U[1, aniso] (thin Gaussians)")
a = ap.parse_args()
dev = torch.device("cuda:0")
D, fi = 2, FUNCS.index(a.function)
means, values, covs, conics = (t.to(dev) for t in syn.gaussians(a.P, D, a.C, seed=0, aniso=a.aniso))
samples = syn.samples(a.N, D, seed=4).to(dev)
dL = syn.grad_out(a.N, D ** fi, a.C, seed=5).to(dev).reshape((a.N,) + (D,) * fi + (a.C,))
R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
prep_ms = []
for _ in range(a.prep):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
    torch.cuda.synchronize()
    prep_ms.append((time.perf_counter() - t0) * 1e3)
name = "sample_gaussians" + ["", "_derivative", "_laplacian", "_third_derivative"][fi]
fwd, bwd = getattr(dgs._C, name), getattr(dgs._C, name + "_backward")


def step():
    fwd(means, values, conics, samples, R, gb, sb, rg, srg, False)
    bwd(means, values, conics, samples, R, dL, gb, sb, rg, srg, False)


for _ in range(a.warmup):
    step()
torch.cuda.synchronize()
dgs._C.timing_read(0)
dgs._C.timing_read(1)
dgs._C.timing_enable(True)
t0 = time.perf_counter()
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
el = time.perf_counter() - t0
dgs._C.timing_enable(False)
nf, fms = dgs._C.timing_read(0)
nb, bms = dgs._C.timing_read(1)
print(json.dumps({"lib": os.path.dirname(dgs.__file__), "fwd_ms": fms / max(nf, 1),
                  "bwd_ms": bms / max(nb, 1), "call_pair_ms": el * 1e3 / a.steps,
                  "prep_ms": sorted(prep_ms)[len(prep_ms) // 2] if prep_ms else 0.0}), flush=True)

"""The call-time path alone at the headline (1M x 2M): preprocess, an in-place step of the means,
then K forward + backward calls on the stale binning (each one verifies, finds the difference and
takes the reference's tile pair set with the passed means).  For rocprofv3 kernel traces.

    python tools/calltime_bench.py [--steps 3] [--aniso 1]
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

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--N", type=int, default=2_000_000)
ap.add_argument("--aniso", type=float, default=1.0)
a = ap.parse_args()
dev = torch.device("cuda:0")
means, values, covs, conics = (t.to(dev) for t in syn.gaussians(a.P, 2, 1, seed=0, aniso=a.aniso))
samples = syn.samples(a.N, 2, seed=4).to(dev)
dL = syn.grad_out(a.N, 1, 1, seed=5).to(dev)
R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
moved = means + torch.randn(means.shape, generator=torch.Generator().manual_seed(9)).to(dev) * (0.1 * 2.0 / a.P ** 0.5)
ms = []
for k in range(a.steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = dgs._C.sample_gaussians(moved, values, conics, samples, R, gb, sb, rg, srg, False)
    g = dgs._C.sample_gaussians_backward(moved, values, conics, samples, R, dL, gb, sb, rg, srg, False)
    torch.cuda.synchronize()
    ms.append((time.perf_counter() - t0) * 1e3)
print(json.dumps({"calltime_ms": ms, "median": sorted(ms)[len(ms) // 2]}), flush=True)

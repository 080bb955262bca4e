"""Phase breakdown of k_backward from a DGS_BWD_STAMPS build (tools/variant.sh stamps
"-DDGS_BWD_STAMPS=1"): per-unit wave-time sums (s_memtime ticks, lane 0 of each wave) of the
setup (unit, entry and rows landed), the pair loop + finish, and the stores / atomics, at the
headline workload.  Wave time, not issue time: ~7 waves share a SIMD.

    PYTHONPATH=variants/stamps python tools/bwd_stamps.py [--aniso 1]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.append(os.path.join(REPO, "diff-gaussian-sampling_amd"))
import torch  # noqa: E402

import diff_gaussian_sampling as dgs  # noqa: E402
from diff_gaussian_sampling import synthetic as syn  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--aniso", type=float, default=1.0)
ap.add_argument("--steps", type=int, default=10)
a = ap.parse_args()
lib = ctypes.CDLL(os.path.join(os.path.dirname(dgs.__file__), "libdgs.so"))
dev = torch.device("cuda:0")
means, values, covs, conics = (t.to(dev) for t in syn.gaussians(1_000_000, 2, 1, seed=0, aniso=a.aniso))
samples = syn.samples(2_000_000, 2, seed=4).to(dev)
dL = syn.grad_out(2_000_000, 1, 1, seed=5).to(dev)
R, gb, sb, rg, srg, _ = dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
args = (means, values, conics, samples, R, gb, sb, rg, srg)
buf = (ctypes.c_ulonglong * 8)()
bwd_ms = []
for it in range(a.steps + 5):
    dgs._C.sample_gaussians(*args, False)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    dgs._C.sample_gaussians_backward(means, values, conics, samples, R, dL, gb, sb, rg, srg, False)
    e1.record()
    torch.cuda.synchronize()
    if it >= 5:
        bwd_ms.append(e0.elapsed_time(e1))
    if it == 4:
        assert lib.dgs_debug_bwd_stamps(buf) == 0, "not a DGS_BWD_STAMPS build"
assert lib.dgs_debug_bwd_stamps(buf) == 0
units = buf[3]
res = {"bwd_call_ms": sorted(bwd_ms)[len(bwd_ms) // 2], "units_per_call": units / a.steps, "setup_ticks_per_unit": buf[0] / units,
       "pairs_ticks_per_unit": buf[1] / units, "store_ticks_per_unit": buf[2] / units}
tot = buf[0] + buf[1] + buf[2]
res.update({k + "_share": round(buf[i] / tot, 4) for i, k in enumerate(["setup", "pairs", "store"])})
print(json.dumps(res))

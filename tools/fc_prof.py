"""k_fine_count phase breakdown from a DGS_FC_PROF build (tuning only):
DGS_EXTRA_CFLAGS=-DDGS_FC_PROF=1 python diff-gaussian-sampling_amd/build.py, then run this on a GPU."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "diff-gaussian-sampling_amd"))
import torch  # noqa: E402

import diff_gaussian_sampling as dgs  # noqa: E402
from diff_gaussian_sampling import synthetic as syn  # noqa: E402

aniso = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
dev = torch.device("cuda:0")
P, N = 1_000_000, 2_000_000
means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, 2, 1, seed=0, aniso=aniso))
samples = syn.samples(N, 2).to(dev)
dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
torch.cuda.synchronize()
dgs._C.debug_fc_prof()
reps = 5
for _ in range(reps):
    dgs._C.preprocess_gaussians(means, values, covs, conics, samples, False)
torch.cuda.synchronize()
v = dgs._C.debug_fc_prof()
waves = reps * ((P + 63) // 64)
names = ["fallback_bits", "loads+copies", "cut+reach", "local_rows", "fallback/enumerate", "whole"]
print(json.dumps({"aniso": aniso, "cycles_per_wave": {n: round(v[k] / waves) for k, n in enumerate(names)}}))

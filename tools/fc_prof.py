"""k_fine_count phase breakdown from a DGS_FC_PROF build (tuning only):
tools/variant.sh fcprof -DDGS_FC_PROF=1, then on a GPU: python tools/fc_prof.py [ANISO] (it loads
variants/fcprof)."""
import json
import os
import sys

_root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(_root, "diff-gaussian-sampling_amd"))
sys.path.insert(0, os.path.join(_root, "variants", os.environ.get("DGS_VARIANT", "fcprof")))
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
names = ["fallback_bits", "loads", "cut+reach", "local_rows", "fallback_only+queue", "whole"]
print(json.dumps({"lib": dgs._C.__file__, "aniso": aniso, "cycles_per_wave": {n: round(v[k] / waves) for k, n in enumerate(names)}}))

"""Time SupportExchange's one-time set construction (distributed.py) at the config-4 shape in ONE process:
1M headline Gaussians, 8 strips of [-1, 1) along y as the rank extents (no collective runs in
the constructor).  Prints the warm median per rank and the rows each rank moves.

    python tools/xchg_bench.py [--world 8] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "diff-gaussian-sampling_amd"))
from diff_gaussian_sampling import synthetic as syn  # noqa: E402
from diff_gaussian_sampling.distributed import SupportExchange  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--P", type=int, default=1_000_000)
a = ap.parse_args()
dev = torch.device("cuda:0")
means, values, covs, conics = (t.to(dev) for t in syn.gaussians(a.P, 2, 1, seed=0))
W = a.world
edges = torch.linspace(-1.0, 1.0, W + 1, device=dev)
ext = torch.stack([edges[:-1], edges[1:]], 1)
res = {}
for r in (0, W // 2):
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x = SupportExchange(means, conics, ext, r)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    res[f"rank{r}"] = {"setup_ms_median": sorted(ts)[len(ts) // 2], "rows_sent": x.rows_moved(),
                       "rows_received": sum(x.recv_splits), "held": int(x.held.sum())}
print(json.dumps(res))

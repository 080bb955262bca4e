"""Neighbour-aggregation timing at SURVEY config 5: P = 1M 2-D Gaussians (the headline
Gaussians; radii from preprocess_gaussians), K = L = 16, F = 4 (E = 17).

    python tools/agg_bench.py [--P 1000000] [--steps 5] [--warmup 2]

Prints one JSON line: list length, ms per preprocess / forward / backward (HIP events on the
current stream), and slots per second.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("DGS_PKG_ROOT", os.path.join(REPO, "diff-gaussian-sampling_amd")))  # variants: tools/variant.sh

import torch  # noqa: E402

import diff_gaussian_sampling as dgs  # noqa: E402
from diff_gaussian_sampling import synthetic as syn  # noqa: E402


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        r = fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--N", type=int, default=2_000_000)
    ap.add_argument("--L", type=int, default=16)
    ap.add_argument("--K", type=int, default=16)
    ap.add_argument("--F", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(a.P, 2, 1, seed=0))
    samples = syn.samples(a.N, 2).to(dev)
    radii = dgs.preprocess_gaussians(means, values, covs, conics, samples, False)[5]
    D, E = 2, 2 * 2 * a.F + 1
    g = torch.Generator(device="cpu").manual_seed(7)
    rnd = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
    feats = [rnd(a.P, a.L), rnd(a.L, a.L) / a.L, rnd(a.P, a.K), rnd(a.P, a.K),
             (torch.rand(a.F, generator=g) * 2.5 + 0.5).to(dev), rnd(2 * E)]
    t_pre, pre = timed(lambda: dgs._C.preprocess_aggregate(means, conics, radii, False), a.steps, a.warmup)
    idx, rg, X, dn, inv = pre
    Lnb = int(idx.numel())
    t_fwd, fw = timed(lambda: dgs._C.aggregate_neighbors(*feats, idx, rg, X, dn, inv, False), a.steps, a.warmup)
    w, e, f, out = fw
    dL = torch.randn_like(out)
    t_bwd, _ = timed(lambda: dgs._C.aggregate_neighbors_backward(*feats, idx, rg, X, dn, w, e, f, inv, dL, False),
                     a.steps, a.warmup)
    print(json.dumps({
        "P": a.P, "L": a.L, "K": a.K, "F": a.F, "neighbours": Lnb, "per_row": Lnb / a.P,
        "invalid_slots": int((idx < 0).sum()),
        "ms_preprocess": round(t_pre, 3), "ms_forward": round(t_fwd, 3), "ms_backward": round(t_bwd, 3),
        "slots_per_s_fwd_bwd": Lnb / ((t_fwd + t_bwd) * 1e-3),
        "max_hbm_gib": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2),
    }))


if __name__ == "__main__":
    main()

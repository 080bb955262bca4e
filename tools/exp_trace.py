"""Experiment: per-unit forward timeline (needs libdgs built with -DDGS_EXP_TRACE)."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "diff-gaussian-sampling_amd"))
import diff_gaussian_sampling as dgs
from diff_gaussian_sampling import synthetic as syn
lib = ctypes.CDLL(os.path.join(os.path.dirname(dgs.__file__), "libdgs.so"))
dev = "cuda"
m, v, cv, c = (t.to(dev) for t in syn.gaussians(1_000_000, 2, 1, seed=0))
s = syn.samples(2_000_000, 2, seed=4).to(dev)
R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
for _ in range(3):
    out = dgs._C.sample_gaussians(m, v, c, s, R, gb, sb, rg, srg, False)
torch.cuda.synchronize()
n = 4 * 40000
buf = (ctypes.c_ulonglong * n)()
assert lib.dgs_exp_trace(buf, ctypes.c_size_t(n)) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4)
a = a[a[:, 1] > 0]
t0, t1 = a[:, 0].astype(np.int64), a[:, 1].astype(np.int64)
base = t0.min(); t0 -= base; t1 -= base
hw = (a[:, 2] & 0xffffffff).astype(np.int64); xcc = (a[:, 2] >> 32).astype(np.int64) & 0xf
cu = (hw >> 8) & 0xf; sh = (hw >> 12) & 1; se = (hw >> 13) & 0x7; simd = (hw >> 4) & 3
cuid = ((xcc * 8 + se) * 2 + sh) * 16 + cu
ns = (a[:, 3] >> 32).astype(np.int64); ne = (a[:, 3] & 0xffffffff).astype(np.int64)
dur = t1 - t0
print("units", len(a), "span ticks(10ns)", t1.max(), "=", t1.max() * 0.01, "us")
print("unit duration us: mean %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f" % tuple(np.r_[dur.mean(), np.percentile(dur, [10, 50, 90]), dur.max()] * 0.01))
print("entries: mean %.0f p10 %.0f p90 %.0f max %d; samples mean %.1f" % (ne.mean(), *np.percentile(ne, [10, 90]), ne.max(), ns.mean()))
print("corr(dur, entries)", np.corrcoef(dur, ne)[0, 1], " us per 1000 entries (f2 units):", 1000 * 0.01 * np.median(dur[ns > 64] / ne[ns > 64]))
print("distinct CUs", len(np.unique(cuid)), "xcc", np.unique(xcc), "se", np.unique(se))
# per-CU busy and finish
last = np.zeros(cuid.max() + 1); first = np.full(cuid.max() + 1, 1e18); busy = np.zeros(cuid.max() + 1)
for i in range(len(a)):
    last[cuid[i]] = max(last[cuid[i]], t1[i]); first[cuid[i]] = min(first[cuid[i]], t0[i])
used = last > 0
print("CU finish time us: min %.1f p50 %.1f max %.1f" % (last[used].min() * 0.01, np.median(last[used]) * 0.01, last[used].max() * 0.01))
# concurrency timeline
T = int(t1.max()); bins_ = 50
edges = np.linspace(0, T, bins_ + 1)
conc = [np.sum((t0 < e1) & (t1 > e0) ) for e0, e1 in zip(edges[:-1], edges[1:])]
print("concurrent units per 1/50 of span:", conc)
# start-time distribution
print("unit start quantiles us:", np.percentile(t0, [0, 25, 50, 75, 90, 99, 100]) * 0.01)

import os, sys, time, torch
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "diff-gaussian-sampling_amd"))
t0 = time.perf_counter()
import diff_gaussian_sampling as dgs
from diff_gaussian_sampling import synthetic as syn
dev = torch.device("cuda:0")
torch.zeros(1, device=dev); torch.cuda.synchronize()
t1 = time.perf_counter()
def prep(P, N, seed=0):
    m, v, cv, c = (t.to(dev) for t in syn.gaussians(P, 2, 1, seed=seed))
    s = syn.samples(N, 2, seed=seed + 4).to(dev)
    torch.cuda.synchronize(); a = time.perf_counter()
    r = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
    torch.cuda.synchronize(); return (time.perf_counter() - a) * 1e3
mode = sys.argv[1]
if mode == "tiny_first":
    print("tiny", prep(100, 400)); print("full after tiny", prep(1_000_000, 2_000_000)); print("full again", prep(1_000_000, 2_000_000))
else:
    print("full first", prep(1_000_000, 2_000_000)); print("full again", prep(1_000_000, 2_000_000))

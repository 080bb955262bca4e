"""Where a fresh process's first preprocess_gaussians call spends its time:
import, device init, the library's code-object load (dgs_warmup), the first binning at the
headline size, a repeat.  One fresh process per run:

    python tools/first_call.py [--no-warmup]
"""
import os
import sys
import time

T0 = time.perf_counter()
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "diff-gaussian-sampling_amd"))


def ms(a):
    return round((time.perf_counter() - a) * 1e3, 2)


out = {"import_torch_ms": ms(T0)}
t = time.perf_counter()
dev = torch.device("cuda:0")
torch.zeros(1, device=dev)
torch.cuda.synchronize()
out["device_init_ms"] = ms(t)
t = time.perf_counter()
import diff_gaussian_sampling as dgs  # noqa: E402
from diff_gaussian_sampling import synthetic as syn  # noqa: E402
out["import_dgs_ms"] = ms(t)
if "--no-warmup" not in sys.argv:
    t = time.perf_counter()
    dgs.warmup()
    out["warmup_ms"] = ms(t)
m, v, cv, c = (x.to(dev) for x in syn.gaussians(1_000_000, 2, 1, seed=0))
s = syn.samples(2_000_000, 2, seed=4).to(dev)
for k in ("first_call_ms", "second_call_ms", "third_call_ms"):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
    torch.cuda.synchronize()
    out[k] = ms(t)
out["torch_reserved_MB"] = round(torch.cuda.memory_reserved() / 2 ** 20)
print(out)

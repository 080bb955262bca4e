"""Graph-capture probe (diagnostic): one scenario per process, `python tools/graph_probe.py K`.
  0: plain torch ops          1: torch autograd (a small MLP's forward + grad)
  2: dgs forward (_C direct)  3: dgs forward + backward (_C direct, no autograd)
  4: dgs forward + grad through the autograd Function"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "diff-gaussian-sampling_amd"))


def capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    g.replay()
    torch.cuda.synchronize()
    return out


def main(k):
    dev = torch.device("cuda")
    if k == 0:
        x = torch.randn(1000, device=dev)
        capture(lambda: x * 2 + 1)
    elif k == 1:
        w = torch.randn(64, 64, device=dev, requires_grad=True)
        x = torch.randn(32, 64, device=dev)
        capture(lambda: torch.autograd.grad((x @ w).tanh().sum(), w))
    else:
        import diff_gaussian_sampling as dgs
        from diff_gaussian_sampling import synthetic as syn
        P, N = 20000, 60000
        means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, 2, 1, seed=3))
        samples = syn.samples(N, 2, seed=9).to(dev)
        R, gb, sb, rg, srg, _ = dgs.preprocess_gaussians(means, values, covs, conics, samples, False)
        dL = torch.randn(N, 1, device=dev)
        C = dgs._C
        if k == 2:
            capture(lambda: C.sample_gaussians(means, values, conics, samples, R, gb, sb, rg, srg, False))
        elif k == 3:
            def fb():
                out = C.sample_gaussians(means, values, conics, samples, R, gb, sb, rg, srg, False)
                return out, C.sample_gaussians_backward(means, values, conics, samples, R, dL, gb, sb, rg, srg,
                                                        False)
            capture(fb)
        else:
            for t in (means, values, conics):
                t.requires_grad_(True)

            def step():
                out = dgs.sample_gaussians(means, values, conics, samples, R, gb, sb, rg, srg, False)
                return torch.autograd.grad(out, (means, values, conics), dL)
            capture(step)
    print(f"probe {k}: ok", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]))

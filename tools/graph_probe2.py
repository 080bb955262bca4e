"""Graph-capture probe for the PIGS training pattern: `loss.backward()` accumulating into `.grad`
inside torch.cuda.graph.  One scenario per process:

    python tools/graph_probe2.py SCENARIO

  torch_recipe            a small MLP, torch's whole-network recipe: warm-up iterations on a side
                          stream, zero_grad(set_to_none=True), then loss.backward() captured
  dgs_recipe              the same recipe with diff_gaussian_sampling.sample_gaussians in the loss
  torch_eager_then_capture  an eager forward + backward on the DEFAULT stream first (its
                          AccumulateGrad nodes and .grad live on that stream), then the capture of
                          loss.backward() into the existing .grad -- the round-4 failing pattern,
                          with torch ops only
  dgs_eager_then_capture  the same with the sampler
  dgs_after_history       round 4's crash came after 15 other tests in the same process
                          (gpurun_out/r04g/tests.log): eager binnings, forwards and backwards of
                          other sizes, functions and C first (their host-side records and freed
                          buffers), then dgs_recipe's capture

Prints "<scenario>: ok" (plus the max gradient difference replay vs eager) on success.
tools/gpu.sh graph runs them from the safest to the riskiest and stops at a crash.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "diff-gaussian-sampling_amd"))


def make_torch():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    w1 = torch.randn(64, 128, device=dev, generator=g, requires_grad=True)
    w2 = torch.randn(128, 1, device=dev, generator=g, requires_grad=True)
    x = torch.randn(256, 64, device=dev, generator=g)

    def loss():
        return ((x @ w1).tanh() @ w2).square().sum()
    return [w1, w2], loss


def make_dgs():
    import diff_gaussian_sampling as dgs
    from diff_gaussian_sampling import synthetic as syn
    dev = torch.device("cuda")
    P, N = 20000, 60000
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, 2, 1, seed=3))
    samples = syn.samples(N, 2, seed=9).to(dev)
    sampler = dgs.GaussianSampler(False)
    params = [means, values, conics]
    for t in params:
        t.requires_grad_(True)
    sampler.preprocess(means, values, covs, conics, samples)
    target = torch.randn(N, 1, device=dev, generator=torch.Generator(device=dev).manual_seed(5))

    def loss():
        return (sampler.sample_gaussians() - target).square().sum()
    return params, loss


def history():
    import diff_gaussian_sampling as dgs
    from diff_gaussian_sampling import synthetic as syn
    dev = torch.device("cuda")
    for k, (P, N, C, fn) in enumerate([(500, 2000, 1, "gaussian"), (3000, 9000, 3, "derivative"),
                                       (800, 4000, 16, "laplacian"), (5000, 20000, 1, "third"),
                                       (20000, 60000, 1, "gaussian")]):
        means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, 2, C, seed=20 + k))
        samples = syn.samples(N, 2, seed=40 + k).to(dev)
        for t in (means, values, conics):
            t.requires_grad_(True)
        sampler = dgs.GaussianSampler(False)
        sampler.preprocess(means, values, covs, conics, samples)
        f = {"gaussian": sampler.sample_gaussians, "derivative": sampler.sample_gaussians_derivative,
             "laplacian": sampler.sample_gaussians_laplacian, "third": sampler.sample_gaussians_third_derivative}[fn]
        for _ in range(3):
            f().square().sum().backward()
        with torch.no_grad():
            means.add_(1e-3)  # an in-place step: the next call verifies and takes the call-time path
        f().sum().backward()
        del sampler, means, values, covs, conics, samples
    torch.cuda.synchronize()


def run(scenario):
    if scenario == "dgs_after_history":
        history()
        scenario = "dgs_recipe"
    params, loss = (make_dgs if scenario.startswith("dgs") else make_torch)()
    eager_first = scenario.endswith("eager_then_capture")
    if eager_first:  # default stream: AccumulateGrad / .grad made here
        loss().backward()
        torch.cuda.synchronize()
    ref = None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            if not eager_first:
                for p in params:
                    p.grad = None
            loss().backward()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    if not eager_first:
        for p in params:
            p.grad = None
        # eager reference of one step from zero grads
        loss().backward()
        ref = [p.grad.clone() for p in params]
        for p in params:
            p.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = loss()
        out.backward()
    torch.cuda.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    msg = ""
    if ref is not None:  # the capture's .grad tensors hold one step's gradients after a replay
        d = max(float((p.grad - r).abs().max() / (r.abs().max() + 1e-30)) for p, r in zip(params, ref))
        msg = f" (replay vs eager, max rel diff {d:.2e})"
        assert d < 1e-4, msg
    print(f"{scenario}: ok{msg}", flush=True)


if __name__ == "__main__":
    run(sys.argv[1])

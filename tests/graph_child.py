"""Child process of tests/test_gpu_graph.py (one scenario per process, so that a failure inside
the HIP runtime's graph capture fails the test instead of ending the pytest process):
`python tests/graph_child.py forward_backward gaussian|derivative` or `python tests/graph_child.py
requires_binned`.  Prints "ok" on success."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diff-gaussian-sampling_amd"))

import diff_gaussian_sampling as dgs  # noqa: E402
from diff_gaussian_sampling import synthetic as syn  # noqa: E402

RTOL, ATOL = 1e-5, 1e-6


def _close(a, b, what):
    scale = float(b.abs().max()) if b.numel() else 0.0
    err = (a - b).abs()
    bound = RTOL * b.abs() + ATOL * scale
    assert bool((err <= bound).all()), f"{what}: max |d| {float(err.max()):.3e} (scale {scale:.3e})"


def forward_backward(fname):
    dev = torch.device("cuda")
    P, N, C = 20000, 60000, 1
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, 2, C, seed=3))
    samples = syn.samples(N, 2, seed=9).to(dev)
    K = 2 if fname == "derivative" else 1
    fwd = {"gaussian": dgs.sample_gaussians, "derivative": dgs.sample_gaussians_derivative}[fname]
    R, gb, sb, rg, srg, _ = dgs.preprocess_gaussians(means, values, covs, conics, samples, False)
    dL = torch.randn((N,) + (2,) * (K - 1) + (C,), device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    for t in (means, values, conics):
        t.requires_grad_(True)

    def step():  # (detached output: no autograd graph outlives a step; INTEGRATION.md §4 has the
        # capture recipe and what is known about round 4's capture-time crash)
        out = fwd(means, values, conics, samples, R, gb, sb, rg, srg, False)
        g = torch.autograd.grad(out, (means, values, conics), dL)
        return out.detach(), g

    # eager reference, then warm-up on a side stream (torch.cuda.graph's recipe)
    ref_out, ref_g = step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g_out, g_g = step()
    for _ in range(2):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(g_out, ref_out), "forward replay differs from the eager call"
        for a, b, w in zip(g_g, ref_g, ("dmeans", "dvalues", "dconics")):
            _close(a, b, f"replay {w}")
    # values and dL change in place: the replay follows them (the rows are re-packed in the graph)
    with torch.no_grad():
        values.mul_(-0.5).add_(0.25)
        dL.mul_(2.0)
    graph.replay()
    torch.cuda.synchronize()
    # (the eager check after the change: values' version moved, so nothing cached is reused)
    new_out, new_g = step()
    assert torch.equal(g_out, new_out), "forward replay after the values change differs"
    for a, b, w in zip(g_g, new_g, ("dmeans", "dvalues", "dconics")):
        _close(a, b, f"replay after change {w}")
    assert not torch.equal(new_out, ref_out)


def rebin_step(fname, fixed=False):
    """the whole PIGS step -- re-binning (preprocess_gaussians_capturable),
    forward, loss and loss.backward() into .grad -- captured as ONE graph with torch's
    whole-network recipe (warm-up on a side stream, grads set to None before the capture), then
    replayed after in-place steps of the means (the optimizer's move): every replay must match an
    eager preprocess + forward + backward of the moved means at the parity bound, with status 0.
    fixed: the captured binning copies the sample side of the first eager binning
    (samples_binned, DGS_BIN_SAMPLES_FIXED) instead of sorting the unchanged samples per replay."""
    dev = torch.device("cuda")
    P, N, C = 20000, 60000, 1
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, 2, C, seed=3))
    samples = syn.samples(N, 2, seed=9).to(dev)
    K = 2 if fname == "derivative" else 1
    fwd = {"gaussian": dgs.sample_gaussians, "derivative": dgs.sample_gaussians_derivative}[fname]
    target = torch.randn((N,) + (2,) * (K - 1) + (C,), device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    R0, gb0, sb0, _, _, _ = dgs.preprocess_gaussians(means, values, covs, conics, samples, False)
    grid, off = dgs._C.tile_grid(samples)
    cap = dgs.capacity_from(gb0, sb0, slack=0.25)
    for t in (means, values, conics):
        t.requires_grad_(True)

    def step():
        R, gb, sb, rg, srg, _, st = dgs.preprocess_gaussians_capturable(means.detach(), values.detach(), covs,
                                                                         conics.detach(), samples, grid, off, cap,
                                                                         samples_binned=sb0 if fixed else None)
        out = fwd(means, values, conics, samples, cap[2], gb, sb, rg, srg, False)
        (out - target).square().sum().backward()
        return out, st, R

    def eager():
        R, gb, sb, rg, srg, _ = dgs.preprocess_gaussians(means.detach(), values.detach(), covs, conics.detach(),
                                                         samples, False)
        out = fwd(means, values, conics, samples, R, gb, sb, rg, srg, False)
        g = torch.autograd.grad((out - target).square().sum(), (means, values, conics))
        return out.detach(), g, R

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            for t in (means, values, conics):
                t.grad = None
            step()
    torch.cuda.current_stream().wait_stream(s)
    for t in (means, values, conics):
        t.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g_out, g_st, g_R = step()
    gen = torch.Generator(device=dev).manual_seed(11)
    for it in range(3):
        with torch.no_grad():  # the optimizer's in-place move of the means (no re-capture)
            means.add_(torch.randn(means.shape, device=dev, generator=gen) * 2e-3)
        graph.replay()
        torch.cuda.synchronize()
        assert int(g_st.item()) == 0, f"replay {it}: status {int(g_st.item())}"
        ref_out, ref_g, ref_R = eager()
        assert int(g_R.item()) == ref_R, f"replay {it}: num_rendered {int(g_R.item())} != {ref_R}"
        _close(g_out.detach(), ref_out, f"replay {it} forward")
        for p, r, w in zip((means, values, conics), ref_g, ("dmeans", "dvalues", "dconics")):
            _close(p.grad, r, f"replay {it} {w}")
    # a capacity overflow is reported, never out of bounds: a tiny capacity, eager
    R, gb, sb, rg, srg, _, st = dgs.preprocess_gaussians_capturable(means.detach(), values.detach(), covs,
                                                                     conics.detach(), samples, grid, off,
                                                                     [4096, 1024, 4096])
    out = dgs._C.sample_gaussians(means.detach(), values.detach(), conics.detach(), samples, 0, gb, sb, rg, srg,
                                  False)
    torch.cuda.synchronize()
    assert int(st.item()) & 1, f"overflow not reported: status {int(st.item())}"
    assert torch.isfinite(out).all()
    # other means on that binning would take the call-time path over its clamped lists: refused
    # loudly instead (no out-of-bounds tile lists)
    try:
        dgs._C.sample_gaussians(means.detach() + 1e-3, values.detach(), conics.detach(), samples, 0, gb, sb, rg,
                                srg, False)
        torch.cuda.synchronize()
    except RuntimeError as e:
        assert "status" in str(e), str(e)
    else:
        raise AssertionError("a call-time evaluation on an overflowed binning did not raise")


def overflow_monitor():
    """a captured PIGS step whose binning overflows at replay k is reported by
    BinningStatusMonitor.check() after replay k + 1 at the latest, with no host sync inside the
    step (the sticky status word is copied to pinned memory by a node of the graph)."""
    dev = torch.device("cuda")
    P, N = 20000, 60000
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, 2, 1, seed=3))
    samples = syn.samples(N, 2, seed=9).to(dev)
    target = torch.randn((N, 1), device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    _, gb0, sb0, _, _, _ = dgs.preprocess_gaussians(means, values, covs, conics, samples, False)
    grid, off = dgs._C.tile_grid(samples)
    cap = dgs.capacity_from(gb0, sb0, slack=0.25)
    mon = dgs.BinningStatusMonitor(dev)
    for t in (means, values, conics):
        t.requires_grad_(True)

    def step():
        R, gb, sb, rg, srg, _, st = dgs.preprocess_gaussians_capturable(
            means.detach(), values.detach(), covs, conics.detach(), samples, grid, off, cap, status=mon.status)
        mon.record()
        out = dgs.sample_gaussians(means, values, conics, samples, 0, gb, sb, rg, srg, False)
        (out - target).square().sum().backward()
        return st

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            for t in (means, values, conics):
                t.grad = None
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert int(mon.status.item()) == 0
    for t in (means, values, conics):
        t.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g_st = step()
    assert g_st.data_ptr() == mon.status.data_ptr()
    k = 3
    raised_at = None
    for it in range(k + 3):
        if it == k:  # the Gaussians grow 4x in area in place: the captured capacity overflows
            with torch.no_grad():
                covs.mul_(4.0)
                conics.mul_(0.25)
        graph.replay()
        try:
            mon.check()
        except dgs.BinningOverflow as e:
            raised_at = it
            print("raised:", e, flush=True)
            break
    assert raised_at is not None, "the overflow was never reported"
    assert k <= raised_at <= k + 1, f"overflow at replay {k} reported at replay {raised_at}"
    torch.cuda.synchronize()
    assert int(mon.status.item()) & 1
    mon.reset()
    assert int(mon.status.item()) == 0


def requires_binned():
    dev = torch.device("cuda")
    P, N = 2000, 6000
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, 2, 1, seed=4))
    samples = syn.samples(N, 2, seed=10).to(dev)
    R, gb, sb, rg, srg, _ = dgs.preprocess_gaussians(means, values, covs, conics, samples, False)
    other = means.clone()  # equal values, another tensor: not provably the binned one
    dgs.sample_gaussians(other, values, conics, samples, R, gb, sb, rg, srg, False)  # eager: fine
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(graph):
            dgs.sample_gaussians(other, values, conics, samples, R, gb, sb, rg, srg, False)
    except RuntimeError as e:
        # (the library's refusal, or -- should ending the capture also fail -- its context)
        msg = str(e) + " " + str(e.__context__)
        assert "graph capture" in msg, msg
    else:
        raise AssertionError("a capture with tensors other than the binned ones did not raise")
    torch.cuda.synchronize()


if __name__ == "__main__":
    if sys.argv[1] == "forward_backward":
        forward_backward(sys.argv[2])
    elif sys.argv[1] == "rebin_step":
        rebin_step(sys.argv[2], fixed=len(sys.argv) > 3 and sys.argv[3] == "fixed")
    elif sys.argv[1] == "overflow_monitor":
        overflow_monitor()
    else:
        requires_binned()
    print("ok", flush=True)

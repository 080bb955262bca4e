"""GPU parity of the render calls when their means / conics / samples are NOT the tensors the
binning was built from.

The reference bins at preprocess (tile lists from the preprocess-time means, covariances and
samples; its preprocess never reads conics: sample_points.cu:38-98, forward.cu:24-83) but reads
means, conics, values and samples from the tensors passed to every forward / backward call
(forward.cu:136-145, backward.cu:76-85).  So a caller that updates the means in place (an
optimizer step) and samples again without re-binning, or passes preprocess other conics,
gets the preprocess-time pair set evaluated with the call-time tensors.  The oracle expresses
exactly that: OracleBins(preprocess tensors).forward/backward(..., call-time tensors).

Checked here: every function x D in {1, 2} x C in {1, 3} with in-place perturbed means, conics
passed to preprocess that differ from the sampled ones, perturbed samples, the fused entry
point, and that the binned (fast) path is taken again after re-binning.
Tolerances as test_gpu_parity.py.
"""
import pytest
import torch

from diff_gaussian_sampling import synthetic as syn
from helpers import FUNCS, FWD_NAME, close

pytestmark = pytest.mark.gpu

RTOL, ATOL_FWD, ATOL_BWD = 1e-5, 1e-6, 1e-6  # SURVEY 8c (backward: atol 1e-6 max|ref|)


def _run(dgs, oracle, function, pre, call, dL):
    """pre / call: (means, values, covs, conics, samples) at preprocess / at the render call."""
    dev = torch.device("cuda:0")
    pm, pv, pcv, pc, ps = (t.to(dev) for t in pre)
    R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(pm, pv, pcv, pc, ps, False)
    cm, cv_, _, cc, cs = (t.to(dev) for t in call)
    match = dgs._C.inputs_match(cm, cc, cs, gb, sb)
    out = getattr(dgs._C, FWD_NAME[function])(cm, cv_, cc, cs, R, gb, sb, rg, srg, False)
    grads = getattr(dgs._C, FWD_NAME[function] + "_backward")(
        cm, cv_, cc, cs, R, dL.to(dev).reshape(out.shape), gb, sb, rg, srg, False)
    ob = oracle.OracleBins(pre[0].numpy(), pre[2].numpy(), pre[4].numpy())
    assert R == ob.num_rendered
    N, C = call[4].shape[0], call[1].shape[1]
    ref = ob.forward(function, call[1].numpy(), call[3].numpy(), means=call[0].numpy(), samples=call[4].numpy())
    close(out.cpu().numpy().reshape(N, -1, C), ref, RTOL, ATOL_FWD, f"{function} forward (call-time inputs)")
    dm, dv, dc = ob.backward(function, call[1].numpy(), call[3].numpy(), dL.numpy(),
                             means=call[0].numpy(), samples=call[4].numpy(), exact=True)
    close(grads[0].cpu().numpy(), dm, RTOL, ATOL_BWD, f"{function} dL/dmeans (call-time inputs)")
    close(grads[1].cpu().numpy(), dv, RTOL, ATOL_BWD, f"{function} dL/dvalues (call-time inputs)")
    close(grads[2].cpu().numpy(), dc, RTOL, ATOL_BWD, f"{function} dL/dconics (call-time inputs)")
    return match


def _problem(P, N, D, C, seed):
    means, values, covs, conics = syn.gaussians(P, D, C, seed=seed)
    samples = syn.samples(N, D, seed=seed + 1)
    return means, values, covs, conics, samples


@pytest.mark.parametrize("function", FUNCS)
@pytest.mark.parametrize("D,C", [(2, 1), (2, 3), (1, 1)])
def test_means_updated_in_place(dgs, oracle, function, D, C):
    """An optimizer-like in-place step on the means between preprocess and sampling."""
    P, N = 2000, 12000
    pre = _problem(P, N, D, C, seed=401)
    g = torch.Generator().manual_seed(402)
    step = (torch.randn(P, D, generator=g) * (0.5 * 2.0 / P ** (1.0 / D))).float()
    call = (pre[0] + step, pre[1], pre[2], pre[3], pre[4])
    dL = syn.grad_out(N, syn.out_components(function, D), C, seed=403)
    assert not _run(dgs, oracle, function, pre, call, dL)


@pytest.mark.parametrize("function", FUNCS)
def test_preprocess_conics_differ(dgs, oracle, function):
    """preprocess given other conics than the ones sampled with: the reference's binning never
    reads conics, so the result must not depend on them."""
    P, N, D, C = 2000, 12000, 2, 1
    pre = _problem(P, N, D, C, seed=411)
    wrong = pre[3] * torch.tensor([4.0, 0.0, 0.25])  # a different (still PD) conic per Gaussian
    dL = syn.grad_out(N, syn.out_components(function, D), C, seed=413)
    assert not _run(dgs, oracle, function, (pre[0], pre[1], pre[2], wrong, pre[4]), pre, dL)


@pytest.mark.parametrize("function", ["gaussian", "laplacian"])
def test_samples_moved(dgs, oracle, function):
    """Query points moved after binning: evaluated at their call-time positions over the
    preprocess-time tile lists (a moved point stays in its binned tile)."""
    P, N, D, C = 2000, 12000, 2, 2
    pre = _problem(P, N, D, C, seed=421)
    g = torch.Generator().manual_seed(422)
    moved = (pre[4] + torch.randn(N, D, generator=g) * 0.01).float()
    dL = syn.grad_out(N, syn.out_components(function, D), C, seed=423)
    assert not _run(dgs, oracle, function, pre, (pre[0], pre[1], pre[2], pre[3], moved), dL)


def test_binned_inputs_take_the_fast_path(dgs, oracle):
    """The normal case (the binned tensors passed back, as GaussianSampler does) is detected as
    such -- also for equal-valued copies -- and still matches the oracle."""
    P, N, D, C = 3000, 15000, 2, 1
    pre = _problem(P, N, D, C, seed=431)
    dL = syn.grad_out(N, 1, C, seed=433)
    assert _run(dgs, oracle, "gaussian", pre, tuple(t.clone() for t in pre), dL)


def test_fused_call_with_moved_means(dgs, oracle):
    """sample_gaussians_multi (one traversal for several functions) on the call-time path."""
    P, N, D, C = 2000, 10000, 2, 1
    means, values, covs, conics, samples = _problem(P, N, D, C, seed=441)
    dev = torch.device("cuda:0")
    m, v, cv, c, s = (t.to(dev) for t in (means, values, covs, conics, samples))
    R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
    g = torch.Generator().manual_seed(442)
    m1 = (means + torch.randn(P, D, generator=g) * 0.01).float()
    fns = [0, 2, 3]
    outs = dgs._C.sample_gaussians_multi(fns, m1.to(dev), v, c, s, gb, sb, False)
    dLs = [syn.grad_out(N, D ** f, C, seed=443 + f) for f in fns]
    gm, gv, gc = dgs._C.sample_gaussians_multi_backward(
        fns, m1.to(dev), v, c, s, [d.to(dev).reshape(o.shape) for d, o in zip(dLs, outs)], gb, sb, False)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    sdm = sdv = sdc = 0
    for f, o, d in zip(fns, outs, dLs):
        name = FUNCS[f]
        ref = ob.forward(name, values.numpy(), conics.numpy(), means=m1.numpy())
        close(o.cpu().numpy().reshape(ref.shape), ref, RTOL, ATOL_FWD, f"fused {name} forward")
        dm, dv, dc = ob.backward(name, values.numpy(), conics.numpy(), d.numpy(), means=m1.numpy(), exact=True)
        sdm, sdv, sdc = sdm + dm, sdv + dv, sdc + dc
    close(gm.cpu().numpy(), sdm, RTOL, ATOL_BWD, "fused dL/dmeans")
    close(gv.cpu().numpy(), sdv, RTOL, ATOL_BWD, "fused dL/dvalues")
    close(gc.cpu().numpy(), sdc, RTOL, ATOL_BWD, "fused dL/dconics")


def test_sampler_after_optimizer_step(dgs, oracle):
    """GaussianSampler: an in-place update of the means Parameter after preprocess changes the
    result as in the reference; re-binning restores the binned path with the new means."""
    P, N, D, C = 2000, 10000, 2, 1
    means, values, covs, conics, samples = _problem(P, N, D, C, seed=451)
    dev = torch.device("cuda:0")
    m = torch.nn.Parameter(means.to(dev))
    v, cv, c, s = (t.to(dev) for t in (values, covs, conics, samples))
    sampler = dgs.GaussianSampler(False)
    sampler.preprocess(m, v, cv, c, s)
    assert dgs._C.inputs_match(m.detach(), c, s, sampler.binning_buffer, sampler.sample_binning_buffer)
    with torch.no_grad():
        m.add_(0.002)
    assert not dgs._C.inputs_match(m.detach(), c, s, sampler.binning_buffer, sampler.sample_binning_buffer)
    out = sampler.sample_gaussians()
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    m1 = m.detach().cpu().numpy()
    close(out.detach().cpu().numpy().reshape(N, 1, 1), ob.forward("gaussian", values.numpy(), conics.numpy(), means=m1),
          RTOL, ATOL_FWD, "sampler forward after in-place step")
    sampler.preprocess(m, v, cv, c, s)
    assert dgs._C.inputs_match(m.detach(), c, s, sampler.binning_buffer, sampler.sample_binning_buffer)
    out2 = sampler.sample_gaussians()
    ob2 = oracle.OracleBins(m1, covs.numpy(), samples.numpy())
    close(out2.detach().cpu().numpy().reshape(N, 1, 1), ob2.forward("gaussian", values.numpy(), conics.numpy()),
          RTOL, ATOL_FWD, "sampler forward after re-binning")


def test_step_cache_rows_and_identity(dgs, oracle):
    """The torch extension's per-step shortcuts (dgs_sample_options): a forward whose inputs are
    the binned tensor objects skips the device-side comparison, and its packed Gaussian rows are
    reused by the backward.  Checked: autograd forward + backward; a second step after in-place
    updates of values and means (version counters bumped: rows repacked, the call-time path
    taken); two backward calls after one forward (the second repacks)."""
    P, N, D, C = 2500, 12000, 2, 1
    means, values, covs, conics, samples = _problem(P, N, D, C, seed=461)
    dev = torch.device("cuda:0")
    m = torch.nn.Parameter(means.to(dev))
    v = torch.nn.Parameter(values.to(dev))
    cv, c, s = (t.to(dev) for t in (covs, conics, samples))
    dL = syn.grad_out(N, 1, C, seed=463)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    sampler = dgs.GaussianSampler(False)
    sampler.preprocess(m, v, cv, c, s)
    out = sampler.sample_gaussians()
    (out * dL.to(dev).reshape(out.shape)).sum().backward()
    close(out.detach().cpu().numpy().reshape(N, 1, C), ob.forward("gaussian", values.numpy(), conics.numpy()),
          RTOL, ATOL_FWD, "step 1 forward")
    dm, dv, dc = ob.backward("gaussian", values.numpy(), conics.numpy(), dL.numpy(), exact=True)
    close(m.grad.cpu().numpy(), dm, RTOL, ATOL_BWD, "step 1 dL/dmeans")
    close(v.grad.cpu().numpy(), dv, RTOL, ATOL_BWD, "step 1 dL/dvalues")
    # in-place updates without re-binning: values (rows repacked) and means (call-time path)
    with torch.no_grad():
        v.mul_(1.5)
        m.add_(0.001)
    m.grad = v.grad = None
    out = sampler.sample_gaussians()
    (out * dL.to(dev).reshape(out.shape)).sum().backward()
    v1, m1 = v.detach().cpu().numpy(), m.detach().cpu().numpy()
    close(out.detach().cpu().numpy().reshape(N, 1, C), ob.forward("gaussian", v1, conics.numpy(), means=m1),
          RTOL, ATOL_FWD, "step 2 forward (values and means updated in place)")
    dm, dv, dc = ob.backward("gaussian", v1, conics.numpy(), dL.numpy(), means=m1, exact=True)
    close(m.grad.cpu().numpy(), dm, RTOL, ATOL_BWD, "step 2 dL/dmeans")
    close(v.grad.cpu().numpy(), dv, RTOL, ATOL_BWD, "step 2 dL/dvalues")
    # raw _C: one forward (rows kept: values requires grad), two backwards
    sampler.preprocess(m, v, cv, c, s)
    args = (m, v, c, s, sampler.num_rendered)
    bufs = (sampler.binning_buffer, sampler.sample_binning_buffer, sampler.ranges, sampler.sample_ranges)
    with torch.no_grad():
        dgs._C.sample_gaussians(*args, *bufs, False)
        g1 = dgs._C.sample_gaussians_backward(*args, dL.to(dev).reshape(N, 1), *bufs, False)
        g2 = dgs._C.sample_gaussians_backward(*args, dL.to(dev).reshape(N, 1), *bufs, False)
    ob2 = oracle.OracleBins(m1, covs.numpy(), samples.numpy())
    dm, dv, dc = ob2.backward("gaussian", v1, conics.numpy(), dL.numpy(), exact=True)
    for k, g in enumerate((g1, g2)):
        close(g[0].cpu().numpy(), dm, RTOL, ATOL_BWD, f"backward {k} dL/dmeans")
        close(g[1].cpu().numpy(), dv, RTOL, ATOL_BWD, f"backward {k} dL/dvalues")
        close(g[2].cpu().numpy(), dc, RTOL, ATOL_BWD, f"backward {k} dL/dconics")


@pytest.mark.parametrize("function", ["gaussian", "derivative"])
@pytest.mark.parametrize("D", [1, 2])
def test_seam_means_moved(dgs, oracle, function, D):
    """Means near the torus seams moved in place (some across x = +-1): the stale tile lists hold
    Gaussians that reach a tile through the torus (wrapped rect keys), and the call-time cull
    tests them after the reference's constant wrap shift over the unit's box (ref_may_touch)."""
    import cases
    pre = cases.seam_case(D=D)
    g = torch.Generator().manual_seed(432)
    P = pre[0].shape[0]
    step = (torch.randn(P, D, generator=g) * 0.02).float()
    call = (pre[0] + step, pre[1], pre[2], pre[3], pre[4])
    N = pre[4].shape[0]
    dL = syn.grad_out(N, syn.out_components(function, D), pre[1].shape[1], seed=433)
    assert not _run(dgs, oracle, function, pre, call, dL)

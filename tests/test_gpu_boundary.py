"""The C-ABI boundary's promises on the GPU (include/dgs.h):
  * the binning / sampling hot path allocates no device memory on its own: a thin-field
    preprocess + forward + backward through ctypes, with a counting allocation callback, leaves
    dgs_internal_allocations() unchanged (the backward's slot sums live in the caller's workspace,
    sized by dgs_sample_workspace_size_binned; a plain-size workspace takes the atomics);
  * torch.inference_mode() tensors work (no version counters: the device-side check runs);
  * writes that bypass autograd's version counter (tensor.data) are missed by the torch layer's
    DGS_SAMPLE_INPUTS_BINNED shortcut and caught with debug=True (which always verifies).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

import cases
from diff_gaussian_sampling import synthetic as syn
from helpers import close

pytestmark = pytest.mark.gpu

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "diff-gaussian-sampling_amd",
                    "diff_gaussian_sampling", "libdgs.so")
_P, _I, _I64, _SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t)


class Opts(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint32)]


def _lib():
    lib = ctypes.CDLL(os.path.abspath(_LIB))
    lib.dgs_last_error.restype = ctypes.c_char_p
    lib.dgs_internal_allocations.restype = _I64
    lib.dgs_preprocess.argtypes = [_I, _I, _I, _P, _P, _P, _P, _P, _P, _P, ALLOC_FN, _P, ctypes.POINTER(_I64), _P, _I]
    lib.dgs_sample_workspace_size.restype = _SZ
    lib.dgs_sample_workspace_size.argtypes = [_I] * 6
    lib.dgs_sample_workspace_size_binned.restype = _SZ
    lib.dgs_sample_workspace_size_binned.argtypes = [_I] * 6 + [_P, _SZ, _P, _SZ]
    lib.dgs_sample_forward_ex.argtypes = [_I] * 5 + [_P] * 4 + [_P, _SZ, _P, _SZ, _P, _P, _SZ, _P, _P, _I]
    lib.dgs_sample_backward_ex.argtypes = [_I] * 5 + [_P] * 5 + [_P, _SZ, _P, _SZ, _P, _P, _P, _P, _SZ, _P, _P, _I]
    lib.dgs_binning_info.argtypes = [_P, _SZ, _P, _SZ, _P]
    return lib


def _ok(lib, rc):
    assert rc == 0, lib.dgs_last_error().decode()


def test_no_internal_allocation_thin_field(oracle):
    lib = _lib()
    dev = torch.device("cuda:0")
    means, values, covs, conics, samples = cases.thin_case(P=20000, n=80000)
    m, v, cv, c, s = (t.to(dev).contiguous() for t in (means, values, covs, conics, samples))
    P, D, N, C = m.shape[0], 2, s.shape[0], 1
    grid, off = oracle.tile_grid(samples.numpy())  # (dgs_tile_grid has scratch of its own: dgs.h)
    held, requests = {}, []

    def alloc(ctx, which, nbytes):
        t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
        held.setdefault(which, []).append(t)
        requests.append((which, int(nbytes)))
        return t.data_ptr()

    cb = ALLOC_FN(alloc)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    radii = torch.zeros(P, device=dev)
    R = ctypes.c_int64(0)
    g = (ctypes.c_int * 2)(*[int(x) for x in grid])
    o = (ctypes.c_float * 2)(*[float(x) for x in off])
    before = lib.dgs_internal_allocations()
    _ok(lib, lib.dgs_preprocess(P, D, N, m.data_ptr(), cv.data_ptr(), c.data_ptr(), s.data_ptr(), g, o,
                                radii.data_ptr(), cb, None, ctypes.byref(R), stream, 0))
    assert requests, "the binning's buffers come from the callback"
    gb, sb = held[0][-1], held[1][-1]
    info = (ctypes.c_int64 * 6)()
    _ok(lib, lib.dgs_binning_info(gb.data_ptr(), gb.numel(), sb.data_ptr(), sb.numel(), info))
    plain = lib.dgs_sample_workspace_size(0, P, D, N, C, 1)
    binned = lib.dgs_sample_workspace_size_binned(1, P, D, N, C, 1, gb.data_ptr(), gb.numel(), sb.data_ptr(),
                                                  sb.numel())
    assert binned > plain, "a thin field's binning wants the slot-sum region"
    opts = Opts(1)  # DGS_SAMPLE_INPUTS_BINNED
    out = torch.zeros(N, 1, device=dev)
    outs = (ctypes.c_void_p * 4)(out.data_ptr(), None, None, None)
    ws = torch.empty(binned, dtype=torch.uint8, device=dev)
    _ok(lib, lib.dgs_sample_forward_ex(1, P, D, N, C, m.data_ptr(), v.data_ptr(), c.data_ptr(), s.data_ptr(),
                                       gb.data_ptr(), gb.numel(), sb.data_ptr(), sb.numel(), outs, ws.data_ptr(),
                                       ws.numel(), ctypes.byref(opts), stream, 0))
    dL = syn.grad_out(N, 1, 1, seed=9).to(dev)
    dls = (ctypes.c_void_p * 4)(dL.data_ptr(), None, None, None)
    grads = {}
    for name, size in (("slots", binned), ("atomics", plain)):
        ws = torch.empty(size, dtype=torch.uint8, device=dev)
        gm, gv, gc = torch.empty(P, 2, device=dev), torch.empty(P, 1, device=dev), torch.empty(P, 3, device=dev)
        _ok(lib, lib.dgs_sample_backward_ex(1, P, D, N, C, m.data_ptr(), v.data_ptr(), c.data_ptr(), s.data_ptr(),
                                            dls, gb.data_ptr(), gb.numel(), sb.data_ptr(), sb.numel(), gm.data_ptr(),
                                            gv.data_ptr(), gc.data_ptr(), ws.data_ptr(), ws.numel(),
                                            ctypes.byref(opts), stream, 0))
        grads[name] = (gm, gv, gc)
    torch.cuda.synchronize()
    assert lib.dgs_internal_allocations() == before, "the hot path allocated on its own"
    n_req = len(requests)
    for a, b in zip(grads["slots"], grads["atomics"]):  # two summation orders of the same terms
        a, b = a.cpu().numpy(), b.cpu().numpy()
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6 * float(np.abs(b).max()))
    assert len(requests) == n_req  # forward / backward never call back


def test_inference_mode(dgs, oracle):
    """preprocess + forward under torch.inference_mode() (version counters of
    inference tensors), against the oracle; and the aggregation's preprocess + forward."""
    dev = torch.device("cuda:0")
    means, values, covs, conics = syn.gaussians(1500, 2, 1, seed=201)
    samples = syn.samples(6000, 2, seed=202)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    with torch.inference_mode():
        m, v, cv, c, s = (t.to(dev) for t in (means, values, covs, conics, samples))
        sampler = dgs.GaussianSampler(False)
        sampler.preprocess(m, v, cv, c, s)
        for fn in ("gaussian", "derivative"):
            out = (sampler.sample_gaussians() if fn == "gaussian" else sampler.sample_gaussians_derivative())
            ref = ob.forward(fn, values.numpy(), conics.numpy()).reshape(out.shape)
            close(out.cpu().numpy(), ref, 1e-5, 1e-6, f"inference-mode {fn}")
        # a second call on the same binning, and an in-place step (must be seen: device-side check)
        m.add_(0.001)
        out = sampler.sample_gaussians()
        ref = ob.forward("gaussian", values.numpy(), conics.numpy(), means=(means + 0.001).numpy()).reshape(out.shape)
        close(out.cpu().numpy(), ref, 1e-5, 1e-6, "inference-mode after an in-place step")
        sampler.preprocess_aggregate()
        assert sampler.indices.numel() > 0
        g = torch.Generator().manual_seed(5)
        feats = [torch.randn(1500, 8, generator=g), torch.randn(8, 8, generator=g) / 8, torch.randn(1500, 8, generator=g),
                 torch.randn(1500, 8, generator=g), torch.rand(3, generator=g) + 0.5,
                 torch.randn(2 * (4 * 3 + 1), generator=g)]
        a = sampler.aggregate_neighbors(*[t.to(dev) for t in feats])
        assert torch.isfinite(a).all()


def test_data_write_missed_without_verify_caught_with_debug(dgs, oracle):
    """the torch layer trusts tensor identity + version counters
    (DGS_SAMPLE_INPUTS_BINNED).  A write through .data bypasses the counter: the default call
    then reads the binned copies (the stale means), while debug=True always runs the device-side
    comparison and takes the reference's call-time path with the written means
    (forward.cu:136-145).  INTEGRATION.md documents this."""
    dev = torch.device("cuda:0")
    means, values, covs, conics = syn.gaussians(1500, 2, 1, seed=211)
    samples = syn.samples(6000, 2, seed=212)
    m, v, cv, c, s = (t.to(dev) for t in (means, values, covs, conics, samples))
    R, gb, sb, rg, srg, _ = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
    m.data.add_(0.002)  # no version bump
    stale = dgs._C.sample_gaussians(m, v, c, s, R, gb, sb, rg, srg, False)
    fresh = dgs._C.sample_gaussians(m, v, c, s, R, gb, sb, rg, srg, True)
    ob = oracle.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    ref_old = ob.forward("gaussian", values.numpy(), conics.numpy()).reshape(stale.shape)
    ref_new = ob.forward("gaussian", values.numpy(), conics.numpy(), means=(means + 0.002).numpy()).reshape(stale.shape)
    close(stale.cpu().numpy(), ref_old, 1e-5, 1e-6, "the .data write is missed (binned copies)")
    close(fresh.cpu().numpy(), ref_new, 1e-5, 1e-6, "debug=True catches it (call-time path)")


def test_allreduce_grads_one_rank_communicator():
    """dgs_allreduce_grads through ctypes on a 1-rank RCCL communicator made by
    dgs_comm_init: the sum over one rank is the input, whole and in chunks; the call is
    asynchronous on the stream.  (More ranks need more GPUs: the driver's multi-GPU bench runs
    the torch.distributed path.)"""
    lib = _lib()
    lib.dgs_comm_id_bytes.restype = _SZ
    lib.dgs_comm_unique_id.argtypes = [_P]
    lib.dgs_comm_init.argtypes = [ctypes.POINTER(_P), _I, _P, _I]
    lib.dgs_comm_destroy.argtypes = [_P]
    lib.dgs_allreduce_grads.argtypes = [_P, _SZ, _P, _SZ, _P]
    uid = ctypes.create_string_buffer(int(lib.dgs_comm_id_bytes()))
    _ok(lib, lib.dgs_comm_unique_id(uid))
    comm = _P()
    torch.cuda.set_device(0)
    _ok(lib, lib.dgs_comm_init(ctypes.byref(comm), 1, uid, 0))
    try:
        g = torch.randn(1_000_003, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
        ref = g.clone()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for chunk in (0, 65536):
            _ok(lib, lib.dgs_allreduce_grads(g.data_ptr(), g.numel(), comm, chunk, stream))
            torch.cuda.synchronize()
            assert torch.equal(g, ref)
    finally:
        _ok(lib, lib.dgs_comm_destroy(comm))

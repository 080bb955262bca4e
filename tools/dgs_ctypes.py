"""ctypes binding of libdgs.so (include/dgs.h) exposing the reference's `_C` surface.

This is the binding a maintainer of kr4b/diff-gaussian-sampling would add in place of the
CUDA extension (`diff_gaussian_sampling/_C`, ext.cpp:20-31) when the torch C++ extension
cannot be built: it needs only ctypes, torch tensors for memory, and libdgs.so.  Install it as
`diff_gaussian_sampling/_C.py` (or `sys.modules["diff_gaussian_sampling._C"] = dgs_ctypes`)
and the reference's Python layer runs unchanged.  tests/test_gpu_ctypes.py checks it against
the compiled extension.

Every function takes and returns torch tensors exactly as the reference's `_C` does.  Device
memory comes from torch (the allocation callback hands out uint8 tensors that this module keeps
alive and returns); kernels run on torch's current stream.
"""
import ctypes
import os

import torch

_LIB_PATH = os.environ.get("DGS_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..", "diff-gaussian-sampling_amd",
    "diff_gaussian_sampling", "libdgs.so")
_lib = ctypes.CDLL(os.path.abspath(_LIB_PATH))

_P, _I, _I64, _SZ, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t)
_lib.dgs_last_error.restype = ctypes.c_char_p
_lib.dgs_tile_grid.argtypes = [_I, _I, _P, _P, _P, _P]
_lib.dgs_preprocess.argtypes = [_I, _I, _I, _P, _P, _P, _P, _P, _P, _P, ALLOC_FN, _P,
                                ctypes.POINTER(_I64), _P, _I]
_lib.dgs_sample_workspace_size.restype = _SZ
_lib.dgs_sample_workspace_size.argtypes = [_I] * 6
_lib.dgs_sample_forward.argtypes = [_I] * 5 + [_P] * 4 + [_P, _SZ, _P, _SZ, _P, _P, _SZ, _P, _I]
_lib.dgs_sample_backward.argtypes = [_I] * 5 + [_P] * 5 + [_P, _SZ, _P, _SZ, _P, _P, _P, _P, _SZ, _P, _I]

FUNCTIONS = {"sample_gaussians": 0, "sample_gaussians_derivative": 1,
             "sample_gaussians_laplacian": 2, "sample_gaussians_third_derivative": 3}


def _check(rc):
    if rc != 0:
        raise RuntimeError(_lib.dgs_last_error().decode())


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _f32(t):
    if t.dtype != torch.float32:
        raise RuntimeError("expected float32 tensors")
    return t.contiguous()


def preprocess_gaussians(means, values, covariances, conics, samples, debug):
    """sample_points.h:20-27 -> (num_rendered, binning, sample_binning, ranges, sample_ranges, radii)."""
    means, covariances, conics, samples = map(_f32, (means, covariances, conics, samples))
    P, D = means.shape
    N = samples.shape[0]
    dev = means.device
    radii = torch.zeros(P, device=dev)
    buffers = {}

    def alloc(ctx, which, nbytes):  # DGS_BUF_* -> device memory owned by torch
        t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
        buffers.setdefault(which, []).append(t)
        return t.data_ptr()

    cb = ALLOC_FN(alloc)
    grid = (ctypes.c_int * 2)()
    off = (ctypes.c_float * 2)()
    if N > 0:
        _check(_lib.dgs_tile_grid(N, D, _ptr(samples), grid, off, _stream()))
    R = ctypes.c_int64(0)
    _check(_lib.dgs_preprocess(P, D, N, _ptr(means), _ptr(covariances), _ptr(conics),
                               _ptr(samples), grid, off, _ptr(radii), cb, None,
                               ctypes.byref(R), _stream(), int(bool(debug))))
    empty = torch.empty(0, dtype=torch.uint8, device=dev)
    get = lambda k: buffers[k][-1] if k in buffers else empty
    return R.value, get(0), get(1), get(2), get(3), radii


def _forward(name, means, values, conics, samples, num_rendered, binning, sample_binning,
             ranges, sample_ranges, debug):
    means, values, conics, samples = map(_f32, (means, values, conics, samples))
    fn = FUNCTIONS[name]
    P, D = means.shape
    N, C = samples.shape[0], values.shape[1]
    out = torch.zeros((N,) + (D,) * fn + (C,), device=means.device)
    ws = torch.empty(_lib.dgs_sample_workspace_size(fn, P, D, N, C, 0), dtype=torch.uint8,
                     device=means.device)
    _check(_lib.dgs_sample_forward(fn, P, D, N, C, _ptr(means), _ptr(values), _ptr(conics),
                                   _ptr(samples), _ptr(binning), binning.numel(),
                                   _ptr(sample_binning), sample_binning.numel(), _ptr(out),
                                   _ptr(ws), ws.numel(), _stream(), int(bool(debug))))
    return out


def _backward(name, means, values, conics, samples, num_rendered, dL_dout, binning,
              sample_binning, ranges, sample_ranges, debug):
    means, values, conics, samples, dL_dout = map(_f32, (means, values, conics, samples, dL_dout))
    fn = FUNCTIONS[name]
    P, D = means.shape
    N, C = samples.shape[0], values.shape[1]
    S = D * (D + 1) // 2
    dm = torch.zeros(P, D, device=means.device)
    dv = torch.zeros(P, C, device=means.device)
    dc = torch.zeros(P, S, device=means.device)
    ws = torch.empty(_lib.dgs_sample_workspace_size(fn, P, D, N, C, 1), dtype=torch.uint8,
                     device=means.device)
    _check(_lib.dgs_sample_backward(fn, P, D, N, C, _ptr(means), _ptr(values), _ptr(conics),
                                    _ptr(samples), _ptr(dL_dout), _ptr(binning), binning.numel(),
                                    _ptr(sample_binning), sample_binning.numel(), _ptr(dm),
                                    _ptr(dv), _ptr(dc), _ptr(ws), ws.numel(), _stream(),
                                    int(bool(debug))))
    return dm, dv, dc


def _make(name):
    fwd = lambda *a: _forward(name, *a)
    bwd = lambda *a: _backward(name, *a)
    fwd.__name__, bwd.__name__ = name, name + "_backward"
    return fwd, bwd


sample_gaussians, sample_gaussians_backward = _make("sample_gaussians")
sample_gaussians_derivative, sample_gaussians_derivative_backward = _make("sample_gaussians_derivative")
sample_gaussians_laplacian, sample_gaussians_laplacian_backward = _make("sample_gaussians_laplacian")
sample_gaussians_third_derivative, sample_gaussians_third_derivative_backward = _make(
    "sample_gaussians_third_derivative")



# ---- fused functions (dgs_sample_{forward,backward}_multi; not on the reference API) --------
_lib.dgs_sample_workspace_size_multi.restype = _SZ
_lib.dgs_sample_workspace_size_multi.argtypes = [_I] * 6
_PP = ctypes.c_void_p * 4
_lib.dgs_sample_forward_multi.argtypes = [_I] * 5 + [_P] * 4 + [_P, _SZ, _P, _SZ, _PP, _P, _SZ, _P, _I]
_lib.dgs_sample_backward_multi.argtypes = [_I] * 5 + [_P] * 4 + [_PP, _P, _SZ, _P, _SZ, _P, _P, _P, _P, _SZ, _P, _I]


def sample_gaussians_multi(codes, means, values, conics, samples, binning, sample_binning, debug):
    """Outputs of the functions `codes` (0..3, each once; D = 2, C = 1 for two or more) in one
    traversal of the pairs, in the order given."""
    means, values, conics, samples = map(_f32, (means, values, conics, samples))
    P, D = means.shape
    N, C = samples.shape[0], values.shape[1]
    mask = sum(1 << c for c in codes)
    outs = {c: torch.zeros((N,) + (D,) * c + (C,), device=means.device) for c in codes}
    ptrs = _PP(*[outs[c].data_ptr() if c in outs else None for c in range(4)])
    ws = torch.empty(_lib.dgs_sample_workspace_size_multi(mask, P, D, N, C, 0), dtype=torch.uint8,
                     device=means.device)
    _check(_lib.dgs_sample_forward_multi(mask, P, D, N, C, _ptr(means), _ptr(values), _ptr(conics),
                                         _ptr(samples), _ptr(binning), binning.numel(),
                                         _ptr(sample_binning), sample_binning.numel(), ptrs,
                                         _ptr(ws), ws.numel(), _stream(), int(bool(debug))))
    return [outs[c] for c in codes]


def sample_gaussians_multi_backward(codes, means, values, conics, samples, dLs, binning,
                                    sample_binning, debug):
    """Gradients of sum_f <dLs[f], out_f> for the functions `codes`."""
    means, values, conics, samples = map(_f32, (means, values, conics, samples))
    dLs = {c: _f32(d) for c, d in zip(codes, dLs)}
    P, D = means.shape
    N, C = samples.shape[0], values.shape[1]
    mask = sum(1 << c for c in codes)
    dm = torch.zeros(P, D, device=means.device)
    dv = torch.zeros(P, C, device=means.device)
    dc = torch.zeros(P, D * (D + 1) // 2, device=means.device)
    ptrs = _PP(*[dLs[c].data_ptr() if c in dLs else None for c in range(4)])
    ws = torch.empty(_lib.dgs_sample_workspace_size_multi(mask, P, D, N, C, 1), dtype=torch.uint8,
                     device=means.device)
    _check(_lib.dgs_sample_backward_multi(mask, P, D, N, C, _ptr(means), _ptr(values), _ptr(conics),
                                          _ptr(samples), ptrs, _ptr(binning), binning.numel(),
                                          _ptr(sample_binning), sample_binning.numel(), _ptr(dm),
                                          _ptr(dv), _ptr(dc), _ptr(ws), ws.numel(), _stream(),
                                          int(bool(debug))))
    return dm, dv, dc

# ---- neighbour aggregation (aggregate_neighbors.h:11-47) ---------------------------------
_lib.dgs_agg_preprocess.argtypes = [_I, _I, _P, _P, _P, _P, _P, _P, ALLOC_FN, _P, ctypes.POINTER(_I64), _P, _I]
_lib.dgs_agg_forward.argtypes = [_I] * 5 + [_P] * 11 + [_P] + [_P] * 4 + [_P, _I]
_lib.dgs_agg_backward.argtypes = [_I] * 5 + [_P] * 14 + [_P] + [_P] * 7 + [_P, _SZ, _P, _I]
_lib.dgs_agg_workspace_size.restype = _SZ
_lib.dgs_agg_workspace_size.argtypes = [_I, _I]
_lib.dgs_agg_transpose.argtypes = [_I, _I64, _P, _P, _P, _P, _P, _P, ALLOC_FN, _P, _P, _I]
_lib.dgs_agg_workspace_size_tr.restype = _SZ
_lib.dgs_agg_workspace_size_tr.argtypes = [_I, _I, _I64]
_lib.dgs_agg_backward_tr.argtypes = [_I] * 5 + [_P] * 14 + [_P] + [_P, _P, _P, _I64] + [_P] * 7 + [_P, _SZ, _P, _I]
_orders = {}  # indices data_ptr -> (P, row order tensor): the scheduling hint of dgs_agg_preprocess


def _i64(t):
    if t.dtype != torch.int64:
        raise RuntimeError("expected int64 tensors")
    return t.contiguous()


def preprocess_aggregate(means, conics, radii, debug):
    """aggregate_neighbors.h:11-15 -> (indices, ranges, dists, densities, inv_total_densities)."""
    means, conics, radii = map(_f32, (means, conics, radii))
    P, D = means.shape
    dev = means.device
    ranges = torch.zeros(P, dtype=torch.int64, device=dev)
    inv = torch.zeros(P, device=dev)
    order = torch.empty(P, dtype=torch.int32, device=dev)
    buffers = {}

    def alloc(ctx, which, nbytes):
        t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
        buffers.setdefault(which, []).append(t)
        return t.data_ptr()

    length = ctypes.c_int64(0)
    if P > 0:
        _check(_lib.dgs_agg_preprocess(P, D, _ptr(means), _ptr(conics), _ptr(radii), _ptr(ranges), _ptr(inv),
                                       _ptr(order), ALLOC_FN(alloc), None, ctypes.byref(length), _stream(),
                                       int(bool(debug))))
    n = length.value
    if n == 0:
        return (torch.empty(0, dtype=torch.int64, device=dev), ranges, torch.empty(0, D, device=dev),
                torch.empty(0, device=dev), inv)
    indices = buffers[5][-1].view(torch.int64)[:n]
    _orders.clear()
    _orders[indices.data_ptr()] = (P, order)
    return (indices, ranges, buffers[6][-1].view(torch.float32)[:n * D].view(n, D),
            buffers[7][-1].view(torch.float32)[:n], inv)


def _agg_sizes(features, queries, distance_transform, dists):
    return (features.shape[0], dists.shape[-1] if dists.dim() == 2 else 1, features.shape[-1],
            queries.shape[-1], distance_transform.shape[-1] // 2)


def _order(indices, P):
    e = _orders.get(indices.data_ptr())
    return e[1] if e is not None and e[0] == P else None


def aggregate_neighbors(features, transform, queries, keys, frequencies, distance_transform, indices, ranges,
                        dists, densities, inv_total_densities, debug):
    """aggregate_neighbors.h:17-29 -> (weights, embeddings, factors, neighbor_features)."""
    f, T, q, k, fr, dt, X, dn, inv = map(_f32, (features, transform, queries, keys, frequencies,
                                               distance_transform, dists, densities, inv_total_densities))
    idx, rg = _i64(indices), _i64(ranges)
    P, D, L, K, E = _agg_sizes(f, q, dt, X)
    w, e, fa = (torch.zeros_like(dn) for _ in range(3))
    out = torch.zeros(P, L, device=f.device)
    _check(_lib.dgs_agg_forward(P, D, L, K, E, _ptr(f), _ptr(T), _ptr(q), _ptr(k), _ptr(fr), _ptr(dt), _ptr(idx),
                                _ptr(rg), _ptr(X), _ptr(dn), _ptr(inv), _ptr(_order(idx, P)), _ptr(w), _ptr(e),
                                _ptr(fa), _ptr(out), _stream(), int(bool(debug))))
    return w, e, fa, out


def aggregate_neighbors_backward(features, transform, queries, keys, frequencies, distance_transform, indices,
                                 ranges, dists, densities, weights, embeddings, factors, inv_total_densities,
                                 dL_dneighbor_features, debug, transposed=True):
    """aggregate_neighbors.h:31-47 -> the six gradients (transposed: dgs_agg_transpose +
    dgs_agg_backward_tr, as the extension does for L + K <= 64; else dgs_agg_backward)."""
    f, T, q, k, fr, dt, X, dn, w, e, fa, inv, g = map(
        _f32, (features, transform, queries, keys, frequencies, distance_transform, dists, densities, weights,
               embeddings, factors, inv_total_densities, dL_dneighbor_features))
    idx, rg = _i64(indices), _i64(ranges)
    P, D, L, K, E = _agg_sizes(f, q, dt, X)
    outs = [torch.zeros_like(t) for t in (f, T, q, k, fr, dt)]
    n = idx.numel()
    if transposed and P > 0 and L + K <= 64:
        # the transposed lists (dgs_agg_transpose), then the gather form of the backward
        tstart = torch.empty(P + 1, dtype=torch.int32, device=f.device)
        tslot = torch.empty(max(n, 1), dtype=torch.int32, device=f.device)
        keep = []

        def alloc(ctx, which, nbytes):
            t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=f.device)
            keep.append(t)
            return t.data_ptr()

        rstart = torch.empty(P, dtype=torch.int32, device=f.device)
        order = _order(idx, P)
        _check(_lib.dgs_agg_transpose(P, n, _ptr(idx), _ptr(rg), _ptr(order), _ptr(tstart), _ptr(tslot), _ptr(rstart),
                                      ALLOC_FN(alloc), None, _stream(), int(bool(debug))))
        ws = torch.empty(_lib.dgs_agg_workspace_size_tr(P, L, n), dtype=torch.uint8, device=f.device)
        _check(_lib.dgs_agg_backward_tr(P, D, L, K, E, _ptr(f), _ptr(T), _ptr(q), _ptr(k), _ptr(fr), _ptr(dt),
                                        _ptr(idx), _ptr(rg), _ptr(X), _ptr(dn), _ptr(w), _ptr(e), _ptr(fa), _ptr(inv),
                                        _ptr(order), _ptr(tstart), _ptr(tslot), _ptr(rstart), n, _ptr(g),
                                        *[_ptr(o) for o in outs], _ptr(ws), ws.numel(), _stream(), int(bool(debug))))
        return tuple(outs)
    ws = torch.empty(_lib.dgs_agg_workspace_size(P, L), dtype=torch.uint8, device=f.device)
    _check(_lib.dgs_agg_backward(P, D, L, K, E, _ptr(f), _ptr(T), _ptr(q), _ptr(k), _ptr(fr), _ptr(dt), _ptr(idx),
                                 _ptr(rg), _ptr(X), _ptr(dn), _ptr(w), _ptr(e), _ptr(fa), _ptr(inv),
                                 _ptr(_order(idx, P)), _ptr(g), *[_ptr(o) for o in outs], _ptr(ws), ws.numel(),
                                 _stream(), int(bool(debug))))
    return tuple(outs)

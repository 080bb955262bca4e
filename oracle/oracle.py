"""ctypes wrapper around oracle/_build/liboracle.so -- the CPU restatement of the reference.

TEST INFRASTRUCTURE ONLY (see oracle.c header): imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, never by the product package.

Parity status: "parity unpinned" -- no reference outputs exist (see oracle.c).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FMA contraction models (oracle.c header, oracle/Makefile): "nocontract" is the model the GPU
# path and the parity tests are built against; "fmad" / "fmad_alt" model nvcc's default
# --fmad=true (the reference's setup.py:30 sets no --fmad=false) with the two fusing choices at
# a*b + c*d sites.
MODELS = {"nocontract": "liboracle.so", "fmad": "liboracle_fmad.so", "fmad_alt": "liboracle_fmad_alt.so"}
_LIB_PATH = os.path.join(_HERE, "_build", MODELS["nocontract"])
_lib = None
_libs = {}

FUNCTIONS = {"gaussian": 0, "derivative": 1, "laplacian": 2, "third": 3}


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load(model="nocontract"):
    global _lib
    if model in _libs:
        return _libs[model]
    path = os.path.join(_HERE, "_build", MODELS[model])
    if not os.path.exists(path):
        build()
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    i32, i64 = ctypes.c_int, ctypes.c_int64
    lib.orc_bin.restype = P
    lib.orc_bin.argtypes = [i32, i32, i32, P, P, P, P, P, P]
    lib.orc_free.argtypes = [P]
    lib.orc_T.argtypes = [P]
    lib.orc_R.argtypes = [P]
    lib.orc_R.restype = i64
    lib.orc_grid.argtypes = [P, P, P]
    lib.orc_ranges.argtypes = [P, P, P]
    lib.orc_sample_keys.argtypes = [P, P]
    lib.orc_tile_gaussians.argtypes = [P, i32, P]
    lib.orc_tile_gaussians.restype = i64
    lib.orc_forward.argtypes = [P, i32, i32, P, P, P, P, P, i32, P]
    lib.orc_backward.argtypes = [P, i32, i32, P, P, P, P, P, P, P, P, i32, P]
    lib.orc_backward64.argtypes = [P, i32, i32, P, P, P, P, P, P, P, P, i32, P]
    lib.orc_forward_bound.argtypes = [P, i32, i32, P, P, P, P, P, i32, P]
    lib.orc_backward_bound.argtypes = [P, i32, i32, P, P, P, P, P, P, P, P, i32, P]
    lib.orc_count_pairs.argtypes = [P, P, P, P, ctypes.c_double, i32, P, P, P]
    lib.orc_tile_grid.argtypes = [i32, i32, P, P, P]
    lib.orc_agg_counts.argtypes = [i32, i32, P, P, P]
    lib.orc_agg_fill.argtypes = [i32, i32, P, P, P, P, P, P, P, P]
    lib.orc_agg_counts_rows.argtypes = [i32, i32, P, P, i32, P, P]
    lib.orc_agg_fill_rows.argtypes = [i32, i32, P, P, P, i32, P, P, P, P, P, P]
    lib.orc_agg_forward.argtypes = [i32] * 5 + [P] * 15
    lib.orc_agg_backward.argtypes = [i32] * 5 + [P] * 21
    lib.orc_agg_forward64.argtypes = [i32] * 5 + [P] * 15
    lib.orc_agg_backward64.argtypes = [i32] * 5 + [P] * 21
    lib.orc_fmad_model.restype = i32
    _libs[model] = lib
    if model == "nocontract":
        _lib = lib
    return lib


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def out_components(function, D):
    return D ** FUNCTIONS[function]


def tile_grid(samples):
    lib = _load()
    s = _f32(samples)
    N, D = s.shape
    grid = np.zeros(2, np.int32)
    off = np.zeros(2, np.float32)
    lib.orc_tile_grid(N, D, _ptr(s), _ptr(grid), _ptr(off))
    return grid[:D].copy(), off[:D].copy()


class OracleBins:
    """Reference binning (sample_points.cu:38-98, sampler_impl.cu:216-330) on the CPU."""

    def __init__(self, means, covariances, samples, grid=None, offset=None, model="nocontract"):
        self.model = model
        lib = self._lib = _load(model)
        self.means = _f32(means)
        self.covariances = _f32(covariances)
        self.samples = _f32(samples)
        self.P, self.D = self.means.shape
        self.N = self.samples.shape[0]
        self.radii = np.zeros(self.P, np.float32)
        g = o = None
        if grid is not None:
            g = np.zeros(2, np.int32)
            g[: len(grid)] = grid
            o = np.zeros(2, np.float32)
            o[: len(offset)] = offset
        self._h = lib.orc_bin(self.P, self.D, self.N, _ptr(self.means), _ptr(self.covariances),
                              _ptr(self.samples), _ptr(g), _ptr(o), _ptr(self.radii))
        if not self._h:
            raise MemoryError("orc_bin failed")
        self.T = lib.orc_T(self._h)
        self.num_rendered = int(lib.orc_R(self._h))
        grid2 = np.zeros(2, np.int32)
        off2 = np.zeros(2, np.float32)
        lib.orc_grid(self._h, _ptr(grid2), _ptr(off2))
        self.grid = grid2[: self.D].copy()
        self.offset = off2[: self.D].copy()

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and getattr(self, "_lib", None) is not None:
            try:
                self._lib.orc_free(h)
            except Exception:  # interpreter shutdown
                pass

    def ranges(self):
        r = np.zeros(2 * self.T, np.uint32)
        s = np.zeros(2 * self.T, np.uint32)
        self._lib.orc_ranges(self._h, _ptr(r), _ptr(s))
        return r.reshape(self.T, 2), s.reshape(self.T, 2)

    def sample_keys(self):
        k = np.zeros(self.N, np.int32)
        self._lib.orc_sample_keys(self._h, _ptr(k))
        return k

    def tile_gaussians(self, t):
        n = self._lib.orc_tile_gaussians(self._h, t, None)
        out = np.zeros(max(n, 1), np.int32)
        self._lib.orc_tile_gaussians(self._h, t, _ptr(out))
        return out[:n]

    def forward(self, function, values, conics, subset=None, samples=None, means=None):
        lib = self._lib
        v = _f32(values)
        c = _f32(conics)
        m = self.means if means is None else _f32(means)
        s = self.samples if samples is None else _f32(samples)
        C = v.shape[1]
        K = out_components(function, self.D)
        out = np.zeros((self.N, K, C), np.float32)
        sub = None if subset is None else np.ascontiguousarray(subset, dtype=np.int32)
        lib.orc_forward(self._h, FUNCTIONS[function], C, _ptr(m), _ptr(v), _ptr(c), _ptr(s),
                        _ptr(out), 0 if sub is None else len(sub), _ptr(sub))
        return out

    def backward(self, function, values, conics, dL_dout, subset=None, samples=None, means=None, exact=False):
        """backward.cu:26-106.  exact=False: the float sums in serial order (one of the reference's
        atomic orders); exact=True: the same float per-pair terms summed in double (float64 arrays),
        the value every atomic order scatters around -- the GPU parity tests' reference."""
        lib = self._lib
        v = _f32(values)
        c = _f32(conics)
        m = self.means if means is None else _f32(means)
        s = self.samples if samples is None else _f32(samples)
        C = v.shape[1]
        S = self.D * (self.D + 1) // 2
        dL = _f32(dL_dout).reshape(self.N, -1)
        ft = np.float64 if exact else np.float32
        dm = np.zeros((self.P, self.D), ft)
        dv = np.zeros((self.P, C), ft)
        dc = np.zeros((self.P, S), ft)
        sub = None if subset is None else np.ascontiguousarray(subset, dtype=np.int32)
        (lib.orc_backward64 if exact else lib.orc_backward)(self._h, FUNCTIONS[function], C, _ptr(m), _ptr(v), _ptr(c), _ptr(s),
                         _ptr(dL), _ptr(dm), _ptr(dv), _ptr(dc),
                         0 if sub is None else len(sub), _ptr(sub))
        return dm, dv, dc

    def order_bound(self, function, values, conics, dL_dout=None, subset=None):
        """The a-priori bound of the exponent's evaluation order (oracle.c orc_forward_bound /
        orc_backward_bound): per output element, sum over its pairs of |term| x
        (exp(gamma_6 M) - 1), M = 0.5|c0 X0^2| + |c1 X0 X1| + 0.5|c2 X1^2|.  Returns the forward's
        [N, K, C] bound, or with dL_dout the gradients' (dmeans, dvalues, dconics) bounds; float64."""
        lib = self._lib
        v = _f32(values)
        c = _f32(conics)
        C = v.shape[1]
        sub = None if subset is None else np.ascontiguousarray(subset, dtype=np.int32)
        ns = 0 if sub is None else len(sub)
        if dL_dout is None:
            K = out_components(function, self.D)
            out = np.zeros((self.N, K, C), np.float64)
            lib.orc_forward_bound(self._h, FUNCTIONS[function], C, _ptr(self.means), _ptr(v), _ptr(c),
                                  _ptr(self.samples), _ptr(out), ns, _ptr(sub))
            return out
        S = self.D * (self.D + 1) // 2
        dL = _f32(dL_dout).reshape(self.N, -1)
        dm = np.zeros((self.P, self.D), np.float64)
        dv = np.zeros((self.P, C), np.float64)
        dc = np.zeros((self.P, S), np.float64)
        lib.orc_backward_bound(self._h, FUNCTIONS[function], C, _ptr(self.means), _ptr(v), _ptr(c),
                               _ptr(self.samples), _ptr(dL), _ptr(dm), _ptr(dv), _ptr(dc), ns, _ptr(sub))
        return dm, dv, dc

    def count_pairs(self, conics, thr=-104.0, subset=None):
        lib = self._lib
        c = _f32(conics)
        sub = None if subset is None else np.ascontiguousarray(subset, dtype=np.int32)
        w_ref = ctypes.c_int64()
        w_live = ctypes.c_int64()
        lib.orc_count_pairs(self._h, _ptr(self.means), _ptr(c), _ptr(self.samples), thr,
                            0 if sub is None else len(sub), _ptr(sub),
                            ctypes.byref(w_ref), ctypes.byref(w_live))
        return w_ref.value, w_live.value


# ------------------------------------------------------------------ neighbour aggregation
def _i64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64))


def agg_preprocess(means, conics, radii, model="nocontract"):
    """preprocess_aggregate (aggregate_neighbors.cu:323-367): (indices i64[Lnb], ranges
    i64[P] inclusive cumsum, dists [Lnb, D], densities [Lnb], inv_total [P])."""
    lib = _load(model)
    m, c, r = _f32(means), _f32(conics), _f32(radii)
    P, D = m.shape
    counts = np.zeros(P, np.int64)
    lib.orc_agg_counts(P, D, _ptr(m), _ptr(r), _ptr(counts))
    ranges = np.cumsum(counts).astype(np.int64)
    n = int(ranges[-1]) if P else 0
    indices = np.full(n, -1, np.int64)
    dists = np.zeros((n, D), np.float32)
    dens = np.zeros(n, np.float32)
    inv = np.zeros(P, np.float32)
    lib.orc_agg_fill(P, D, _ptr(m), _ptr(c), _ptr(r), _ptr(ranges), _ptr(indices), _ptr(dists),
                     _ptr(dens), _ptr(inv))
    return indices, ranges, dists, dens, inv


def agg_preprocess_rows(means, conics, radii, rows, model="nocontract"):
    """preprocess_aggregate restricted to the rows `rows` (each an O(P) scan): compact lists
    (indices, ranges [len(rows)] inclusive cumsum, dists, densities, inv_total [len(rows)])
    equal to those rows' slices of agg_preprocess."""
    lib = _load(model)
    m, c, r = _f32(means), _f32(conics), _f32(radii)
    rw = np.ascontiguousarray(rows, dtype=np.int32)
    P, D = m.shape
    counts = np.zeros(len(rw), np.int64)
    lib.orc_agg_counts_rows(P, D, _ptr(m), _ptr(r), len(rw), _ptr(rw), _ptr(counts))
    ranges = np.cumsum(counts).astype(np.int64)
    n = int(ranges[-1]) if len(rw) else 0
    indices = np.full(n, -1, np.int64)
    dists = np.zeros((n, D), np.float32)
    dens = np.zeros(n, np.float32)
    inv = np.zeros(len(rw), np.float32)
    lib.orc_agg_fill_rows(P, D, _ptr(m), _ptr(c), _ptr(r), len(rw), _ptr(rw), _ptr(ranges),
                          _ptr(indices), _ptr(dists), _ptr(dens), _ptr(inv))
    return indices, ranges, dists, dens, inv


def agg_forward(features, transform, queries, keys, frequencies, distance_transform, indices,
                ranges, dists, densities, inv_total, rows=None, exact=False):
    """aggregate_neighbors forward: (weights, embeddings, factors, neighbor_features).
    rows: evaluate only the first `rows` rows (a bounded CPU-baseline sample).
    exact: neighbor_features with exact (double) accumulation of the reference's per-slot float
    terms (float64), instead of the reference's own float summation order."""
    lib = _load()
    f, T, q, k = _f32(features), _f32(transform), _f32(queries), _f32(keys)
    fr, dt = _f32(frequencies), _f32(distance_transform)
    idx, rg, X, dn, inv = _i64(indices), _i64(ranges), _f32(dists), _f32(densities), _f32(inv_total)
    P, L = f.shape
    K = q.shape[1]
    D = X.shape[1] if X.ndim == 2 else 1
    E = dt.size // 2
    n = idx.size
    w, emb, fac = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    out = np.zeros((P, L), np.float64 if exact else np.float32)
    fn = lib.orc_agg_forward64 if exact else lib.orc_agg_forward
    fn(P if rows is None else min(rows, P), D, L, K, E, _ptr(f), _ptr(T), _ptr(q), _ptr(k), _ptr(fr), _ptr(dt),
                        _ptr(idx), _ptr(rg), _ptr(X), _ptr(dn), _ptr(inv), _ptr(w), _ptr(emb),
                        _ptr(fac), _ptr(out))
    return w, emb, fac, out


def agg_backward(features, transform, queries, keys, frequencies, distance_transform, indices,
                 ranges, dists, densities, weights, embeddings, factors, inv_total, dL, rows=None,
                 exact=False):
    """aggregate_neighbors backward: the six gradients (features, transform, queries, keys,
    frequencies, distance_transform).  exact: accumulated exactly (float64 results), see
    agg_forward."""
    lib = _load()
    f, T, q, k = _f32(features), _f32(transform), _f32(queries), _f32(keys)
    fr, dt = _f32(frequencies), _f32(distance_transform)
    idx, rg, X, dn = _i64(indices), _i64(ranges), _f32(dists), _f32(densities)
    w, emb, fac, inv, g = _f32(weights), _f32(embeddings), _f32(factors), _f32(inv_total), _f32(dL)
    P, L = f.shape
    K = q.shape[1]
    D = X.shape[1] if X.ndim == 2 else 1
    E = dt.size // 2
    ot = np.float64 if exact else np.float32
    outs = [np.zeros(a.shape, ot) for a in (f, T, q, k, fr, dt)]
    fn = lib.orc_agg_backward64 if exact else lib.orc_agg_backward
    fn(P if rows is None else min(rows, P), D, L, K, E, _ptr(f), _ptr(T), _ptr(q), _ptr(k), _ptr(fr), _ptr(dt),
                         _ptr(idx), _ptr(rg), _ptr(X), _ptr(dn), _ptr(w), _ptr(emb), _ptr(fac),
                         _ptr(inv), _ptr(g), *[_ptr(o) for o in outs])
    return tuple(outs)


def agg_forward_rows(features, transform, queries, keys, frequencies, distance_transform, rows,
                     indices, ranges, dists, densities, inv_total, exact=False):
    """agg_forward over the rows `rows` only, on the compact lists of agg_preprocess_rows:
    (weights, embeddings, factors) of those slots and neighbor_features [len(rows), L]."""
    lib = _load()
    f, T, k = _f32(features), _f32(transform), _f32(keys)
    q = _f32(np.asarray(queries)[np.asarray(rows)])
    fr, dt = _f32(frequencies), _f32(distance_transform)
    idx, rg, X, dn, inv = _i64(indices), _i64(ranges), _f32(dists), _f32(densities), _f32(inv_total)
    L, K, n = f.shape[1], q.shape[1], idx.size
    D = X.shape[1] if X.ndim == 2 else 1
    E = dt.size // 2
    w, emb, fac = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    out = np.zeros((len(rows), L), np.float64 if exact else np.float32)
    (lib.orc_agg_forward64 if exact else lib.orc_agg_forward)(len(rows), D, L, K, E, _ptr(f), _ptr(T), _ptr(q), _ptr(k), _ptr(fr), _ptr(dt),
                        _ptr(idx), _ptr(rg), _ptr(X), _ptr(dn), _ptr(inv), _ptr(w), _ptr(emb),
                        _ptr(fac), _ptr(out))
    return w, emb, fac, out


def agg_backward_rows(features, transform, queries, keys, frequencies, distance_transform, rows,
                      indices, ranges, dists, densities, weights, embeddings, factors, inv_total, dL_rows,
                      exact=False):
    """agg_backward with dL/dneighbor_features non-zero on the rows `rows` only (dL_rows
    [len(rows), L]), on their compact lists: the six gradients (queries' gradient full-size,
    zero outside `rows`)."""
    lib = _load()
    f, T, k = _f32(features), _f32(transform), _f32(keys)
    qf = _f32(queries)
    q = _f32(qf[np.asarray(rows)])
    fr, dt = _f32(frequencies), _f32(distance_transform)
    idx, rg, X, dn = _i64(indices), _i64(ranges), _f32(dists), _f32(densities)
    w, emb, fac, inv, g = _f32(weights), _f32(embeddings), _f32(factors), _f32(inv_total), _f32(dL_rows)
    L, K = f.shape[1], q.shape[1]
    D = X.shape[1] if X.ndim == 2 else 1
    E = dt.size // 2
    ot = np.float64 if exact else np.float32
    dq_rows = np.zeros(q.shape, ot)
    outs = [np.zeros(f.shape, ot), np.zeros(T.shape, ot), dq_rows, np.zeros(k.shape, ot),
            np.zeros(fr.shape, ot), np.zeros(dt.shape, ot)]
    (lib.orc_agg_backward64 if exact else lib.orc_agg_backward)(len(rows), D, L, K, E, _ptr(f), _ptr(T), _ptr(q), _ptr(k), _ptr(fr), _ptr(dt),
                         _ptr(idx), _ptr(rg), _ptr(X), _ptr(dn), _ptr(w), _ptr(emb), _ptr(fac),
                         _ptr(inv), _ptr(g), *[_ptr(o) for o in outs])
    dq = np.zeros(qf.shape, ot)
    dq[np.asarray(rows)] = dq_rows
    return outs[0], outs[1], dq, outs[3], outs[4], outs[5]

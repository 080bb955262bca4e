"""How much does nvcc's default FMA contraction move the reference's outputs?

The reference is built by nvcc with its default --fmad=true (setup.py:30 passes no
--fmad=false), so the compiled reference may fuse its a*b +- c sites (forward.cu:55,59,177,182,
199,223,252; backward.cu:122,141,147-148 and the other functions' equivalents).  The oracle has
three builds (oracle/Makefile, oracle.c header): "nocontract" (every product rounded; the model
the GPU path is built against), "fmad" (LLVM's own contraction, ties fused left) and "fmad_alt"
(ties fused right).  This script compares them on every BASELINE config and every golden /
parity case and writes profiles/r05_contraction.json:

  binning  : Gaussians whose radius differs, whose presence (radius > 0) differs, det == 0
             decisions per model (forward.cu:55-56, counted exactly in numpy), num_rendered and
             reference-layout ranges differences;
  forward  : per function, max |model - nocontract| / (1e-5 |nocontract| + 1e-6 max|nocontract|),
             the SURVEY 8c parity bound the GPU tests use (< 1: inside the bound);
  backward : the same for the exact-sum gradients (dmeans, dvalues, dconics);
  aggregate: neighbour lists (indices / ranges / densities) of config 5 on a row subset.

    python tools/contraction_study.py [--out profiles/r05_contraction.json] [--quick]

CPU only (test infrastructure: imports the oracle as the checker, never the product path).
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "diff-gaussian-sampling_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

FUNCS = ["gaussian", "derivative", "laplacian", "third"]
MODELS = ["fmad", "fmad_alt"]
RTOL, ATOL = 1e-5, 1e-6


def margin(got, ref):
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    if not ref.size:
        return 0.0
    b = RTOL * np.abs(ref) + ATOL * float(np.max(np.abs(ref))) + 1e-300
    return float(np.max(np.abs(got - ref) / b))


def det_zero_counts(covs):
    """det == 0 decisions (forward.cu:55-56) per model, exact: fl(c0 c2) - fl(c1 c1) == 0,
    fma(c0, c2, -fl(c1 c1)) == 0 (fused left), fma(-c1, c1, fl(c0 c2)) == 0 (fused right)."""
    c = np.asarray(covs, np.float32)
    if c.shape[1] != 3:
        return None
    c0, c1, c2 = (c[:, k] for k in range(3))
    p02 = (c0 * c2).astype(np.float32)
    p11 = (c1 * c1).astype(np.float32)
    e02 = c0.astype(np.float64) * c2.astype(np.float64)  # exact in double (24 + 24 bits)
    e11 = c1.astype(np.float64) * c1.astype(np.float64)
    z0 = p02 == p11
    z1 = e02 == p11.astype(np.float64)
    z2 = p02.astype(np.float64) == e11
    return {"nocontract": int(z0.sum()), "fmad": int(z1.sum()), "fmad_alt": int(z2.sum()),
            "differ_fmad": int((z0 != z1).sum()), "differ_fmad_alt": int((z0 != z2).sum())}


def study_case(args):
    name, build, opts = args
    from oracle import oracle as orc
    t0 = time.time()
    means, values, covs, conics, samples = build_inputs(build)
    means, values, covs, conics, samples = (np.asarray(t, np.float32) for t in (means, values, covs, conics, samples))
    P, D = means.shape
    N = samples.shape[0]
    C = values.shape[1]
    rec = {"P": P, "N": N, "D": D, "C": C}
    bins = {m: orc.OracleBins(means, covs, samples, model=m) for m in ["nocontract"] + MODELS}
    b0 = bins["nocontract"]
    r0, s0 = b0.ranges()
    rec["num_rendered"] = b0.num_rendered
    binning = {}
    for m in MODELS:
        b = bins[m]
        r, s = b.ranges()
        binning[m] = {
            "radii_differ": int(np.sum(b.radii != b0.radii)),
            "presence_differ": int(np.sum((b.radii > 0) != (b0.radii > 0))),
            "num_rendered_diff": int(b.num_rendered - b0.num_rendered),
            "ranges_differ": int(np.sum(r != r0)),
            "sample_ranges_differ": int(np.sum(s != s0)),
        }
    binning["det_zero"] = det_zero_counts(covs) if D == 2 else None
    rec["binning"] = binning
    # float outputs on a subset of samples (the whole set for small cases)
    sub_n = opts.get("subset")
    rng = np.random.default_rng(7)
    keys = b0.sample_keys()
    rendered = np.nonzero(keys < b0.T)[0]
    sub = None
    if sub_n is not None and sub_n < N:
        sub = np.sort(rng.choice(rendered, size=min(sub_n, rendered.size), replace=False)).astype(np.int32)
    rec["samples_evaluated"] = int(N if sub is None else sub.size)
    g = np.random.default_rng(5)
    fwd, bwd = {}, {}
    for fn in opts.get("functions", FUNCS):
        K = D ** FUNCS.index(fn)
        dL = g.standard_normal((N, K, C)).astype(np.float32)
        outs = {m: bins[m].forward(fn, values, conics, subset=sub) for m in ["nocontract"] + MODELS}
        grads = {m: bins[m].backward(fn, values, conics, dL, subset=sub, exact=True) for m in ["nocontract"] + MODELS}
        ref = outs["nocontract"] if sub is None else outs["nocontract"][sub]
        fwd[fn] = {}
        bwd[fn] = {}
        for m in MODELS:
            got = outs[m] if sub is None else outs[m][sub]
            fwd[fn][m] = margin(got, ref)
            bwd[fn][m] = {nm: margin(a, b) for nm, a, b in zip(("dmeans", "dvalues", "dconics"), grads[m], grads["nocontract"])}
        gotf = outs["fmad"] if sub is None else outs["fmad"][sub]
        gota = outs["fmad_alt"] if sub is None else outs["fmad_alt"][sub]
        fwd[fn]["fmad_vs_fmad_alt"] = margin(gota, gotf)
    rec["forward_margin_vs_nocontract"] = fwd
    rec["backward_margin_vs_nocontract"] = bwd
    rec["seconds"] = round(time.time() - t0, 1)
    return name, rec


def study_aggregate(args):
    """Config 5's neighbour lists (aggregate_neighbors.cu:18-127) on a row subset, per model."""
    name, P, nrows = args
    from oracle import oracle as orc
    from diff_gaussian_sampling import synthetic as syn
    t0 = time.time()
    means, values, covs, conics = (t.numpy() for t in syn.gaussians(P, 2, 1, seed=0))
    samples = syn.samples(min(P, 200000), 2, seed=4).numpy()
    radii = orc.OracleBins(means, covs, samples).radii
    rows = np.sort(np.random.default_rng(3).choice(P, size=nrows, replace=False)).astype(np.int32)
    lists = {m: orc.agg_preprocess_rows(means, conics, radii, rows, model=m) for m in ["nocontract"] + MODELS}
    i0, rg0, X0, d0, inv0 = lists["nocontract"]
    rec = {"P": P, "rows": nrows, "slots": int(i0.size)}
    for m in MODELS:
        i1, rg1, X1, d1, inv1 = lists[m]
        same_shape = i1.size == i0.size
        rec[m] = {"ranges_differ": int(np.sum(rg1 != rg0)), "slot_count_diff": int(i1.size - i0.size),
                  "indices_differ": int(np.sum(i1 != i0)) if same_shape else None,
                  "dists_differ": int(np.sum(X1 != X0)) if same_shape else None,
                  "densities_margin": margin(d1, d0) if same_shape else None,
                  "inv_total_margin": margin(inv1, inv0)}
    rec["seconds"] = round(time.time() - t0, 1)
    return name, rec


def _golden(name):
    return ("golden", name)


def _synthetic(P, N, D, C, aniso=1.0):
    return ("synthetic", P, N, D, C, aniso)


def _case(fn_name, **kw):
    return ("case", fn_name, kw)


def build_inputs(spec):
    kind = spec[0]
    if kind == "golden":
        z = np.load(os.path.join(REPO, "tests", "golden", spec[1] + ".npz"))
        return z["means"], z["values"], z["covariances"], z["conics"], z["samples"]
    if kind == "synthetic":
        from diff_gaussian_sampling import synthetic as syn
        _, P, N, D, C, aniso = spec
        m, v, cv, c = syn.gaussians(P, D, C, seed=0, aniso=aniso)
        return m, v, cv, c, syn.samples(N, D, seed=4)
    import cases
    return getattr(cases, spec[1])(**spec[2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05_contraction.json"))
    ap.add_argument("--quick", action="store_true", help="golden fixtures and small cases only")
    ap.add_argument("--workers", type=int, default=6)
    a = ap.parse_args()
    jobs = []
    for g in sorted(f[:-4] for f in os.listdir(os.path.join(REPO, "tests", "golden")) if f.endswith(".npz")):
        jobs.append(("golden/" + g, _golden(g), {}))
    jobs += [
        ("case/edge", _case("edge_case"), {}),
        ("case/aliasing", _case("aliasing_case"), {}),
        ("case/far_means", _case("far_means_case"), {}),
        ("case/seam_d2", _case("seam_case"), {}),
        ("case/thin_c1", _case("thin_case"), {"subset": 6000}),
        ("case/clustered", _case("clustered_case"), {"subset": 4000}),
        ("case/mixed_scales", _case("mixed_scales_case"), {"subset": 4000}),
        ("case/wide_domain", _case("wide_domain_case"), {}),
        ("config1/1k_4k_c1", _synthetic(1000, 4000, 2, 1), {}),
    ]
    if not a.quick:
        jobs += [
            ("config2/100k_256k_c16", _synthetic(100_000, 256_000, 2, 16), {"subset": 256}),
            ("config3/1M_2M_c1", _synthetic(1_000_000, 2_000_000, 2, 1), {"subset": 192}),
            ("config3_aniso25/1M_2M_c1", _synthetic(1_000_000, 2_000_000, 2, 1, aniso=25.0), {"subset": 192}),
            ("config4/1M_8M_c1", _synthetic(1_000_000, 8_000_000, 2, 1), {"subset": 96, "functions": ["gaussian"]}),
        ]
    out = {"what": __doc__.strip().splitlines()[0],
           "models": {"nocontract": "every product and sum rounded (gcc -ffp-contract=off); the GPU path's model",
                      "fmad": "nvcc --fmad=true modelled by LLVM contraction (clang -ffp-contract=fast -mfma), a*b+c*d fused left",
                      "fmad_alt": "as fmad, every explicit a*b+c*d site fused right"},
           "bound": "max |x - nocontract| / (1e-5 |nocontract| + 1e-6 max|nocontract|)",
           "cases": {}}
    t0 = time.time()
    with ProcessPoolExecutor(a.workers) as ex:
        futs = [ex.submit(study_case, j) for j in jobs]
        if not a.quick:
            futs.append(ex.submit(study_aggregate, ("config5/aggregate_1M_rows", 1_000_000, 48)))
        futs.append(ex.submit(study_aggregate, ("config5/aggregate_20k_all_rows", 20_000, 20_000)))
        for f in futs:
            name, rec = f.result()
            out["cases"][name] = rec
            print(name, json.dumps(rec)[:400], flush=True)
    out["seconds"] = round(time.time() - t0, 1)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()

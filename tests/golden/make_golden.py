"""Generates the committed golden fixtures under tests/golden/.  Run in the build container:

    python tests/golden/make_golden.py            # both parts
    python tests/golden/make_golden.py --api      # api_trace.json only
    python tests/golden/make_golden.py --vectors  # *.npz only

1. api_trace.json -- the reference's own Python layer (/root/reference/diff_gaussian_sampling/
   __init__.py) driven through tests/plumbing.py's scenario with a recording stub `_C`.  The
   module is compiled from its SOURCE TEXT (never from the __pycache__ shipped inside the
   reference) into a throwaway module object; nothing of it is stored except the trace.
2. <case>.npz -- inputs and oracle outputs (num_rendered, radii, reference-layout ranges,
   forward and backward of every Function) for the SURVEY 8c golden cases.  The oracle is the
   CPU restatement pinned by tests/test_oracle.py; the GPU tests compare the HIP path against
   these files without needing the oracle, and tests/test_golden.py re-derives them with the
   oracle to catch drift.
"""
import argparse
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
REPO = os.path.dirname(TESTS)
for p in (TESTS, REPO, os.path.join(REPO, "diff-gaussian-sampling_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

REFERENCE_INIT = "/root/reference/diff_gaussian_sampling/__init__.py"


def load_reference_python_layer(stub):
    """The reference package module, compiled from source with `stub` as its `_C`."""
    name = "_reference_dgs"
    pkg = types.ModuleType(name)
    pkg.__path__ = []
    pkg.__package__ = name
    pkg.__file__ = REFERENCE_INIT
    sys.modules[name] = pkg
    sys.modules[name + "._C"] = stub
    with open(REFERENCE_INIT) as f:
        code = compile(f.read(), REFERENCE_INIT, "exec")
    exec(code, pkg.__dict__)
    return pkg


def make_api():
    import plumbing
    stub = plumbing.RecordingC()
    ref = load_reference_python_layer(stub)
    torch.manual_seed(0)
    res = plumbing.scenario(ref, stub)
    path = os.path.join(HERE, "api_trace.json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", path)


def golden_cases():
    import cases
    from diff_gaussian_sampling import synthetic as syn
    return {
        # 1k x 4k D=2 C=1 (configs[0]), 256 x 1024 D=1 C=2, C=16 small, edge cases
        "d2_c1_1k_4k": lambda: syn.gaussians(1000, 2, 1, seed=0) + (syn.samples(4000, 2, seed=4),),
        "d1_c2_256_1k": lambda: syn.gaussians(256, 1, 2, seed=7) + (syn.samples(1024, 1, seed=8),),
        "d2_c16_200_800": lambda: syn.gaussians(200, 2, 16, seed=9) + (syn.samples(800, 2, seed=10),),
        "edge": lambda: cases.edge_case(n_random=1000),
        "aliasing": lambda: cases.aliasing_case(n=1000, P=200),
        "far_means": lambda: cases.far_means_case(n=1000),
        "d1_zero_variance": cases.d1_zero_variance_case,
        "seam_d1": lambda: cases.seam_case(D=1, n=1500),
        "seam_d2": lambda: cases.seam_case(D=2, n=1500),
    }


FUNCS = ["gaussian", "derivative", "laplacian", "third"]


def compute_case(orc, means, values, covs, conics, samples):
    """Dict of arrays: inputs + oracle outputs for every Function."""
    from diff_gaussian_sampling import synthetic as syn
    m, v, cv, c, s = (np.ascontiguousarray(t.numpy(), np.float32) for t in (means, values, covs, conics, samples))
    ob = orc.OracleBins(m, cv, s)
    rg, srg = ob.ranges()
    out = {"means": m, "values": v, "covariances": cv, "conics": c, "samples": s,
           "num_rendered": np.int64(ob.num_rendered), "radii": ob.radii,
           "ranges": rg, "sample_ranges": srg, "grid": ob.grid, "offset": ob.offset}
    N, D = s.shape
    C = v.shape[1]
    for i, fn in enumerate(FUNCS):
        K = syn.out_components(fn, D)
        dL = syn.grad_out(N, K, C, seed=1000 + i).numpy()
        out[fn + "_dL"] = dL
        out[fn + "_out"] = ob.forward(fn, v, c)
        dm, dv, dc = ob.backward(fn, v, c, dL)
        out[fn + "_dmeans"], out[fn + "_dvalues"], out[fn + "_dconics"] = dm, dv, dc
    return out


def make_vectors():
    from oracle import oracle as orc
    orc.build()
    for name, gen in golden_cases().items():
        data = compute_case(orc, *gen())
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **data)
        print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--api", action="store_true")
    ap.add_argument("--vectors", action="store_true")
    a = ap.parse_args()
    both = not (a.api or a.vectors)
    if a.api or both:
        make_api()
    if a.vectors or both:
        make_vectors()

"""The package's host logic against the reference's own Python layer (CPU, no GPU).

tests/golden/api_trace.json was recorded by running tests/plumbing.py's scenario against the
reference's diff_gaussian_sampling/__init__.py with a recording stub `_C`
(tests/golden/make_golden.py).  Here the same scenario runs against this repository's package
with the same stub patched in for its `_C`; the public signatures, every `_C` call with its
argument identities, the gradients delivered to each input, and the debug snapshot behaviour
must be identical.
"""
import json
import os

import pytest
import torch

import plumbing

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "api_trace.json")


@pytest.fixture
def pkg(monkeypatch):
    import diff_gaussian_sampling as dgs
    stub = plumbing.RecordingC()
    monkeypatch.setattr(dgs, "_C", stub)
    return dgs, stub


def test_plumbing_matches_reference_python_layer(pkg):
    dgs, stub = pkg
    torch.manual_seed(0)
    got = json.loads(json.dumps(plumbing.scenario(dgs, stub)))
    ref = json.load(open(GOLDEN))
    for key in ref:
        assert got[key] == ref[key], key


def test_package_imports_the_native_extension():
    """No CPU fallback: the package's _C is the built extension over libdgs.so."""
    import diff_gaussian_sampling as dgs
    f = dgs._C.__file__
    assert f.endswith(".so") and os.path.dirname(f) == os.path.dirname(dgs.__file__)
    for name in ["preprocess_gaussians", "sample_gaussians", "sample_gaussians_backward",
                 "sample_gaussians_derivative", "sample_gaussians_derivative_backward",
                 "sample_gaussians_laplacian", "sample_gaussians_laplacian_backward",
                 "sample_gaussians_third_derivative", "sample_gaussians_third_derivative_backward"]:
        assert callable(getattr(dgs._C, name)), name


def test_cpu_tensors_are_rejected():
    """The extension runs on the GPU only; CPU inputs raise instead of silently computing."""
    import diff_gaussian_sampling as dgs
    from diff_gaussian_sampling import synthetic as syn
    means, values, covs, conics = syn.gaussians(10, 2, 1)
    with pytest.raises(RuntimeError):
        dgs._C.preprocess_gaussians(means, values, covs, conics, syn.samples(20), False)

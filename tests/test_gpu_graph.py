"""Graph capture of the render calls (the binning has one host sync, the
sample calls none).  A forward + backward through the autograd Functions is captured into a
torch.cuda.CUDAGraph (a HIP graph) on a fixed binning and replayed: the forward must equal the
eager call bit for bit and the gradients (float atomics, order-dependent) within the parity
tolerance, also after `values` and dL change in place between replays (the graph re-packs the
Gaussian rows; no cached rows are reused).  A capture with tensors other than the binned ones
raises.  Each scenario runs in a child process (tests/graph_child.py)."""
import os
import subprocess
import sys

import pytest
import torch

# (A child process per scenario: a capture that an autograd graph of an earlier eager step on
# another stream breaks -- torch's AccumulateGrad stream-mismatch warning -- ends in a segfault
# inside capture_end on this image, which would otherwise take the pytest process with it.)
pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _child(*args):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "graph_child.py"), *args],
                       capture_output=True, text=True, timeout=240)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), f"rc {r.returncode}: {tail}"


@pytest.mark.parametrize("fname", ["gaussian", "derivative"])
def test_graph_capture_forward_backward(fname):
    _child("forward_backward", fname)


@pytest.mark.parametrize("fname", ["gaussian", "derivative"])
def test_graph_capture_rebin_step(fname):
    """The whole PIGS step in one graph: capturable re-binning + forward + loss.backward() into
    .grad, replayed after in-place moves of the means (graph_child.rebin_step)."""
    _child("rebin_step", fname)


def test_graph_capture_requires_binned_tensors():
    _child("requires_binned")

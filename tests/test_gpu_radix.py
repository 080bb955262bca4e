"""The binning's radix sort (dgs_radix.h) on its own: a stable sort of (key, value) pairs,
checked against numpy's stable argsort on keys with many duplicates, at tile-boundary sizes
(one sort tile = 4096 items) and for every digit-place count the binning uses."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from diff_gaussian_sampling import _C
    return _C


@pytest.mark.parametrize("n", [1, 63, 4095, 4096, 4097, 3 * 4096 + 5, 1 << 20, 2_000_003])
@pytest.mark.parametrize("bits,kbytes", [(4, 4), (8, 4), (14, 4), (15, 2), (16, 2), (20, 4), (32, 4)])
def test_radix_stable(C, n, bits, kbytes):
    rng = np.random.default_rng(n * 131 + bits)
    hi = 1 << bits
    # few distinct keys for the small widths (long equal runs: stability matters), skewed otherwise
    keys = (rng.integers(0, hi, n, dtype=np.uint64) if bits > 8 else rng.integers(0, min(hi, 7), n, dtype=np.uint64))
    if bits > 8:
        keys[rng.random(n) < 0.3] = hi - 1  # one heavy digit in every place
    vals = rng.permutation(n).astype(np.int64)
    kdt = np.uint16 if kbytes == 2 else np.uint32
    kt = torch.from_numpy(keys.astype(kdt).view(np.int16 if kbytes == 2 else np.int32)).cuda()
    vt = torch.from_numpy(vals.astype(np.uint32).view(np.int32)).cuda()
    ko, vo = C.radix_sort_test(kt, vt, bits)
    ko = ko.cpu().numpy().view(kdt).astype(np.uint64)
    vo = vo.cpu().numpy().view(np.uint32).astype(np.int64)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(ko, keys[order])
    assert np.array_equal(vo, vals[order])


def test_radix_empty(C):
    k = torch.empty(0, dtype=torch.int32, device="cuda")
    ko, vo = C.radix_sort_test(k, k.clone(), 8)
    assert ko.numel() == 0 and vo.numel() == 0

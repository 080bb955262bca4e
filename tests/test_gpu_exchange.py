"""The native exchange-set kernel of spatial sharding (dgs_exchange_sets) against
the host path of distributed.exchange_sets (the same predicate in torch ops, exercised by the
gloo tests): the same touch masks and owners, hence the same SupportExchange row lists; strips of
[-1, 1) with torus images, overlapping and unordered extents, and a non-PD conic that reaches
every rank."""
import pytest
import torch

from diff_gaussian_sampling import synthetic as syn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layout", ["strips", "overlap", "shuffled"])
@pytest.mark.parametrize("D", [1, 2])
def test_exchange_sets_native_equals_host(dgs, layout, D):
    from diff_gaussian_sampling.distributed import SupportExchange, exchange_sets
    means, values, covs, conics = syn.gaussians(30000, D, 1, seed=341 + D)
    conics[7] = -conics[7]  # not positive definite: every rank
    W = 5
    edges = torch.linspace(-1.0, 1.0, W + 1)
    ext = torch.stack([edges[:-1], edges[1:]], 1)
    if layout == "overlap":
        ext = ext + torch.tensor([[-0.05, 0.05]])
    elif layout == "shuffled":
        ext = ext[[3, 0, 4, 1, 2]]
    mh, oh = exchange_sets(means, conics, ext)
    md, od = exchange_sets(means.cuda(), conics.cuda(), ext)
    assert torch.equal(mh, md.cpu()) and torch.equal(oh, od.cpu())
    assert int(mh[7]) == (1 << W) - 1
    touched = mh != 0
    assert bool(((mh[touched] >> oh[touched]) & 1).all())  # owners touch their rows
    for rank in range(W):
        host = SupportExchange(means, conics, ext, rank)
        dev = SupportExchange(means.cuda(), conics.cuda(), ext, rank)
        assert torch.equal(host.owned, dev.owned.cpu()) and torch.equal(host.held, dev.held.cpu())
        assert host.send_splits == dev.send_splits and host.recv_splits == dev.recv_splits
        assert torch.equal(host.send_cat, dev.send_cat.cpu()) and torch.equal(host.recv_cat, dev.recv_cat.cpu())

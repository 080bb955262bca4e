"""Query-point sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Each rank holds all P Gaussians (replicated) and its own shard of the query points.  The
reference derives the tile grid from the samples it is given (sample_points.cu:70-74), so a
shard must use the GLOBAL grid -- the min/max over all shards -- or its tile membership, and
therefore its results, would differ from the single-GPU run.  `global_tile_grid` obtains it
with two tiny all-reduces (MIN and MAX of D floats) and then applies the reference formula.

The forward needs no communication (a query point's value depends only on the Gaussians);
the backward's per-Gaussian gradients are partial sums over each rank's points.

* ShardedGaussianSampler: any split of the points; ONE all-reduce of the packed
  [dmeans | dvalues | dconics] buffer (P (D + C + S) floats: 24 MB at 1M Gaussians, C = 1).
* SpatialShardedGaussianSampler: a domain decomposition.  Rank r owns a
  fixed strip of the points and a fixed set of Gaussians (their owner rank).  A Gaussian's
  partial gradient can be non-zero only on the ranks whose strip meets its exact-zero cut
  (X^T A X <= 210, the binning's culling bound; with the torus images 2k), so the backward sends
  only those rows, to the owner (one all-to-all): afterwards a rank's gradient is the global
  gradient on the rows it OWNS and 0 elsewhere, and an ordinary optimizer over the full tensors
  updates exactly the owned rows.  `push` then sends the owners' updated rows to every rank
  whose strip the updated cut reaches.  A rank bins only the rows it holds current copies of
  (owned or pushed), so its results never read a stale row.  With strips, only the Gaussians
  near a strip boundary travel (~1-2 MB per rank per step at config 4 against 24 MB).
"""
import math

import torch
import torch.distributed as dist

from . import _C, call_debug

_FWD = {"gaussian": "sample_gaussians", "derivative": "sample_gaussians_derivative",
        "laplacian": "sample_gaussians_laplacian", "third": "sample_gaussians_third_derivative"}


def _world(group=None):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def global_tile_grid(samples, group=None):
    """(grid, offset) of the union of every rank's `samples` (reference formula, torch ops)."""
    mn = samples.min(0).values.clone()
    mx = samples.max(0).values.clone()
    if _world(group) > 1:
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    grid = torch.ceil((mx - mn + 1e-6) / 0.51).to(torch.int32)
    return [int(g) for g in grid.cpu()], [float(o) for o in mn.cpu()]


def allreduce_grads(grads, group=None, chunks=1):
    """Sums (dmeans, dvalues, dconics) over ranks: the packed rows [dmeans | dvalues | dconics]
    (P x (D + C + S) floats), one collective, or `chunks` row blocks whose collectives are issued
    back to back (async_op): block k's all-reduce runs on the communication stream while block
    k + 1 is packed on the compute stream, and RCCL pipelines the blocks over xGMI.  The sum of an
    element does not depend on the blocking at world 2 (a + b); at more ranks the ring's order
    may differ in the last bit (tests/test_distributed.py checks world 2 bit for bit)."""
    if _world(group) == 1:
        return grads
    P = grads[0].shape[0]
    if P == 0:  # (nothing to sum; reshape(0, -1) would raise -- ADVICE r05)
        return grads
    cols = [g.reshape(P, -1) for g in grads]
    widths = [c.shape[1] for c in cols]
    chunks = max(1, min(int(chunks), P)) if P else 1
    bounds = [P * k // chunks for k in range(chunks + 1)]
    blocks, works = [], []
    for k in range(chunks):  # pack block k, then start its collective (async)
        r0, r1 = bounds[k], bounds[k + 1]
        blk = torch.cat([c[r0:r1] for c in cols], dim=1).contiguous()
        blocks.append(blk)
        works.append(dist.all_reduce(blk, group=group, async_op=True))
    for w in works:
        w.wait()
    packed = blocks[0] if chunks == 1 else torch.cat(blocks, dim=0)
    out, o = [], 0
    for g, w in zip(grads, widths):
        out.append(packed[:, o:o + w].reshape(g.shape))
        o += w
    return tuple(out)


class _ShardedSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, function, comm, means, values, conics, samples, num_rendered, binning,
                sample_binning, ranges, sample_ranges, debug):
        fwd = getattr(_C, _FWD[function])
        out = call_debug(fwd, debug, "shard_fw", means, values, conics, samples, num_rendered,
                         binning, sample_binning, ranges, sample_ranges, debug)
        ctx.function, ctx.debug, ctx.num_rendered = function, debug, num_rendered
        ctx.group, ctx.chunks = comm  # (process group, row blocks of the gradient all-reduce)
        ctx.save_for_backward(means, values, conics, samples, binning, sample_binning, ranges,
                              sample_ranges)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        means, values, conics, samples, binning, sample_binning, ranges, sample_ranges = ctx.saved_tensors
        bwd = getattr(_C, _FWD[ctx.function] + "_backward")
        grads = call_debug(bwd, ctx.debug, "shard_bw", means, values, conics, samples,
                           ctx.num_rendered, grad_out.contiguous(), binning, sample_binning,
                           ranges, sample_ranges, ctx.debug)
        gm, gv, gc = allreduce_grads(grads, ctx.group, ctx.chunks)
        return (None, None, gm, gv, gc) + (None,) * 7


class ShardedGaussianSampler:
    """GaussianSampler over a process group: this rank's `samples` are its shard; gradients
    flowing back to (means, values, conics) are the sums over all shards (allreduce_grads, in
    `chunks` pipelined row blocks)."""

    def __init__(self, debug=False, group=None, chunks=4):
        self.debug = debug
        self.group = group
        self.chunks = max(1, int(chunks))

    def preprocess(self, means, values, covariances, conics, samples):
        grid, offset = global_tile_grid(samples, self.group)
        (self.num_rendered, self.binning_buffer, self.sample_binning_buffer, self.ranges,
         self.sample_ranges, self.radii) = call_debug(
            _C.preprocess_gaussians_bounded, self.debug, "shard_preprocess", means, values,
            covariances, conics, samples, grid, offset, self.debug)
        self.grid, self.offset = grid, offset
        self.means, self.values, self.conics, self.samples = means, values, conics, samples

    def _sample(self, function):
        return _ShardedSample.apply(function, (self.group, self.chunks), self.means, self.values, self.conics,
                                    self.samples, self.num_rendered, self.binning_buffer,
                                    self.sample_binning_buffer, self.ranges, self.sample_ranges,
                                    self.debug)

    def sample_gaussians(self):
        return self._sample("gaussian")

    def sample_gaussians_derivative(self):
        return self._sample("derivative")

    def sample_gaussians_laplacian(self):
        return self._sample("laplacian")

    def sample_gaussians_third_derivative(self):
        return self._sample("third")


# ------------------------------------------------------------------------ spatial shards (f3)
Q_CUT = 210.0  # X^T A X above this gives expf(-q / 2) == +0 in fp32 (dgs_internal.h kQCut)
RHO2_MAX = 0.9995  # conics with c1^2 >= RHO2_MAX c0 c2 are not culled (dgs_internal.h kRho2Max)


def support_halfwidth(means, conics):
    """Half-width along the sharding axis (y at D = 2, x at D = 1) of every Gaussian's
    exact-zero cut {X : X^T A X <= Q_CUT}: sqrt(Q_CUT * (A^-1)_axis).  inf for conics that are not
    positive definite (their pairs are bounded by no ellipse).  float64, widened by 1e-5."""
    D = means.shape[1]
    c = conics.detach().double()
    if D == 2:
        c0, c1, c2 = c[:, 0], c[:, 1], c[:, 2]
        det = c0 * c2 - c1 * c1
        pd = (c0 > 0) & (det > 0) & torch.isfinite(det) & torch.isfinite(c0) & torch.isfinite(c2)
        pd &= c1 * c1 < RHO2_MAX * (c0 * c2)  # (the binning keeps whole tiles past it: gauss_cut)
        e = torch.sqrt(Q_CUT * c0 / torch.where(pd, det, torch.ones_like(det)))
    else:
        c0 = c[:, 0]
        pd = (c0 > 0) & torch.isfinite(c0)
        e = torch.sqrt(Q_CUT / torch.where(pd, c0, torch.ones_like(c0)))
    e = e * (1.0 + 1e-5) + 1e-6
    return torch.where(pd, e, torch.full_like(e, math.inf))


def exchange_sets(means, conics, extents):
    """(mask int64 [P], owner int64 [P]) for the rank ranges `extents` [W, 2] = [lo, hi] along the
    sharding axis: bit r of mask[g] is set when rank r's range meets the cut of g or of one of its
    torus images m + 2k (forward.cu:149-157 wraps X with period 2), i.e. when rank r's partial
    gradient for g can be non-zero; owner[g] is the rank nearest the mean among those it touches
    (the nearest of all when it touches none; first on ties).  GPU tensors: the native kernel
    (dgs_exchange_sets, W <= 32); host tensors: the same predicate in torch ops."""
    D = means.shape[1]
    dev = means.device
    ext = torch.as_tensor(extents).detach().double().cpu()
    W = ext.shape[0]
    if W > 63:  # (the rank bits live in one int64 per Gaussian)
        raise ValueError(f"exchange_sets: at most 63 ranks (got {W})")
    if means.is_cuda and W <= 32:
        mask, owner = _C.exchange_sets(means.detach(), conics.detach(), [float(v) for v in ext.reshape(-1)])
        return mask.long() & 0xFFFFFFFF, owner.long()
    y = means.detach()[:, D - 1].double()
    e = support_halfwidth(means, conics)
    lo, hi = ext[:, 0].to(dev), ext[:, 1].to(dev)
    span = float(ext[:, 1].max() - ext[:, 0].min()) if W else 0.0
    kmax = int(math.ceil(span / 2.0)) + 1
    touch = torch.zeros(y.numel(), W, dtype=torch.bool, device=dev)
    for k in range(-kmax, kmax + 1):
        a, b = y + 2.0 * k - e, y + 2.0 * k + e
        touch |= (a[:, None] <= hi[None, :]) & (b[:, None] >= lo[None, :])
    dist_r = torch.clamp(torch.maximum(lo[None, :] - y[:, None], y[:, None] - hi[None, :]), min=0.0)
    near_all = torch.argmin(dist_r, dim=1)  # first minimum: deterministic
    near_touch = torch.argmin(torch.where(touch, dist_r, torch.full_like(dist_r, math.inf)), dim=1)
    owner = torch.where(touch.any(1), near_touch, near_all)
    mask = (touch.long() << torch.arange(W, device=dev)).sum(1)
    return mask, owner


def _bits(mask, r):
    return ((mask >> r) & 1).bool()


class SupportExchange:
    """The sparse communication of a spatially sharded run.

    Every Gaussian g has a fixed owner rank, chosen once from the parameters given here (the
    same on every rank).  Per step:

    * `reduce(G)` (in the backward): rank r sends its partial rows of the Gaussians it touches but
      does not own to their owners (one all-to-all); the owner adds them, in rank order, to its own
      partial.  Afterwards a rank's rows are the sums over all ranks on the rows it owns and 0
      elsewhere -- so an ordinary optimizer over the full tensors updates the owned rows only.
    * `push(tensors, means, conics)` (after the optimizer step): each owner recomputes the ranks
      its updated Gaussians touch and sends those rows of `tensors` to them (ids + rows, one
      count exchange).  A rank then HOLDS current copies of the rows it owns or was pushed --
      every row whose cut reaches its strip -- and bins only those (`held`).  The push also fixes
      the next reduce's row lists on both sides: the owner receives back exactly the rows it
      pushed, so the reduce needs no count exchange.

    `extents` [W, 2]: every rank's range [lo, hi] along the sharding axis (y at D = 2), fixed for
    the run.  The constructor derives the first lists from the replicated parameters alone."""

    def __init__(self, means, conics, extents, rank, group=None, debug=False):
        dev = means.device
        self.extents = torch.as_tensor(extents).detach().double().cpu().clone()
        W = self.extents.shape[0]
        self.rank, self.world, self.group, self.debug = rank, W, group, debug
        mask, owner = exchange_sets(means, conics, self.extents)
        self.owner = owner
        self.owned = owner == rank
        self.owned_idx = torch.nonzero(self.owned).flatten()  # (owners never change)
        touch_me = _bits(mask, rank)
        self.held = touch_me | self.owned
        # rows sent in the reduce, grouped by owner (ascending id within a group)
        snd = torch.nonzero(touch_me & ~self.owned).flatten()
        so = owner[snd]
        snd = snd[torch.argsort(so, stable=True)]
        send_n = torch.bincount(so, minlength=W)
        recv, recv_n = self._by_rank(mask, self.owned_idx)
        n = torch.stack([send_n, recv_n]).cpu()
        self._set_lists(list(torch.split(snd, [int(v) for v in n[0]])), list(torch.split(recv, [int(v) for v in n[1]])))
        # the sync-free push (push(..., sync=False)): per (owner -> rank) pair a row capacity,
        # the same on both sides (both know the pair's count of the last exact exchange)
        self._set_caps([int(v) for v in n[1]], [int(v) for v in n[0]])
        self.overflow = None  # device flag of the last sync-free push (checked at the next preprocess)
        self._last_push = None
        # the padded push writes its padding slots to an owned row of the receiver: usable only
        # when every rank owns one (decided once, the same on every rank)
        self._padded_ok = self.owned_idx.numel() > 0
        if W > 1 and dist.is_available() and dist.is_initialized():  # (no group: a set-only exchange)
            ok = torch.tensor([int(self._padded_ok)],
                              device=torch.device("cpu") if dist.get_backend(group) == "gloo" else dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
            self._padded_ok = bool(int(ok.item()))

    def _by_rank(self, mask, rows):
        """`rows` grouped by every other rank whose bit is set in mask[rows] (a row appears once per
        such rank; ascending within a group), and the group sizes (device)."""
        W = self.world
        bits = ((mask[rows][None, :] >> torch.arange(W, device=rows.device)[:, None]) & 1).bool()
        bits[self.rank] = False
        q, j = torch.nonzero(bits, as_tuple=True)  # rank-major, ascending row within a rank
        return rows[j], torch.bincount(q, minlength=W)

    def _set_lists(self, send, recv):
        self.send_splits = [int(x.numel()) for x in send]
        self.recv_splits = [int(x.numel()) for x in recv]
        self.send_idx, self.recv_idx = send, recv
        self.send_cat = torch.cat(send)
        self.recv_cat = torch.cat(recv)
        self.padded = None  # exact lists (set by the sync-free push: padded ones)

    @staticmethod
    def cap_of(n):
        """Row capacity of an (owner -> rank) pair whose last exact exchange moved n rows."""
        return n + n // 4 + 16 if n else 0

    def _set_caps(self, push_send, push_recv):
        """push_send[r]: rows this rank (owner) sent to r in the last exact push; push_recv[q]: rows
        it received from owner q.  Pairs with no rows stay at capacity 0 until an exact push."""
        self.cap_send = [self.cap_of(v) if r != self.rank else 0 for r, v in enumerate(push_send)]
        self.cap_recv = [self.cap_of(v) if q != self.rank else 0 for q, v in enumerate(push_recv)]
        # their device forms, built here (at an exact exchange, which synchronises anyway) so the
        # sync-free push and reduce build nothing from host lists (a pageable H2D copy blocks)
        dev = self.owner.device
        self._caps_dev = torch.tensor(self.cap_send, dtype=torch.int64, device=dev)
        rtot = int(sum(self.cap_recv))
        self._slot_in = (torch.cat([torch.arange(n, device=dev) for n in self.cap_recv]) if rtot
                         else torch.zeros(0, dtype=torch.long, device=dev))
        self._owner_of = (torch.repeat_interleave(torch.arange(self.world, device=dev),
                                                  torch.tensor(self.cap_recv, device=dev), output_size=rtot)
                          if rtot else self._slot_in)
        stot = int(sum(self.cap_send))
        self._slot_out = (torch.cat([torch.arange(n, device=dev) for n in self.cap_send]) if stot
                          else torch.zeros(0, dtype=torch.long, device=dev))
        self._dest_of = (torch.repeat_interleave(torch.arange(self.world, device=dev),
                                                 torch.tensor(self.cap_send, device=dev), output_size=stot)
                         if stot else self._slot_out)
        # the padded push's one all-to-all: per (owner -> rank) pair a block of capacity + 1 rows,
        # [count | ids and rows], so the counts, ids and rows travel in ONE collective
        def layout(caps):
            blk = [n + 1 if n else 0 for n in caps]
            pos, hdr_rows, hdr_ranks, o = [], [], [], 0
            for r, n in enumerate(caps):
                if n:
                    hdr_rows.append(o)
                    hdr_ranks.append(r)
                    pos.extend(range(o + 1, o + 1 + n))
                o += blk[r]
            t = lambda v: torch.tensor(v, dtype=torch.long, device=dev)  # noqa: E731
            return blk, t(pos), t(hdr_rows), t(hdr_ranks)
        self._pk_send_splits, self._pk_pos_send, self._pk_hdr_send, self._pk_hdr_send_ranks = layout(self.cap_send)
        self._pk_recv_splits, self._pk_pos_recv, self._pk_hdr_recv, self._pk_hdr_recv_ranks = layout(self.cap_recv)

    def _counts_a2a(self, counts):
        """all-to-all of one int per rank pair (host lists in, host list out)."""
        dev = torch.device("cpu") if dist.get_backend(self.group) == "gloo" else self.owner.device
        mine = torch.tensor(counts, dtype=torch.long, device=dev)
        got = torch.empty_like(mine)
        dist.all_to_all_single(got, mine, [1] * self.world, [1] * self.world, group=self.group)
        return [int(v) for v in got.cpu()]

    def rows_moved(self):
        """Gaussian rows this rank sends in one reduce (the padded blocks' capacities after a
        sync-free push)."""
        return sum(self.cap_recv) if self.padded is not None else sum(self.send_splits)

    def _a2a(self, out, inp, out_splits, in_splits):
        if inp.is_cuda and dist.get_backend(self.group) == "gloo":  # gloo: host staging
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def _check_splits(self):
        """debug: every rank's send count to q equals q's receive count from it (else raise on
        every rank, before a mismatched all-to-all can hang or corrupt rows)."""
        got = self._counts_a2a(self.send_splits)
        dev = torch.device("cpu") if dist.get_backend(self.group) == "gloo" else self.owner.device
        bad = torch.tensor([int(got != self.recv_splits)], device=dev)
        dist.all_reduce(bad, group=self.group)
        if int(bad.item()):
            raise RuntimeError("SupportExchange: the ranks' row lists disagree -- the parameters were changed "
                               "without push() (or differed between ranks at construction)")

    def reduce(self, G):
        """G [P, F] float32, this rank's partial sums (modified in place): afterwards the rows this
        rank owns hold the sum over all ranks and every other row is 0."""
        if self.world == 1:
            return G
        if self.padded is not None:
            return self._reduce_padded(G)
        if self.debug:
            self._check_splits()
        F = G.shape[1]
        send = G.index_select(0, self.send_cat).contiguous()
        recv = torch.empty((sum(self.recv_splits), F), dtype=G.dtype, device=G.device)
        self._a2a(recv, send, self.recv_splits, self.send_splits)
        G.masked_fill_(~self.owned[:, None], 0.0)
        o = 0
        for r in range(self.world):  # added in rank order: deterministic
            n = self.recv_splits[r]
            if n:
                G.index_add_(0, self.recv_idx[r], recv[o:o + n])
            o += n
        return G

    def _reduce_padded(self, G):
        """reduce() on the sync-free push's padded lists: every pair's block has its capacity of
        rows (host-known splits); a block's valid rows are counted on the device, the others are
        sent for the padding id (an owned row of the receiver) and added as exact zeros."""
        pd = self.padded
        F = G.shape[1]
        send = G.index_select(0, pd["red_send_ids"]).contiguous()
        recv = torch.empty((sum(self.cap_send), F), dtype=G.dtype, device=G.device)
        self._a2a(recv, send, self.cap_send, self.cap_recv)
        G.masked_fill_(~self.owned[:, None], 0.0)
        # padding slots (beyond a block's device-side count) add exact zeros: masked with where,
        # not multiplied (0 * inf would be NaN)
        valid = self._slot_out < pd["send_cnt"][self._dest_of]
        recv = torch.where(valid[:, None], recv, torch.zeros((), dtype=recv.dtype, device=recv.device))
        o = 0
        for r in range(self.world):  # added in rank order: deterministic
            n = self.cap_send[r]
            if n:
                G.index_add_(0, pd["push_send_ids"][o:o + n], recv[o:o + n])
            o += n
        return G

    @torch.no_grad()
    def push(self, tensors, means, conics, sync=True):
        """After the optimizer step on the owned rows: send every owner's rows of `tensors` (each
        [P, ...], float32; updated in place on the receivers) to the ranks its updated cut
        reaches, computed from `means` / `conics` (the updated ones; only the owned rows are
        read).  Updates `held` and the next reduce's row lists.  Returns the rows sent (a device
        count with sync=False).

        sync=False: no host synchronisation.  Every (owner -> rank) pair moves a block of its
        capacity (the last exact push's count + 25 % + 16, the same on both sides) with the valid
        rows counted on the device; a pair with more rows than its capacity sets the device flag
        `overflow`, which the next SpatialShardedGaussianSampler.preprocess reads in its one host
        transfer and answers with an exact push (all ranks together) before binning."""
        W = self.world
        if W == 1:
            return 0
        self._last_push = (tensors, means, conics)
        if not sync and self._padded_ok:
            return self._push_padded(tensors, means, conics)
        return self._push_exact(tensors, means, conics)

    @torch.no_grad()
    def _push_padded(self, tensors, means, conics):
        W, me = self.world, self.rank
        dev = self.owner.device
        oi = self.owned_idx
        dummy = oi[:1]  # an owned row: no rank ever sends it to its owner
        mask, _ = exchange_sets(means.index_select(0, oi), conics.index_select(0, oi), self.extents)
        bits = ((mask[None, :] >> torch.arange(W, device=dev)[:, None]) & 1).bool()  # [W, n_owned]
        bits[me] = False
        cnt = bits.sum(1)  # rows per destination (device)
        pos = torch.cumsum(bits.to(torch.int64), 1) - 1
        caps = self._caps_dev
        base = torch.cumsum(caps, 0) - caps
        tot = int(sum(self.cap_send))
        keep = bits & (pos < caps[:, None])
        slot = torch.where(keep, base[:, None] + pos, torch.full_like(pos, tot))
        buf = dummy.expand(tot + 1).clone()
        buf.scatter_(0, slot.reshape(-1), oi.expand(W, -1).reshape(-1))
        send_ids = buf[:tot]
        overflow = (cnt > caps).any()
        cols = [t.reshape(t.shape[0], -1) for t in tensors]
        F = sum(c.shape[1] for c in cols)
        rtot = int(sum(self.cap_recv))
        # one collective: per destination block [count | (id, row) x capacity], ids and counts as
        # int32 bits in the float32 column 0 (an all-to-all moves bytes)
        pk = torch.zeros((sum(self._pk_send_splits), 1 + F), dtype=torch.float32, device=dev)
        pk[self._pk_hdr_send, 0] = cnt.index_select(0, self._pk_hdr_send_ranks).to(torch.int32).view(torch.float32)
        pk[self._pk_pos_send, 0] = send_ids.to(torch.int32).view(torch.float32)
        pk[self._pk_pos_send, 1:] = torch.cat([c.index_select(0, send_ids) for c in cols], 1).float()
        got = torch.empty((sum(self._pk_recv_splits), 1 + F), dtype=torch.float32, device=dev)
        self._a2a(got, pk, self._pk_recv_splits, self._pk_send_splits)
        recv_cnt = torch.zeros(W, dtype=torch.int32, device=dev)
        recv_cnt[self._pk_hdr_recv_ranks] = got[self._pk_hdr_recv, 0].contiguous().view(torch.int32)
        got_ids = got[self._pk_pos_recv, 0].contiguous().view(torch.int32).long()
        got_rows = got[self._pk_pos_recv, 1:]
        valid = self._slot_in < recv_cnt[self._owner_of]
        ids = torch.where(valid, got_ids, dummy.expand(rtot))
        o = 0
        for t, c in zip(tensors, cols):
            k = c.shape[1]
            new = torch.where(valid[:, None], got_rows[:, o:o + k].to(c.dtype), c.index_select(0, ids))
            c.index_copy_(0, ids, new)  # (the padding slots write the dummy row's own value back)
            if c.data_ptr() != t.data_ptr():
                t.copy_(c.reshape(t.shape))
            o += k
        held = self.owned.clone()
        held.index_fill_(0, ids, True)
        self.held = held
        # the next reduce: send back what was received (per owner block), receive into the blocks
        # this rank pushed, valid counts as pushed
        self.padded = {"red_send_ids": ids, "push_send_ids": send_ids, "send_cnt": cnt}
        self.overflow = overflow
        return cnt.sum()

    @torch.no_grad()
    def _push_exact(self, tensors, means, conics):
        W, me = self.world, self.rank
        dev = self.owner.device
        oi = self.owned_idx
        m_o, _ = exchange_sets(means.index_select(0, oi), conics.index_select(0, oi), self.extents)
        mask = torch.zeros(self.owner.numel(), dtype=m_o.dtype, device=dev)
        mask[oi] = m_o
        ids, send_n = self._by_rank(mask, oi)
        if dist.get_backend(self.group) == "gloo":
            out_splits = [int(v) for v in send_n.cpu()]
            in_splits = self._counts_a2a(out_splits)
        else:  # the counts exchanged on the device, both read back in one host transfer
            recv_n = torch.empty_like(send_n)
            dist.all_to_all_single(recv_n, send_n, [1] * W, [1] * W, group=self.group)
            n = torch.stack([send_n, recv_n]).cpu()
            out_splits, in_splits = [int(v) for v in n[0]], [int(v) for v in n[1]]
        out_ids = list(torch.split(ids, out_splits))
        cols = [t.reshape(t.shape[0], -1) for t in tensors]
        F = sum(c.shape[1] for c in cols)
        rows = torch.cat([c.index_select(0, ids) for c in cols], 1) if F else torch.empty(0, 0, device=dev)
        got_ids = torch.empty(sum(in_splits), dtype=torch.long, device=dev)
        got_rows = torch.empty((sum(in_splits), F), dtype=torch.float32, device=dev)
        self._a2a(got_ids, ids, in_splits, out_splits)
        self._a2a(got_rows, rows.float().contiguous(), in_splits, out_splits)
        o = 0
        for t, c in zip(tensors, cols):
            k = c.shape[1]
            c.index_copy_(0, got_ids, got_rows[:, o:o + k].to(c.dtype))
            if c.data_ptr() != t.data_ptr():  # a non-contiguous tensor: write back
                t.copy_(c.reshape(t.shape))
            o += k
        held = self.owned.clone()
        held[got_ids] = True
        self.held = held
        send = list(torch.split(got_ids, in_splits))  # ascending per owner (the owner sent them so)
        self._set_lists(send, out_ids)
        self._set_caps(out_splits, in_splits)
        self.overflow = None
        return int(ids.numel())


def shard_extents(samples, group=None):
    """[W, 2] point range [min, max] of every rank along the sharding axis (all-gather)."""
    D = samples.shape[1]
    ax = samples.detach()[:, D - 1]
    mine = torch.stack([ax.min(), ax.max()]) if ax.numel() else torch.tensor(
        [math.inf, -math.inf], device=samples.device)
    W = _world(group)
    if W == 1:
        return mine[None, :]
    out = [torch.empty_like(mine) for _ in range(W)]
    dist.all_gather(out, mine.contiguous(), group=group)
    return torch.stack(out)


def grid_and_box(samples, group=None, strip=None, flag=None):
    """(grid, offset) of the union of every rank's samples (global_tile_grid) and this rank's
    own bounding box (lo[D], hi[D]), read back in ONE host transfer.  strip = (lo, hi) of this
    rank along the sharding axis: also returns whether ANY rank's samples leave its strip (folded
    into the MAX all-reduce, so every rank learns it together), else None.  flag (a device
    bool, e.g. the sync-free push's overflow): also returns whether it is set on ANY rank."""
    D = samples.shape[1]
    mn = samples.min(0).values
    mx = samples.max(0).values
    gmn, gmx = mn.clone(), mx.clone()
    extra = []
    if strip is not None:
        extra.append(((mn[D - 1] < strip[0]) | (mx[D - 1] > strip[1])).float().reshape(1))
    if flag is not None:
        extra.append(torch.as_tensor(flag, device=mx.device).float().reshape(1))
    gmx = torch.cat([gmx] + extra)
    if _world(group) > 1:
        dist.all_reduce(gmn, op=dist.ReduceOp.MIN, group=group)
        dist.all_reduce(gmx, op=dist.ReduceOp.MAX, group=group)
    grid = torch.ceil((gmx[:D] - gmn + 1e-6) / 0.51).to(torch.float32)
    rows = [grid, gmn, mn, mx]
    for k in range(len(extra)):  # the flags ride along in the same transfer
        rows.append(torch.cat([gmx[D + k:D + k + 1], torch.zeros(D - 1, dtype=gmx.dtype, device=gmx.device)]))
    h = torch.stack(rows).cpu()
    res = ([int(g) for g in h[0]], [float(o) for o in h[1]], [float(v) for v in h[2]],
           [float(v) for v in h[3]])
    if strip is not None:
        res = res + (bool(h[4][0] > 0),)
    if flag is not None:
        res = res + (bool(h[-1][0] > 0),)
    return res


def pack_grads(grads):
    """(dmeans [P,D], dvalues [P,C], dconics [P,S]) -> one [P, D + C + S] buffer."""
    return torch.cat([g.reshape(g.shape[0], -1) for g in grads], dim=1)


def unpack_grads(G, like):
    out, o = [], 0
    for g in like:
        k = g.reshape(g.shape[0], -1).shape[1]
        out.append(G[:, o:o + k].reshape(g.shape))
        o += k
    return tuple(out)


class _SpatialSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, function, xchg, means, values, conics, samples, num_rendered, binning,
                sample_binning, ranges, sample_ranges, debug):
        fwd = getattr(_C, _FWD[function])
        out = call_debug(fwd, debug, "spatial_fw", means, values, conics, samples, num_rendered,
                         binning, sample_binning, ranges, sample_ranges, debug)
        ctx.function, ctx.xchg, ctx.debug, ctx.num_rendered = function, xchg, debug, num_rendered
        ctx.save_for_backward(means, values, conics, samples, binning, sample_binning, ranges,
                              sample_ranges)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        means, values, conics, samples, binning, sample_binning, ranges, sample_ranges = ctx.saved_tensors
        bwd = getattr(_C, _FWD[ctx.function] + "_backward")
        grads = call_debug(bwd, ctx.debug, "spatial_bw", means, values, conics, samples,
                           ctx.num_rendered, grad_out.contiguous(), binning, sample_binning,
                           ranges, sample_ranges, ctx.debug)
        G = ctx.xchg.reduce(pack_grads(grads))
        gm, gv, gc = unpack_grads(G, grads)
        return (None, None, gm, gv, gc) + (None,) * 7


class SpatialShardedGaussianSampler(ShardedGaussianSampler):
    """ShardedGaussianSampler as a domain decomposition (see SupportExchange).

    Rank r's `samples` must stay inside its strip along the sharding axis (y at D = 2): `extents`
    [W, 2], or, by default, the all-gathered ranges of the first preprocess call.  The Gaussian
    tensors keep all P rows on every rank, but only the rows this rank holds are current and
    binned.  Training loop per step:

        sampler.preprocess(means, values, covariances, conics, samples)
        loss(sampler.sample_gaussians(), ...).backward()  # grads: global sums on the owned rows, 0 elsewhere
        optimizer.step()                                    # moves the owned rows only
        sampler.push([params...], means, conics)            # owners -> every rank their cut reaches

    All ranks start from identical parameters.  Changing means, conics or samples in place between
    preprocess and a sampling call raises (the exchange lists are those of the binned tensors)."""

    def __init__(self, debug=False, group=None, extents=None):
        super().__init__(debug, group)
        self.xchg = None
        self.extents = extents

    def preprocess(self, means, values, covariances, conics, samples):
        W = _world(self.group)
        rank = dist.get_rank(self.group) if W > 1 else 0
        D = samples.shape[1]
        known = self.xchg.extents if self.xchg is not None else self.extents
        strip = None
        if known is not None:
            e = torch.as_tensor(known).detach().double().cpu()[rank]
            strip = (float(e[0]), float(e[1])) if samples.shape[0] else (-math.inf, math.inf)
        # (an empty rank never leaves its strip)
        ovf = self.xchg.overflow if self.xchg is not None else None
        grid, offset, lo, hi, *flags = grid_and_box(samples, self.group, strip, ovf)
        left = flags[:1] if strip is not None else []
        if ovf is not None and flags[-1]:  # some pair outgrew its capacity: every rank re-pushes exactly
            self.xchg._push_exact(*self.xchg._last_push)
        if left and left[0]:  # raised on every rank together (no rank left waiting in a collective)
            raise ValueError(f"rank {rank}: the samples of some rank leave its strip along the sharding axis "
                             f"(this rank: [{lo[D - 1]}, {hi[D - 1]}] in [{strip[0]}, {strip[1]}]); pass "
                             f"extents covering every call's points")
        if self.xchg is None:
            ext = self.extents if self.extents is not None else shard_extents(samples, self.group)
            self.xchg = SupportExchange(means, conics, ext, rank, self.group, self.debug)
        area = 1.0
        for d in range(D):
            area *= max(hi[d] - lo[d], 0.0)
        (self.num_rendered, self.binning_buffer, self.sample_binning_buffer, self.ranges,
         self.sample_ranges, self.radii) = call_debug(
            _C.preprocess_gaussians_sharded, self.debug, "spatial_preprocess", means, values,
            covariances, conics, samples, grid, offset, self.xchg.held, area, self.debug)
        self.grid, self.offset = grid, offset
        self.means, self.values, self.conics, self.samples = means, values, conics, samples
        self._versions = self._now()

    def _now(self):
        ts = (self.means, self.conics, self.samples)
        return None if any(t.is_inference() for t in ts) else tuple(t._version for t in ts)

    def push(self, tensors, means=None, conics=None):
        """After optimizer.step(): the owners' rows of `tensors` to every rank their updated cut
        reaches (SupportExchange.push).  `means` / `conics` default to the tensors the last
        preprocess was given (right when they are the optimised leaves themselves)."""
        return self.xchg.push(tensors, self.means if means is None else means,
                              self.conics if conics is None else conics)

    def _sample(self, function):
        if self._now() != self._versions:  # (inference tensors: unknown, not checked)
            raise RuntimeError("SpatialShardedGaussianSampler: means, conics or samples were modified in place "
                               "after preprocess; call push() (after an optimizer step) and preprocess() again")
        return _SpatialSample.apply(function, self.xchg, self.means, self.values, self.conics,
                                    self.samples, self.num_rendered, self.binning_buffer,
                                    self.sample_binning_buffer, self.ranges, self.sample_ranges,
                                    self.debug)

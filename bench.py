"""Benchmark: sampled points/s (forward + backward) of the MI355X Gaussian sampler.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--function gaussian] [--no-cpu]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Workload (BASELINE.json configs): 1M anisotropic 2-D Gaussians, C = 1.
  * N = 1: configs[2], the headline -- 1M Gaussians x 2M query points on one GPU.
  * N > 1: configs[3] -- 1M Gaussians x 1M query points PER GPU (1M x 8M at N = 8), the tile
    grid the global one (all-reduce MIN/MAX of the sample bounds, sample_points.cu:70-74).  Two
    ways to sum the per-Gaussian gradients:
      --shard spatial (default): rank r's points are the strip r along y; the backward sends each
        partial row to its owner rank only (one RCCL all-to-all, SupportExchange.reduce) and the
        owners send their rows back to every rank that holds them (SupportExchange.push, an id
        and a row all-to-all) -- both inside the timed step;
      --shard dense: uniform points on every rank, ONE RCCL all-reduce (sum) of the packed
        [dmeans | dvalues | dconics] gradients per step (the north star's formulation).
    `--weak` keeps 2M query points per GPU instead.
One step = forward + backward through the autograd Function (+ the gradient exchange for N > 1);
binning (preprocess) is timed separately, as the metric asks.  kernels_ms and the roofline come
from HIP events on the render kernels' stream over every 4th timed step and the last (an event
record opens a ~5 us gap between kernels: events on every step would add ~1.4 % to it).

`python bench.py --gpus N` without a torch.distributed environment starts the N ranks itself
(a torch.distributed.run child, before this process touches the GPU) and exits with its code;
with fewer than N visible GPUs it fails loudly instead of reporting a 1-GPU number.

Printed: one JSON line on rank 0 (DESIGN.md section 5 explains every field).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# (DGS_TEST_PKG_ROOT: time a tools/variant.sh build, variants/NAME, as the tests can)
sys.path.insert(0, os.environ.get("DGS_TEST_PKG_ROOT") or os.path.join(REPO, "diff-gaussian-sampling_amd"))
sys.path.insert(0, REPO)

PEAK_FP32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E peak (6.29 TB/s measured copy)
PEAK_ATOMIC_GBS = 1300.0       # MI355X_MICROARCH.md "Global float atomics": chip-wide added-byte rate
FUNCS = {"gaussian": 0, "derivative": 1, "laplacian": 2, "third": 3}

# FLOP-eq per live pair at D = 2, counting every +, -, x (and unary minus) of the reference's
# expressions literally, per channel terms times C, plus one exp = 4 (its v_exp_f32 issue cost
# is ~2 FMAs).  (fixed, per-channel) for forward.cu:168-275 / backward.cu:108-416;
# the derivation is tabulated in DESIGN.md section 5.  gaussian = SURVEY 8d's 11+2C / 37+4C.
FLOPS_D2 = {
    "gaussian":   {"fwd": (11 + 4, 2), "bwd": (37 + 4, 4)},
    "derivative": {"fwd": (11 + 4, 10), "bwd": (60 + 4, 9)},
    "laplacian":  {"fwd": (15 + 4, 20), "bwd": (153 + 4, 17)},
    "third":      {"fwd": (39 + 4, 24), "bwd": (332 + 4, 33)},
}


def traffic_key(fn, C, P, N, aniso=1.0, grid=0):
    """profiles/traffic.json's workload key: the measured bytes of one workload are never
    reported for another (thin fields, lattices)."""
    return (f"{fn},C={C},P={P},N={N}" + (f",aniso={aniso:g}" if aniso > 1 else "")
            + (f",grid={grid}" if grid else ""))


def flops_per_live_pair(function, C):
    f = FLOPS_D2[function]
    return f["fwd"][0] + f["fwd"][1] * C, f["bwd"][0] + f["bwd"][1] * C


def algorithmic_bytes(function, P, N, C, D=2):
    """HBM bytes each render kernel must move at least: the forward reads the
    Gaussian parameters (means, conics, values) and the samples and writes the output; the
    backward reads the parameters, the samples and dL/dout and writes the three gradients."""
    S = D * (D + 1) // 2
    K = D ** FUNCS[function]
    params = 4 * P * (D + S + C)
    fwd = params + 4 * N * D + 4 * N * K * C
    bwd = 2 * params + 4 * N * D + 4 * N * K * C
    return fwd, bwd


def _count(n):
    """1000000 -> '1M', 256000 -> '256k' (metric labels)."""
    return f"{n // 1_000_000}M" if n % 1_000_000 == 0 else (f"{n // 1000}k" if n % 1000 == 0 else str(n))


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`--gpus N` outside torch.distributed: start the N ranks as a child process (nothing here
    has touched the GPU yet) and return its exit code."""
    import torch  # device_count() does not initialise the GPU on this image
    have = torch.cuda.device_count()
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {have}; "
              f"refusing to report a {have}-GPU number as {args.gpus}", file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--function", default="gaussian", choices=list(FUNCS))
    ap.add_argument("--functions", default=None,
                    help="comma-separated functions evaluated by ONE fused call per step "
                         "(sample_gaussians_multi, SURVEY 8f f2), e.g. gaussian,derivative,laplacian,third")
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--N", type=int, default=None,
                    help="query points per GPU (default: 2M on one GPU, 1M per GPU for N > 1)")
    ap.add_argument("--weak", action="store_true", help="N > 1: 2M query points per GPU")
    ap.add_argument("--ar-chunks", type=int, default=4,
                    help="--shard dense: row blocks of the pipelined gradient all-reduce")
    ap.add_argument("--push-sync", action="store_true",
                    help="--shard spatial: the exact push (one host sync per step) instead of the sync-free one")
    ap.add_argument("--shard", default="spatial", choices=["spatial", "dense"],
                    help="N > 1: spatial = rank r owns the strip r of the points along y and the "
                         "gradient sum moves only the Gaussians that reach another strip "
                         "(distributed.SupportExchange, SURVEY 8f f3); dense = uniform points on "
                         "every rank and one all-reduce of every gradient")
    ap.add_argument("--C", type=int, default=1)
    ap.add_argument("--aniso", type=float, default=1.0,
                    help="axis ratios U[1, aniso] at the headline's areas (thin Gaussians: 25)")
    ap.add_argument("--grid", type=int, default=0,
                    help="query points on a regular g x g lattice instead of uniform (SURVEY 8d config 5: 4096)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baselines")
    ap.add_argument("--cpu-samples", type=int, default=2048,
                    help="query points of the PyTorch-eager CPU baseline sample")
    ap.add_argument("--cpu-oracle-samples", type=int, default=2048,
                    help="query points of the 1-thread C-oracle CPU baseline sample")
    ap.add_argument("--pre-reps", type=int, default=5, help="warm preprocess repetitions (median)")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed steps for this long before the timed ones (0: none; the clock ramp)")
    ap.add_argument("--grid3", type=int, default=128,
                    help="--op volume: query points on a g^3 lattice (BASELINE config 5 names 256)")
    ap.add_argument("--op", default="sample", choices=["sample", "aggregate", "volume"],
                    help="sample: the headline (default); aggregate: aggregate_neighbors at SURVEY "
                         "config 5 (P = 1M, K = L = 16, F = 4), one GPU or N replicas")
    ap.add_argument("--cpu-rows", type=int, default=20000, help="aggregate CPU-baseline rows")
    ap.add_argument("--calltime", action="store_true",
                    help="also time fwd + bwd after an in-place step on the means WITHOUT re-binning: the "
                         "call-time path (the reference's whole tile pair set, dgs_reference.hip), next to "
                         "re-binning + the binned step")
    ap.add_argument("--pigs-graph", action="store_true",
                    help="also time the PIGS step -- re-binning + forward + backward -- eagerly and as ONE "
                         "captured HIP graph (preprocess_gaussians_capturable, SURVEY 8f row f1)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, sys.argv[1:])

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr, flush=True)
        return 2
    # DGS_BENCH_SHARE_GPU=1: rehearsal of the N-rank path with the ranks sharing the visible
    # GPU(s) (a 1-GPU box; RCCL refuses two ranks on one device, so gloo); never a measurement
    share = os.environ.get("DGS_BENCH_SHARE_GPU") == "1"
    if share:
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    if args.op == "aggregate":
        return bench_aggregate(args, world, rank, dev, torch, dist)
    if args.op == "volume":
        return bench_volume(args, world, rank, dev, torch, dist)
    return bench_sample(args, world, rank, dev, torch, dist)


def bench_sample(args, world, rank, dev, torch, dist):
    import diff_gaussian_sampling as dgs
    from diff_gaussian_sampling import synthetic as syn
    from diff_gaussian_sampling.distributed import (SupportExchange, allreduce_grads, grid_and_box, pack_grads,
                                                    shard_extents)

    P, C, D = args.P, args.C, 2
    N = args.N if args.N is not None else (2_000_000 if (world == 1 or args.weak) else 1_000_000)
    fn = args.function
    K = D ** FUNCS[fn]
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, D, C, seed=0, aniso=args.aniso))
    if args.grid:
        g = args.grid
        allpts = syn.grid_samples(g, D)
        per = (allpts.shape[0] + world - 1) // world
        samples = allpts[rank * per:(rank + 1) * per].to(dev)
        N = samples.shape[0]
    else:
        if world > 1 and args.shard == "spatial":  # strip r of [-1, 1) along y: the union is uniform
            samples = syn.strip_samples(N, D, rank, world, seed=4 + 1000 * rank).to(dev)
        else:
            samples = syn.samples(N, D, seed=4 + 1000 * rank).to(dev)
    spatial = world > 1 and args.shard == "spatial"
    dL = syn.grad_out(N, K, C, seed=5 + 1000 * rank).to(dev)
    for t in (means, values, conics):
        t.requires_grad_(True)

    # ---- preprocess (binning), reported separately: the first call (cold: code-object load,
    # allocator growth) and the warm median of --pre-reps further calls (the PIGS loop re-bins
    # every step because the means move)
    # one GPU: the reference API (grid computed on the device, one host sync per call); N > 1:
    # every shard bins with the global grid (distributed.global_tile_grid)
    grid = off = None
    xchg, xsetup_ms, area = None, 0.0, 0.0
    if world > 1:
        grid, off, lo, hi = grid_and_box(samples)
    if spatial:  # the owner / held sets: built once per run from the replicated parameters
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        xchg = SupportExchange(means, conics, shard_extents(samples), rank)
        torch.cuda.synchronize()
        xsetup_ms = (time.perf_counter() - t0) * 1e3
        area = (hi[0] - lo[0]) * (hi[1] - lo[1])  # fine cells sized for the strip's own density
    # the library's code objects onto the device (dgs_warmup; a training loop does it once at
    # start-up), timed on its own: preprocess_first_call_ms below is the first binning after it
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dgs.warmup()
    warmup_ms = (time.perf_counter() - t0) * 1e3
    pre_times = []
    for _ in range(1 + args.pre_reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if spatial:  # only the rows this rank holds (owned or reaching its strip)
            binned = dgs._C.preprocess_gaussians_sharded(means.detach(), values.detach(), covs,
                                                         conics.detach(), samples, grid, off, xchg.held,
                                                         area, False)
        elif world > 1:
            binned = dgs._C.preprocess_gaussians_bounded(means.detach(), values.detach(), covs,
                                                         conics.detach(), samples, grid, off, False)
        else:
            binned = dgs._C.preprocess_gaussians(means.detach(), values.detach(), covs,
                                                 conics.detach(), samples, False)
        torch.cuda.synchronize()
        pre_times.append((time.perf_counter() - t0) * 1e3)
    pre_first_ms = pre_times[0]
    pre_ms = sorted(pre_times[1:])[len(pre_times[1:]) // 2] if args.pre_reps > 0 else pre_first_ms
    R, gb, sb, rg, srg, radii = binned
    pre_extra = {}
    if world == 1 and args.pre_reps > 0:
        # the PIGS loop's other binning patterns (one GPU, reference API): fresh collocation points
        # every call (samples.min -- the grid offset -- moves each time), and two samplers whose
        # domains alternate (interior / boundary points); inputs generated before the clock starts
        med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
        fresh = [torch.rand(N, D, device=dev) * 2.0 - 1.0 for _ in range(args.pre_reps + 1)]
        # a second sampler's points: an independent draw over the same domain (another grid
        # offset, the same density and binning cost)
        other = torch.rand(N, D, device=dev, generator=torch.Generator(device=dev).manual_seed(77)) * 2.0 - 1.0
        pats = {"preprocess_resampled_ms": [fresh[i] for i in range(args.pre_reps + 1)],
                "preprocess_alternating_ms": [samples if i % 2 == 0 else other for i in range(2 * args.pre_reps + 2)]}
        for key, seq in pats.items():
            ts = []
            for sm in seq:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                dgs._C.preprocess_gaussians(means.detach(), values.detach(), covs, conics.detach(), sm, False)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            pre_extra[key] = med(ts[2:])
        del fresh, other
    fwd = {"gaussian": dgs.sample_gaussians, "derivative": dgs.sample_gaussians_derivative,
           "laplacian": dgs.sample_gaussians_laplacian,
           "third": dgs.sample_gaussians_third_derivative}[fn]
    dLv = dL.reshape((N,) + (D,) * FUNCS[fn] + (C,))
    flat = torch.empty(P * (D + C + D * (D + 1) // 2), device=dev)
    multi = args.functions.split(",") if args.functions else None
    if multi:  # one dL per function of the fused call
        dLm = [syn.grad_out(N, D ** FUNCS[f], C, seed=5 + 1000 * rank + 17 * i).to(dev).reshape(
            (N,) + (D,) * FUNCS[f] + (C,)) for i, f in enumerate(multi)]
    ar_ev = []  # (start, end) events around the gradient sum, on its stream
    push_ev = []  # (start, end) events around the spatial push

    def step(timed=False):
        for t in (means, values, conics):
            t.grad = None
        if multi:
            outs = dgs.sample_gaussians_multi(multi, means, values, conics, samples, R, gb, sb, rg, srg, False)
            torch.autograd.backward(list(outs), dLm)
        else:
            out = fwd(means, values, conics, samples, R, gb, sb, rg, srg, False)
            out.backward(dLv)
        if world > 1:
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            if spatial:  # partial rows to their owners (owner-side optimizer, SupportExchange)
                xchg.reduce(pack_grads((means.grad, values.grad, conics.grad)))
            else:  # the packed gradients in pipelined row blocks (distributed.allreduce_grads)
                g = allreduce_grads((means.grad, values.grad, conics.grad), chunks=args.ar_chunks)
                means.grad, values.grad, conics.grad = g
            if timed:
                e1.record()
                ar_ev.append((e0, e1))
            if spatial:  # the owners' rows to every rank their cut reaches (once per optimizer step)
                if timed:
                    p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    p0.record()
                xchg.push([means, values, conics], means, conics, sync=args.push_sync)
                if timed:
                    p1.record()
                    push_ev.append((p0, p1))

    for _ in range(args.warmup):
        step()

    def timed_block(events):
        # HIP events around the two render kernels (kernels_ms, the roofline) on every 4th timed
        # step (and the last): an event record opens a ~5 us gap between the step's kernels, 4
        # per step, so events on every step would add ~1.4 % to the step they time.
        ar_ev.clear()
        push_ev.clear()
        dgs._C.timing_read(0)
        dgs._C.timing_read(1)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for k in range(args.steps):
            dgs._C.timing_enable(events and (k % 4 == 3 or k == args.steps - 1))
            step(timed=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        dgs._C.timing_enable(False)
        return el

    # The render kernels run ~25 % slower for the first ~30 ms of sustained work (the clock ramp,
    # profiles/r04_clock_ramp.txt): K steps right after the W warmup steps are timed
    # and reported (ms_per_step_unsettled), then steps run until --settle-ms of them have passed,
    # and the K timed steps of the line follow, at the clocks a training loop runs at.
    unsettled_ms = timed_block(False) * 1e3 / args.steps if args.settle_ms > 0 else None
    settle_steps, t_settle = 0, time.perf_counter()

    def settling():  # (N > 1: rank 0's clock decides, every rank steps the same number of times)
        go = args.settle_ms > 0 and settle_steps < 1000 and (time.perf_counter() - t_settle) * 1e3 < args.settle_ms
        if world > 1:
            flag = torch.tensor([1.0 if go else 0.0], device=dev)
            dist.broadcast(flag, 0)
            go = bool(flag.item() > 0)
        return go

    while settling():
        for _ in range(4):
            step()
        settle_steps += 4
        torch.cuda.synchronize()
    settle_ms = (time.perf_counter() - t_settle) * 1e3
    elapsed = timed_block(True)
    nf, fms = dgs._C.timing_read(0)
    nb, bms = dgs._C.timing_read(1)
    rank_ms = elapsed * 1e3 / args.steps
    ar_ms = sum(a.elapsed_time(b) for a, b in ar_ev) / len(ar_ev) if ar_ev else 0.0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        per_rank = torch.zeros(world, device=dev, dtype=torch.float64)
        per_rank[rank] = rank_ms
        dist.all_reduce(per_rank)
        per_rank_ms = [float(x) for x in per_rank.cpu()]
    else:
        per_rank_ms = [rank_ms]
    ms_per_step = elapsed * 1e3 / args.steps
    value = N * world / (ms_per_step / 1e3)

    push_ms = sum(a.elapsed_time(b) for a, b in push_ev) / len(push_ev) if push_ev else 0.0
    # ---- live-pair count (diagnostic kernel, outside the timed region)
    w_cand, w_live = dgs._C.count_pairs(means.detach(), conics.detach(), samples, gb, sb, -104.0)
    avg_f = fms / max(nf, 1)
    avg_b = bms / max(nb, 1)
    fname = "+".join(multi) if multi else fn
    roofline = hbm = None
    if not multi:
        f_fwd, f_bwd = flops_per_live_pair(fn, C)
        b_fwd, b_bwd = algorithmic_bytes(fn, P, N, C)
        kern = {"forward_render": (avg_f, f_fwd, b_fwd), "backward_render": (avg_b, f_bwd, b_bwd)}
        dom = max(kern, key=lambda k: kern[k][0])
        dom_ms, dom_flops, dom_bytes = kern[dom]
        achieved = w_live * dom_flops / (dom_ms * 1e-3) / 1e12 if dom_ms > 0 else 0.0
        traffic = None
        tpath = os.path.join(REPO, "profiles", "traffic.json")
        if os.path.exists(tpath):
            try:
                tj = json.load(open(tpath))
                wl = tj.get("workloads", {}).get(traffic_key(fn, C, P, N, args.aniso, args.grid), {})
                traffic = wl.get(dom)
            except Exception:
                traffic = None
        roofline = {"bound": "valu", "kernel": dom, "achieved": achieved,
                    "peak": PEAK_FP32_VALU_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / PEAK_FP32_VALU_TFLOPS, "traffic": traffic,
                    "flops_per_live_pair": dom_flops, "flops_basis": "reference-literal, DESIGN.md 5"}
        gbs = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        hbm = {"kernel": dom, "algorithmic_bytes": dom_bytes, "achieved_GBs": gbs,
               "peak_GBs": PEAK_HBM_GBS, "frac": gbs / PEAK_HBM_GBS,
               "measured_bytes": traffic}

    workload = (f"{P // 1000}k Gaussians x {N // 1000}k query points per GPU"
                + (f" ({args.grid}^2 lattice)" if args.grid else "")
                + f", D=2, C={C}, function={fname}, fwd+bwd"
                + (f", axis ratios U[1, {args.aniso:g}]" if args.aniso > 1 else "")
                + ((", spatial strips + sparse gradient exchange" if spatial else ", RCCL all-reduce of grads")
                   if world > 1 else ""))
    result = {
        "metric": f"sampled points/sec (fwd+bwd), {_count(P)} Gaussians x "
                  + (f"{_count(N * world)} queries over {world} GPUs" if world > 1 else f"{_count(N)} queries")
                  + (f", fused functions {fname}" if multi else "")
                  + (f", function {fn}" if fn != "gaussian" and not multi else ""),
        "value": value,
        "unit": "points/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded uniform means/samples, anisotropic covariances, N(0,1) values)",
        # untimed steps between the warmup and the timed ones, and the K steps timed right after
        # the warmup (before them): the render kernels' clock ramp
        "settle": {"steps": settle_steps, "ms": settle_ms, "ms_per_step_unsettled": unsettled_ms},
        "config": {"workload": workload, "gaussians": P, "query_points_per_gpu": N,
                   "query_points_total": N * world, "channels": C, "function": fname,
                   "parallelism": f"query-point shards x{world}, Gaussians replicated"
                                  + ((", spatial strips, sparse gradient exchange (RCCL all-to-all)" if spatial
                                      else ", 1 RCCL all-reduce per step") if world > 1 else "")},
        "preprocess_ms": pre_ms,
        # the Physics-Informed-GS loop re-bins every step (means move): its step time
        "total_ms_per_step_incl_preprocess": ms_per_step + pre_ms,
        "preprocess_first_call_ms": pre_first_ms,
        "library_warmup_ms": warmup_ms,
        **pre_extra,
        "kernels_ms": {"forward_render": avg_f, "backward_render": avg_b},
        "pairs": {"W_cand": w_cand, "W_live": w_live, "num_rendered": R},
        "entries": dict(zip(("num_rendered", "fine_entries", "literal_path_entries", "fine_cells", "thin_entries",
                             "sort_path_entries"),
                            dgs._C.binning_info(gb, sb))),
        "roofline": roofline,
        "hbm": hbm,
        "cpu_baseline": None,
    }
    if world > 1:
        F = D + C + D * (D + 1) // 2
        result["distributed"] = {"backend": dist.get_backend(), "world_size": world, "shard": args.shard,
                                 "per_rank_ms_per_step": per_rank_ms,
                                 "gradient_sum_ms_rank0": ar_ms,
                                 "gradient_sum_bytes_rank0": (int(xchg.rows_moved() * F * 4) if spatial
                                                              else int(flat.numel() * 4)),
                                 "dense_allreduce_bytes": int(flat.numel() * 4),
                                 "exchange_setup_ms_once": xsetup_ms,
                                 "push_ms_rank0_in_step": push_ms,
                                 "held_rows_rank0": int(xchg.held.sum()) if spatial else P,
                                 "w_cand_per_point_rank0": w_cand / N}

    if args.calltime and world == 1 and not multi:
        # an optimizer-like in-place step on the means (1/10 of the mean spacing), then sampling
        # with the stale binning: every call compares its inputs with the binned copies and takes
        # the reference's own pair set (forward.cu:119-162 over every tile pair, W_ref ~ 2.3e11 at
        # the headline), as the reference would.  Against: re-binning, then the binned step.
        m_keep = means.detach().clone()
        with torch.no_grad():
            step_m = torch.randn(means.shape, generator=torch.Generator().manual_seed(9)).to(dev) * (0.1 * 2.0 / P ** 0.5)
            means.add_(step_m)
        ct = []
        for k in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            ct.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        R, gb, sb, rg, srg, _ = dgs._C.preprocess_gaussians(means.detach(), values.detach(), covs, conics.detach(),
                                                             samples, False)
        step()
        torch.cuda.synchronize()
        rebin_ms = (time.perf_counter() - t0) * 1e3
        with torch.no_grad():
            means.copy_(m_keep)
        result["calltime"] = {"ms_per_step_stale_binning": sorted(ct)[1],
                              "ms_rebin_plus_step": rebin_ms,
                              "note": "fwd + bwd after an in-place means update without re-preprocess (the "
                                      "reference's tile pair set, evaluated on the GPU) vs preprocess + fwd + bwd"}
    if args.pigs_graph and world == 1 and not multi:
        # The PIGS loop re-bins after every optimizer step.  Eager: preprocess (one host sync) +
        # forward + backward.  Graph: the same three captured once with torch.cuda.graph
        # (the capturable binning keeps R / E / status on the device) and replayed; the binning
        # runs in full at every replay.  Both from the same tensors, K steps each, medians.
        grid, off = dgs._C.tile_grid(samples)
        cap = dgs.capacity_from(gb, sb, slack=0.125)
        md, vd, cd = means.detach(), values.detach(), conics.detach()

        def pigs_eager():
            for t in (means, values, conics):
                t.grad = None
            R2, gb2, sb2, rg2, srg2, _ = dgs._C.preprocess_gaussians(md, vd, covs, cd, samples, False)
            fwd(means, values, conics, samples, R2, gb2, sb2, rg2, srg2, False).backward(dLv)

        fixed_sb = sb  # (the collocation points stay put: the captured binning copies their sample side)

        def pigs_body():
            R2, gb2, sb2, rg2, srg2, _, st2 = dgs.preprocess_gaussians_capturable(md, vd, covs, cd, samples, grid,
                                                                                    off, cap, samples_binned=fixed_sb)
            fwd(means, values, conics, samples, cap[2], gb2, sb2, rg2, srg2, False).backward(dLv)
            return st2

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                for t in (means, values, conics):
                    t.grad = None
                pigs_body()
        torch.cuda.current_stream().wait_stream(side)
        for t in (means, values, conics):
            t.grad = None
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_st = pigs_body()
        times = {}
        for name, run_step in (("eager", pigs_eager), ("graph", graph.replay)):
            for _ in range(3):
                run_step()
            torch.cuda.synchronize()
            ms = []
            for _ in range(max(args.steps, 5)):
                t0 = time.perf_counter()
                run_step()
                torch.cuda.synchronize()
                ms.append((time.perf_counter() - t0) * 1e3)
            times[name] = sorted(ms)[len(ms) // 2]
        result["pigs_graph"] = {"ms_per_step_eager": times["eager"], "ms_per_step_graph": times["graph"],
                                "graph_status": int(g_st.item()), "capacity": cap,
                                "note": "re-binning + fwd + bwd per step, host-timed medians; graph = one "
                                        "torch.cuda.graph replay of preprocess_gaussians_capturable + the sample "
                                        "call + backward; both copy the fixed samples' sample side from an "
                                        "earlier binning (samples_binned) instead of sorting them per step"}
        del graph
    if rank == 0 and world == 1 and not args.no_cpu and not multi:
        cpu_baselines(result, means.detach().cpu(), values.detach().cpu(), covs.cpu(),
                      conics.detach().cpu(), samples.cpu(), dL.cpu(), fn, w_live, N, args, torch)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def cpu_baselines(result, means, values, covs, conics, samples, dL, fn, w_live_total, N, args, torch):
    """Two host-side baselines on a bounded sample of the same workload, binning excluded:
      cpu_baseline        PyTorch eager (oracle/torch_eager.py) on all host threads torch uses,
                          as BASELINE.json's north_star asks, extrapolated to the whole workload
                          by W_live(total) / W_live(sample) (BASELINE.md CPU plan);
      cpu_baseline_oracle the 1-thread C oracle (the literal per-pair loop), same extrapolation.
    The first points in tile-sorted order are the sample."""
    import numpy as np
    from oracle import oracle as orc
    orc.build()
    ob = orc.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    order = np.argsort(ob.sample_keys(), kind="stable").astype(np.int32)

    def sample_live(sub):
        return ob.count_pairs(conics.numpy(), -104.0, subset=sub)[1]

    if fn == "gaussian":
        from oracle import torch_eager as te
        sub = order[:args.cpu_samples]
        t0 = time.perf_counter()
        te.gaussian_fwd_bwd(ob, means.numpy(), values.numpy(), conics.numpy(), samples.numpy(),
                            dL.numpy(), sub)
        dt = time.perf_counter() - t0
        wl = max(sample_live(sub), 1)
        t_all = dt * w_live_total / wl
        result["cpu_baseline"] = {
            "value": N / t_all, "unit": "points/s", "cores": torch.get_num_threads(), "kind": "port",
            "extrapolated": True,
            "sample": f"first {len(sub)} of the {N} query points in tile order (W_live {wl}), every "
                      f"Gaussian of their tiles, torch eager fwd + autograd bwd, binning excluded "
                      f"({dt:.1f} s); scaled by W_live(total) {w_live_total} / W_live(sample)"}
    sub = order[:args.cpu_oracle_samples]
    t0 = time.perf_counter()
    ob.forward(fn, values.numpy(), conics.numpy(), subset=sub)
    ob.backward(fn, values.numpy(), conics.numpy(), dL.numpy(), subset=sub)
    dt = time.perf_counter() - t0
    wl = max(sample_live(sub), 1)
    key = "cpu_baseline_oracle" if fn == "gaussian" else "cpu_baseline"
    result[key] = {"value": N / (dt * w_live_total / wl), "unit": "points/s", "cores": 1, "kind": "port",
                   "extrapolated": True,
                   "sample": f"first {len(sub)} of the {N} query points in tile order (W_live {wl}), "
                             f"1-thread C oracle fwd+bwd, binning excluded ({dt:.1f} s); scaled by "
                             f"W_live(total) / W_live(sample)"}


def bench_volume(args, world, rank, dev, torch, dist):
    """D = 3 fields (beyond the reference): P Gaussians (default 1M) against a
    g^3 lattice of query points (--grid3, config 5's "256^3 grid"), one function, forward +
    backward through VolumeSampler's autograd Function per step; the binning (preprocess) is
    timed separately.  N > 1 runs N independent replicas."""
    from diff_gaussian_sampling import synthetic as syn
    from diff_gaussian_sampling.volume import VolumeSampler
    P, C, fn = args.P, args.C, args.function
    code = FUNCS[fn]
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians3(P, C, seed=0))
    samples = syn.grid_samples3(args.grid3).to(dev)
    N = samples.shape[0]
    for t in (means, values, conics):
        t.requires_grad_(True)
    vs = VolumeSampler(False)
    pre = []
    for _ in range(1 + max(args.pre_reps, 1)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vs.preprocess(means, values, covs, conics, samples)
        torch.cuda.synchronize()
        pre.append((time.perf_counter() - t0) * 1e3)
    pre_ms = sorted(pre[1:])[len(pre[1:]) // 2]
    run = [vs.sample_gaussians, vs.sample_gaussians_derivative, vs.sample_gaussians_laplacian,
           vs.sample_gaussians_third_derivative][code]
    dL = torch.randn((N,) + (3,) * code + (C,), generator=torch.Generator().manual_seed(5)).to(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fwd_ms, bwd_ms = [], []

    def step(timed):
        for t in (means, values, conics):
            t.grad = None
        if timed:
            ev[0].record()
        out = run()
        if timed:
            ev[1].record()
        out.backward(dL)
        if timed:
            ev[2].record()
            torch.cuda.synchronize()
            fwd_ms.append(ev[0].elapsed_time(ev[1]))
            bwd_ms.append(ev[1].elapsed_time(ev[2]))

    # the first step also builds the transposed lists (at its backward, once per
    # preprocess_aggregate: a loop that re-runs the neighbour search every step pays it per step)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    step(False)
    torch.cuda.synchronize()
    first_step_ms = (time.perf_counter() - t1) * 1e3
    for _ in range(args.warmup - 1):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    step(True)
    ms = elapsed * 1e3 / args.steps
    from diff_gaussian_sampling import _C
    w_eval, w_live = _C.volume_count_pairs(means.detach(), conics.detach(), samples, vs.binning)
    # forward FLOPs per live pair of the D = 3 expressions (include/dgs_volume.h), C = 1: X 3,
    # the two quadratic sums 8 + 8, power 2, expf 4 (FLOP-eq), a = A X 15 (functions >= 1), the
    # unique terms (laplacian 6 x 2, third 10 x 8) and v G t accumulated, 3 per unique component
    # and channel
    KU = [1, 3, 6, 10][code]
    f_fwd = 25 + [0, 15, 15, 15][code] + [0, 0, 12, 80][code] + 3 * KU * C
    fwd_s = fwd_ms[-1] * 1e-3
    ach = w_live * f_fwd / fwd_s / 1e12
    result = {
        "metric": f"sampled points/sec (fwd+bwd), D=3, {P // 1000}k Gaussians x {args.grid3}^3 lattice",
        "value": N * world / (ms / 1e3), "unit": "points/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded uniform means, rotated anisotropic covariances, N(0,1) values)",
        "config": {"workload": f"D=3 {fn}, P={P}, {args.grid3}^3 query lattice, C={C}, fwd+bwd",
                   "query_points": N, "parallelism": f"replicas x{world}",
                   "note": "beyond the reference (no D = 3 path there); SURVEY 8f row f4"},
        "preprocess_ms": pre_ms, "preprocess_first_call_ms": pre[0],
        "phases_ms": {"forward": fwd_ms[-1], "backward": bwd_ms[-1]},
        "pairs": {"W_eval": int(w_eval), "W_live": int(w_live)},
        "roofline": {"bound": "valu", "kernel": "k_vol_forward", "achieved": ach, "peak": PEAK_FP32_VALU_TFLOPS,
                     "unit": "TFLOP/s", "frac": ach / PEAK_FP32_VALU_TFLOPS, "traffic": None,
                     "flops_per_live_pair": f_fwd, "flops_basis": "D = 3 expressions, DESIGN.md 4.8"},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def bench_aggregate(args, world, rank, dev, torch, dist):
    """aggregate_neighbors: P = 1M Gaussians (the headline's, radii from
    preprocess_gaussians), K = L = 16, F = 4.  A step = forward + backward through the autograd
    Function on resident neighbour lists; preprocess_aggregate is timed separately.  N > 1 runs
    N independent replicas (the rows shard, but nothing in a step is exchanged)."""
    import diff_gaussian_sampling as dgs
    from diff_gaussian_sampling import synthetic as syn
    P, L, K, F, D = args.P, 16, 16, 4, 2
    E = 2 * D * F + 1
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, D, 1, seed=0))
    samples = syn.samples(args.N or 2_000_000, D, seed=4).to(dev)
    radii = dgs.preprocess_gaussians(means, values, covs, conics, samples, False)[5]
    del samples
    g = torch.Generator().manual_seed(7)
    feats = [torch.randn(P, L, generator=g), torch.randn(L, L, generator=g) / L,
             torch.randn(P, K, generator=g), torch.randn(P, K, generator=g),
             torch.rand(F, generator=g) * 2.5 + 0.5, torch.randn(2 * E, generator=g)]
    feats_d = [t.to(dev).requires_grad_(True) for t in feats]
    dL = torch.randn(P, L, generator=torch.Generator().manual_seed(5)).to(dev)
    sampler = dgs.GaussianSampler(False)
    sampler.means, sampler.conics, sampler.radii = means, conics, radii
    pre_times = []  # first call (cold: code-object load, allocator growth), then warm calls
    for _ in range(1 + max(args.pre_reps, 1)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sampler.preprocess_aggregate()
        torch.cuda.synchronize()
        pre_times.append((time.perf_counter() - t0) * 1e3)
    pre_ms = sorted(pre_times[1:])[len(pre_times[1:]) // 2]
    Lnb = int(sampler.indices.numel())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fwd_ms, bwd_ms = [], []

    def step(timed):
        for t in feats_d:
            t.grad = None
        if timed:
            ev[0].record()
        out = sampler.aggregate_neighbors(*feats_d)
        if timed:
            ev[1].record()
        out.backward(dL)
        if timed:
            ev[2].record()
            torch.cuda.synchronize()
            fwd_ms.append(ev[0].elapsed_time(ev[1]))
            bwd_ms.append(ev[1].elapsed_time(ev[2]))

    # the first step also builds the transposed lists (at its backward, once per
    # preprocess_aggregate: a loop that re-runs the neighbour search every step pays it per step)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    step(False)
    torch.cuda.synchronize()
    first_step_ms = (time.perf_counter() - t1) * 1e3
    for _ in range(args.warmup - 1):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    for _ in range(3):  # per-phase event times, outside the timed region
        step(True)
    ms_per_step = elapsed * 1e3 / args.steps
    f_ms, b_ms = sorted(fwd_ms)[1], sorted(bwd_ms)[1]
    # algorithmic bytes: per slot the backward streams indices (8), dists (8), densities (4),
    # weights / embeddings / factors (12) and adds L + K floats into neighbour rows
    stream_b = 32.0 * Lnb + 4.0 * P * (3 * L + 3 * K)
    atomic_b = 4.0 * (L + K) * Lnb
    if os.environ.get("DGS_AGG_TRANSPOSE", "1") != "0" and L + K <= 64:
        # transposed backward: no float atomics on the neighbour rows; the row pass
        # streams the slot arrays and stores one 16-byte record per slot, the per-neighbour sum
        # reads the transposed slot ids (4 B) and the records (16 B, gathered): HBM-bound
        rec_b = 36.0 * Lnb
        roof_bwd = {"bound": "hbm", "kernel": "k_agg_backward_s + k_agg_tgather",
                    "achieved": (stream_b + rec_b) / (b_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": (stream_b + rec_b) / (b_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                    "bytes_basis": "slot streams 32 B + per-row terms, plus the 36 B per slot of the "
                                   "transposed records (written, gathered, slot ids)", "traffic": None}
    else:
        # the atomic form is bound by the memory-side float-atomic rate (its added bytes)
        roof_bwd = {"bound": "atomic", "kernel": "k_agg_backward_s",
                    "achieved": atomic_b / (b_ms * 1e-3) / 1e9, "peak": PEAK_ATOMIC_GBS,
                    "unit": "GB/s (float-atomic added bytes)",
                    "frac": atomic_b / (b_ms * 1e-3) / 1e9 / PEAK_ATOMIC_GBS, "traffic": None}
    result = {
        "metric": "aggregated neighbour slots/sec (aggregate_neighbors fwd+bwd), 1M Gaussians",
        "value": Lnb * world / (ms_per_step / 1e3),
        "unit": "slots/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (the headline Gaussians; N(0,1) features, queries, keys, transform/L)",
        "config": {"workload": f"aggregate_neighbors, P={P}, K={K}, L={L}, F={F}, D=2, fwd+bwd",
                   "neighbour_slots": Lnb, "parallelism": f"replicas x{world}"},
        "preprocess_aggregate_ms": pre_ms,
        "preprocess_aggregate_first_call_ms": pre_times[0],
        # the first fwd + bwd on new lists: + the transposition of the lists (built lazily at
        # that backward); preprocess_aggregate + this is a re-binning loop's step
        "first_step_ms_incl_transpose": first_step_ms,
        "phases_ms": {"forward": f_ms, "backward": b_ms},
        "roofline": roof_bwd,
        # the forward: per slot it streams indices / dists / densities (20 B) and writes weights /
        # embeddings / factors (12 B), reads the neighbour's feature and key rows (4 (L + K) B,
        # mostly from cache: neighbours of adjacent rows coincide) and writes out once per row
        "roofline_forward": {"bound": "hbm", "kernel": "k_agg_forward_s",
                             "achieved": (32.0 * Lnb + 4.0 * P * (L + 2 * K + 2 * L)) / (f_ms * 1e-3) / 1e9,
                             "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": (32.0 * Lnb + 4.0 * P * (L + 2 * K + 2 * L)) / (f_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                             "gathered_row_bytes": 4.0 * (L + K) * Lnb, "traffic": None},
        "hbm": {"kernel": "k_agg_backward_s", "algorithmic_bytes": stream_b + atomic_b,
                "achieved_GBs": (stream_b + atomic_b) / (b_ms * 1e-3) / 1e9, "peak_GBs": PEAK_HBM_GBS,
                "frac": (stream_b + atomic_b) / (b_ms * 1e-3) / 1e9 / PEAK_HBM_GBS},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import oracle as orc
        from oracle import torch_eager as te
        orc.build()
        host = lambda t: t.detach().cpu().numpy()  # noqa: E731
        args_np = [host(t) for t in feats_d]
        idx, rg, X, dn, inv = (host(t) for t in (sampler.indices, sampler.ranges, sampler.dists,
                                                sampler.densities, sampler.inv_total_densities))
        rows = min(args.cpu_rows, P)
        nslots = int(rg[rows - 1])
        # PyTorch eager on the host cores (BASELINE.json north_star): the same math vectorised
        # over the rows' slots, autograd backward (oracle/torch_eager.py aggregate_fwd_bwd)
        t0 = time.perf_counter()
        te.aggregate_fwd_bwd(*args_np, idx, rg, X, dn, inv, host(dL), rows=rows)
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": nslots / dt, "unit": "slots/s", "cores": torch.get_num_threads(),
                                  "kind": "port",
                                  "sample": f"first {rows} rows ({nslots} slots) of the same lists, torch eager "
                                            f"fwd + autograd bwd, neighbour search excluded ({dt:.1f} s)"}
        t0 = time.perf_counter()
        w, e_, f_, _ = orc.agg_forward(*args_np, idx, rg, X, dn, inv, rows=rows)
        orc.agg_backward(*args_np, idx, rg, X, dn, w, e_, f_, inv, host(dL), rows=rows)
        dt = time.perf_counter() - t0
        result["cpu_baseline_oracle"] = {"value": nslots / dt, "unit": "slots/s", "cores": 1, "kind": "port",
                                         "sample": f"first {rows} rows ({nslots} slots) of the same lists, "
                                                   f"1-thread C oracle fwd+bwd, neighbour search excluded ({dt:.1f} s)"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Benchmark: sampled points/s (forward + backward) of the MI355X Gaussian sampler.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--function gaussian] [--no-cpu]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Workload (BASELINE.json configs[2], the headline): 1M anisotropic 2-D Gaussians, C = 1, and
2M uniform query points PER GPU (weak scaling; configs[3] is the N = 8 case with 1M per GPU
in spirit -- every rank evaluates the same 1M Gaussians on its own 2M points).  Gaussians are
replicated (same seed on every rank); the tile grid is the global one (all-reduce MIN/MAX of
the sample bounds); one step = forward + backward through the autograd Function, plus, for
N > 1, ONE RCCL all-reduce (sum) of the packed [dmeans | dvalues | dconics] gradients.

Printed: one JSON line on rank 0 (see README of the bench contract in DESIGN.md).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "diff-gaussian-sampling_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_FP32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate
FUNCS = {"gaussian": 0, "derivative": 1, "laplacian": 2, "third": 3}


def flops_per_live_pair(function, C):
    """FLOP-eq per live pair for the gaussian function: forward 11 + 2C, backward
    37 + 4C, each with one exp counted as 4 (its v_exp_f32 issue cost is 2 FMAs)."""
    return 11 + 2 * C + 4, 37 + 4 * C + 4


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


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
    ap.add_argument("--N", type=int, default=2_000_000, help="query points per GPU")
    ap.add_argument("--C", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--cpu-samples", type=int, default=3072)
    ap.add_argument("--cpu-torch-samples", type=int, default=2048,
                    help="query points of the PyTorch-eager CPU baseline")
    ap.add_argument("--pre-reps", type=int, default=5, help="warm preprocess repetitions (median)")
    ap.add_argument("--op", default="sample", choices=["sample", "aggregate"],
                    help="sample: the headline (default); aggregate: aggregate_neighbors at SURVEY "
                         "config 5 (P = 1M, K = L = 16, F = 4), one GPU or N replicas")
    ap.add_argument("--cpu-rows", type=int, default=20000, help="aggregate CPU-baseline rows")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    if args.op == "aggregate":
        return bench_aggregate(args, world, rank, dev)

    import diff_gaussian_sampling as dgs
    from diff_gaussian_sampling import synthetic as syn
    from diff_gaussian_sampling.distributed import global_tile_grid

    P, N, C, D = args.P, args.N, args.C, 2
    fn = args.function
    K = D ** FUNCS[fn]
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, D, C, seed=0))
    samples = syn.samples(N, D, seed=4 + 1000 * rank).to(dev)
    dL = syn.grad_out(N, K, C, seed=5 + 1000 * rank).to(dev)
    for t in (means, values, conics):
        t.requires_grad_(True)

    # ---- preprocess (binning), reported separately
    # first call (cold: code-object load, allocator growth) and the warm median of
    # --pre-reps further calls (the PIGS loop re-bins every step because means change)
    grid, off = global_tile_grid(samples)
    pre_times = []
    for _ in range(1 + args.pre_reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        binned = dgs._C.preprocess_gaussians_bounded(means.detach(), values.detach(), covs,
                                                     conics.detach(), samples, grid, off, False)
        torch.cuda.synchronize()
        pre_times.append((time.perf_counter() - t0) * 1e3)
    pre_first_ms = pre_times[0]
    pre_ms = sorted(pre_times[1:])[len(pre_times[1:]) // 2] if args.pre_reps > 0 else pre_first_ms
    R, gb, sb, rg, srg, radii = binned
    fwd = {"gaussian": dgs.sample_gaussians, "derivative": dgs.sample_gaussians_derivative,
           "laplacian": dgs.sample_gaussians_laplacian,
           "third": dgs.sample_gaussians_third_derivative}[fn]
    dLv = dL.reshape((N,) + (D,) * FUNCS[fn] + (C,))
    flat = torch.empty(P * (D + C + D * (D + 1) // 2), device=dev)
    multi = args.functions.split(",") if args.functions else None
    if multi:  # one dL per function of the fused call
        dLm = [syn.grad_out(N, D ** FUNCS[f], C, seed=5 + 1000 * rank + 17 * i).to(dev).reshape(
            (N,) + (D,) * FUNCS[f] + (C,)) for i, f in enumerate(multi)]

    def step():
        for t in (means, values, conics):
            t.grad = None
        if multi:
            outs = dgs.sample_gaussians_multi(multi, means, values, conics, samples, R, gb, sb, rg, srg, False)
            torch.autograd.backward(list(outs), dLm)
        else:
            out = fwd(means, values, conics, samples, R, gb, sb, rg, srg, False)
            out.backward(dLv)
        if world > 1:
            torch.cat([means.grad.reshape(-1), values.grad.reshape(-1), conics.grad.reshape(-1)], out=flat)
            dist.all_reduce(flat)

    for _ in range(args.warmup):
        step()
    dgs._C.timing_read(0)
    dgs._C.timing_read(1)
    dgs._C.timing_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    dgs._C.timing_enable(False)
    nf, fms = dgs._C.timing_read(0)
    nb, bms = dgs._C.timing_read(1)
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    ms_per_step = elapsed * 1e3 / args.steps
    value = N * world / (ms_per_step / 1e3)

    # ---- live-pair count (diagnostic kernel, outside the timed region)
    w_cand, w_live = dgs._C.count_pairs(means.detach(), conics.detach(), samples, gb, sb, -104.0)
    f_fwd, f_bwd = flops_per_live_pair(fn, C)
    avg_f = fms / max(nf, 1)
    avg_b = bms / max(nb, 1)
    kern = {"forward_render": (avg_f, f_fwd), "backward_render": (avg_b, f_bwd)}
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms, dom_flops = kern[dom]
    achieved = w_live * dom_flops / (dom_ms * 1e-3) / 1e12 if dom_ms > 0 else 0.0
    traffic = None
    tpath = os.path.join(REPO, "profiles", "traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            traffic = tj.get(dom)
        except Exception:
            traffic = None

    if multi:  # per-pair FLOPs of the fused functions are not in SURVEY 8d: no roofline line
        fn = "+".join(multi)
    result = {
        "metric": "sampled points/sec (fwd+bwd), 1M Gaussians x 2M queries per GPU"
                  + (f", fused functions {fn}" if multi else ""),
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
        "config": {"workload": f"{P // 1000}k Gaussians x {N // 1000}k query points per GPU, D=2, "
                               f"C={C}, function={fn}, fwd+bwd" + (", RCCL all-reduce of grads" if world > 1 else ""),
                   "gaussians": P, "query_points_per_gpu": N, "channels": C, "function": fn,
                   "parallelism": f"query-point shards x{world}, Gaussians replicated"},
        "preprocess_ms": pre_ms,
        # the Physics-Informed-GS loop re-bins every step (means move): its step time
        "total_ms_per_step_incl_preprocess": ms_per_step + pre_ms,
        "preprocess_first_call_ms": pre_first_ms,
        "kernels_ms": {"forward_render": avg_f, "backward_render": avg_b},
        "pairs": {"W_cand": w_cand, "W_live": w_live, "num_rendered": R},
        "roofline": {"bound": "valu", "kernel": dom, "achieved": achieved,
                     "peak": PEAK_FP32_VALU_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_FP32_VALU_TFLOPS, "traffic": traffic,
                     "flops_per_live_pair": dom_flops},
        "cpu_baseline": None,
    }

    if multi:
        result["roofline"] = None
    if rank == 0 and world == 1 and not args.no_cpu and not multi:
        result["cpu_baseline"] = cpu_baseline(means.detach().cpu(), values.detach().cpu(),
                                              covs.cpu(), conics.detach().cpu(), samples.cpu(),
                                              dL.cpu(), fn, args.cpu_samples)
        if fn == "gaussian":  # BASELINE north_star: PyTorch-eager CPU on the host cores, beside it
            result["cpu_baseline_torch_eager"] = cpu_baseline_torch(
                means.detach().cpu(), values.detach().cpu(), covs.cpu(), conics.detach().cpu(),
                samples.cpu(), dL.cpu(), args.cpu_torch_samples)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E peak
PEAK_ATOMIC_GBS = 1300.0     # MI355X_MICROARCH.md "Global float atomics": chip-wide added-byte rate


def bench_aggregate(args, world, rank, dev):
    """aggregate_neighbors: P = 1M Gaussians (the headline's, radii from
    preprocess_gaussians), K = L = 16, F = 4.  A step = forward + backward through the autograd
    Function on resident neighbour lists; preprocess_aggregate is timed separately.  N > 1 runs
    N independent replicas (the rows shard, but nothing in a step is exchanged)."""
    import diff_gaussian_sampling as dgs
    from diff_gaussian_sampling import synthetic as syn
    P, L, K, F, D = args.P, 16, 16, 4, 2
    E = 2 * D * F + 1
    means, values, covs, conics = (t.to(dev) for t in syn.gaussians(P, D, 1, seed=0))
    samples = syn.samples(args.N, D, seed=4).to(dev)
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

    for _ in range(args.warmup):
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
        "phases_ms": {"forward": f_ms, "backward": b_ms},
        "roofline": {"bound": "hbm", "kernel": "k_agg_backward_s", "achieved": stream_b / (b_ms * 1e-3) / 1e9,
                     "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": stream_b / (b_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, "traffic": None,
                     "atomic_added_GBs": atomic_b / (b_ms * 1e-3) / 1e9, "atomic_peak_GBs": PEAK_ATOMIC_GBS,
                     "atomic_frac": atomic_b / (b_ms * 1e-3) / 1e9 / PEAK_ATOMIC_GBS},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        import numpy as np
        from oracle import oracle as orc
        orc.build()
        host = lambda t: t.detach().cpu().numpy()  # noqa: E731
        args_np = [host(t) for t in feats_d]
        idx, rg, X, dn, inv = (host(t) for t in (sampler.indices, sampler.ranges, sampler.dists,
                                                sampler.densities, sampler.inv_total_densities))
        rows = min(args.cpu_rows, P)
        t0 = time.perf_counter()
        w, e_, f_, _ = orc.agg_forward(*args_np, idx, rg, X, dn, inv, rows=rows)
        orc.agg_backward(*args_np, idx, rg, X, dn, w, e_, f_, inv, host(dL), rows=rows)
        dt = time.perf_counter() - t0
        nslots = int(rg[rows - 1])
        result["cpu_baseline"] = {"value": nslots / dt, "unit": "slots/s", "cores": 1, "kind": "port",
                                  "sample": f"first {rows} rows ({nslots} slots) of the same lists, "
                                            f"fwd+bwd, neighbour search excluded ({dt:.1f} s)"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(means, values, covs, conics, samples, dL, fn, nsub):
    """The oracle (literal CPU restatement of the reference: every pair of the tile, in gid
    order, 1 thread) on the first `nsub` query points: forward + backward, binning excluded."""
    import numpy as np
    from oracle import oracle as orc
    orc.build()
    ob = orc.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    sub = np.arange(nsub, dtype=np.int32)
    t0 = time.perf_counter()
    ob.forward(fn, values.numpy(), conics.numpy(), subset=sub)
    ob.backward(fn, values.numpy(), conics.numpy(), dL.numpy(), subset=sub)
    dt = time.perf_counter() - t0
    return {"value": nsub / dt, "unit": "points/s", "cores": 1, "kind": "port",
            "sample": f"first {nsub} of the 2M query points of the same workload, fwd+bwd, "
                      f"binning excluded ({dt:.1f} s)"}


def cpu_baseline_torch(means, values, covs, conics, samples, dL, nsub):
    """PyTorch eager (float32, all host threads torch uses) on the first `nsub` query points:
    the same pair set and math, forward + backward by autograd (oracle/torch_eager.py)."""
    import numpy as np
    from oracle import oracle as orc
    from oracle import torch_eager as te
    orc.build()
    ob = orc.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
    sub = np.arange(nsub, dtype=np.int32)
    t0 = time.perf_counter()
    te.gaussian_fwd_bwd(ob, means.numpy(), values.numpy(), conics.numpy(), samples.numpy(),
                        dL.numpy(), sub)
    dt = time.perf_counter() - t0
    return {"value": nsub / dt, "unit": "points/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"first {nsub} of the 2M query points, every Gaussian of their tiles, "
                      f"torch eager fwd + autograd bwd, binning excluded ({dt:.1f} s)"}


if __name__ == "__main__":
    main()

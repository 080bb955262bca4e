"""A/B timing of package variants (tools/variant.sh) in alternating child processes on one GPU,
so clock drift and device differences hit every variant alike.

    python tools/ab.py [--rounds 4] [--kbench-args "..."] base variants/X variants/Y ...

`base` means the in-tree package; `path:K=V,K2=V2` adds environment variables to that run.  Prints per-variant medians of tools/kbench.py's numbers.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--kbench-args", default="")
ap.add_argument("variants", nargs="+")
a = ap.parse_args()
res = {v: [] for v in a.variants}
for v in a.variants:  # a mistyped variant would silently time the in-tree build
    pv = v.partition(":")[0]
    if pv != "base" and not os.path.isdir(os.path.join(REPO, pv, "diff_gaussian_sampling")):
        sys.exit(f"no variant package at {os.path.join(REPO, pv)} (tools/variant.sh builds variants/NAME)")
for r in range(a.rounds):
    for v in a.variants:
        env = dict(os.environ)
        pv, _, extra = v.partition(":")
        for kv in filter(None, extra.split(",")):
            k, _, val = kv.partition("=")
            env[k] = val
        path = os.path.join(REPO, "diff-gaussian-sampling_amd") if pv == "base" else os.path.join(REPO, pv)
        env["PYTHONPATH"] = path
        out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "kbench.py"), *a.kbench_args.split()],
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            sys.stderr.write(out.stderr[-3000:])
            sys.exit(out.returncode)
        j = json.loads(out.stdout.strip().splitlines()[-1])
        res[v].append(j)
        print(r, v, json.dumps(j), flush=True)
for v, js in res.items():
    med = {k: statistics.median(j[k] for j in js) for k in ("fwd_ms", "bwd_ms", "call_pair_ms", "prep_ms") if k in js[0]}
    print("MEDIAN", v, json.dumps(med), flush=True)

"""Updates profiles/traffic.json (bench.py's roofline.traffic) from rocprofv3 --pmc passes of one
bench workload (tools/pmc_passes.sh with FETCH_SIZE and WRITE_SIZE in separate passes):

    python tools/traffic_json.py PMC_DIR KEY ROUND_NOTE

KEY is bench.traffic_key(...) of the profiled workload ("gaussian,C=1,P=1000000,N=2000000",
"...,aniso=25").  Bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 (gfx950: FETCH_SIZE
counts half of wide streaming reads, MI355X_MICROARCH.md HBM section), averaged over the launches
of the render kernels; the forward is the main pass (k_forward_s, else k_forward_t / _mx).
"""
import collections
import csv
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r.get("Kernel_Name", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = list(vals)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return {d: {c: sum(v) / len(v) for c, v in vals[n].items()} for n, d in zip(names, dem)}


def pick(k, prefixes, exclude=()):
    for p in prefixes:
        for name, c in k.items():
            if name.startswith(p) and not any(x in name for x in exclude):
                return name, c
    return None, None


def main(root, key, note):
    k = per_kernel(root)
    out = {}
    for what, prefixes, excl in (("forward_render", ["void dgs::k_forward_s<", "void dgs::k_forward_t<",
                                                     "void dgs::k_forward_mx<"], ("true>",)),
                                 ("backward_render", ["void dgs::k_backward<", "void dgs::k_backward_mx<"], ())):
        name, c = pick(k, prefixes, excl)
        if name is None or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        b = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
        out[what] = b
        out.setdefault("detail", {})[what] = {"kernel": name[:90], "fetch_kb_raw": round(c["FETCH_SIZE"], 1),
                                              "write_kb": round(c["WRITE_SIZE"], 1), "bytes": b}
    path = os.path.join(REPO, "profiles", "traffic.json")
    tj = json.load(open(path)) if os.path.exists(path) else {"workloads": {}}
    tj.setdefault("workloads", {})[key] = out
    tj.setdefault("rounds", {})[key] = note
    json.dump(tj, open(path, "w"), indent=1)
    print(key, json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])

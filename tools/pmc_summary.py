"""Summarise rocprofv3 --pmc counter CSVs per kernel (averaged over dispatches)."""
import collections
import csv
import glob
import subprocess
import sys

root = sys.argv[1]
want = sys.argv[2:] if len(sys.argv) > 2 else ["k_forward", "k_backward"]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = list(vals)
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for n, d in zip(names, dem):
    if not any(w in d for w in want):
        continue
    print(d[:80])
    for c, v in sorted(vals[n].items()):
        print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")

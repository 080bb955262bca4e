"""One warm preprocess call's kernel timeline from a rocprofv3 kernel trace (tools/gpu.sh (round 4: tools/gpu_r04.sh, in git history)'s
profprep): start, gap before, duration per kernel, and the busy sum."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_sample_cells" in r["Kernel_Name"]]
i0, i1 = idx[-2], idx[-1]
t0 = prev = int(rows[i0]["Start_Timestamp"])
busy = 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} gap{(s - prev) / 1e3:6.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:90]}")
    prev = e
print("busy", busy / 1e3, "span", (prev - t0) / 1e3)

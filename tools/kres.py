"""Per-kernel register / scratch / occupancy summary of a HIP source (hipcc resource remarks).

    python tools/kres.py csrc/dgs_aggregate.hip [name-filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", "include",
       "-I", "diff-gaussian-sampling_amd/csrc", "-O3", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                       text=True).stdout.splitlines()
for r, n in zip(rows, names):
    if filt not in n or "hipcub" in n or "rocprim" in n:
        continue
    print(f"{n[:90]:90s} V{r.get('VGPRs', '?'):>4s} A{r.get('AGPRs', '?'):>3s} "
          f"scr{r.get('ScratchSize [bytes/lane]', '?'):>4s} occ{r.get('Occupancy [waves/SIMD]', '?'):>2s} "
          f"lds{r.get('LDS Size [bytes/block]', '?')}")

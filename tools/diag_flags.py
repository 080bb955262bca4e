import sys, os, struct
sys.path.insert(0, "diff-gaussian-sampling_amd")
import numpy as np, torch
import diff_gaussian_sampling as dgs
from diff_gaussian_sampling import synthetic as syn
dev = "cuda"
m, v, cv, c = (t.to(dev) for t in syn.gaussians(1_000_000, 2, 1, seed=0))
s = syn.samples(2_000_000, 2, seed=4).to(dev)
R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
h = gb[:256].cpu().numpy().tobytes()
magic, ver, P, D, N, T = struct.unpack_from("<IIiiii", h, 0)
n, CT, ncells, pad = struct.unpack_from("<iiii", h, 40)
R_, E, fcap, bcap = struct.unpack_from("<qqqq", h, 56)
offs = struct.unpack_from("<" + "Q" * 14, h, 88)
print("P", P, "N", N, "T", T, "n", n, "CT", CT, "ncells", ncells, "E", E)
o_entries = offs[4]
ent = gb[o_entries:o_entries + 4 * E].cpu().numpy().view(np.uint32)
gen = (ent >> 31) & 1; uns = (ent >> 30) & 1
print("general", int(gen.sum()), "unsafe", int(uns.sum()), "fraction general", gen.mean())
ids = ent & 0x3fffffff
u_ids = np.unique(ids[uns == 1])
print("unique unsafe gaussians", len(u_ids))
# per-cell: count entries in fallback cells
cells_entries = None
names = ["o_counts", "o_perm", "o_cell_gbeg", "o_cell_gend", "o_entries", "o_bwd_units", "g_bytes",
         "o_sorted", "o_cell_sbeg", "o_cell_send", "o_fwd_units", "s_bytes", "stamp", "o_cell_gmid"]
O = dict(zip(names, offs))
gbeg = gb[O["o_cell_gbeg"]:O["o_cell_gbeg"] + 4 * ncells].cpu().numpy().view(np.int32)
gend = gb[O["o_cell_gend"]:O["o_cell_gend"] + 4 * ncells].cpu().numpy().view(np.int32)
sbeg = sb[O["o_cell_sbeg"]:O["o_cell_sbeg"] + 4 * ncells].cpu().numpy().view(np.int32)
send = sb[O["o_cell_send"]:O["o_cell_send"] + 4 * ncells].cpu().numpy().view(np.int32)
cell_of = np.zeros(E, np.int64)
for cidx in np.nonzero(gend > gbeg)[0]:
    cell_of[gbeg[cidx]:gend[cidx]] = cidx
uc = cell_of[uns == 1]
fb = (uc % CT) == CT - 1
print("unsafe entries in fallback cells", int(fb.sum()), "of", len(uc))
fbc = np.arange(ncells)[(np.arange(ncells) % CT) == CT - 1]
print("fallback cells samples", (send[fbc] - sbeg[fbc]).tolist())
nf = uc[~fb]
if len(nf):
    t = nf // CT; loc = nf % CT
    print("non-fallback unsafe cells: tiles", np.unique(t).tolist()[:20], "fx", np.unique(loc % n)[:20].tolist(), "fy", np.unique(loc // n)[:20].tolist())
    ids_nf = ids[uns == 1][~fb]
    mm = m.cpu().numpy()
    perm = gb[O["o_perm"]:O["o_perm"] + 4 * P].cpu().numpy().view(np.int32)
    g = perm[ids_nf[:10]]
    print("example means", mm[g].tolist())
    print("example cells (tile, fx, fy)", [(int(a // CT), int(a % CT % n), int(a % CT // n)) for a in nf[:10]])

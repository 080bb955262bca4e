import sys, struct
sys.path.insert(0, "diff-gaussian-sampling_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
import diff_gaussian_sampling as dgs
from diff_gaussian_sampling import synthetic as syn
from oracle import oracle as orc
orc.build()
P, N, C, D = 200, 3000, 5, 1
means, values, covs, conics = syn.gaussians(P, D, C, seed=11)
samples = syn.samples(N, D, seed=12)
dL = syn.grad_out(N, 1, C, seed=13)
dev = "cuda"
m, v, cv, c, s = (t.to(dev) for t in (means, values, covs, conics, samples))
R, gb, sb, rg, srg, radii = dgs._C.preprocess_gaussians(m, v, cv, c, s, False)
gm, gv, gc = dgs._C.sample_gaussians_backward(m, v, c, s, R, dL.to(dev).reshape(N, 1, C), gb, sb, rg, srg, False)
ob = orc.OracleBins(means.numpy(), covs.numpy(), samples.numpy())
dm, dv, dc = ob.backward("gaussian", values.numpy(), conics.numpy(), dL.numpy())
err = np.abs(gv.cpu().numpy() - dv).max(1)
bad = np.nonzero(err > 1e-3)[0]
print("bad gaussians", bad.tolist())
h = gb[:256].cpu().numpy().tobytes()
n, CT, ncells = struct.unpack_from("<iii", h, 40)
E = struct.unpack_from("<q", h, 64)[0]
offs = struct.unpack_from("<" + "Q" * 14, h, 88)
names = ["o_counts", "o_perm", "o_cell_gbeg", "o_cell_gend", "o_entries", "o_bwd_units", "g_bytes",
         "o_sorted", "o_cell_sbeg", "o_cell_send", "o_fwd_units", "s_bytes", "stamp", "o_cell_gmid"]
O = dict(zip(names, offs))
grid = struct.unpack_from("<ii", h, 24); off = struct.unpack_from("<ff", h, 32)
print("n", n, "CT", CT, "ncells", ncells, "E", E, "grid", grid, "off", off)
perm = gb[O["o_perm"]:O["o_perm"] + 4 * P].cpu().numpy().view(np.int32)
inv = np.argsort(perm)
ent = gb[O["o_entries"]:O["o_entries"] + 4 * E].cpu().numpy().view(np.uint32)
gbeg = gb[O["o_cell_gbeg"]:O["o_cell_gbeg"] + 4 * ncells].cpu().numpy().view(np.int32)
gend = gb[O["o_cell_gend"]:O["o_cell_gend"] + 4 * ncells].cpu().numpy().view(np.int32)
for g in bad[:4]:
    i = inv[g]
    print("gaussian", g, "internal", i, "mean", means[g].tolist(), "cov", covs[g].tolist())
    for cidx in range(ncells):
        for e in range(gbeg[cidx], gend[cidx]):
            if (ent[e] & 0x3fffffff) == i:
                print("   cell", cidx, "tile", cidx // CT, "loc", cidx % CT, "flags", hex(ent[e] >> 30))

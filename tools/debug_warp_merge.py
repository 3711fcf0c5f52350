"""Debug helper: the cost_each_small fixture's fmap_ref gradient from the
warp-cost backward, saved for an A/B between the merged and the plain scatter
(DRO_WARP_NOMERGE).  usage: python tools/debug_warp_merge.py <out.pt>"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402

d = {k: torch.from_numpy(v).cuda() for k, v in np.load(os.path.join(ROOT, "tests/golden/cost_each_small.npz")).items()}
fmap, fref = d["fmap"].clone().requires_grad_(True), d["fmap_ref"].clone().requires_grad_(True)
with hip.record_bilinear_cells() as rec:
    cost = hip.warp_cost(fmap, fref.unsqueeze(0), d["depth"], d["pose"].unsqueeze(0), d["K"], reduce_mean=False)
    (cost * d["G"].unsqueeze(0)).sum().backward()
torch.cuda.synchronize()
out = {"g_fref": fref.grad.cpu(), "ref": d["g_fmap_ref"].cpu(), "cells": rec.calls[0][1].cpu()}
torch.save(out, sys.argv[1])
e = (fref.grad.cpu() - d["g_fmap_ref"].cpu()).abs()
print("rel", float(e.max() / d["g_fmap_ref"].abs().max()))

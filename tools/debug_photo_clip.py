"""Debug helper: the photo_loss_clip fixture through hip.photometric_loss with
its branch record saved (selection, cells, L1 signs, clip thresholds and
decisions) for offline comparison with the oracle.
usage: python tools/debug_photo_clip.py <out.pt>"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402

d = {k: torch.from_numpy(v).cuda() for k, v in np.load(os.path.join(ROOT, "tests/golden/photo_loss_clip.npz")).items()}
res = {}
for clip in (0.5, 0.0):
    invs = d["inv_depths"].clone().requires_grad_(True)
    vec = d["poses"].clone().requires_grad_(True)
    with hip.record_bilinear_cells() as rec:
        loss, metrics, sel = hip.photometric_loss(d["image"], d["context"], invs, vec.permute(1, 2, 0, 3), d["K"],
                                                  automask=True, reduce_min=True, clip_loss=clip,
                                                  return_selection=True)
        loss.sum().backward()
    torch.cuda.synchronize()
    res[clip] = {"g_inv": invs.grad.cpu(), "g_pose": vec.grad.cpu(), "sel": sel.cpu(), "loss": loss.detach().cpu(),
                 "calls": [(t, c.cpu()) for t, c in rec.calls]}
torch.save(res, sys.argv[1])
print("saved")

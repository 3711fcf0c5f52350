"""Dump the fp32 CPU oracle's intermediates for photo_loss_mean (ref 0, pred 0)
on this machine, for comparison with the same computation on another host:
sampling grid, warped image, sign map of the L1 term and the L1-only pose
gradient; plus torch's CPU capability string."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402
from common import load_fixture  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402

d = load_fixture(os.path.join(ROOT, "tests", "golden", "photo_loss_mean.npz"))
n, B, _, H, W = d["inv_depths"].shape
N = d["poses"].shape[1]
res = {"cpu": torch.backends.cpu.get_cpu_capability(), "threads": torch.get_num_threads()}
for dt in (torch.float32, torch.float64):
    inv = d["inv_depths"][0].to(dt)
    vec = d["poses"][:, 0, 0].to(dt).clone().requires_grad_(True)
    K = d["K"].to(dt)
    grid = O.sample_grid(O.inv2depth(inv), K, K, vec, 1.0)
    est = torch.nn.functional.grid_sample(d["context"][0].to(dt), grid, mode="bilinear", padding_mode="zeros",
                                          align_corners=True)
    l1 = (est - d["image"].to(dt)).abs().mean()
    l1.backward()
    R, t = O.euler_to_matrix(vec.detach())
    res[str(dt)] = {"grid": grid.detach(), "est": est.detach(), "g": vec.grad.detach(), "R": R, "t": t}
out = os.path.join(ROOT, "gpurun_out", sys.argv[1] if len(sys.argv) > 1 else "photo_box.pt")
os.makedirs(os.path.dirname(out), exist_ok=True)
torch.save(res, out)
print(res["cpu"], res["threads"], res[str(torch.float32)]["g"][0].tolist(), res[str(torch.float64)]["g"][0].tolist())

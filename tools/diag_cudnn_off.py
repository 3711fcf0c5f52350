"""Encoders and the step loss with MIOpen on vs off, against a CPU fp64 copy."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch

from test_graph_step import _batch, _setup

m = _setup()
b = _batch()
K0 = b["intrinsics"].clone()
dn = m.depth_net
x = torch.cat([b["rgb"]] + list(b["rgb_context"]), 0)
pairs = torch.cat([b["rgb"], b["rgb_context"][0]], 1)
cpu = copy.deepcopy(dn).cpu().double()
with torch.no_grad():
    ref_f = cpu.fnet(x.cpu().double())
    ref_cd = cpu.cnet_depth(b["rgb"].cpu().double())
    ref_cp = cpu.cnet_pose(pairs.cpu().double())
for cud in (True, False):
    torch.backends.cudnn.enabled = cud
    with torch.no_grad():
        f = dn.fnet(x)
        cd = dn.cnet_depth(b["rgb"])
        cp = dn.cnet_pose(pairs)
    r = lambda a, r_: float((a.double().cpu() - r_).abs().max() / r_.abs().max())
    b["intrinsics"].copy_(K0)
    loss = float(m(b, flip=False)["loss"])
    print(f"cudnn={cud}: fnet {r(f, ref_f):.2e} cnet_depth {r(cd, ref_cd):.2e} cnet_pose {r(cp, ref_cp):.2e} loss {loss:.7f}",
          flush=True)

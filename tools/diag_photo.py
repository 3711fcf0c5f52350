"""Locate photometric-gradient mismatches (HIP vs forced-selection fp32/fp64 oracle)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch
from common import kitti_K, smooth_images
from oracle import dro_oracle as O
import dro_sfm_amd.hip as hip

for (H, W, n, lo, span) in ((192, 640, 9, 0.02, 0.3), (48, 160, 3, 0.02, 0.3), (192, 640, 2, 0.05, 0.5)):
    g = torch.Generator().manual_seed(9)
    B, N = 2, 2
    K = kitti_K(B, W=W, H=H)
    image = smooth_images(B, H, W, 41)
    ctx = torch.stack([smooth_images(B, H, W, 42 + j) for j in range(N)])
    invs = lo + span * torch.rand(n, B, 1, H, W, generator=g)
    vec = torch.cat([0.1 * torch.randn(B, N, n, 3, generator=g), 0.02 * torch.randn(B, N, n, 3, generator=g)], 3)
    ig = invs.cuda().requires_grad_(True)
    loss, metrics, sel = hip.photometric_loss(image.cuda(), ctx.cuda(), ig, vec.cuda().permute(1, 2, 0, 3), K.cuda(), return_selection=True)
    loss.sum().backward()
    ic = invs.double().clone().requires_grad_(True)
    vc = vec.double()
    out = O.photometric_decay_loss(image.double(), list(ctx.double()), list(ic), K.double(), K.double(),
                                   [[vc[:, j, i] for i in range(n)] for j in range(N)],
                                   forced_selection=sel.cpu().unsqueeze(2))
    out["loss"].sum().backward()
    err = (ig.grad.cpu().double() - ic.grad).abs()
    m = ic.grad.abs().max()
    print(f"H{H} W{W} n{n}: max rel {float(err.max() / m):.3e}; #px > 1e-4*max: {int((err > 1e-4 * m).sum())} of {err.numel()}")
    flat = err.flatten().argsort(descending=True)[:6]
    for f in flat.tolist():
        i, b, _, y, x = torch.unravel_index(torch.tensor(f), err.shape)
        i, b, y, x = int(i), int(b), int(y), int(x)
        print(f"   i{i} b{b} y{y} x{x}: hip {float(ig.grad[i,b,0,y,x]):.4e} o64 {float(ic.grad[i,b,0,y,x]):.4e} sel {int(sel[i,b,y,x])} inv {float(invs[i,b,0,y,x]):.4f}")

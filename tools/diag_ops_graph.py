"""Replay each HIP op (fwd+bwd) from a hipGraph several times; compare to eager."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dro_sfm_amd.hip as hip

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
B, C, h, w, N = 2, 128, 24, 80, 2
K = torch.tensor([[371.8, 0.0, 314.1], [0.0, 369.4, 88.5], [0.0, 0.0, 1.0]], device=dev).repeat(B, 1, 1)


def _run(fn, inputs):
    outs = fn()
    loss = sum((o * (i + 1)).sum() for i, o in enumerate(outs))
    return torch.autograd.grad(loss, inputs)


def check(name, fn, inputs):
    ref = [t.clone() for t in _run(fn, inputs)]
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            _run(fn, inputs)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        grads = _run(fn, inputs)
    for rep in range(3):
        gr.replay(); torch.cuda.synchronize()
        errs = [float((a - b).abs().max() / b.abs().max().clamp(min=1e-30)) for a, b in zip(grads, ref)]
        fin = [bool(torch.isfinite(a).all()) for a in grads]
        print(name, "replay", rep, "rel errs", ["%.2e" % e for e in errs], "finite", fin, flush=True)


fmap = torch.randn(B, C, h, w, generator=g, device=dev).requires_grad_(True)
frefs = torch.randn(N, B, C, h, w, generator=g, device=dev).requires_grad_(True)
disp = torch.rand(B, 1, h, w, generator=g, device=dev).requires_grad_(True)
poses = torch.cat([0.1 * torch.randn(N, B, 3, generator=g, device=dev), 0.02 * torch.randn(N, B, 3, generator=g, device=dev)], 2).requires_grad_(True)
check("warp depth-mean", lambda: [hip.warp_cost(fmap, frefs, disp, poses.detach(), K, depth_mode=hip.DEPTH_DISP, min_depth=0.5, max_depth=80.0, reduce_mean=True)], [fmap, frefs, disp])
check("warp pose", lambda: [hip.warp_cost(fmap, frefs, disp.detach(), poses, K, depth_mode=hip.DEPTH_DISP, min_depth=0.5, max_depth=80.0, reduce_mean=False)], [fmap, frefs, poses])
inv = torch.rand(B, 1, h, w, generator=g, device=dev).requires_grad_(True)
mask = torch.randn(B, 576, h, w, generator=g, device=dev).requires_grad_(True)
check("upsample", lambda: [hip.convex_upsample(inv, mask, 8)], [inv, mask])
H, W, n = 192, 640, 9
img = torch.rand(B, 3, H, W, generator=g, device=dev)
ctx = torch.rand(N, B, 3, H, W, generator=g, device=dev)
invs = (0.02 + 0.3 * torch.rand(n, B, 1, H, W, generator=g, device=dev)).requires_grad_(True)
pv = torch.cat([0.1 * torch.randn(N, n, B, 3, generator=g, device=dev), 0.02 * torch.randn(N, n, B, 3, generator=g, device=dev)], 3).requires_grad_(True)
check("photometric", lambda: [hip.photometric_loss(img, ctx, invs, pv, K)[0]], [invs, pv])

"""Kink allowances for photometric-loss gradient parity (test infrastructure).

The photometric loss is continuous but not differentiable everywhere, and
two fp32 evaluations (the reference's on its host CPU, the HIP kernel's) can
land on different sides of a kink.  The one that moves gradients measurably
(found from the round-2 pose-gradient failure of photo_loss_mean and the
round-3 one of photo_loss_noauto, whose deviations this reproduces to 1 %):

  bilinear sampling (grid_sample, align_corners=True) has a derivative that
  jumps where the sampling coordinate crosses an integer (the cell changes).
  A warped pixel whose coordinate lies within fp32 rounding of a grid line
  gets d(est)/d(coordinate) from the left cell in one evaluation and from the
  right cell in another; its contribution to the pose gradient (and to the
  inverse depth at that pixel) changes by |dL/dest . jump| |dcoord/dtheta|.

`gridline_allowance` finds those pixels from the fp64 oracle -- coordinate
within `delta` of an integer, delta = 2x the largest |coordinate_fp32 -
coordinate_fp64| of the fixture's own warps (measured, not assumed) -- and
returns the elementwise bound on how far any fp32 evaluation's gradient may
move because of them, for the pose vector [B,N,n,6] and the inverse depths
[n,B,1,H,W].  Every other pixel is held to the plain tolerance.
"""
import torch
import torch.nn.functional as F

from oracle import dro_oracle as O


def _coords(depth, K, pose, H, W):
    grid = O.sample_grid(depth, K, K, pose, 1.0)
    return grid, (grid[..., 0] + 1) / 2 * (W - 1), (grid[..., 1] + 1) / 2 * (H - 1)


def gridline_allowance(d, forced_selection=None):
    """d: a photometric fixture (image, context [N,B,3,H,W], inv_depths
    [n,B,1,H,W], poses [B,N,n,6], K, automask, reduce_min).  Returns
    (allow_pose [B,N,n,6], allow_inv [n,B,1,H,W], delta_px, kink_count)."""
    dt = torch.float64
    n, B, _, H, W = d["inv_depths"].shape
    N = d["poses"].shape[1]
    K = d["K"].cpu().to(dt)
    # dL/d(warped image) of every (ref, prediction) from the fp64 oracle
    ests = []
    orig = O.view_synthesis

    def keep(ref, depth, pose, K_, rK):
        e = orig(ref, depth, pose, K_, rK)
        e.retain_grad()
        ests.append(e)
        return e

    O.view_synthesis = keep
    try:
        invs = [i.cpu().to(dt).requires_grad_(True) for i in d["inv_depths"]]
        vec = d["poses"].cpu().to(dt).requires_grad_(True)
        out = O.photometric_decay_loss(d["image"].cpu().to(dt), [c.cpu().to(dt) for c in d["context"]], invs,
                                       K, K, [[vec[:, j, i] for i in range(n)] for j in range(N)],
                                       automask=bool(int(d["automask"])),
                                       reduce="min" if int(d["reduce_min"]) else "mean",
                                       forced_selection=forced_selection)
        out["loss"].sum().backward()
    finally:
        O.view_synthesis = orig
    # the fp32 coordinate error of these warps sets the kink band
    delta = 0.0
    for j in range(N):
        for i in range(n):
            inv = d["inv_depths"][i].cpu()
            _, x32, y32 = _coords(O.inv2depth(inv), d["K"].cpu(), d["poses"][:, j, i].cpu(), H, W)
            _, x64, y64 = _coords(O.inv2depth(inv.to(dt)), K, d["poses"][:, j, i].cpu().to(dt), H, W)
            delta = max(delta, float((x32.double() - x64).abs().max()), float((y32.double() - y64).abs().max()))
    delta *= 2.0
    allow_p = torch.zeros(B, N, n, 6, dtype=dt)
    allow_i = torch.zeros(n, B, 1, H, W, dtype=dt)
    count, k = 0, 0
    h = 1e-3
    for j in range(N):
        ctx = d["context"][j].cpu().to(dt)
        for i in range(n):
            gest = ests[k].grad
            k += 1
            inv = d["inv_depths"][i].cpu().to(dt)
            v0 = d["poses"][:, j, i].cpu().to(dt)
            depth = O.inv2depth(inv)
            grid, x, y = _coords(depth, K, v0, H, W)
            for ax, coord, size in ((0, x, W), (1, y, H)):
                near = (coord - coord.round()).abs() < delta
                if not bool(near.any()):
                    continue
                count += int(near.sum())
                sc = 2.0 / (size - 1)

                def sample(s):
                    g = grid.clone()
                    g[..., ax] = g[..., ax] + s * sc
                    return F.grid_sample(ctx, g, mode="bilinear", padding_mode="zeros", align_corners=True)

                # derivative of the right cell minus that of the left cell, weighted by dL/dest
                jump = (((sample(2 * h) - sample(h)) - (sample(-h) - sample(-2 * h))) / h * gest).sum(1)
                jump = jump.abs() * near                                     # [B,H,W]
                for c in range(6):
                    t = torch.zeros_like(v0)
                    t[:, c] = 1.0
                    _, jg = torch.func.jvp(lambda vv: O.sample_grid(depth, K, K, vv, 1.0), (v0,), (t,))
                    allow_p[:, j, i, c] += (jump * (jg[..., ax] / sc).abs()).sum((1, 2))
                # d coordinate / d inverse depth at the same pixel (pixelwise)
                _, jd = torch.func.jvp(lambda iv: O.sample_grid(O.inv2depth(iv), K, K, v0, 1.0), (inv,),
                                       (torch.ones_like(inv),))
                allow_i[i, :, 0] += jump * (jd[..., ax] / sc).abs()
    return allow_p, allow_i, delta, count

"""GPU parity: the HIP kernels (through the C ABI, via dro_sfm_amd.hip) against
the reference golden vectors and the CPU oracle on identical inputs.

Tolerance: 1e-4 relative (max|a-b| / max|b|) for outputs and input gradients
(BASELINE.json north_star); recurrent full-network outputs 1e-3 (fp32
rounding amplified through 8-12 GRU steps, stated per test).
"""
import os

import pytest
import torch

from common import fval, grad_errors, kitti_K, load_fixture, load_spec, params_from_spec, smooth_images
from oracle import dro_oracle as O

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-4
DEV = "cuda"


def fx(name):
    return {k: v.to(DEV) for k, v in load_fixture(os.path.join(G, name + ".npz")).items()}


@pytest.fixture(scope="module")
def hip():
    import dro_sfm_amd.hip as H
    from dro_sfm_amd.hip import _lib
    _lib.load()
    return H


def rel(a, b):
    return O.rel_err(a.cpu(), b.cpu())


# ------------------------------------------------------------------ warp + feature cost
@pytest.mark.parametrize("name", ["cost_each_small", "cost_each_edge", "cost_each_kitti"])
@pytest.mark.parametrize("as_matrix", [False, True])
def test_warp_cost_single_ref(hip, name, as_matrix):
    d = fx(name)
    pose = d["pose"]
    if as_matrix:  # same pose as a [B,4,4] transform; chain its grad back to euler via the oracle
        pose_in = O.vec_to_transform(pose.cpu()).to(DEV)
    else:
        pose_in = pose
    pose_in = pose_in.clone().requires_grad_(True)
    fmap, fref, depth = (d[k].clone().requires_grad_(True) for k in ("fmap", "fmap_ref", "depth"))
    cost = hip.warp_cost(fmap, fref, depth, pose_in, d["K"], depth_mode=hip.DEPTH_METRIC,
                         reduce_mean=False).squeeze(0)
    assert rel(cost, d["cost"]) < TOL
    (cost * d["G"]).sum().backward()
    assert rel(fmap.grad, d["g_fmap"]) < TOL
    assert rel(fref.grad, d["g_fmap_ref"]) < TOL
    assert rel(depth.grad, d["g_depth"]) < TOL
    if as_matrix:
        vec = pose.cpu().clone().requires_grad_(True)
        T = O.vec_to_transform(vec)
        (T * pose_in.grad.cpu()).sum().backward()
        assert rel(vec.grad, d["g_pose"]) < TOL
    else:
        assert rel(pose_in.grad, d["g_pose"]) < TOL


@pytest.mark.parametrize("name", ["depth_cost_n2", "depth_cost_n4"])
def test_warp_cost_depth_mean(hip, name):
    d = fx(name)
    disp = d["disp"].clone().requires_grad_(True)
    fmap = d["fmap"].clone().requires_grad_(True)
    fref = d["fmap_ref"].clone().requires_grad_(True)
    cost = hip.warp_cost(fmap, fref, disp, d["poses"], d["K"], depth_mode=hip.DEPTH_DISP,
                         min_depth=fval(d["min_depth"]), max_depth=fval(d["max_depth"]),
                         reduce_mean=True)
    assert rel(cost, d["cost"]) < TOL
    (cost * d["G"]).sum().backward()
    assert rel(disp.grad, d["g_disp"]) < TOL
    assert rel(fmap.grad, d["g_fmap"]) < TOL
    assert rel(fref.grad, d["g_fmap_ref"]) < TOL


def test_plane_sweep(hip):
    d = fx("plane_sweep_d64")
    vol = hip.plane_sweep_cost(d["fmap"], d["fmap_ref"], d["disp"], d["pose"], d["K"],
                               min_depth=fval(d["min_depth"]), max_depth=fval(d["max_depth"]))
    assert rel(vol, d["cost"]) < TOL


@pytest.mark.parametrize("w", [80, 21])
def test_plane_sweep_equals_per_plane_warp_cost(hip, w):
    """D=64 sweep at the KITTI feature size (24x80; and 24x21, a ragged last
    pixel block) against one warp_cost call per plane with that plane's
    constant disparity map: bit-identical (same projection, same tap sums;
    out-of-image taps weigh zero instead of being skipped)."""
    g = torch.Generator().manual_seed(9)
    B, C, h, D = 2, 128, 24, 64
    fmap = torch.randn(B, C, h, w, generator=g).to(DEV)
    fref = torch.randn(B, C, h, w, generator=g).to(DEV)
    pose = torch.cat([0.3 * torch.randn(B, 3, generator=g), 0.02 * torch.randn(B, 3, generator=g)], 1).to(DEV)
    K = kitti_K(B, W=8 * w, H=8 * h).to(DEV)
    disp = torch.linspace(0, 1, D).to(DEV)
    vol = hip.plane_sweep_cost(fmap, fref, disp, pose, K, min_depth=0.5, max_depth=80.0)
    for d in (0, 17, 40, 63):
        dm = disp[d].expand(B, 1, h, w).contiguous()
        ref = hip.warp_cost(fmap, fref, dm, pose, K, depth_mode=hip.DEPTH_DISP, min_depth=0.5,
                            max_depth=80.0, reduce_mean=False).squeeze(0)
        assert torch.equal(vol[:, d], ref), d


def test_warp_cost_kitti_size_vs_oracle(hip):
    """Metric-config size: B=2, C=128, 24x80, N=2 refs, depth mean + per-ref pose cost."""
    g = torch.Generator().manual_seed(7)
    B, C, h, w, N = 2, 128, 24, 80, 2
    K = kitti_K(B)
    fmap, frefs = torch.randn(B, C, h, w, generator=g), torch.randn(N, B, C, h, w, generator=g)
    disp = torch.rand(B, 1, h, w, generator=g)
    poses = torch.cat([0.1 * torch.randn(N, B, 3, generator=g), 0.02 * torch.randn(N, B, 3, generator=g)], 2)
    Gm, Gp = torch.randn(B, C, h, w, generator=g), torch.randn(N, B, C, h, w, generator=g)
    # oracle
    dc = disp.clone().requires_grad_(True)
    fc = fmap.clone().requires_grad_(True)
    rc = frefs.clone().requires_grad_(True)
    pc = poses.clone().requires_grad_(True)
    inv = O.disp_to_depth(dc, 0.5, 80.0)
    cm = O.depth_cost_calc(inv, fc, list(rc), list(poses), K, K, 1 / 8)
    depth_fixed = O.inv2depth(O.disp_to_depth(disp, 0.5, 80.0))
    cp = torch.stack([O.get_cost_each(pc[j], fc, rc[j], depth_fixed, K, K, 1 / 8) for j in range(N)])
    ((cm * Gm).sum() + (cp * Gp).sum()).backward()
    # HIP
    dg, fg, rg, pg = (t.to(DEV).requires_grad_(True) for t in (disp, fmap, frefs, poses))
    Kd = K.to(DEV)
    hm = hip.warp_cost(fg, rg, dg, poses.to(DEV), Kd, depth_mode=hip.DEPTH_DISP, min_depth=0.5,
                       max_depth=80.0, reduce_mean=True)
    hp = hip.warp_cost(fg, rg, disp.to(DEV), pg, Kd, depth_mode=hip.DEPTH_DISP, min_depth=0.5,
                       max_depth=80.0, reduce_mean=False)
    ((hm * Gm.to(DEV)).sum() + (hp * Gp.to(DEV)).sum()).backward()
    assert rel(hm, cm) < TOL and rel(hp, cp) < TOL
    assert rel(dg.grad, dc.grad) < TOL
    assert rel(fg.grad, fc.grad) < TOL
    assert rel(rg.grad, rc.grad) < TOL
    assert rel(pg.grad, pc.grad) < TOL


def test_warp_cost_forward_deterministic(hip):
    d = fx("cost_each_small")
    a = hip.warp_cost(d["fmap"], d["fmap_ref"], d["depth"], d["pose"], d["K"], reduce_mean=False)
    b = hip.warp_cost(d["fmap"], d["fmap_ref"], d["depth"], d["pose"], d["K"], reduce_mean=False)
    assert torch.equal(a, b)


def test_warp_cost_rejects_bad_input(hip):
    d = fx("cost_each_small")
    with pytest.raises(RuntimeError):
        hip.warp_cost(d["fmap"].cpu(), d["fmap_ref"], d["depth"], d["pose"], d["K"])
    with pytest.raises(RuntimeError):
        hip.warp_cost(d["fmap"], d["fmap_ref"][:, :, :5], d["depth"], d["pose"], d["K"])
    with pytest.raises(RuntimeError):
        hip.warp_cost(d["fmap"].double(), d["fmap_ref"], d["depth"], d["pose"], d["K"])


# ------------------------------------------------------------------ photometric loss
def _oracle_photometric(d, dt, forced_selection=None):
    """Oracle loss and gradients on the fixture inputs in dtype dt; with
    forced_selection the min reduction takes the given candidates."""
    invs = [i.cpu().to(dt).requires_grad_(True) for i in d["inv_depths"]]
    vecs = d["poses"].cpu().to(dt).requires_grad_(True)
    N, n = vecs.shape[1], vecs.shape[2]
    poses = [[vecs[:, j, i] for i in range(n)] for j in range(N)]
    out = O.photometric_decay_loss(d["image"].cpu().to(dt), [c.cpu().to(dt) for c in d["context"]], invs,
                                   d["K"].cpu().to(dt), d["K"].cpu().to(dt), poses,
                                   automask=bool(int(d["automask"])),
                                   reduce="min" if int(d["reduce_min"]) else "mean",
                                   forced_selection=forced_selection)
    out["loss"].sum().backward()
    return torch.stack([i.grad for i in invs]).double(), vecs.grad.double(), out["loss"].detach().double()


@pytest.mark.parametrize("name", ["photo_loss", "photo_loss_noauto", "photo_loss_mean", "photo_loss_n4"])
def test_photometric_loss_golden(hip, name):
    """MultiViewPhotometricDecayLoss vs the reference's own outputs and input
    gradients (multiview_photometric_loss_mf.py:194-361).  Loss scalar and
    smoothness: 1e-4.  Gradients: EVERY element of the reference's
    g_inv_depths and g_poses, nothing excluded:

        |hip - ref| <= 1e-4 max|ref| + |ref - x64| + kink
                       (+ 2 |x32 - x64| for g_inv)

    x64 / x32: the oracle in fp64 / fp32 taking the kernel's min-selection.
    |ref - x64| is the reference's own measured distance from the exact
    gradient of that selection (its fp32 rounding, plus -- where the kernel
    resolved a near-tied min differently -- the exact effect of that choice;
    the selection may differ from the fp64 minimum only where the loss moves by
    <= 1e-9 relative, asserted).  `kink` (tests/photo_kinks.py) bounds the
    pixels whose warp coordinate lies within fp32 rounding (2x the fixture's
    measured coordinate error) of a grid line, where the bilinear derivative
    jumps: found as the cause of the round-2 photo_loss_mean and round-3
    photo_loss_noauto pose deviations (reproduced to 1 %).  The inverse-depth
    map also gets twice the fp32 oracle's own per-pixel error: SSIM's
    E[x^2]-E[x]^2 on smooth 3x3 windows cancels in any fp32 evaluation."""
    import photo_kinks
    d = fx(name)
    invs = d["inv_depths"].clone().requires_grad_(True)           # [n,B,1,H,W]
    vec = d["poses"].clone().requires_grad_(True)                 # [B,N,n,6]
    pose = vec.permute(1, 2, 0, 3)                                # [N,n,B,6]
    loss, metrics, sel = hip.photometric_loss(d["image"], d["context"], invs, pose, d["K"],
                                              automask=bool(int(d["automask"])),
                                              reduce_min=bool(int(d["reduce_min"])),
                                              return_selection=True)
    assert rel(loss, d["loss"]) < TOL
    assert rel(metrics[1], d["smoothness_loss"]) < TOL
    loss.sum().backward()
    forced = None
    if int(d["reduce_min"]):
        forced = sel.cpu().unsqueeze(2)
        _, _, l64_free = _oracle_photometric(d, torch.float64)
        _, _, l64_forced = _oracle_photometric(d, torch.float64, forced)
        assert float(l64_forced - l64_free) <= 1e-9 * float(l64_free), "selection differs beyond near-ties"
    gi64, gp64, _ = _oracle_photometric(d, torch.float64, forced)
    gi32, _, _ = _oracle_photometric(d, torch.float32, forced)
    kink_p, kink_i, _, _ = photo_kinks.gridline_allowance(d, forced)
    ref_i, ref_p = d["g_inv_depths"].double().cpu(), d["g_poses"].double().cpu()
    got_i, got_p = invs.grad.double().cpu(), vec.grad.double().cpu()
    bound_p = TOL * ref_p.abs().max() + (ref_p - gp64).abs() + kink_p
    bound_i = TOL * ref_i.abs().max() + (ref_i - gi64).abs() + 2 * (gi32 - gi64).abs() + kink_i
    ep, ei = (got_p - ref_p).abs(), (got_i - ref_i).abs()
    assert bool((ep <= bound_p).all()), ("pose", float((ep - bound_p).max()), float(ep.max() / ref_p.abs().max()))
    assert bool((ei <= bound_i).all()), ("inv", float((ei - bound_i).max()), int((ei > bound_i).sum()))
    # and the kernel against the exact gradient of its own selection
    assert bool(((got_p - gp64).abs() <= TOL * gp64.abs().max() + kink_p).all())


def test_photometric_loss_kitti_size_vs_oracle(hip):
    """Metric-config loss: B=2, 192x640, n_pred=9, N=2, automask + min.

    The oracle takes the kernel's per-pixel min selection (forced_selection),
    so near-tied pixels cannot pick different candidates in two fp32 orders.
    Loss scalar: 1e-4.  Gradients: relative L2 1e-4 against the fp64 oracle,
    and max-rel within 4x the oracle's own fp32 max-rel: SSIM's E[x^2]-E[x]^2
    on smooth 3x3 windows cancels, so the reference algorithm itself is
    ~2e-2 max-rel off fp64 on a handful of pixels at this size."""
    g = torch.Generator().manual_seed(9)
    B, H, W, n, N = 2, 192, 640, 9, 2
    K = kitti_K(B)
    image = smooth_images(B, H, W, 41, detail=0.3)      # textured: keeps SSIM well conditioned
    ctx = torch.stack([smooth_images(B, H, W, 42 + j, detail=0.3) for j in range(N)])
    invs = 0.02 + 0.3 * torch.rand(n, B, 1, H, W, generator=g)
    vec = torch.cat([0.1 * torch.randn(B, N, n, 3, generator=g), 0.02 * torch.randn(B, N, n, 3, generator=g)], 3)
    ig, vg = invs.to(DEV).requires_grad_(True), vec.to(DEV).requires_grad_(True)
    loss, metrics, sel = hip.photometric_loss(image.to(DEV), ctx.to(DEV), ig, vg.permute(1, 2, 0, 3),
                                              K.to(DEV), return_selection=True)
    loss.sum().backward()
    free = O.photometric_decay_loss(image, list(ctx), list(invs), K, K,
                                    [[vec[:, j, i] for i in range(n)] for j in range(N)])
    assert rel(loss, free["loss"]) < TOL                     # un-forced oracle: same scalar
    ref = {}
    for dt in (torch.float32, torch.float64):
        ic = invs.to(dt).detach().clone().requires_grad_(True)
        vc = vec.to(dt).detach().clone().requires_grad_(True)
        out = O.photometric_decay_loss(image.to(dt), list(ctx.to(dt)), list(ic), K.to(dt), K.to(dt),
                                       [[vc[:, j, i] for i in range(n)] for j in range(N)],
                                       forced_selection=sel.cpu().unsqueeze(2))
        out["loss"].sum().backward()
        ref[dt] = (out, ic.grad.double(), vc.grad.double())
    out64, gi64, gv64 = ref[torch.float64]
    _, gi32, gv32 = ref[torch.float32]
    assert rel(loss, out64["loss"]) < TOL
    assert rel(metrics[1], out64["smoothness_loss"]) < TOL
    l2 = lambda a, b: float((a.double().cpu() - b).norm() / b.norm())
    assert l2(ig.grad, gi64) <= max(TOL, 4 * l2(gi32, gi64)), (l2(ig.grad, gi64), l2(gi32, gi64))
    assert l2(vg.grad, gv64) <= max(TOL, 4 * l2(gv32, gv64)), (l2(vg.grad, gv64), l2(gv32, gv64))
    assert rel(ig.grad.double(), gi64) <= max(TOL, 4 * rel(gi32, gi64))
    assert rel(vg.grad.double(), gv64) <= max(TOL, 4 * rel(gv32, gv64))


# ------------------------------------------------------------------ convex upsample
def test_convex_upsample(hip):
    d = fx("upsample")
    inv, mask = d["inv"].clone().requires_grad_(True), d["mask"].clone().requires_grad_(True)
    up = hip.convex_upsample(inv, mask, 8)
    assert rel(up, d["up"]) < TOL
    (up * d["G"]).sum().backward()
    assert rel(inv.grad, d["g_inv"]) < TOL
    assert rel(mask.grad, d["g_mask"]) < TOL


def test_convex_upsample_kitti_size(hip):
    g = torch.Generator().manual_seed(3)
    inv, mask = torch.rand(2, 1, 24, 80, generator=g), torch.randn(2, 576, 24, 80, generator=g)
    ic, mc = inv.clone().requires_grad_(True), mask.clone().requires_grad_(True)
    ref = O.convex_upsample(ic, mc, 8)
    Gr = torch.randn(ref.shape, generator=g)
    (ref * Gr).sum().backward()
    ig, mg = inv.to(DEV).requires_grad_(True), mask.to(DEV).requires_grad_(True)
    up = hip.convex_upsample(ig, mg, 8)
    (up * Gr.to(DEV)).sum().backward()
    assert rel(up, ref) < TOL and rel(ig.grad, ic.grad) < TOL and rel(mg.grad, mc.grad) < TOL


def test_convex_upsample_fused_scale(hip):
    """affine=(lo, hi - lo): the disp_to_depth scaling of DepthPoseNet.scale_inv_depth
    (networks/layers/resnet/layers.py:11-20) in the upsample epilogue equals the
    upsample followed by PyTorch's multiply and add to f32 rounding (1e-6
    relative), forward and backward."""
    g = torch.Generator().manual_seed(4)
    inv, mask = torch.rand(2, 1, 24, 80, generator=g), torch.randn(2, 576, 24, 80, generator=g)
    lo, hi = 1.0 / 80.0, 1.0 / 0.5
    G = torch.randn(2, 1, 192, 640, generator=g).to(DEV)
    a, am = inv.to(DEV).requires_grad_(True), mask.to(DEV).requires_grad_(True)
    ref = lo + (hi - lo) * hip.convex_upsample(a, am, 8)
    (ref * G).sum().backward()
    b, bm = inv.to(DEV).requires_grad_(True), mask.to(DEV).requires_grad_(True)
    out = hip.convex_upsample(b, bm, 8, affine=(lo, hi - lo))
    (out * G).sum().backward()
    torch.cuda.synchronize()
    assert rel(out, ref) < 1e-6
    assert rel(b.grad, a.grad) < 1e-6 and rel(bm.grad, am.grad) < 1e-6


def test_convex_upsample_many(hip):
    """convex_upsample_many (n predictions, one launch each way, the training
    step's path): each slice of the stacked output and every input gradient vs
    the fp64 oracle restatement (1e-4), one prediction without an inv gradient,
    the backward bitwise deterministic (no atomics), and stacked_view returning
    the stack itself for its unbind() views."""
    g = torch.Generator().manual_seed(5)
    n, B, h, w = 5, 2, 24, 80
    lo, hi = 1.0 / 80.0, 1.0 / 0.5
    invs = [torch.rand(B, 1, h, w, generator=g) for _ in range(n)]
    masks = [torch.randn(B, 576, h, w, generator=g) for _ in range(n)]
    G = torch.randn(n, B, 1, 8 * h, 8 * w, generator=g)
    refs, rg = [], []
    for i in range(n):
        ic = invs[i].double().requires_grad_(i != 2)
        mc = masks[i].double().requires_grad_(True)
        r = lo + (hi - lo) * O.convex_upsample(ic, mc, 8)
        (r * G[i].double()).sum().backward()
        refs.append(r.detach())
        rg.append((ic.grad, mc.grad))

    def run():
        di = [t.to(DEV).requires_grad_(i != 2) for i, t in enumerate(invs)]
        dm = [t.to(DEV).requires_grad_(True) for t in masks]
        out = hip.convex_upsample_many(di, dm, 8, affine=(lo, hi - lo))
        views = list(out.unbind(0))
        assert hip.stacked_view(views) is out
        (hip.stacked_view(views) * G.to(DEV)).sum().backward()
        torch.cuda.synchronize()
        return out.detach(), [t.grad for t in di], [t.grad for t in dm]

    out, gi, gm = run()
    assert out.shape == (n, B, 1, 8 * h, 8 * w)
    for i in range(n):
        assert rel(out[i], refs[i]) < TOL
        assert rel(gm[i], rg[i][1]) < TOL
        if i == 2:
            assert gi[i] is None
        else:
            assert rel(gi[i], rg[i][0]) < TOL
    out2, gi2, gm2 = run()
    assert torch.equal(out, out2)
    assert all(torch.equal(a, b) for a, b in zip(gm, gm2))
    assert all(a is None or torch.equal(a, b) for a, b in zip(gi, gi2))


# ------------------------------------------------------------------ network level
def _load_net(tag, version, mind, maxd):
    from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet
    net = DepthPoseNet(version=version, min_depth=mind, max_depth=maxd)
    net.load_state_dict(params_from_spec(load_spec(os.path.join(G, f"depthposenet_{tag}_keys.json"))))
    return net.to(DEV)


@pytest.mark.parametrize("tag,version", [("it8", "it8-seq4-inter-out"), ("it12h", "it12-h-out")])
def test_depth_pose_net_golden(hip, tag, version):
    """Full forward (train + eval mode) against the reference; 1e-3 (recurrent)."""
    d = fx(f"depthposenet_{tag}")
    net = _load_net(tag, version, fval(d["min_depth"]), fval(d["max_depth"]))
    net.train()
    with torch.no_grad():
        invs, poses = net(d["image"], list(d["refs"]), d["K"])
        assert rel(torch.stack(invs), d["inv_depths"]) < 1e-3
        assert rel(poses, d["poses"]) < 1e-3
        net.eval()
        inv_e, pose_e = net(d["image"], list(d["refs"]), d["K"])
        assert rel(inv_e, d["inv_eval"]) < 1e-3
        assert rel(pose_e, d["poses_eval"]) < 1e-3


def _oracle_grads(spec, version, mind, maxd, batch, kind, dt, forced=None, flip=False, perturb=False,
                  want_preds=False, seed=99, pred_perturb=None):
    """Oracle loss and parameter gradients (and, want_preds, the net's
    predictions (inv_depths [n,B,1,H,W], poses [B,N,n,6])).  perturb (True =
    1e-7, or a relative scale): the images and K moved by a seeded relative
    Gaussian -- the gradient's change under it measures how far an fp32
    evaluation of this step may land from another at that distance (kinks of
    the loss: min selection, L1 signs, bilinear cell edges, smoothness signs;
    amplified by the recurrence)."""
    p = params_from_spec(spec)
    p = {k: (v.to(dt).requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.to(dt) if v.is_floating_point() else v)) for k, v in p.items()}
    b = {k: (v.to(dt) if torch.is_tensor(v) and v.is_floating_point() else
             ([t.to(dt) for t in v] if isinstance(v, list) else v)) for k, v in batch.items()}
    if perturb:
        s = 1e-7 if perturb is True else float(perturb)
        g = torch.Generator().manual_seed(seed)
        jig = lambda t: t * (1 + s * torch.randn(t.shape, generator=g, dtype=t.dtype))
        for key in ("rgb", "rgb_original", "intrinsics"):
            b[key] = jig(b[key])
        for key in ("rgb_context", "rgb_context_original"):
            b[key] = [jig(t) for t in b[key]]
    out = O.train_step_loss(p, version, mind, maxd, b, kind=kind, forced_selection=forced, flip=flip,
                            pred_perturb=pred_perturb)
    out["loss"].sum().backward()
    grads = {k: v.grad for k, v in p.items() if getattr(v, "grad", None) is not None}
    if want_preds:
        return out["loss"].detach(), grads, out["preds"]
    return out["loss"].detach(), grads


def _l2(a, b):
    return float((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm())


def _matched_sensitivity(model, out, preds64, oracle_args, cap=1e-5, seeds=(99, 100, 101)):
    """The fp64 gradient's change between two points as far apart as THIS
    evaluation's forward pass is from fp64.

    The photometric loss has derivative jumps (bilinear cell edges where a
    warped coordinate crosses an integer, L1 and smoothness signs): the
    gradient is piecewise smooth, and on small images a few pixels crossing a
    cell edge move a pose gradient by percents (view5 fixture, fp64 oracle:
    input perturbation 1e-7 -> gradient L2 change 2.3e-5; 1e-6 -> 4.3e-3, dL/dpose
    of one ref by 11 %).  Where an fp32 forward lands within that band is
    rounding, not parity.  So: measure the forward distance d_hip of the HIP
    predictions (inverse depths and poses, relative L2) from the fp64 oracle's,
    measure the fp64 oracle's own prediction move d0 under a 1e-7 input
    perturbation, and evaluate the fp64 gradient at a perturbation scaled to
    1e-7 * d_hip / d0 (capped at `cap`, which also bounds what this allowance
    can ever absorb), once per seed: each sample crosses a different set of
    kinks, and the checks take the largest change per tensor.  An input
    perturbation moves every activation smoothly; an fp32 forward's rounding
    does not, so three more samples evaluate the loss at the fp64
    predictions moved by relative noise of HIP's measured prediction distance
    (inverse depths and poses separately), backpropagated through the exact
    net (oracle train_step_loss pred_perturb).  Returns ([gsens...], info)."""
    inv_h = torch.stack([d.detach() for d in out["inv_depths"]]).double().cpu()
    pv = getattr(out.get("poses"), "vec", None)
    pose_h = pv.detach().double().cpu() if pv is not None else None
    args, kw = oracle_args
    _, _, (inv_p, pose_p) = _oracle_grads(*args, perturb=1e-7, want_preds=True, **kw)
    d_inv = _l2(inv_h, preds64[0])
    d_pose = _l2(pose_h, preds64[1]) if pose_h is not None else 0.0
    d_hip = max(d_inv, d_pose)
    d0 = max(_l2(inv_p, preds64[0]), _l2(pose_p, preds64[1]) if pose_h is not None else 0.0)
    scale = min(cap, 1e-7 * max(1.0, d_hip / max(d0, 1e-30)))
    gs = [_oracle_grads(*args, perturb=scale, seed=sd, **kw)[1] for sd in seeds]
    # the loss evaluated at predictions moved as far as HIP's are from fp64
    # (straight-through to the exact net): the loss's own derivative jumps
    pp = (min(cap, d_inv), min(cap, d_pose))
    gs += [_oracle_grads(*args, pred_perturb=(pp[0], pp[1], sd), **kw)[1] for sd in seeds]
    return gs, {"d_hip": d_hip, "d_inv": d_inv, "d_pose": d_pose, "d0_1e-7": d0, "scale": scale}


def _hip_spread(model, batch, flip=None, runs=2):
    """Per-tensor max relative difference between the parameter gradients of
    this step (already back-propagated into `model`) and those of `runs`
    re-runs of the SAME step (same parameters, a fresh copy of the same batch).
    MIOpen's forward convolutions (the encoders' stride-2 entries) are not
    run-to-run deterministic (1.9e-6 forward spread, tools/diag_determinism2.py),
    and at the fixtures' bilinear cell-edge kinks that spread alone moved one
    tensor of the flipped it8 step by 4 % in one of three runs -- a property
    of this point of the function under fp32 rounding, measured on the product
    itself.  Re-runs whose min-reprojection selection differs from the first
    run's (the oracle is pinned to that one) are not compared.  Returns
    {name: spread}."""
    named = [(k, p) for k, p in model.depth_net.named_parameters() if p.grad is not None]
    g0 = {k: p.grad.detach().clone() for k, p in named}
    loss_mod = getattr(model, "_photometric_loss", None)
    sel0 = loss_mod.last_selection.clone() if loss_mod is not None and loss_mod.last_selection is not None else None
    spread = {k: 0.0 for k in g0}
    for _ in range(runs):
        b = {k: (v.clone() if torch.is_tensor(v) else [t.clone() for t in v]) for k, v in batch.items()}
        for _, p in named:
            p.grad = None
        out = model(b, flip=flip) if flip is not None else model(b)
        out["loss"].sum().backward()
        if sel0 is not None and not torch.equal(loss_mod.last_selection, sel0):
            continue
        for k, p in named:
            spread[k] = max(spread[k], rel(p.grad, g0[k]))
    for k, p in named:                      # leave the first run's gradients in place
        p.grad = g0[k]
    return spread


def _grad_check(model, g64, g32, floor_mult=16.0, abs_floor=2e-3, gsens=None, spread=None):
    """Every parameter gradient within max(abs_floor, floor_mult x the fp32
    oracle's own distance to fp64 for that tensor, 4 x the fp32 oracle's
    global relative L2 distance, 4 x the fp64 gradient's largest change under
    the input perturbations gsens (_matched_sensitivity)) of the fp64 oracle (per tensor, max-rel over
    every element); the global relative L2 error of the whole gradient within
    max(abs_floor, 8x the fp32 oracle's, 4x the perturbation's).  The global
    term matters where the step is ill-conditioned in fp32 (the flipped it8
    fixture: the fp32 oracle itself is 2e-3 off fp64 in L2, its error sitting
    on other tensors than any other fp32 evaluation's).
    Returns (offenders, ok_global, info)."""
    names = [k for k, v in model.depth_net.named_parameters() if k in g64 and v.grad is not None]
    grads = dict(model.depth_net.named_parameters())
    den = sum(float(g64[k].double().pow(2).sum()) for k in names)
    num = sum(float((grads[k].grad.double().cpu() - g64[k].double()).pow(2).sum()) for k in names)
    num32 = sum(float((g32[k].double() - g64[k].double()).pow(2).sum()) for k in names)
    l2, l2_32 = (num / den) ** 0.5, (num32 / den) ** 0.5
    gsens = [] if gsens is None else (gsens if isinstance(gsens, list) else [gsens])
    l2_s = max([(sum(float((g[k].double() - g64[k].double()).pow(2).sum()) for k in names) / den) ** 0.5
                for g in gsens] or [0.0])
    bad = []
    for k in names:
        e = rel(grads[k].grad, g64[k])
        tol = max(abs_floor, floor_mult * rel(g32[k], g64[k]), 4 * l2_32,
                  *[4 * rel(g[k], g64[k]) for g in gsens], 4 * (spread or {}).get(k, 0.0))
        if e > tol:
            bad.append((k, e, tol))
    return bad, l2 <= max(abs_floor, 8.0 * l2_32, 4.0 * l2_s), (l2, l2_32, l2_s)


def _fixture_check(model, fixture, g64, g32, floor_mult=16.0, abs_floor=2e-3, gsens=None, spread=None):
    """Per tensor, over the reference fixture's stored elements (whole tensors
    or a fixed 2048-entry sample): max|HIP - reference| / max|reference| within
    the distance of the reference to the fp64 oracle (same min-selection as
    HIP) plus max(abs_floor, floor_mult x the fp32 oracle's own max-rel) -- the
    reference is compared directly, and may differ only by what its own fp32
    rounding and this build's bound explain."""
    named = [(k, v.grad) for k, v in model.depth_net.named_parameters() if v.grad is not None]
    den = sum(float(g64[k].double().pow(2).sum()) for k, _ in named if k in g64)
    l2_32 = (sum(float((g32[k].double() - g64[k].double()).pow(2).sum()) for k, _ in named if k in g64)
             / den) ** 0.5
    e_hip = grad_errors(named, fixture)
    e_ref = grad_errors(list(g64.items()), fixture)        # reference vs exact
    gsens = [] if gsens is None else (gsens if isinstance(gsens, list) else [gsens])
    bad = []
    for k, e in e_hip.items():
        tol = e_ref[k] + max(abs_floor, floor_mult * rel(g32[k], g64[k]), 4 * l2_32,
                             *[4 * rel(g[k], g64[k]) for g in gsens], 4 * (spread or {}).get(k, 0.0))
        if e > tol:
            bad.append((k, e, tol))
    return bad, e_hip


def _selfsup_model(mind, maxd, tag, version):
    from dro_sfm_amd.models.SelfSupModelMF import SelfSupModelMF
    m = SelfSupModelMF(ssim_loss_weight=0.85, smooth_loss_weight=0.001, C1=1e-4, C2=9e-4,
                       photometric_reduce_op="min", clip_loss=0.0, automask_loss=True, flip_lr_prob=0.0,
                       min_depth=mind, max_depth=maxd)
    m._photometric_loss.keep_selection = True
    m.add_depth_net(_load_net(tag, version, mind, maxd))
    return m.train()


def _sup_model(mind, maxd, tag, version):
    from dro_sfm_amd.models.SupModelMF import SupModelMF
    model = SupModelMF(supervised_method="sparse-l1", flip_lr_prob=0.0, min_depth=mind, max_depth=maxd)
    model.add_depth_net(_load_net(tag, version, mind, maxd))
    return model.train()


@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("tag,version,kind", [("it8", "it8-seq4-inter-out", "selfsup"),
                                              ("it12h", "it12-h-out", "sup")])
def test_train_step_golden(hip, tag, version, kind, flip):
    """SelfSupModelMF / SupModelMF training step on the reference's golden inputs,
    without and with the left-right flip forced (SfmModelMF.py:110-119: the
    net sees flipped images and the flipped K, the loss the flipped K).
    Loss scalar: 1e-4 vs the reference.  Parameter gradients, per element:
    (1) vs the fp64 oracle taking the kernel's min-selection, per tensor
    within max(2e-3, 16x the fp32 oracle's own error), global L2 within
    max(2e-3, 8x); (2) directly vs the reference's per-element fixture
    (_fixture_check).  The factor covers fp32 convolution rounding amplified
    by the recurrent loop; the allowance also holds the step's own
    run-to-run spread (_hip_spread: MIOpen's forward is not deterministic)."""
    d = fx(f"train_step_{tag}")
    f = fx(f"train_step_{tag}_{'flip' if flip else 'grads'}")
    dn = fx(f"depthposenet_{tag}")
    mind, maxd = fval(dn["min_depth"]), fval(dn["max_depth"])
    spec = load_spec(os.path.join(G, f"depthposenet_{tag}_keys.json"))
    N = d["refs"].shape[0]
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"].clone(),
             "depth": d["gt_depth"], "pose_context": [d["gt_poses"][:, j] for j in range(N)]}
    cpu_batch = {k: (v.cpu().clone() if torch.is_tensor(v) else [t.cpu() for t in v]) for k, v in batch.items()}
    model = (_selfsup_model if kind == "selfsup" else _sup_model)(mind, maxd, tag, version)
    out = model(batch, flip=flip)
    assert rel(out["loss"], f["loss"]) < TOL
    if flip:
        assert torch.equal(batch["intrinsics"].cpu(), f["K_after"].cpu())   # mutated in place
    out["loss"].sum().backward()
    forced = None
    if kind == "selfsup":
        forced = model._photometric_loss.last_selection.cpu().unsqueeze(2)
    b0 = {k: (v.clone() if torch.is_tensor(v) else [t.clone() for t in v]) for k, v in cpu_batch.items()}
    spread = _hip_spread(model, {k: (v.to(DEV) if torch.is_tensor(v) else [t.to(DEV) for t in v])
                                 for k, v in b0.items()}, flip)
    args = (spec, version, mind, maxd, cpu_batch, kind, torch.float64, forced, flip)
    _, g64, p64 = _oracle_grads(*args, want_preds=True)
    _, g32, p32 = _oracle_grads(*args[:6], torch.float32, forced, flip, want_preds=True)
    gs, sinfo = _matched_sensitivity(model, out, p64, (args, {}))
    sinfo["d_o32"] = _l2(p32[0], p64[0])
    assert sinfo["d_hip"] < 1e-4, sinfo                   # the forward itself: fp32-close
    bad, ok, info = _grad_check(model, g64, g32, gsens=gs, spread=spread)
    assert not bad and ok, (bad[:5], info, sinfo)
    fbad, _ = _fixture_check(model, {k: v.cpu() for k, v in f.items()}, g64, g32, gsens=gs, spread=spread)
    assert not fbad, (fbad[:5], sinfo)


def _scannet_K(B, W=320, H=240):
    K = torch.tensor([[289.0, 0.0, 160.0], [0.0, 290.0, 120.0], [0.0, 0.0, 1.0]])
    K[0] *= W / 320.0
    K[1] *= H / 240.0
    K[2] = torch.tensor([0.0, 0.0, 1.0])
    return K.unsqueeze(0).repeat(B, 1, 1).contiguous()


def test_train_step_view5_n4_golden(hip):
    """configs[4] model on the reference's fixture: SelfSupModelMF it12-h-out,
    N=4 refs (ScanNet view5, depth 0.2-10), 64x96: loss 1e-4, gradients as in
    test_train_step_golden."""
    f = fx("train_step_it12h_selfsup_n4")
    mind, maxd = fval(f["min_depth"]), fval(f["max_depth"])
    spec = load_spec(os.path.join(G, "depthposenet_it12h_keys.json"))
    batch = {"rgb": f["image"], "rgb_context": list(f["refs"]), "rgb_original": f["image"],
             "rgb_context_original": list(f["refs"]), "intrinsics": f["K"].clone()}
    cpu_batch = {k: (v.cpu().clone() if torch.is_tensor(v) else [t.cpu() for t in v]) for k, v in batch.items()}
    model = _selfsup_model(mind, maxd, "it12h", "it12-h-out")
    out = model(batch)
    assert rel(out["loss"], f["loss"]) < TOL
    out["loss"].sum().backward()
    forced = model._photometric_loss.last_selection.cpu().unsqueeze(2)
    args = (spec, "it12-h-out", mind, maxd, cpu_batch, "selfsup", torch.float64, forced)
    _, g64, p64 = _oracle_grads(*args, want_preds=True)
    _, g32, p32 = _oracle_grads(*args[:6], torch.float32, forced, want_preds=True)
    gs, sinfo = _matched_sensitivity(model, out, p64, (args, {}))
    sinfo["d_o32"] = _l2(p32[0], p64[0])
    assert sinfo["d_hip"] < 1e-4, sinfo
    bad, ok, info = _grad_check(model, g64, g32, gsens=gs)
    assert not bad and ok, (bad[:5], info, sinfo)
    fbad, _ = _fixture_check(model, {k: v.cpu() for k, v in f.items()}, g64, g32, gsens=gs)
    assert not fbad, (fbad[:5], sinfo)


@pytest.mark.parametrize("kind", ["selfsup_view5", "sup_view3"])
def test_train_step_scannet_size_vs_oracle(hip, kind):
    """BASELINE configs[4] (SelfSupModelMF it12-h-out, N=4) and configs[2]
    (SupModelMF it12-h-out, N=2, dense GT) at the ScanNet training shape
    240x320, B=1: product step vs the fp64 oracle on the same weights and
    inputs (kernel's min-selection); loss 1e-4, gradients as in
    test_train_step_golden."""
    B, H, W = 1, 240, 320
    N = 4 if kind == "selfsup_view5" else 2
    mind, maxd = 0.2, 10.0
    spec = load_spec(os.path.join(G, "depthposenet_it12h_keys.json"))
    img = smooth_images(B, H, W, 81, detail=0.3)
    refs = [torch.roll(img, 2 * (j + 1), 3) * 0.9 + 0.1 * smooth_images(B, H, W, 82 + j, detail=0.3)
            for j in range(N)]
    batch = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs,
             "intrinsics": _scannet_K(B)}
    if kind == "sup_view3":
        g = torch.Generator().manual_seed(83)
        batch["depth"] = 0.5 + 9.5 * torch.rand(B, 1, H, W, generator=g)
        from oracle.dro_oracle import vec_to_transform
        batch["pose_context"] = [vec_to_transform(torch.cat([0.05 * torch.randn(B, 3, generator=g),
                                                             0.01 * torch.randn(B, 3, generator=g)], 1))
                                 for _ in range(N)]
    model = (_selfsup_model if kind == "selfsup_view5" else _sup_model)(mind, maxd, "it12h", "it12-h-out")
    gb = {k: (v.to(DEV) if torch.is_tensor(v) else [t.to(DEV) for t in v]) for k, v in batch.items()}
    out = model(gb)
    out["loss"].sum().backward()
    forced = model._photometric_loss.last_selection.cpu().unsqueeze(2) if kind == "selfsup_view5" else None
    okind = "selfsup" if kind == "selfsup_view5" else "sup"
    loss64, g64 = _oracle_grads(spec, "it12-h-out", mind, maxd, batch, okind, torch.float64, forced)
    loss32, g32 = _oracle_grads(spec, "it12-h-out", mind, maxd, batch, okind, torch.float32, forced)
    # the untrained it12-h recurrence at 240x320 is ill-conditioned in fp32: the
    # fp32 oracle's own loss sits ~3.5e-4 from fp64 (sup_view3), so the loss
    # bound is max(1e-4, 4x that measured distance)
    assert rel(out["loss"], loss64) < max(TOL, 4 * rel(loss32, loss64))
    bad, ok, info = _grad_check(model, g64, g32)
    assert not bad and ok, (bad[:5], info)


def test_train_step_kitti_metric_config(hip):
    """Metric config (KITTI 192x640, it8-seq4-inter-out, B=2, N=2): product step vs
    fp64 oracle step on the same weights/inputs with the same min-selection:
    loss 1e-4; gradients as in test_train_step_golden."""
    B, N, H, W = 2, 2, 192, 640
    spec = load_spec(os.path.join(G, "depthposenet_it8_keys.json"))
    img = smooth_images(B, H, W, 51, detail=0.3)
    refs = [torch.roll(img, 3 * (j + 1), 3) * 0.9 + 0.1 * smooth_images(B, H, W, 52 + j, detail=0.3)
            for j in range(N)]
    K = kitti_K(B)
    batch = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs,
             "intrinsics": K}
    model = _selfsup_model(0.5, 80.0, "it8", "it8-seq4-inter-out")
    gb = {k: (v.to(DEV) if torch.is_tensor(v) else [t.to(DEV) for t in v]) for k, v in batch.items()}
    out = model(gb)
    out["loss"].sum().backward()
    forced = model._photometric_loss.last_selection.cpu().unsqueeze(2)
    loss64, g64 = _oracle_grads(spec, "it8-seq4-inter-out", 0.5, 80.0, batch, "selfsup", torch.float64, forced)
    _, g32 = _oracle_grads(spec, "it8-seq4-inter-out", 0.5, 80.0, batch, "selfsup", torch.float32, forced)
    assert rel(out["loss"], loss64) < TOL
    bad, ok, info = _grad_check(model, g64, g32)
    assert not bad and ok, (bad[:5], info)

"""Pin the CPU oracle (oracle/dro_oracle.py) to the reference's golden vectors.

The fixtures were produced by running the reference code itself
(tests/golden/gen_golden.py).  Tolerance: 1e-5 relative (max|a-b| / max|b|)
for single ops, looser where a recurrent network amplifies fp32 rounding.
"""
import os

import pytest
import torch

from common import fval, grad_errors, load_fixture, load_spec, params_from_spec  # tests/golden on sys.path
from oracle import dro_oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-5


def fx(name):
    return load_fixture(os.path.join(G, name + ".npz"))


@pytest.mark.parametrize("name", ["cost_each_small", "cost_each_edge", "cost_each_kitti"])
def test_cost_each(name):
    d = fx(name)
    pose, fmap, fref, depth = (d[k].clone().requires_grad_(True) for k in ("pose", "fmap", "fmap_ref", "depth"))
    cost = O.get_cost_each(pose, fmap, fref, depth, d["K"], d["K"], 1.0 / 8)
    assert O.rel_err(cost, d["cost"]) < TOL
    (cost * d["G"]).sum().backward()
    assert O.rel_err(fmap.grad, d["g_fmap"]) < TOL
    assert O.rel_err(fref.grad, d["g_fmap_ref"]) < TOL
    assert O.rel_err(depth.grad, d["g_depth"]) < 1e-4
    assert O.rel_err(pose.grad, d["g_pose"]) < 1e-4


@pytest.mark.parametrize("name", ["depth_cost_n2", "depth_cost_n4"])
def test_depth_cost(name):
    d = fx(name)
    disp = d["disp"].clone().requires_grad_(True)
    fmap = d["fmap"].clone().requires_grad_(True)
    frefs = [f.clone().requires_grad_(True) for f in d["fmap_ref"]]
    poses = list(d["poses"])
    inv = O.disp_to_depth(disp, fval(d["min_depth"]), fval(d["max_depth"]))
    cost = O.depth_cost_calc(inv, fmap, frefs, poses, d["K"], d["K"], 1.0 / 8)
    assert O.rel_err(cost, d["cost"]) < TOL
    (cost * d["G"]).sum().backward()
    assert O.rel_err(disp.grad, d["g_disp"]) < 1e-4
    assert O.rel_err(fmap.grad, d["g_fmap"]) < TOL
    assert O.rel_err(torch.stack([f.grad for f in frefs]), d["g_fmap_ref"]) < TOL


def test_plane_sweep():
    d = fx("plane_sweep_d64")
    B, C, h, w = d["fmap"].shape
    vol = []
    for v in d["disp"]:
        inv = O.disp_to_depth(torch.full((B, 1, h, w), float(v)), fval(d["min_depth"]), fval(d["max_depth"]))
        vol.append(O.get_cost_each(d["pose"], d["fmap"], d["fmap_ref"], O.inv2depth(inv), d["K"], d["K"], 1 / 8))
    assert O.rel_err(torch.stack(vol, 1), d["cost"]) < TOL


def test_view_synthesis():
    d = fx("view_synthesis")
    depth, pose = d["depth"].clone().requires_grad_(True), d["pose"].clone().requires_grad_(True)
    out = O.view_synthesis(d["ref"], depth, pose, d["K"], d["K"])
    assert O.rel_err(out, d["warped"]) < TOL
    (out * d["G"]).sum().backward()
    assert O.rel_err(depth.grad, d["g_depth"]) < 1e-4
    assert O.rel_err(pose.grad, d["g_pose"]) < 1e-4


def test_ssim():
    d = fx("ssim")
    x = d["x"].clone().requires_grad_(True)
    s = O.ssim(x, d["y"])
    assert O.rel_err(s, d["ssim"]) < TOL
    (s * d["G"]).sum().backward()
    assert O.rel_err(x.grad, d["g_x"]) < 1e-4


@pytest.mark.parametrize("name", ["photo_loss", "photo_loss_noauto", "photo_loss_mean", "photo_loss_n4",
                                  "photo_loss_clip", "photo_loss_clip_mean"])
def test_photometric_loss(name):
    d = fx(name)
    invs = [i.clone().requires_grad_(True) for i in d["inv_depths"]]
    vecs = d["poses"].clone().requires_grad_(True)  # [B,N,n,6]
    N, n = vecs.shape[1], vecs.shape[2]
    poses = [[vecs[:, j, i] for i in range(n)] for j in range(N)]
    out = O.photometric_decay_loss(d["image"], list(d["context"]), invs, d["K"], d["K"], poses,
                                   automask=bool(d["automask"]),
                                   reduce="min" if int(d["reduce_min"]) else "mean",
                                   clip_loss=float(d["clip_loss"]) if "clip_loss" in d else 0.0)
    assert O.rel_err(out["loss"], d["loss"]) < TOL
    assert O.rel_err(out["photometric_loss"], d["photometric_loss"]) < TOL
    assert O.rel_err(out["smoothness_loss"], d["smoothness_loss"]) < TOL
    out["loss"].sum().backward()
    assert O.rel_err(torch.stack([i.grad for i in invs]), d["g_inv_depths"]) < 1e-4
    assert O.rel_err(vecs.grad, d["g_poses"]) < 1e-4


def test_supervised_loss():
    d = fx("sup_loss")
    invs = [i.clone().requires_grad_(True) for i in d["inv_depths"]]
    vecs = d["poses"].clone().requires_grad_(True)
    N, n = vecs.shape[1], vecs.shape[2]
    poses = [[vecs[:, j, i] for i in range(n)] for j in range(N)]
    gt = d["gt_depth"]
    gt_inv = torch.where(gt <= 0, torch.zeros_like(gt), 1.0 / gt.clamp(min=1e-6))
    out = O.supervised_depth_pose_loss(invs, gt_inv, [d["gt_poses"][:, j] for j in range(N)], poses,
                                       d["K"], d["K"], fval(d["min_depth"]), fval(d["max_depth"]))
    assert O.rel_err(out["loss"], d["loss"]) < TOL
    assert O.rel_err(out["depth_loss"], d["depth_loss"]) < TOL
    assert O.rel_err(out["pose_loss"], d["pose_loss"]) < TOL
    out["loss"].sum().backward()
    assert O.rel_err(torch.stack([i.grad for i in invs]), d["g_inv_depths"]) < 1e-4
    assert O.rel_err(vecs.grad, d["g_poses"]) < 1e-4


def test_upsample():
    d = fx("upsample")
    inv, mask = d["inv"].clone().requires_grad_(True), d["mask"].clone().requires_grad_(True)
    up = O.convex_upsample(inv, mask, 8)
    assert O.rel_err(up, d["up"]) < TOL
    (up * d["G"]).sum().backward()
    assert O.rel_err(inv.grad, d["g_inv"]) < TOL
    assert O.rel_err(mask.grad, d["g_mask"]) < TOL


def spec_params(name, grad=False):
    p = params_from_spec(load_spec(os.path.join(G, name + "_keys.json")))
    if grad:
        p = {k: (v.requires_grad_(True) if v.is_floating_point() and "running" not in k else v)
             for k, v in p.items()}
    return p


@pytest.mark.parametrize("hd", [64, 128])
def test_sepconvgru(hd):
    d = fx(f"sepconvgru_h{hd}")
    p = spec_params(f"sepconvgru_h{hd}", grad=True)
    h, x = d["h"].clone().requires_grad_(True), d["x"].clone().requires_grad_(True)
    out = O.sep_conv_gru(p, "", h, x)
    assert O.rel_err(out, d["out"]) < TOL
    (out * d["G"]).sum().backward()
    assert O.rel_err(h.grad, d["g_h"]) < 1e-4
    assert O.rel_err(x.grad, d["g_x"]) < 1e-4
    for k, v in p.items():
        ref = d["gsum." + k]
        got = v.grad.double()
        assert abs(float(got.sum()) - float(ref[0])) <= 1e-4 * float(ref[1]) + 1e-6, k


def test_update_block_depth():
    d = fx("update_depth")
    p = spec_params("update_depth", grad=True)
    net = d["net"].clone().requires_grad_(True)
    fmap = d["fmap"].clone().requires_grad_(True)
    frefs = [f.clone().requires_grad_(True) for f in d["fmap_ref"]]
    poses = list(d["poses"])
    cost_fn = lambda x: O.depth_cost_calc(x, fmap, frefs, poses, d["K"], d["K"], 1.0 / 8)
    scale = lambda x: O.disp_to_depth(x, 0.5, 80.0)
    out, masks, invs = O.update_block_depth(p, "", net, cost_fn, d["disp"], d["ctx"], 2, scale)
    assert O.rel_err(out, d["net_out"]) < 1e-4
    assert O.rel_err(torch.stack(invs), d["invs"]) < 1e-4
    assert O.rel_err(torch.stack(masks)[:, :, :24], d["masks"]) < 1e-4
    ((out * d["Gn"]).sum() + (invs[-1] * d["Gi"]).sum() + (masks[-1] * d["Gm"]).sum()).backward()
    assert O.rel_err(net.grad, d["g_net"]) < 1e-4
    assert O.rel_err(fmap.grad, d["g_fmap"]) < 1e-4
    assert O.rel_err(torch.stack([f.grad for f in frefs]), d["g_fmap_ref"]) < 1e-4
    for k, v in p.items():
        if v.requires_grad:
            ref = d["gsum." + k]
            assert abs(float(v.grad.double().sum()) - float(ref[0])) <= 1e-4 * float(ref[1]) + 1e-6, k


def test_update_block_pose():
    d = fx("update_pose")
    p = spec_params("update_pose", grad=True)
    fmap = d["fmap"].clone().requires_grad_(True)
    fref = d["fmap_ref"].clone().requires_grad_(True)
    pose = d["pose"].clone().requires_grad_(True)
    cost_fn = lambda q: O.get_cost_each(q, fmap, fref, d["depth"], d["K"], d["K"], 1.0 / 8)
    out, seqs = O.update_block_pose(p, "", d["net"], cost_fn, pose, d["ctx"], 2)
    assert O.rel_err(out, d["net_out"]) < 1e-4
    assert O.rel_err(torch.stack(seqs), d["poses"]) < 1e-4
    ((out * d["Gn"]).sum() + (seqs[-1] * d["Gp"]).sum()).backward()
    assert O.rel_err(pose.grad, d["g_pose"]) < 1e-4
    assert O.rel_err(fmap.grad, d["g_fmap"]) < 1e-4
    assert O.rel_err(fref.grad, d["g_fmap_ref"]) < 1e-4


@pytest.mark.parametrize("tag,version", [("it8", "it8-seq4-inter-out"), ("it12h", "it12-h-out")])
def test_depth_pose_net(tag, version):
    d = fx(f"depthposenet_{tag}")
    p = spec_params(f"depthposenet_{tag}")
    mind, maxd = fval(d["min_depth"]), fval(d["max_depth"])
    with torch.no_grad():
        invs, poses = O.depth_pose_net(dict(p), version, mind, maxd, d["image"], list(d["refs"]),
                                       d["K"], training=True)
        assert O.rel_err(torch.stack(invs), d["inv_depths"]) < 1e-4
        assert O.rel_err(poses, d["poses"]) < 1e-4
        # the reference eval pass runs after the train pass updated BN running stats
        inv_e, pose_e = O.depth_pose_net(p, version, mind, maxd, d["image"], list(d["refs"]),
                                         d["K"], training=False)
        assert O.rel_err(inv_e, d["inv_eval"]) < 1e-4
        assert O.rel_err(pose_e, d["poses_eval"]) < 1e-4


@pytest.mark.parametrize("tag,version,kind", [("it8", "it8-seq4-inter-out", "selfsup"),
                                              ("it12h", "it12-h-out", "sup")])
def test_train_step(tag, version, kind):
    d = fx(f"train_step_{tag}")
    dn = fx(f"depthposenet_{tag}")
    p = spec_params(f"depthposenet_{tag}", grad=True)
    mind, maxd = fval(dn["min_depth"]), fval(dn["max_depth"])
    N = d["refs"].shape[0]
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"], "depth": d["gt_depth"],
             "pose_context": [d["gt_poses"][:, j] for j in range(N)]}
    out = O.train_step_loss(p, version, mind, maxd, batch, kind=kind)
    assert O.rel_err(out["loss"], d["loss"]) < 1e-4
    out["loss"].sum().backward()
    worst = 0.0
    for k, v in p.items():
        key = "gsum." + k
        if key in d and v.grad is not None:
            ref = d[key]
            worst = max(worst, abs(float(v.grad.double().sum()) - float(ref[0])) / (float(ref[1]) + 1e-12))
    assert worst < 1e-3


@pytest.mark.parametrize("name", ["metrics_garg", "metrics_nocrop"])
@pytest.mark.parametrize("scaled", [True, False])
def test_depth_metrics(name, scaled):
    """compute_depth_metrics (utils/depth.py:259-343): the restatement reproduces
    the reference's nine metrics bit for bit on sparse LiDAR-like ground truth
    (garg crop + upsampled prediction; no crop; an image without valid pixels)."""
    d = load_fixture(os.path.join(G, name + ".npz"))
    crop = {0: "", 1: "garg", 2: "eigen_nyu"}[int(d["crop"])]
    out = O.depth_metrics(d["gt"], d["pred"], fval(d["min_depth"]), fval(d["max_depth"]), crop, scaled)
    assert torch.equal(out, d["metrics_scaled" if scaled else "metrics_unscaled"])


@pytest.mark.parametrize("shape", [((375, 1242), (192, 640)), ((480, 640), (240, 320)), ((50, 40), (96, 81))])
def test_resize_matches_pillow(shape):
    """The Pillow BILINEAR restatement (the reference's Resize on PIL frames,
    datasets/augmentations.py:69-111) reproduces PIL itself bit for bit."""
    import numpy as np
    from PIL import Image
    (h0, w0), (H, W) = shape
    a = np.random.default_rng(h0).integers(0, 256, (h0, w0, 3), dtype=np.uint8)
    want = np.asarray(Image.fromarray(a).resize((W, H), Image.BILINEAR))
    assert np.array_equal(O.resize_bilinear_pil(a, H, W), want)


def _train_step_oracle(spec_name, version, mind, maxd, batch, kind, dt, flip=False):
    p = spec_params(spec_name)
    p = {k: (v.to(dt).requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.to(dt) if v.is_floating_point() else v)) for k, v in p.items()}
    b = {k: (v.to(dt) if torch.is_tensor(v) and v.is_floating_point() else
             ([t.to(dt) for t in v] if isinstance(v, list) else v)) for k, v in batch.items()}
    out = O.train_step_loss(p, version, mind, maxd, b, kind=kind, flip=flip)
    out["loss"].sum().backward()
    return out, [(k, v.grad) for k, v in p.items() if getattr(v, "grad", None) is not None]


def _grad_pin(fixture, g32, g64, floor=2e-5, frac=0.1):
    """Per tensor, over the fixture's stored elements: the fp32 oracle within
    max(floor, frac x the reference fp32 gradient's own max-rel distance to
    the fp64 oracle) of the reference.  The reference is itself that far from
    the exact gradient (BatchNorm parameter gradients are sums with heavy
    cancellation, the recurrent loop amplifies rounding); a restatement
    error would show up as a fixed fraction of the gradient, not below it."""
    e32, e64 = grad_errors(g32, fixture), grad_errors(g64, fixture)
    assert e32.keys() == e64.keys() and len(e32) > 100
    bad = [(k, e32[k], e64[k]) for k in e32 if e32[k] > max(floor, frac * e64[k])]
    return bad, max(e32.values())


@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("tag,version,kind", [("it8", "it8-seq4-inter-out", "selfsup"),
                                              ("it12h", "it12-h-out", "sup")])
def test_train_step_gradients_per_element(tag, version, kind, flip):
    """Training step (SelfSupModelMF it8 / SupModelMF it12-h) without and with
    the left-right flip forced (SfmModelMF.py:110-119: K flipped in place,
    the loss sees it): loss 1e-5 and every parameter gradient per element
    (it8: update blocks and heads whole; encoders at a fixed sample of 2048
    entries per tensor) against the reference's own fixtures."""
    d = fx(f"train_step_{tag}")
    dn = fx(f"depthposenet_{tag}")
    f = fx(f"train_step_{tag}_{'flip' if flip else 'grads'}")
    mind, maxd = fval(dn["min_depth"]), fval(dn["max_depth"])
    N = d["refs"].shape[0]
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"], "depth": d["gt_depth"],
             "pose_context": [d["gt_poses"][:, j] for j in range(N)]}
    out, g32 = _train_step_oracle(f"depthposenet_{tag}", version, mind, maxd, batch, kind, torch.float32, flip)
    assert O.rel_err(out["loss"], f["loss"]) < 1e-5
    if flip:
        assert torch.equal(O.flip_lr_intr(d["K"], d["image"].shape[3]), f["K_after"])
    _, g64 = _train_step_oracle(f"depthposenet_{tag}", version, mind, maxd, batch, kind, torch.float64, flip)
    bad, worst = _grad_pin(f, g32, g64)
    assert not bad, bad[:5]


def test_train_step_selfsup_view5_n4():
    """configs[4] model: SelfSupModelMF it12-h-out with N=4 refs (ScanNet view5,
    depth 0.2-10) -- loss and per-element gradients vs the reference."""
    f = fx("train_step_it12h_selfsup_n4")
    N = f["refs"].shape[0]
    batch = {"rgb": f["image"], "rgb_context": list(f["refs"]), "rgb_original": f["image"],
             "rgb_context_original": list(f["refs"]), "intrinsics": f["K"]}
    mind, maxd = fval(f["min_depth"]), fval(f["max_depth"])
    assert N == 4
    out, g32 = _train_step_oracle("depthposenet_it12h", "it12-h-out", mind, maxd, batch, "selfsup", torch.float32)
    assert O.rel_err(out["loss"], f["loss"]) < 1e-5
    _, g64 = _train_step_oracle("depthposenet_it12h", "it12-h-out", mind, maxd, batch, "selfsup", torch.float64)
    bad, worst = _grad_pin(f, g32, g64)
    assert not bad, bad[:5]


@pytest.mark.parametrize("scaled", [True, False])
def test_depth_metrics_demon(scaled):
    """compute_depth_metrics_demon (utils/depth.py:343-398): the restatement
    reproduces the reference's metrics bit for bit (dense ScanNet-like gt, a
    lower-resolution prediction, the gt translation normalisation, an image
    without valid pixels)."""
    d = load_fixture(os.path.join(G, "metrics_demon.npz"))
    out = O.depth_metrics_demon(d["gt"], d["gt_pose"], d["pred"], fval(d["min_depth"]), fval(d["max_depth"]),
                                scaled)
    assert torch.equal(out, d["metrics_scaled" if scaled else "metrics_unscaled"])


def test_pose_metrics():
    """compute_pose_metrics (utils/depth.py:400-421) on six near pose pairs:
    bit for bit."""
    d = load_fixture(os.path.join(G, "metrics_pose.npz"))
    for k in range(d["gt"].shape[0]):
        assert torch.equal(O.pose_metrics(d["gt"][k], d["pred"][k]), d["metrics"][k]), k


def test_grid_sample_cells_matches_aten():
    """The oracle's forced-cell bilinear sampler (O.Cells, the parity tests'
    branch pinning): with the natural cells recorded and forced back it equals
    F.grid_sample (bilinear, zeros, align_corners=True) in value and in both
    gradients; at a sampling coordinate exactly on a grid line, forcing the
    cell to the left neighbour keeps the value and switches the x-derivative
    to the left cell's slope."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(0)
    img = torch.randn(2, 5, 12, 20, generator=g, dtype=torch.float64)
    grid = torch.rand(2, 12, 20, 2, generator=g, dtype=torch.float64) * 2.4 - 1.2
    rec = O.Cells(record=True)
    ga, gb = grid.clone().requires_grad_(True), grid.clone().requires_grad_(True)
    ia, ib = img.clone().requires_grad_(True), img.clone().requires_grad_(True)
    a = F.grid_sample(ia, ga, mode="bilinear", padding_mode="zeros", align_corners=True)
    assert torch.allclose(rec.sample(img, grid, "k"), a, atol=1e-12)
    b = O.Cells(forced={"k": rec.recorded["k"]}).sample(ib, gb, "k")
    assert torch.allclose(a, b, atol=1e-12)
    a.sum().backward()
    b.sum().backward()
    assert torch.allclose(ga.grad, gb.grad, atol=1e-10) and torch.allclose(ia.grad, ib.grad, atol=1e-12)
    # one output exactly on the grid line x = 7: natural cell x0 = 7, forced x0 = 6
    one = img[:1, :1]
    gx = torch.tensor([[[[2 * 7 / 19 - 1, 2 * 4.25 / 11 - 1]]]], dtype=torch.float64, requires_grad=True)
    nat = O.Cells(record=True)
    v_nat = nat.sample(one, gx, "p")
    c = nat.recorded["p"].clone()
    c = c - 1                                           # x0 + 32768 - 1: the left cell
    v_left = O.Cells(forced={"p": c}).sample(one, gx, "p")
    assert torch.allclose(v_nat, v_left, atol=1e-12)
    d_nat = torch.autograd.grad(nat.sample(one, gx, "p").sum(), gx)[0][..., 0]
    d_left = torch.autograd.grad(O.Cells(forced={"p": c}).sample(one, gx, "p").sum(), gx)[0][..., 0]
    r = one[0, 0, 4] * 0.75 + one[0, 0, 5] * 0.25      # the row interpolated at y = 4.25
    assert torch.allclose(d_nat, (r[8] - r[7]) * 19 / 2, atol=1e-10)
    assert torch.allclose(d_left, (r[7] - r[6]) * 19 / 2, atol=1e-10)


def test_max_pool_forced_argmax():
    """oracle.max_pool_3x3s2: with the natural argmax forced it equals
    F.max_pool2d (values and gradients); on an exact tie the gradient goes to
    the forced window element; a forced index that is not a near-tie is
    ignored."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 3, 9, 11, generator=g, dtype=torch.float64)
    y, ind = F.max_pool2d(x, 3, 2, 1, return_indices=True)
    Ho, Wo = y.shape[-2:]
    oy = torch.arange(Ho).view(1, 1, Ho, 1)
    ox = torch.arange(Wo).view(1, 1, 1, Wo)
    iy, ix = ind // 11, ind % 11
    nat = (iy - (2 * oy - 1)) * 3 + (ix - (2 * ox - 1))
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    G = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (O.max_pool_3x3s2(xa, nat) * G).sum().backward()
    (F.max_pool2d(xb, 3, 2, 1) * G).sum().backward()
    assert torch.allclose(xa.grad, xb.grad, rtol=0, atol=1e-14)
    # exact tie in window (0, 1): input (0, 1) and (0, 2); natural picks the first
    t = torch.zeros(1, 1, 3, 5, dtype=torch.float64)
    t[0, 0, 0, 1] = t[0, 0, 0, 2] = 1.0
    forced = torch.full((1, 1, 2, 3), -1, dtype=torch.int64)
    nat_t = F.max_pool2d(t, 3, 2, 1, return_indices=True)[1]
    forced[0, 0, 0, 1] = 1 * 3 + 1            # window rows -1..1, cols 1..3: input (0, 2) is dy 1, dx 1
    tt = t.clone().requires_grad_(True)
    O.max_pool_3x3s2(tt, forced.clamp_min(0)).sum().backward()
    assert nat_t[0, 0, 0, 1] == 1                      # natural: the first maximum, x = 1
    assert tt.grad[0, 0, 0, 2] >= 1.0                  # forced: routed to x = 2 for that window
    far = torch.zeros_like(forced)                     # index 0 = the (padded / smaller) corner: not a tie
    tf = t.clone().requires_grad_(True)
    O.max_pool_3x3s2(tf, far).sum().backward()
    tn = t.clone().requires_grad_(True)
    F.max_pool2d(tn, 3, 2, 1).sum().backward()
    assert torch.equal(tf.grad, tn.grad)


def test_relu_pinned():
    """oracle.relu_pinned: the natural mask forced == F.relu; a forced mask
    flips the derivative only where |v| is within 1e-5 of the channel scale."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(5)
    v = torch.randn(2, 3, 4, 5, generator=g, dtype=torch.float64)
    v[0, 1, 2, 3] = 1e-9                      # at the kink
    book = O.Cells(forced={("relu", "s"): (v > 0).to(torch.uint8)})
    a = v.clone().requires_grad_(True)
    O.relu_pinned(a, book, "s").sum().backward()
    b = v.clone().requires_grad_(True)
    F.relu(b).sum().backward()
    assert torch.equal(a.grad, b.grad)
    flipped = (v > 0).to(torch.uint8)
    flipped[0, 1, 2, 3] = 0                   # near the kink: taken
    flipped[1, 0, 0, 0] = 1 - flipped[1, 0, 0, 0]   # far from it: ignored
    c = v.clone().requires_grad_(True)
    O.relu_pinned(c, O.Cells(forced={("relu", "s"): flipped}), "s").sum().backward()
    assert c.grad[0, 1, 2, 3] == 0 and c.grad[1, 0, 0, 0] == b.grad[1, 0, 0, 0]


def test_cells_from_calls_keys():
    """oracle.cells_from_calls maps the product's record (tag, map) in call
    order to the oracle's keys: cost calls per inner step and view, the
    photometric calls per (view, prediction), pooling argmax and ReLU masks
    by encoder / BatchNorm site."""
    cost = torch.zeros(2, 1, 3, 4, dtype=torch.int32)                 # [N=2, B=1, h, w]
    photo = torch.zeros(2, 3, 1, 6, 8, dtype=torch.int32)             # [N=2, n=3, B=1, H, W]
    calls = [(("depth", 0), cost), (("depth", 0), cost + 1), (("pose", 0), cost + 2), ("photo", photo),
             (("maxpool", "fnet"), torch.zeros(1, 2, 3, 4, dtype=torch.uint8)),
             (("relu", "fnet.layer1.0.bn1"), torch.ones(1, 2, 3, 4, dtype=torch.uint8))]
    out = O.cells_from_calls(calls)
    assert int(out[("depth", 0, 1, 0)][0, 0, 0]) == 1 and ("depth", 0, 1, 1) in out
    assert int(out[("pose", 0, 0, 1)][0, 0, 0]) == 2
    assert out[("photo", 1, 2)].shape == (1, 6, 8)
    assert out[("maxpool", "fnet")].dtype == torch.int64
    assert int(out[("relu", "fnet.layer1.0.bn1")].sum()) == 24


def test_relu_site_calls_and_views():
    """Conv ReLU sites: the product's ("relu_seq", name) records become
    ("relu", (name, n)) for the n-th call; oracle.relu_site takes view j's rows
    of a stacked record and pins only near-kinks (SEQ_RELU_TOL)."""
    import torch.nn.functional as F
    m0 = torch.ones(4, 2, 3, 3, dtype=torch.uint8)             # [N*B = 2*2, C, h, w]
    m1 = m0.clone()
    m1[2, 1, 0, 0] = 0                                           # view j=1, row 0
    out = O.cells_from_calls([(("relu_seq", "u.convc1"), m0), (("relu_seq", "u.convc1"), m1)])
    assert set(out) == {("relu", ("u.convc1", 0)), ("relu", ("u.convc1", 1))}
    book = O.Cells(forced=out)
    v = torch.full((2, 2, 3, 3), 0.5, dtype=torch.float64)
    v[0, 1, 0, 0] = 1e-9                                         # at the kink, positive
    a = v.clone().requires_grad_(True)
    O.relu_site(a, (book, 1, (1, 2)), "u.convc1").sum().backward()
    assert a.grad[0, 1, 0, 0] == 0 and a.grad.sum() == v.numel() - 1
    b = v.clone().requires_grad_(True)
    O.relu_site(b, (book, 1, (0, 2)), "u.convc1").sum().backward()      # view 0: natural
    c = v.clone().requires_grad_(True)
    F.relu(c).sum().backward()
    assert torch.equal(b.grad, c.grad)
    assert torch.equal(O.relu_site(v, (None, 0, None), "x"), F.relu(v))

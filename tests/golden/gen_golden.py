"""Golden-vector generator (test infrastructure; runs ONLY in the build container).

Imports the read-only reference at /root/reference in-process, through the
import shims of SURVEY.md §8(c), and records inputs, outputs and input
gradients of every hot-path row of SURVEY.md §8(a) into small ``.npz``
fixtures next to this file.  The reference itself never leaves this
container; only these numeric vectors are committed.

Shims (all injected into ``sys.modules`` before the reference is imported):
  * ``cv2``                        -- empty module (imported, unused on the path:
                                      dro_sfm/utils/image.py:2)
  * ``numpy.lib.type_check.imag``  -- removed in numpy 2
                                      (losses/multiview_photometric_loss_mf.py:2)
  * ``yacs.config.CfgNode``        -- dict stand-in (utils/types.py:2)
  * ``torchvision.transforms``     -- empty (utils/depth.py:4)
  * ``torchvision.models``         -- structural stand-in of torchvision's
                                      ResNet-18 (BasicBlock, _make_layer), only
                                      so that ``ResNetEncoder`` (extractor.py:7)
                                      can subclass it; pretrained download is
                                      never attempted (pretrained=False).
  * ``Camera.to(-1)``              -- mapped to 'cpu' (the reference's
                                      ``ref_image.get_device()`` returns -1 on CPU,
                                      multiview_photometric_loss_mf.py:156,162).
Weights are filled by ``common.det_init`` (name-keyed), so fixtures carry no
state_dicts.

Usage:  python tests/golden/gen_golden.py          (writes tests/golden/*.npz)
"""
import os
import sys
import types
from functools import partial

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from common import SCANNET_K_320, det_init, grad_fixture, kitti_K, smooth_images, to_np  # noqa: E402

REF = "/root/reference"


# ----------------------------------------------------------------------------- shims
def _resnet_standin():
    """torchvision.models stand-in: ResNet/BasicBlock with torchvision's structure."""
    tvm = types.ModuleType("torchvision.models")
    res = types.ModuleType("torchvision.models.resnet")

    def conv3x3(i, o, s=1):
        return nn.Conv2d(i, o, 3, stride=s, padding=1, bias=False)

    class BasicBlock(nn.Module):
        expansion = 1

        def __init__(self, inplanes, planes, stride=1, downsample=None, *a, **k):
            super().__init__()
            self.conv1 = conv3x3(inplanes, planes, stride)
            self.bn1 = nn.BatchNorm2d(planes)
            self.relu = nn.ReLU(inplace=True)
            self.conv2 = conv3x3(planes, planes)
            self.bn2 = nn.BatchNorm2d(planes)
            self.downsample = downsample
            self.stride = stride

        def forward(self, x):
            idt = x
            out = self.relu(self.bn1(self.conv1(x)))
            out = self.bn2(self.conv2(out))
            if self.downsample is not None:
                idt = self.downsample(x)
            return self.relu(out + idt)

    class Bottleneck(BasicBlock):
        expansion = 4

    class ResNet(nn.Module):
        def __init__(self, block, layers, num_classes=1000):
            super().__init__()
            self.inplanes = 64
            self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
            self.bn1 = nn.BatchNorm2d(64)
            self.relu = nn.ReLU(inplace=True)
            self.maxpool = nn.MaxPool2d(3, 2, 1)
            self.layer1 = self._make_layer(block, 64, layers[0])
            self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
            self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
            self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
            self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
            self.fc = nn.Linear(512 * block.expansion, num_classes)

        def _make_layer(self, block, planes, blocks, stride=1):
            down = None
            if stride != 1 or self.inplanes != planes * block.expansion:
                down = nn.Sequential(
                    nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride=stride, bias=False),
                    nn.BatchNorm2d(planes * block.expansion))
            mods = [block(self.inplanes, planes, stride, down)]
            self.inplanes = planes * block.expansion
            for _ in range(1, blocks):
                mods.append(block(self.inplanes, planes))
            return nn.Sequential(*mods)

    res.BasicBlock, res.Bottleneck, res.ResNet = BasicBlock, Bottleneck, ResNet
    res.model_urls = {"resnet18": "offline://never-fetched"}
    tvm.resnet, tvm.ResNet = res, ResNet
    return tvm, res


def install_shims():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    import numpy.lib as nplib
    tc = types.ModuleType("numpy.lib.type_check")
    tc.imag = np.imag
    sys.modules["numpy.lib.type_check"] = tc
    nplib.type_check = tc
    yacs = types.ModuleType("yacs")
    yc = types.ModuleType("yacs.config")

    class CfgNode(dict):
        pass

    yc.CfgNode = CfgNode
    yacs.config = yc
    sys.modules["yacs"], sys.modules["yacs.config"] = yacs, yc
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tvm, res = _resnet_standin()
    tv.transforms, tv.models = tvt, tvm
    sys.modules.update({"torchvision": tv, "torchvision.transforms": tvt,
                        "torchvision.models": tvm, "torchvision.models.resnet": res})
    sys.path.insert(0, REF)
    import torch.utils.model_zoo as mz

    def _no_fetch(*a, **k):
        raise RuntimeError("network fetch disabled in golden generation")

    mz.load_url = _no_fetch
    from dro_sfm.geometry import camera as cam_mod
    _orig_to = cam_mod.Camera.to

    def _to(self, *args, **kw):
        args = tuple("cpu" if (isinstance(a, int) and a < 0) else a for a in args)
        return _orig_to(self, *args, **kw)

    cam_mod.Camera.to = _to
    from dro_sfm.networks.optim import extractor
    extractor.ResNetEncoder.__init__.__defaults__ = (18, 1, False, 32, 8)


# ----------------------------------------------------------------------------- helpers
def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    arrs = {k: to_np(v).astype(np.float32) if to_np(v).dtype == np.float64 else to_np(v)
            for k, v in arrays.items()}
    if os.path.exists(path):
        # regenerating an existing fixture must reproduce it exactly: keep the
        # committed file (no byte churn from the zip metadata), fail otherwise
        with np.load(path, allow_pickle=False) as z:
            same = set(z.files) == set(arrs) and all(np.array_equal(z[k], arrs[k]) for k in arrs)
        if same:
            print(f"  {name}.npz unchanged")
            return
        if os.environ.get("GOLDEN_OVERWRITE") != "1":
            raise SystemExit(f"{name}.npz would change (set GOLDEN_OVERWRITE=1 to rewrite it)")
    np.savez_compressed(path, **arrs)
    print(f"  wrote {name}.npz ({os.path.getsize(path) / 1024:.0f} KiB)")


def rand_pose(B, g, t_std=0.1, r_std=0.02):
    t = torch.randn(B, 3, generator=g) * t_std
    r = torch.randn(B, 3, generator=g) * r_std
    return torch.cat([t, r], 1)


def grad_checksums(module, g):
    """Per-parameter gradient fingerprints (sum, |sum|, fixed random projection)."""
    out = {}
    for name, p in module.named_parameters():
        if p.grad is None:
            continue
        proj = torch.randn(p.shape, generator=_proj_gen(name))
        gr = p.grad.double()
        out["gsum." + name] = torch.tensor([gr.sum(), gr.abs().sum(), (gr * proj.double()).sum()])
    return out


def _proj_gen(name):
    import zlib
    gg = torch.Generator()
    gg.manual_seed(zlib.crc32(("proj:" + name).encode()) & 0x7FFFFFFF)
    return gg


# ----------------------------------------------------------------------------- fixtures
def gen_cost():
    from dro_sfm.networks.depth_pose.DepthPoseNet import DepthPoseNet
    from dro_sfm.utils.depth import inv2depth
    from dro_sfm.networks.layers.resnet.layers import disp_to_depth
    cost_each = partial(DepthPoseNet.get_cost_each, None)
    depth_cost = DepthPoseNet.depth_cost_calc

    class _Self:
        get_cost_each = staticmethod(cost_each)

    g = torch.Generator().manual_seed(1)
    # (a) get_cost_each, B=2 C=128 12x20, image 96x160
    cases = {
        "cost_each_small": dict(B=2, C=128, h=12, w=20, oob=False),
        "cost_each_edge": dict(B=2, C=64, h=12, w=20, oob=True),
        "cost_each_kitti": dict(B=1, C=32, h=24, w=80, oob=False),
    }
    for name, c in cases.items():
        B, C, h, w = c["B"], c["C"], c["h"], c["w"]
        K = kitti_K(B, W=8 * w, H=8 * h)
        pose = rand_pose(B, g, 0.1, 0.02)
        inv = 0.05 + 0.5 * torch.rand(B, 1, h, w, generator=g)
        if c["oob"]:
            pose[0, 3:] = torch.tensor([0.05, 0.9, -0.1])       # large yaw: many OOB samples
            pose[1, :3] = torch.tensor([0.0, 0.0, -25.0])       # points behind the camera
            inv[:, :, :2, :3] = -0.1                            # inv <= 0 -> depth 0
            inv[:, :, 5, 7] = 0.0
        depth = inv2depth(inv)
        fmap = torch.randn(B, C, h, w, generator=g)
        fref = torch.randn(B, C, h, w, generator=g)
        G = torch.randn(B, C, h, w, generator=g)
        pose_, fmap_, fref_, depth_ = (x.clone().requires_grad_(True) for x in (pose, fmap, fref, depth))
        cost = cost_each(pose_, fmap_, fref_, depth_, K, K, 1.0 / 8)
        (cost * G).sum().backward()
        save(name, pose=pose, fmap=fmap, fmap_ref=fref, depth=depth, K=K, G=G, cost=cost,
             g_pose=pose_.grad, g_fmap=fmap_.grad, g_fmap_ref=fref_.grad, g_depth=depth_.grad)

    # (b) depth_cost_calc: N refs, mean over refs, grad to the scaled inverse depth
    for name, (B, C, h, w, N) in {"depth_cost_n2": (2, 128, 12, 20, 2),
                                  "depth_cost_n4": (1, 64, 12, 20, 4)}.items():
        K = kitti_K(B, W=8 * w, H=8 * h)
        poses = [rand_pose(B, g) for _ in range(N)]
        disp = torch.rand(B, 1, h, w, generator=g)
        fmap = torch.randn(B, C, h, w, generator=g)
        frefs = [torch.randn(B, C, h, w, generator=g) for _ in range(N)]
        G = torch.randn(B, C, h, w, generator=g)
        disp_ = disp.clone().requires_grad_(True)
        fmap_ = fmap.clone().requires_grad_(True)
        frefs_ = [f.clone().requires_grad_(True) for f in frefs]
        inv_scaled = disp_to_depth(disp_, 0.5, 80.0)[0]
        cost = depth_cost(_Self(), inv_scaled, fmap_, frefs_, poses, K, K, 1.0 / 8)
        (cost * G).sum().backward()
        save(name, disp=disp, fmap=fmap, fmap_ref=torch.stack(frefs), poses=torch.stack(poses),
             K=K, G=G, cost=cost, g_disp=disp_.grad, g_fmap=fmap_.grad,
             g_fmap_ref=torch.stack([f.grad for f in frefs_]), min_depth=np.float32(0.5),
             max_depth=np.float32(80.0))

    # (c) D=64 fronto-parallel hypothesis planes (SURVEY.md §8(d) measurement extension)
    B, C, h, w, D = 1, 16, 12, 20, 64
    K = kitti_K(B, W=8 * w, H=8 * h)
    pose = rand_pose(B, g)
    fmap = torch.randn(B, C, h, w, generator=g)
    fref = torch.randn(B, C, h, w, generator=g)
    disp = torch.linspace(0, 1, D)
    vol = []
    with torch.no_grad():
        for d in disp:
            inv = disp_to_depth(torch.full((B, 1, h, w), float(d)), 0.5, 80.0)[0]
            vol.append(cost_each(pose, fmap, fref, inv2depth(inv), K, K, 1.0 / 8))
    save("plane_sweep_d64", pose=pose, fmap=fmap, fmap_ref=fref, K=K, disp=disp,
         cost=torch.stack(vol, 1), min_depth=np.float32(0.5), max_depth=np.float32(80.0))


def gen_geometry_loss():
    from dro_sfm.geometry.camera import Camera
    from dro_sfm.geometry.pose import Pose
    from dro_sfm.geometry.camera_utils import view_synthesis
    from dro_sfm.losses.multiview_photometric_loss_mf import SSIM, MultiViewPhotometricDecayLoss
    from dro_sfm.losses.supervised_loss import SupervisedDepthPoseLoss
    g = torch.Generator().manual_seed(2)
    B, H, W = 2, 48, 160
    K = kitti_K(B, W=W, H=H)

    # view synthesis (K9): RGB warp at full res
    ref = smooth_images(B, H, W, 11)
    depth = 1.0 / (0.05 + 0.5 * torch.rand(B, 1, H, W, generator=g))
    vec = rand_pose(B, g)
    d_, v_ = depth.clone().requires_grad_(True), vec.clone().requires_grad_(True)
    warped = view_synthesis(ref, d_, Camera(K=K, Tcw=Pose.from_vec(v_, "euler")), Camera(K=K))
    G = torch.randn(warped.shape, generator=g)
    (warped * G).sum().backward()
    save("view_synthesis", ref=ref, depth=depth, pose=vec, K=K, G=G, warped=warped,
         g_depth=d_.grad, g_pose=v_.grad)

    # SSIM (K10)
    x, y = smooth_images(B, H, W, 12), smooth_images(B, H, W, 13)
    x_ = x.clone().requires_grad_(True)
    s = SSIM(x_, y)
    Gs = torch.randn(s.shape, generator=g)
    (s * Gs).sum().backward()
    save("ssim", x=x, y=y, G=Gs, ssim=s, g_x=x_.grad)

    # Photometric decay loss (a18): n_pred=3 full-res predictions, N=2 refs
    for name, kw in {"photo_loss": dict(),
                     "photo_loss_noauto": dict(automask_loss=False),
                     "photo_loss_mean": dict(automask_loss=False, photometric_reduce_op="mean")}.items():
        n, N = 3, 2
        image = smooth_images(B, H, W, 21)
        ctx = [smooth_images(B, H, W, 22 + j) for j in range(N)]
        invs = [0.05 + 0.5 * torch.rand(B, 1, H, W, generator=g) for _ in range(n)]
        vecs = torch.stack([torch.stack([rand_pose(B, g) for _ in range(n)], 1) for _ in range(N)], 1)  # [B,N,n,6]
        args = dict(ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001, C1=1e-4,
                    C2=9e-4, photometric_reduce_op="min", disp_norm=True, clip_loss=0.0,
                    progressive_scaling=0.0, padding_mode="zeros", automask_loss=True)
        args.update(kw)
        loss_fn = MultiViewPhotometricDecayLoss(**args)
        invs_ = [i.clone().requires_grad_(True) for i in invs]
        vecs_ = vecs.clone().requires_grad_(True)
        poses = [[Pose.from_vec(vecs_[:, j, i], "euler") for i in range(n)] for j in range(N)]
        out = loss_fn(image, ctx, invs_, K, K, poses)
        out["loss"].sum().backward()
        save(name, image=image, context=torch.stack(ctx), inv_depths=torch.stack(invs), poses=vecs,
             K=K, loss=out["loss"], photometric_loss=out["metrics"]["photometric_loss"],
             smoothness_loss=out["metrics"]["smoothness_loss"],
             g_inv_depths=torch.stack([i.grad for i in invs_]), g_poses=vecs_.grad,
             automask=np.int32(args["automask_loss"]),
             reduce_min=np.int32(args["photometric_reduce_op"] == "min"))

    # Supervised depth+pose loss (a19)
    n, N = 3, 2
    gt_depth = 1.0 + 79.0 * torch.rand(B, 1, H, W, generator=g)
    gt_depth[torch.rand(B, 1, H, W, generator=g) > 0.3] = 0.0
    invs = [0.02 + 0.5 * torch.rand(B, 1, H, W, generator=g) for _ in range(n)]
    vecs = torch.stack([torch.stack([rand_pose(B, g) for _ in range(n)], 1) for _ in range(N)], 1)
    gt_vecs = torch.stack([rand_pose(B, g) for _ in range(N)], 1)
    gt_mats = torch.stack([Pose.from_vec(gt_vecs[:, j], "euler").mat for j in range(N)], 1)  # [B,N,4,4]
    loss_fn = SupervisedDepthPoseLoss(supervised_method="sparse-l1", supervised_num_scales=4,
                                      min_depth=0.2, max_depth=80.0)
    invs_ = [i.clone().requires_grad_(True) for i in invs]
    vecs_ = vecs.clone().requires_grad_(True)
    poses = [[Pose.from_vec(vecs_[:, j, i], "euler") for i in range(n)] for j in range(N)]
    from dro_sfm.utils.depth import depth2inv
    out = loss_fn(None, None, invs_, depth2inv(gt_depth), [gt_mats[:, j] for j in range(N)], K, K, poses)
    out["loss"].sum().backward()
    save("sup_loss", gt_depth=gt_depth, inv_depths=torch.stack(invs), poses=vecs, gt_poses=gt_mats,
         K=K, loss=out["loss"], depth_loss=out["metrics"]["depth_loss"],
         pose_loss=out["metrics"]["pose_loss"], g_inv_depths=torch.stack([i.grad for i in invs_]),
         g_poses=vecs_.grad, min_depth=np.float32(0.2), max_depth=np.float32(80.0))


def gen_clip():
    """MultiViewPhotometricDecayLoss with clip_loss > 0 (the constructor's
    default 0.5, multiview_photometric_loss_mf.py:93, :223-227): min reduction
    with automask, and mean reduction without."""
    from dro_sfm.geometry.pose import Pose
    from dro_sfm.losses.multiview_photometric_loss_mf import MultiViewPhotometricDecayLoss
    g = torch.Generator().manual_seed(7)
    B, H, W = 2, 48, 160
    K = kitti_K(B, W=W, H=H)
    for name, kw in {"photo_loss_clip": dict(),
                     "photo_loss_clip_mean": dict(automask_loss=False, photometric_reduce_op="mean")}.items():
        n, N = 3, 2
        image = smooth_images(B, H, W, 61)
        ctx = [smooth_images(B, H, W, 62 + j) for j in range(N)]
        invs = [0.05 + 0.5 * torch.rand(B, 1, H, W, generator=g) for _ in range(n)]
        vecs = torch.stack([torch.stack([rand_pose(B, g) for _ in range(n)], 1) for _ in range(N)], 1)  # [B,N,n,6]
        args = dict(ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001, C1=1e-4,
                    C2=9e-4, photometric_reduce_op="min", disp_norm=True, clip_loss=0.5,
                    progressive_scaling=0.0, padding_mode="zeros", automask_loss=True)
        args.update(kw)
        loss_fn = MultiViewPhotometricDecayLoss(**args)
        invs_ = [i.clone().requires_grad_(True) for i in invs]
        vecs_ = vecs.clone().requires_grad_(True)
        poses = [[Pose.from_vec(vecs_[:, j, i], "euler") for i in range(n)] for j in range(N)]
        out = loss_fn(image, ctx, invs_, K, K, poses)
        out["loss"].sum().backward()
        save(name, image=image, context=torch.stack(ctx), inv_depths=torch.stack(invs), poses=vecs,
             K=K, loss=out["loss"], photometric_loss=out["metrics"]["photometric_loss"],
             smoothness_loss=out["metrics"]["smoothness_loss"],
             g_inv_depths=torch.stack([i.grad for i in invs_]), g_poses=vecs_.grad,
             automask=np.int32(args["automask_loss"]),
             reduce_min=np.int32(args["photometric_reduce_op"] == "min"), clip_loss=np.float32(0.5))


def gen_network_parts():
    from dro_sfm.networks.depth_pose.DepthPoseNet import DepthPoseNet
    from dro_sfm.networks.optim.update import SepConvGRU, BasicUpdateBlockDepth, BasicUpdateBlockPose
    from dro_sfm.networks.layers.resnet.layers import disp_to_depth
    g = torch.Generator().manual_seed(3)
    B, h, w = 2, 12, 20

    # convex upsample (a17)
    inv = torch.rand(1, 1, 6, 10, generator=g)
    mask = torch.randn(1, 576, 6, 10, generator=g)
    i_, m_ = inv.clone().requires_grad_(True), mask.clone().requires_grad_(True)
    up = DepthPoseNet.upsample_depth(None, i_, m_, ratio=8)
    G = torch.randn(up.shape, generator=g)
    (up * G).sum().backward()
    save("upsample", inv=inv, mask=mask, G=G, up=up, g_inv=i_.grad, g_mask=m_.grad)

    # SepConvGRU (a14), hdim 64 / 128, cdim 32
    for hd in (64, 128):
        gru = det_init(SepConvGRU(hidden_dim=hd, input_dim=hd + 32))
        hs = torch.tanh(torch.randn(B, hd, h, w, generator=g))
        x = torch.relu(torch.randn(B, hd + 32, h, w, generator=g))
        h_, x_ = hs.clone().requires_grad_(True), x.clone().requires_grad_(True)
        out = gru(h_, x_)
        G = torch.randn(out.shape, generator=g)
        (out * G).sum().backward()
        extra = {"g_" + k.replace(".", "_"): p.grad for k, p in gru.named_parameters()} if hd == 64 else {}
        import json
        with open(os.path.join(HERE, f"sepconvgru_h{hd}_keys.json"), "w") as fh:
            json.dump({k: list(v.shape) for k, v in gru.state_dict().items()}, fh, indent=0)
        save(f"sepconvgru_h{hd}", h=hs, x=x, G=G, out=out, g_h=h_.grad, g_x=x_.grad,
             **extra, **grad_checksums(gru, g))

    # update blocks (a12, a13): hdim 64, seq_len 2, N=2 refs, cost through the reference
    N, C, S = 2, 128, 2
    K = kitti_K(B, W=8 * w, H=8 * h)
    fmap = torch.randn(B, C, h, w, generator=g)
    frefs = [torch.randn(B, C, h, w, generator=g) for _ in range(N)]
    poses = [rand_pose(B, g) for _ in range(N)]

    class _Self:
        get_cost_each = staticmethod(partial(DepthPoseNet.get_cost_each, None))

    scale = partial(disp_to_depth, min_depth=0.5, max_depth=80.0)
    ub = det_init(BasicUpdateBlockDepth(hidden_dim=64, cost_dim=C, ratio=8, context_dim=32))
    import json
    with open(os.path.join(HERE, "update_depth_keys.json"), "w") as fh:
        json.dump({k: list(v.shape) for k, v in ub.state_dict().items()}, fh, indent=0)
    net = torch.tanh(torch.randn(B, 64, h, w, generator=g))
    ctx = torch.relu(torch.randn(B, 32, h, w, generator=g))
    disp = torch.sigmoid(torch.randn(B, 1, h, w, generator=g))
    fmap_ = fmap.clone().requires_grad_(True)
    frefs_ = [f.clone().requires_grad_(True) for f in frefs]
    net_ = net.clone().requires_grad_(True)
    cf = partial(DepthPoseNet.depth_cost_calc, _Self(), fmap=fmap_, fmaps_ref=frefs_, pose_list=poses,
                 K=K, ref_K=K, scale_factor=1.0 / 8)
    net_o, masks, invs = ub(net_, cf, disp, ctx, seq_len=S, scale_func=scale)
    Gn = torch.randn(net_o.shape, generator=g)
    Gi = torch.randn(invs[-1].shape, generator=g)
    Gm = torch.randn(masks[-1].shape, generator=g)
    ((net_o * Gn).sum() + (invs[-1] * Gi).sum() + (masks[-1] * Gm).sum()).backward()
    save("update_depth", net=net, ctx=ctx, disp=disp, fmap=fmap, fmap_ref=torch.stack(frefs),
         poses=torch.stack(poses), K=K, Gn=Gn, Gi=Gi, Gm=Gm, net_out=net_o,
         invs=torch.stack(invs), masks=torch.stack(masks)[:, :, :24], g_net=net_.grad, g_fmap=fmap_.grad,
         g_fmap_ref=torch.stack([f.grad for f in frefs_]), **grad_checksums(ub, g))

    ubp = det_init(BasicUpdateBlockPose(hidden_dim=64, cost_dim=C, context_dim=32))
    with open(os.path.join(HERE, "update_pose_keys.json"), "w") as fh:
        json.dump({k: list(v.shape) for k, v in ubp.state_dict().items()}, fh, indent=0)
    depth = 1.0 / scale(torch.sigmoid(torch.randn(B, 1, h, w, generator=g)))[0]
    pose0 = rand_pose(B, g)
    netp = torch.tanh(torch.randn(B, 64, h, w, generator=g))
    ctxp = torch.relu(torch.randn(B, 32, h, w, generator=g))
    fmap_ = fmap.clone().requires_grad_(True)
    fref_ = frefs[0].clone().requires_grad_(True)
    pose_ = pose0.clone().requires_grad_(True)
    cf = partial(DepthPoseNet.get_cost_each, None, fmap=fmap_, fmap_ref=fref_, depth=depth, K=K,
                 ref_K=K, scale_factor=1.0 / 8)
    net_o, plist = ubp(netp, cf, pose_, ctxp, seq_len=S)
    Gn = torch.randn(net_o.shape, generator=g)
    Gp = torch.randn(plist[-1].shape, generator=g)
    ((net_o * Gn).sum() + (plist[-1] * Gp).sum()).backward()
    save("update_pose", net=netp, ctx=ctxp, depth=depth, pose=pose0, fmap=fmap, fmap_ref=frefs[0],
         K=K, Gn=Gn, Gp=Gp, net_out=net_o, poses=torch.stack(plist), g_pose=pose_.grad,
         g_fmap=fmap_.grad, g_fmap_ref=fref_.grad, **grad_checksums(ubp, g))


def gen_full():
    from dro_sfm.networks.depth_pose.DepthPoseNet import DepthPoseNet
    from dro_sfm.models.SelfSupModelMF import SelfSupModelMF
    from dro_sfm.models.SupModelMF import SupModelMF
    from dro_sfm.geometry.pose import Pose
    B, N, H, W = 2, 2, 64, 96
    torch.manual_seed(0)
    for tag, version, mind, maxd in (("it8", "it8-seq4-inter-out", 0.5, 80.0),
                                     ("it12h", "it12-h-out", 0.2, 80.0)):
        net = det_init(DepthPoseNet(version=version, min_depth=mind, max_depth=maxd))
        import json
        with open(os.path.join(HERE, f"depthposenet_{tag}_keys.json"), "w") as fh:
            json.dump({k: list(v.shape) for k, v in net.state_dict().items()}, fh, indent=0)
        img = smooth_images(B, H, W, 31)
        refs = [smooth_images(B, H, W, 32 + j) for j in range(N)]
        K = kitti_K(B, W=W, H=H)
        net.train()
        invs, poses = net(img, refs, K)
        net.eval()
        with torch.no_grad():
            inv_e, pose_e = net(img, refs, K)
        save(f"depthposenet_{tag}", image=img, refs=torch.stack(refs), K=K,
             inv_depths=torch.stack(invs), poses=poses, inv_eval=inv_e, poses_eval=pose_e,
             min_depth=np.float32(mind), max_depth=np.float32(maxd))

        # full training step: model fwd + loss + backward (flip disabled)
        model_cls = SelfSupModelMF if tag == "it8" else SupModelMF
        kw = dict(ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001, C1=1e-4,
                  C2=9e-4, photometric_reduce_op="min", disp_norm=True, clip_loss=0.0,
                  progressive_scaling=0.0, padding_mode="zeros", automask_loss=True,
                  num_scales=4, flip_lr_prob=0.0, rotation_mode="euler", upsample_depth_maps=True,
                  supervised_method="sparse-l1", supervised_num_scales=4,
                  min_depth=mind, max_depth=maxd)
        model = model_cls(**kw)
        net2 = det_init(DepthPoseNet(version=version, min_depth=mind, max_depth=maxd))
        model.add_depth_net(net2)
        model.train()
        gdepth = 1.0 + 30.0 * torch.rand(B, 1, H, W, generator=torch.Generator().manual_seed(5))
        gvec = torch.stack([torch.cat([0.1 * torch.randn(B, 3), 0.02 * torch.randn(B, 3)], 1)
                            for _ in range(N)], 1)
        gpose = [Pose.from_vec(gvec[:, j], "euler").mat for j in range(N)]
        batch = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs,
                 "intrinsics": K.clone(), "depth": gdepth, "pose_context": gpose}
        out = model(batch)
        out["loss"].sum().backward()
        save(f"train_step_{tag}", image=img, refs=torch.stack(refs), K=K, gt_depth=gdepth,
             gt_poses=torch.stack(gpose, 1), loss=out["loss"],
             **{"metric_" + k: v for k, v in out["metrics"].items()}, **grad_checksums(net2, None))
        # per-element parameter gradients of the same step (it8: update blocks and
        # heads whole, the encoders at a fixed sample of entries), then the same
        # step with the left-right flip forced (SfmModelMF.py:110-119: images
        # flipped, K flipped IN PLACE -- the loss sees fx < 0, cx' = W - cx).
        # Global RNG state is restored so the fixtures after this one are unchanged.
        rng = torch.get_rng_state()
        full = ("update_block_depth", "update_block_pose", "depth_head", "pose_head",
                "upmask_net") if tag == "it8" else ()
        save(f"train_step_{tag}_grads", loss=out["loss"],
             **grad_fixture(((k, q.grad) for k, q in net2.named_parameters()), full))
        model_f = model_cls(**{**kw, "flip_lr_prob": 1.0})
        net3 = det_init(DepthPoseNet(version=version, min_depth=mind, max_depth=maxd))
        model_f.add_depth_net(net3)
        model_f.train()
        batch_f = dict(batch, intrinsics=K.clone())
        out_f = model_f(batch_f)
        out_f["loss"].sum().backward()
        save(f"train_step_{tag}_flip", K_after=batch_f["intrinsics"], loss=out_f["loss"],
             **{"metric_" + k: v for k, v in out_f["metrics"].items()},
             **grad_fixture(((k, q.grad) for k, q in net3.named_parameters()), full))
        torch.set_rng_state(rng)


def gen_scannet():
    """ScanNet-style cases (BASELINE configs[2] / configs[4]): the photometric loss
    at N=4 refs, n=4 predictions (the it12-h count) with automask + min, and a
    SelfSupModelMF it12-h-out training step with N=4 refs (view5, depth 0.2-10)
    at 64x96 -- loss, metrics and per-element gradients."""
    from dro_sfm.networks.depth_pose.DepthPoseNet import DepthPoseNet
    from dro_sfm.models.SelfSupModelMF import SelfSupModelMF
    from dro_sfm.geometry.pose import Pose
    from dro_sfm.losses.multiview_photometric_loss_mf import MultiViewPhotometricDecayLoss
    g = torch.Generator().manual_seed(44)

    def scannet_K(B, W, H):
        K = torch.tensor(SCANNET_K_320, dtype=torch.float32)
        K[0] *= W / 320.0
        K[1] *= H / 240.0
        K[2] = torch.tensor([0.0, 0.0, 1.0])
        return K.unsqueeze(0).repeat(B, 1, 1).contiguous()

    B, H, W, n, N = 2, 48, 64, 4, 4
    K = scannet_K(B, W, H)
    image = smooth_images(B, H, W, 61, detail=0.3)
    ctx = [smooth_images(B, H, W, 62 + j, detail=0.3) for j in range(N)]
    invs = [0.1 + 2.0 * torch.rand(B, 1, H, W, generator=g) for _ in range(n)]
    vecs = torch.stack([torch.stack([rand_pose(B, g, 0.05, 0.02) for _ in range(n)], 1) for _ in range(N)], 1)
    loss_fn = MultiViewPhotometricDecayLoss(ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001,
                                            C1=1e-4, C2=9e-4, photometric_reduce_op="min", disp_norm=True,
                                            clip_loss=0.0, progressive_scaling=0.0, padding_mode="zeros",
                                            automask_loss=True)
    invs_ = [i.clone().requires_grad_(True) for i in invs]
    vecs_ = vecs.clone().requires_grad_(True)
    poses = [[Pose.from_vec(vecs_[:, j, i], "euler") for i in range(n)] for j in range(N)]
    out = loss_fn(image, ctx, invs_, K, K, poses)
    out["loss"].sum().backward()
    save("photo_loss_n4", image=image, context=torch.stack(ctx), inv_depths=torch.stack(invs), poses=vecs,
         K=K, loss=out["loss"], photometric_loss=out["metrics"]["photometric_loss"],
         smoothness_loss=out["metrics"]["smoothness_loss"],
         g_inv_depths=torch.stack([i.grad for i in invs_]), g_poses=vecs_.grad,
         automask=np.int32(1), reduce_min=np.int32(1))

    # view5 self-supervised training step (it12-h-out, N=4)
    B, H, W, N = 1, 64, 96, 4
    mind, maxd = 0.2, 10.0
    K = scannet_K(B, W, H)
    img = smooth_images(B, H, W, 71, detail=0.3)
    refs = [smooth_images(B, H, W, 72 + j, detail=0.3) for j in range(N)]
    model = SelfSupModelMF(ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001, C1=1e-4,
                           C2=9e-4, photometric_reduce_op="min", disp_norm=True, clip_loss=0.0,
                           progressive_scaling=0.0, padding_mode="zeros", automask_loss=True,
                           num_scales=4, flip_lr_prob=0.0, rotation_mode="euler", upsample_depth_maps=True,
                           min_depth=mind, max_depth=maxd)
    net = det_init(DepthPoseNet(version="it12-h-out", min_depth=mind, max_depth=maxd))
    model.add_depth_net(net)
    model.train()
    batch = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs,
             "intrinsics": K.clone()}
    out = model(batch)
    out["loss"].sum().backward()
    save("train_step_it12h_selfsup_n4", image=img, refs=torch.stack(refs), K=K, loss=out["loss"],
         min_depth=np.float32(mind), max_depth=np.float32(maxd),
         **{"metric_" + k: v for k, v in out["metrics"].items()},
         **grad_fixture(((k, q.grad) for k, q in net.named_parameters()), ("depth_head", "pose_head")))


def gen_metrics():
    """compute_depth_metrics (utils/depth.py:259-343) on LiDAR-like sparse ground
    truth: garg crop with a lower-resolution prediction, and no crop with a
    same-resolution prediction; the last image of each batch has no valid pixel."""
    from types import SimpleNamespace
    from dro_sfm.utils.depth import compute_depth_metrics
    g = torch.Generator().manual_seed(77)
    for name, crop, (H, W), (h, w), lo, hi in (("metrics_garg", "garg", (96, 320), (48, 160), 1e-3, 80.0),
                                               ("metrics_nocrop", "", (64, 96), (64, 96), 0.2, 10.0)):
        B = 3
        gt = torch.zeros(B, 1, H, W)
        keep = torch.rand(B, 1, H, W, generator=g) < 0.3
        gt[keep] = (lo + 1.0 + (hi - lo - 1.0) * torch.rand(B, 1, H, W, generator=g))[keep]
        gt[-1] = 0.0                                                   # empty image
        base = torch.nn.functional.interpolate(torch.rand(B, 1, 6, 10, generator=g), size=(h, w),
                                               mode="bilinear", align_corners=False)
        pred = (0.5 + (hi / 2) * base) * (1.0 + 0.05 * torch.randn(B, 1, h, w, generator=g))
        cfg = SimpleNamespace(crop=crop, min_depth=lo, max_depth=hi)
        out_s = compute_depth_metrics(cfg, gt, pred, use_gt_scale=True)
        out_u = compute_depth_metrics(cfg, gt, pred, use_gt_scale=False)
        save(name, gt=gt, pred=pred, metrics_scaled=out_s, metrics_unscaled=out_u,
             min_depth=torch.tensor(lo), max_depth=torch.tensor(hi),
             crop=np.array({"": 0, "garg": 1, "eigen_nyu": 2}[crop], dtype=np.int32))


def gen_demon():
    """compute_depth_metrics_demon (utils/depth.py:343-398: ScanNet/DeMoN
    evaluation -- ground truth normalised by the first reference's gt
    translation norm, median scaling, no crop, no clamp to the depth range)
    and compute_pose_metrics (:400-421: rotation angle, translation angle,
    scale-fitted translation error of the first reference)."""
    from types import SimpleNamespace
    from dro_sfm.geometry.pose import Pose
    from dro_sfm.utils.depth import compute_depth_metrics_demon, compute_pose_metrics
    g = torch.Generator().manual_seed(78)
    B, N, H, W, h, w, lo, hi = 3, 2, 96, 128, 48, 64, 0.2, 10.0
    gt = torch.zeros(B, 1, H, W)
    keep = torch.rand(B, 1, H, W, generator=g) < 0.8
    gt[keep] = (lo + 0.05 + (hi - lo - 0.1) * torch.rand(B, 1, H, W, generator=g))[keep]
    gt[-1] = 0.0                                                       # empty image
    base = torch.nn.functional.interpolate(torch.rand(B, 1, 6, 8, generator=g), size=(h, w),
                                           mode="bilinear", align_corners=False)
    pred = (0.3 + 4.0 * base) * (1.0 + 0.05 * torch.randn(B, 1, h, w, generator=g))
    vec = torch.cat([0.3 * torch.randn(B * N, 3, generator=g), 0.05 * torch.randn(B * N, 3, generator=g)], 1)
    gt_pose = Pose.from_vec(vec, "euler").mat.view(B, N, 4, 4)
    cfg = SimpleNamespace(min_depth=lo, max_depth=hi)
    out_s = compute_depth_metrics_demon(cfg, gt, gt_pose, pred, use_gt_scale=True)
    out_u = compute_depth_metrics_demon(cfg, gt, gt_pose, pred, use_gt_scale=False)
    pose_gt, pose_pred, pose_out = [], [], []
    for k in range(6):
        v1 = torch.cat([0.2 * torch.randn(1, 3, generator=g), 0.05 * torch.randn(1, 3, generator=g)], 1)
        v2 = v1 + torch.cat([0.02 * torch.randn(1, 3, generator=g), 0.005 * torch.randn(1, 3, generator=g)], 1)
        T1 = Pose.from_vec(v1, "euler").mat
        P2 = Pose.from_vec(v2, "euler")
        pose_out.append(compute_pose_metrics(cfg, [T1], [P2]))
        pose_gt.append(T1[0])
        pose_pred.append(P2.mat[0])
    save("metrics_demon", gt=gt, pred=pred, gt_pose=gt_pose, metrics_scaled=out_s, metrics_unscaled=out_u,
         min_depth=torch.tensor(lo), max_depth=torch.tensor(hi))
    save("metrics_pose", gt=torch.stack(pose_gt), pred=torch.stack(pose_pred), metrics=torch.stack(pose_out))


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference not present: golden fixtures can only be regenerated in the build container")
    torch.set_num_threads(8)
    install_shims()
    which = sys.argv[1:] or ["cost", "geom", "parts", "full"]
    if "cost" in which:
        gen_cost()
    if "geom" in which:
        gen_geometry_loss()
    if "clip" in which:
        gen_clip()
    if "parts" in which:
        gen_network_parts()
    if "full" in which:
        gen_full()
    if "metrics" in which:
        gen_metrics()
    if "scannet" in which:
        gen_scannet()
    if "demon" in which:
        gen_demon()

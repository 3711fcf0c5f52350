"""Diagnose hipGraph capture vs eager on the training step (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dro_sfm_amd.models.SelfSupModelMF import SelfSupModelMF
from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet
from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, GraphedTrainStep


def setup(seed=0):
    torch.manual_seed(seed)
    m = SelfSupModelMF(flip_lr_prob=0.5, automask_loss=True, photometric_reduce_op="min", clip_loss=0.0,
                       smooth_loss_weight=0.001, min_depth=0.5, max_depth=80.0)
    m.add_depth_net(DepthPoseNet(version="it8-seq4-inter-out", min_depth=0.5, max_depth=80.0))
    return m.cuda()


def batch(H=192, W=640):
    g = torch.Generator(device="cuda").manual_seed(3)
    B = 2
    lo = torch.rand(B, 3, H // 8, W // 8, generator=g, device="cuda")
    img = torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear").clamp(0, 1)
    refs = [(0.97 * torch.roll(img, 2 + j, 3) + 0.03 * torch.rand(B, 3, H, W, generator=g, device="cuda")) for j in range(2)]
    K = torch.tensor([[371.8, 0.0, 314.1], [0.0, 369.4, 88.5], [0.0, 0.0, 1.0]], device="cuda").repeat(B, 1, 1)
    return {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs, "intrinsics": K}


b = batch()
K0 = b["intrinsics"].clone()
def trial(name, flips_cap, share, seq):
    m = setup()
    tr = DataParallelTrainer(m, capturable=True)
    b["intrinsics"].copy_(K0)
    gs = GraphedTrainStep(tr, b, warmup=3, flips=flips_cap, share_pool=share)
    res = []
    for i, f in enumerate(seq):
        b["intrinsics"].copy_(K0)
        l, _ = gs.step(b, flip=f)
        torch.cuda.synchronize()
        gfin = bool(torch.isfinite(tr.grads.flat).all())
        pfin = all(bool(torch.isfinite(p).all()) for p in m.parameters())
        res.append((round(float(l), 5), gfin, pfin))
        if not pfin:
            break
    print(name, res, flush=True)
    del gs, tr, m
    torch.cuda.synchronize()


trial("V1 only-T", (True,), True, [True] * 4)
trial("V0 only-F", (False,), True, [False] * 4)
trial("V2 F,T separate pools", (False, True), False, [False, True, True, False, True])
trial("V3 F,T shared pool", (False, True), True, [False, True, True, False, True])
trial("V4 T,F shared pool", (True, False), True, [False, True, True, False, True])

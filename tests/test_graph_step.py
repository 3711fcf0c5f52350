"""hipGraph-captured training step == eager training step (GPU)."""
import pytest
import torch

from oracle import dro_oracle as O

pytestmark = pytest.mark.gpu


def _setup(seed=0):
    from dro_sfm_amd.models.SelfSupModelMF import SelfSupModelMF
    from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet
    torch.manual_seed(seed)
    m = SelfSupModelMF(flip_lr_prob=0.5, automask_loss=True, photometric_reduce_op="min", clip_loss=0.0,
                       smooth_loss_weight=0.001, min_depth=0.5, max_depth=80.0)
    m.add_depth_net(DepthPoseNet(version="it8-seq4-inter-out", min_depth=0.5, max_depth=80.0))
    return m.cuda()


def _batch():
    g = torch.Generator(device="cuda").manual_seed(3)
    B, H, W = 2, 64, 96
    img = torch.rand(B, 3, H, W, generator=g, device="cuda")
    refs = [(0.9 * torch.roll(img, 2 + j, 3) + 0.1 * torch.rand(B, 3, H, W, generator=g, device="cuda"))
            for j in range(2)]
    K = torch.tensor([[93.0, 0.0, 47.5], [0.0, 92.0, 31.5], [0.0, 0.0, 1.0]], device="cuda").repeat(B, 1, 1)
    return {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs, "intrinsics": K}


def test_graph_replay_matches_eager():
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, GraphedTrainStep
    batch = _batch()
    K0 = batch["intrinsics"].clone()
    flips = [False, True, False, False, True]
    a = _setup()
    ta = DataParallelTrainer(a, capturable=True)
    losses_a = []
    for f in flips:
        batch["intrinsics"].copy_(K0)
        losses_a.append(ta.step(batch, flip=f)[0].clone())
    b = _setup()
    tb = DataParallelTrainer(b, capturable=True)
    batch["intrinsics"].copy_(K0)                       # the last eager step flipped K in place
    gs = GraphedTrainStep(tb, batch, warmup=3)          # eager warmup: flips F, T, F
    batch["intrinsics"].copy_(K0)
    l3 = gs.step(batch, flip=False)[0].clone()
    l4 = gs.step(batch, flip=True)[0].clone()
    torch.cuda.synchronize()
    assert O.rel_err(l3.cpu(), losses_a[3].cpu()) < 1e-4
    assert O.rel_err(l4.cpu(), losses_a[4].cpu()) < 1e-4
    for (ka, pa), (kb, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert O.rel_err(pb.detach().cpu(), pa.detach().cpu()) < 1e-4, ka

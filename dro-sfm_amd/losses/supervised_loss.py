"""SupervisedDepthPoseLoss on the GPU (drop-in for
dro_sfm/losses/supervised_loss.py:204-371, supervised_method 'sparse-l1').

The reference loops n_pred x N in Python and runs two reconstruct+project
chains per pair (~30 ATen launches each).  Here every (prediction, view) pair
-- and the N ground-truth poses -- is reprojected in ONE batched pass over a
[M, B, H*W] point set, and both loss terms reduce with a handful of launches.
"""
import torch

from ..geometry.pose import Pose, euler2mat
from ..utils.depth import inv2depth
from .loss_base import LossBase, ProgressiveScaling


def _kinv(K):
    Ki = K.clone()
    Ki[:, 0, 0] = 1.0 / K[:, 0, 0]
    Ki[:, 1, 1] = 1.0 / K[:, 1, 1]
    Ki[:, 0, 2] = -1.0 * K[:, 0, 2] / K[:, 0, 0]
    Ki[:, 1, 2] = -1.0 * K[:, 1, 2] / K[:, 1, 1]
    return Ki


def _rt(pose):
    if isinstance(pose, Pose):
        if pose.vec is not None and pose.mode == "euler":
            return euler2mat(pose.vec[:, 3:]), pose.vec[:, :3]
        pose = pose.mat
    return pose[:, :3, :3], pose[:, :3, 3]


def reproject(depth, K, ref_K, R, t):
    """Normalised reference coordinates of every target pixel for M poses at once.
    depth [B,1,H,W]; R [M,B,3,3]; t [M,B,3] -> [M,B,H,W,2]  (camera.py:111-194)."""
    B, _, H, W = depth.shape
    ys, xs = torch.meshgrid(torch.arange(H, device=depth.device, dtype=depth.dtype),
                            torch.arange(W, device=depth.device, dtype=depth.dtype), indexing="ij")
    pix = torch.stack([xs, ys, torch.ones_like(xs)], 0).view(1, 3, H * W)
    X = (_kinv(K) @ pix) * depth.view(B, 1, H * W)               # [B,3,HW]
    x = ref_K.unsqueeze(0) @ (R @ X.unsqueeze(0) + t.unsqueeze(-1))  # [M,B,3,HW]
    Z = x[:, :, 2].clamp(min=1e-5)
    u = 2 * (x[:, :, 0] / Z) / (W - 1) - 1.0
    v = 2 * (x[:, :, 1] / Z) / (H - 1) - 1.0
    return torch.stack([u, v], -1).view(R.shape[0], B, H, W, 2)


class SupervisedDepthPoseLoss(LossBase):
    def __init__(self, supervised_method="sparse-l1", supervised_num_scales=4, progressive_scaling=0.0,
                 min_depth=0.1, max_depth=100, **kwargs):
        super().__init__()
        if supervised_method != "sparse-l1":
            raise NotImplementedError(f"supervised_method {supervised_method!r}: only 'sparse-l1' "
                                      "(used by every reference yaml) is implemented")
        self.supervised_method = supervised_method
        self.n = supervised_num_scales
        self.progressive_scaling = ProgressiveScaling(progressive_scaling, self.n)
        self.min_depth, self.max_depth = min_depth, max_depth

    @property
    def logs(self):
        return {"supervised_num_scales": self.n}

    def _decay(self):
        w = torch.tensor([0.85 ** (self.n - i - 1) for i in range(self.n)])
        return w / w.sum()

    def calculate_loss(self, inv_depths, gt_inv_depths):
        """Masked inverse-depth L1 with normalised 0.85 decay (:244-277)."""
        lo, hi = 1.0 / self.max_depth, 1.0 / self.min_depth
        gt = gt_inv_depths[0]
        valid = ((gt > lo) & (gt < hi)).to(gt.dtype)
        err = (valid.unsqueeze(0) * (gt.unsqueeze(0) - torch.stack(list(inv_depths))).abs())
        per = err.flatten(1).mean(1)
        return (per * self._decay().to(per)).sum()

    def calc_pose_loss(self, pred_poses, gt_pose_context, gt_depth, K, ref_K):
        """Reprojection error under predicted vs ground-truth pose (:293-325)."""
        N, n = len(gt_pose_context), self.n
        Rg, tg = zip(*[_rt(p) for p in gt_pose_context])
        Rp, tp = zip(*[_rt(pred_poses[j][i]) for i in range(n) for j in range(N)])
        R = torch.stack(list(Rg) + list(Rp))
        t = torch.stack(list(tg) + list(tp))
        coords = reproject(gt_depth, K.float(), ref_K.float(), R.float(), t.float())
        inb = (coords >= -1) & (coords <= 1)
        cg, cp = coords[:N], coords[N:].view(n, N, *coords.shape[1:])
        dmask = ((gt_depth > self.min_depth) & (gt_depth < self.max_depth / 4.0)).permute(0, 2, 3, 1)
        valid = inb[:N].unsqueeze(0) & inb[N:].view_as(cp) & dmask
        diff = valid * (cp - cg.unsqueeze(0)).abs().clamp(-1, 1)
        per = diff.flatten(2).mean(2).mean(1)                         # [n]
        return (per * self._decay().to(per)).sum()

    def forward(self, image, context, inv_depths, gt_inv_depth, gt_pose_context, K, ref_K, poses,
                return_logs=False, progress=0.0):
        self.n = len(inv_depths)
        if any(d.shape[-2:] != gt_inv_depth.shape[-2:] for d in inv_depths):
            raise NotImplementedError("predictions must be at the ground-truth resolution")
        loss_depth = self.calculate_loss(inv_depths, [gt_inv_depth])
        loss_pose = self.calc_pose_loss(poses, gt_pose_context, inv2depth(gt_inv_depth), K, ref_K)
        self.add_metric("depth_loss", loss_depth)
        self.add_metric("pose_loss", loss_pose)
        self.add_metric("all_loss", loss_depth + loss_pose)
        loss = loss_depth + loss_pose
        return {"loss": loss.unsqueeze(0), "metrics": self.metrics}

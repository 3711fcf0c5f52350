"""SupervisedDepthPoseLoss on MI355X (drop-in for
dro_sfm/losses/supervised_loss.py:204-371, supervised_method 'sparse-l1').

The reference loops n_pred x N in Python and runs two reconstruct+project
chains per (prediction, view) pair (~60 ATen launches each).  Here the whole
loss -- the masked inverse-depth L1 of every prediction and the reprojection
error of every (prediction, view) pair under predicted vs ground-truth pose --
is one fused HIP op (hip.supervised_loss, csrc/supervised.hip): 2 launches
forward, 2 backward.  There is no CPU path: the op raises on CPU tensors.
"""
import torch

from ..geometry.pose import Pose, kernel_pose_tensor
from ..hip import stacked_view, supervised_loss
from .loss_base import LossBase, ProgressiveScaling


def _gt_matrix(p):
    return p.mat if isinstance(p, Pose) else p


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

    def forward(self, image, context, inv_depths, gt_inv_depth, gt_pose_context, K, ref_K, poses,
                return_logs=False, progress=0.0):
        self.n = len(inv_depths)
        if any(d.shape[-2:] != gt_inv_depth.shape[-2:] for d in inv_depths):
            raise NotImplementedError("predictions must be at the ground-truth resolution")
        n, N = self.n, len(gt_pose_context)
        invs = stacked_view(inv_depths)                                  # [n,B,1,H,W]
        pose_t = kernel_pose_tensor(poses, n)                                    # [N,n,B,6|3x4]
        gt_t = torch.stack([_gt_matrix(p).float() for p in gt_pose_context], 0)  # [N,B,4,4]
        loss, metrics = supervised_loss(gt_inv_depth.float(), invs, pose_t, gt_t, K.float(),
                                        ref_K.float(), min_depth=self.min_depth,
                                        max_depth=self.max_depth)
        self.add_metric("depth_loss", metrics[0])
        self.add_metric("pose_loss", metrics[1])
        self.add_metric("all_loss", loss.detach().reshape(()))
        return {"loss": loss, "metrics": self.metrics}

"""SfmModelMF (drop-in for dro_sfm/models/SfmModelMF.py:11-189)."""
import random

import torch
import torch.nn as nn

from .. import hip
from ..geometry.pose import Pose, PoseGrid


def flip_lr(image):
    return torch.flip(image, [3])


def flip_lr_intr(intr, width):
    """utils/image.py:61-81 -- mutates `intr` IN PLACE (fx -> -fx, cx -> W - cx),
    exactly as the reference does; the loss therefore sees the flipped K."""
    assert intr.shape[1:] == (3, 3)
    intr[:, 0, 0] = -1 * intr[:, 0, 0]
    intr[:, 0, 2] = width - intr[:, 0, 2]
    return intr


class SfmModelMF(nn.Module):
    def __init__(self, depth_net=None, pose_net=None, rotation_mode="euler", flip_lr_prob=0.0,
                 upsample_depth_maps=False, min_depth=0.1, max_depth=100, **kwargs):
        super().__init__()
        self.depth_net, self.pose_net = depth_net, pose_net
        self.rotation_mode = rotation_mode
        self.flip_lr_prob = flip_lr_prob
        self.upsample_depth_maps = upsample_depth_maps
        self.min_depth, self.max_depth = min_depth, max_depth
        self._logs, self._losses = {}, {}
        self._network_requirements = {"depth_net": True, "pose_net": False, "percep_net": False}
        self._train_requirements = {"gt_depth": False, "gt_pose": False}
        self._rng = random.Random()

    logs = property(lambda self: self._logs)
    losses = property(lambda self: self._losses)
    network_requirements = property(lambda self: self._network_requirements)
    train_requirements = property(lambda self: self._train_requirements)

    def add_loss(self, key, val):
        self._losses[key] = val.detach()

    def add_depth_net(self, depth_net):
        self.depth_net = depth_net

    def add_pose_net(self, pose_net):
        self.pose_net = pose_net

    def seed(self, seed):
        """Seed the flip draw (the reference draws from the global `random`)."""
        self._rng.seed(seed)

    def compute_inv_depths(self, image, ref_imgs, intrinsics, flip=None):
        """SfmModelMF.py:106-127.  `flip` overrides the random draw (graph capture)."""
        if flip is None:
            flip = self._rng.random() < self.flip_lr_prob if self.training else False
        if flip:
            intrinsics = flip_lr_intr(intrinsics, width=image.shape[3])
            inv_depths, poses = self.depth_net(flip_lr(image), [flip_lr(r) for r in ref_imgs],
                                               intrinsics)
        else:
            inv_depths, poses = self.depth_net(image, ref_imgs, intrinsics)
        inv_depths = inv_depths if isinstance(inv_depths, (list, tuple)) else [inv_depths]
        if flip:
            # the flip back: one launch over the stacked predictions
            inv_depths = list(torch.flip(hip.stacked_view(inv_depths), [-1]).unbind(0))
        # upsample_depth_maps: predictions are already full resolution (identity)
        return list(inv_depths), poses

    def forward(self, batch, return_logs=False, flip=None):
        inv_depths, pose_vec = self.compute_inv_depths(batch["rgb"], batch["rgb_context"],
                                                       batch["intrinsics"], flip=flip)
        if pose_vec.dim() == 3 and pose_vec.shape[2] == 6:      # eval: [B,N,6]
            poses = [Pose.from_vec(pose_vec[:, j], self.rotation_mode) for j in range(pose_vec.shape[1])]
        elif pose_vec.shape[-2:] == (4, 4):
            poses = [Pose(pose_vec[:, j]) for j in range(pose_vec.shape[1])]
        else:                                                   # train: [B,N,n_pred,6]
            poses = PoseGrid([[Pose.from_vec(pose_vec[:, j, i], self.rotation_mode)
                               for i in range(pose_vec.shape[2])] for j in range(pose_vec.shape[1])],
                             pose_vec, self.rotation_mode)
        return {"inv_depths": inv_depths, "poses": poses}


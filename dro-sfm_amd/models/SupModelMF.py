"""SupModelMF (drop-in for dro_sfm/models/SupModelMF.py:7-118)."""
from ..losses.supervised_loss import SupervisedDepthPoseLoss
from ..utils.depth import depth2inv
from .model_utils import merge_outputs
from .SfmModelMF import SfmModelMF


class SupModelMF(SfmModelMF):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._network_requirements = {"depth_net": True, "pose_net": False, "percep_net": False}
        self._train_requirements = {"gt_depth": True, "gt_pose": True}
        self._loss = SupervisedDepthPoseLoss(**kwargs)

    @property
    def logs(self):
        return {**super().logs, **self._loss.logs}

    def supervised_loss(self, image, ref_images, inv_depths, gt_depth, gt_poses, poses, intrinsics,
                        return_logs=False, progress=0.0):
        return self._loss(image, ref_images, inv_depths, depth2inv(gt_depth), gt_poses, intrinsics,
                          intrinsics, poses, return_logs=return_logs, progress=progress)

    def forward(self, batch, return_logs=False, progress=0.0, flip=None):
        output = super().forward(batch, return_logs=return_logs, flip=flip)
        if not self.training:
            return output
        if output["poses"] is None:
            return None
        sup = self.supervised_loss(batch["rgb_original"], batch["rgb_context_original"],
                                   output["inv_depths"], batch["depth"], batch["pose_context"],
                                   output["poses"], batch["intrinsics"], return_logs=return_logs,
                                   progress=progress)
        return {"loss": sup["loss"], **merge_outputs(output, sup)}

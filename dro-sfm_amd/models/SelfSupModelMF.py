"""SelfSupModelMF (drop-in for dro_sfm/models/SelfSupModelMF.py:7-99)."""
from ..losses.multiview_photometric_loss_mf import MultiViewPhotometricDecayLoss
from .model_utils import merge_outputs
from .SfmModelMF import SfmModelMF


class SelfSupModelMF(SfmModelMF):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._photometric_loss = MultiViewPhotometricDecayLoss(**kwargs)

    @property
    def logs(self):
        return {**super().logs, **self._photometric_loss.logs}

    def self_supervised_loss(self, image, ref_images, inv_depths, poses, intrinsics, return_logs=False,
                             progress=0.0):
        return self._photometric_loss(image, ref_images, inv_depths, intrinsics, intrinsics, poses,
                                      return_logs=return_logs, progress=progress)

    def forward(self, batch, return_logs=False, progress=0.0, flip=None):
        output = super().forward(batch, return_logs=return_logs, flip=flip)
        if not self.training:
            return output
        if output["poses"] is None:
            return None
        sup = self.self_supervised_loss(batch["rgb_original"], batch["rgb_context_original"],
                                        output["inv_depths"], output["poses"], batch["intrinsics"],
                                        return_logs=return_logs, progress=progress)
        return {"loss": sup["loss"], **merge_outputs(output, sup)}

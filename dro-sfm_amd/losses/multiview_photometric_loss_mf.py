"""MultiViewPhotometricDecayLoss on MI355X (drop-in for
dro_sfm/losses/multiview_photometric_loss_mf.py:58-361).

The whole loss -- view synthesis of every (prediction, ref) pair, SSIM + L1,
automask, min/mean reduction with the 0.85^(n-i-1) decay and the edge-aware
smoothness term -- is one fused HIP op (hip.photometric_loss): 3 launches
forward, 2 backward, in place of ~50 ATen launches per (prediction, ref) pair.

Supported: any clip_loss >= 0 (every reference yaml sets 0; the constructor's
default 0.5 clamps each candidate map at mean + 0.5 std of itself, :223-227 --
two forward passes around per-map thresholds in the kernel), padding_mode
'zeros' (every yaml), and inverse-depth predictions at the image resolution
(what DepthPoseNet emits).  Anything else raises NotImplementedError rather
than running a slow path.
"""
import torch

from ..hip import photometric_loss, stacked_view
from ..hip.timeline import stamp_grad
from ..geometry.pose import kernel_pose_tensor
from .loss_base import LossBase, ProgressiveScaling


class MultiViewPhotometricDecayLoss(LossBase):
    def __init__(self, num_scales=4, ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.1,
                 C1=1e-4, C2=9e-4, photometric_reduce_op="mean", disp_norm=True, clip_loss=0.5,
                 progressive_scaling=0.0, padding_mode="zeros", automask_loss=False, **kwargs):
        super().__init__()
        self.n = 1
        self.ssim_loss_weight = ssim_loss_weight
        self.occ_reg_weight = occ_reg_weight
        self.smooth_loss_weight = smooth_loss_weight
        self.C1, self.C2 = C1, C2
        self.photometric_reduce_op = photometric_reduce_op
        self.disp_norm = disp_norm
        self.clip_loss = clip_loss
        self.padding_mode = padding_mode
        self.automask_loss = automask_loss
        self.progressive_scaling = ProgressiveScaling(progressive_scaling, self.n)
        self.keep_selection = False       # tests: keep the per-pixel min-candidate map
        self.last_selection = None
        if self.automask_loss:
            assert self.photometric_reduce_op == "min", \
                "For automasking only the min photometric_reduce_op is supported."

    @property
    def logs(self):
        return {"num_scales": self.n}

    def _check_supported(self, image, inv_depths):
        if self.padding_mode != "zeros":
            raise NotImplementedError("only padding_mode='zeros' is implemented")
        if self.ssim_loss_weight <= 0.0:
            raise NotImplementedError("ssim_loss_weight must be > 0 for the fused kernel")
        if self.photometric_reduce_op not in ("min", "mean"):
            raise NotImplementedError(f"Unknown photometric_reduce_op: {self.photometric_reduce_op}")
        if any(d.shape[-2:] != image.shape[-2:] for d in inv_depths):
            raise NotImplementedError("inverse depths must be at the image resolution")

    def forward(self, image, context, inv_depths, K, ref_K, poses, return_logs=False, progress=0.0):
        self.n = len(inv_depths)
        self._check_supported(image, inv_depths)
        n, N = self.n, len(context)
        ctx = torch.stack(list(context), 0)                                   # [N,B,3,H,W]
        invs = stamp_grad(stacked_view(inv_depths), "bwd:loss_done")                               # [n,B,1,H,W]
        pose_t = kernel_pose_tensor(poses, n)                                 # [N,n,B,6|3x4]
        loss, metrics, sel = photometric_loss(
            image, ctx, invs, pose_t, K.float(), ref_K.float(), ssim_w=self.ssim_loss_weight,
            C1=self.C1, C2=self.C2, smooth_w=self.smooth_loss_weight, automask=self.automask_loss,
            reduce_min=self.photometric_reduce_op == "min", clip_loss=max(float(self.clip_loss), 0.0),
            return_selection=True)
        self.last_selection = sel.clone() if self.keep_selection else None
        # The reference stores a detached alias of the photometric loss and then adds
        # the smoothness in place (:268, :356), so its 'photometric_loss' metric
        # reports the total; mirror that.
        photo_metric = loss.detach().reshape(()) if self.smooth_loss_weight > 0 else metrics[0]
        self.add_metric("photometric_loss", photo_metric)
        if self.smooth_loss_weight > 0.0:
            self.add_metric("smoothness_loss", metrics[1])
        return {"loss": loss, "metrics": self.metrics}

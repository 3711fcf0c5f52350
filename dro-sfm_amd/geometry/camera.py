"""Camera: pinhole lift/project (API of dro_sfm/geometry/camera.py:12-194).

The training hot path never calls these torch implementations -- the fused
HIP kernels inline the same algebra -- they serve callers that want explicit
3-D points or pixel coordinates (evaluation, visualisation).  Unlike the
reference, Kinv/Twc are not lru_cached on the instance (the reference cache
pins up to 128 autograd graphs).
"""
import torch

from .pose import Pose


def scale_intrinsics(K, x_scale, y_scale):
    """geometry/camera_utils.py:13-19 (in place, like the reference)."""
    K[..., 0, 0] *= x_scale
    K[..., 1, 1] *= y_scale
    K[..., 0, 2] = (K[..., 0, 2] + 0.5) * x_scale - 0.5
    K[..., 1, 2] = (K[..., 1, 2] + 0.5) * y_scale - 0.5
    return K


class Camera(torch.nn.Module):
    def __init__(self, K, Tcw=None):
        super().__init__()
        self.K = K
        self.Tcw = Pose.identity(len(K), K.device, K.dtype) if Tcw is None else Tcw

    def __len__(self):
        return len(self.K)

    def to(self, *args, **kwargs):
        self.K = self.K.to(*args, **kwargs)
        self.Tcw = self.Tcw.to(*args, **kwargs)
        return self

    fx = property(lambda self: self.K[:, 0, 0])
    fy = property(lambda self: self.K[:, 1, 1])
    cx = property(lambda self: self.K[:, 0, 2])
    cy = property(lambda self: self.K[:, 1, 2])

    @property
    def Twc(self):
        return self.Tcw.inverse()

    @property
    def Kinv(self):
        Ki = self.K.clone()
        Ki[:, 0, 0] = 1.0 / self.fx
        Ki[:, 1, 1] = 1.0 / self.fy
        Ki[:, 0, 2] = -1.0 * self.cx / self.fx
        Ki[:, 1, 2] = -1.0 * self.cy / self.fy
        return Ki

    def scaled(self, x_scale, y_scale=None):
        y_scale = x_scale if y_scale is None else y_scale
        if x_scale == 1.0 and y_scale == 1.0:
            return self
        return Camera(scale_intrinsics(self.K.clone(), x_scale, y_scale), Tcw=self.Tcw)

    def reconstruct(self, depth, frame="w"):
        B, C, H, W = depth.shape
        assert C == 1
        ys, xs = torch.meshgrid(torch.arange(H, device=depth.device, dtype=depth.dtype),
                                torch.arange(W, device=depth.device, dtype=depth.dtype), indexing="ij")
        grid = torch.stack([xs, ys, torch.ones_like(xs)], 0).view(1, 3, -1).expand(B, 3, H * W)
        Xc = (self.Kinv.bmm(grid)).view(B, 3, H, W) * depth
        if frame == "c":
            return Xc
        if frame == "w":
            return self.Twc @ Xc
        raise ValueError(f"Unknown reference frame {frame}")

    def project(self, X, frame="w", normalize=True):
        B, C, H, W = X.shape
        assert C == 3
        if frame == "c":
            Xc = self.K.bmm(X.view(B, 3, -1))
        elif frame == "w":
            Xc = self.K.bmm((self.Tcw @ X).view(B, 3, -1))
        else:
            raise ValueError(f"Unknown reference frame {frame}")
        Z = Xc[:, 2].clamp(min=1e-5)
        if normalize:
            u, v = 2 * (Xc[:, 0] / Z) / (W - 1) - 1.0, 2 * (Xc[:, 1] / Z) / (H - 1) - 1.0
        else:
            u, v = Xc[:, 0] / Z, Xc[:, 1] / Z
        return torch.stack([u, v], dim=-1).view(B, H, W, 2)

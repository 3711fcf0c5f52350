"""Pose: a batch of rigid transforms (API of dro_sfm/geometry/pose.py:7-98).

A pose built by ``from_vec(vec, 'euler')`` keeps its 6-vector: the fused HIP
kernels consume the vector directly (rotation built in registers) and return
gradients w.r.t. it, so the [B,4,4] matrix is only materialised when a caller
asks for ``.mat``.
"""
import torch


def euler2mat(angle):
    """R = Rx @ Ry @ Rz (geometry/pose_utils.py:40-69), [B,3] -> [B,3,3]."""
    x, y, z = angle.unbind(1)
    cx, sx, cy, sy, cz, sz = x.cos(), x.sin(), y.cos(), y.sin(), z.cos(), z.sin()
    # closed form of Rx @ Ry @ Rz
    r = torch.stack([cy * cz, -cy * sz, sy,
                     sx * sy * cz + cx * sz, -sx * sy * sz + cx * cz, -sx * cy,
                     -cx * sy * cz + sx * sz, cx * sy * sz + sx * cz, cx * cy], 1)
    return r.view(-1, 3, 3)


def axis_angle_to_matrix(aa):
    """Rodrigues' formula (geometry/pose_trans.py:427) for rotation_mode='axis_angle'."""
    theta = aa.norm(dim=1, keepdim=True).clamp(min=1e-12)
    k = aa / theta
    K = torch.zeros(aa.shape[0], 3, 3, dtype=aa.dtype, device=aa.device)
    K[:, 0, 1], K[:, 0, 2], K[:, 1, 2] = -k[:, 2], k[:, 1], -k[:, 0]
    K = K - K.transpose(1, 2)
    s, c = theta.sin().unsqueeze(-1), theta.cos().unsqueeze(-1)
    eye = torch.eye(3, dtype=aa.dtype, device=aa.device).expand_as(K)
    return eye + s * K + (1 - c) * (K @ K)


def pose_vec2mat(vec, mode="euler"):
    """[B,6] -> [B,3,4] (geometry/pose_utils.py:73-85)."""
    if mode is None:
        return vec
    rot = euler2mat(vec[:, 3:]) if mode == "euler" else (
        axis_angle_to_matrix(vec[:, 3:]) if mode == "axis_angle" else None)
    if rot is None:
        raise ValueError(f"Rotation mode not supported {mode}")
    return torch.cat([rot, vec[:, :3].unsqueeze(-1)], 2)


def invert_pose(T):
    """[B,4,4] rigid inverse (geometry/pose_utils.py:89-94)."""
    R, t = T[:, :3, :3], T[:, :3, 3:]
    Rt = R.transpose(1, 2)
    top = torch.cat([Rt, -Rt @ t], 2)
    bottom = T.new_tensor([0, 0, 0, 1]).expand(T.shape[0], 1, 4)
    return torch.cat([top, bottom], 1)


class Pose:
    def __init__(self, mat=None, vec=None, mode="euler"):
        if mat is not None:
            assert tuple(mat.shape[-2:]) == (4, 4)
            if mat.dim() == 2:
                mat = mat.unsqueeze(0)
            assert mat.dim() == 3
        self._mat, self.vec, self.mode = mat, vec, mode

    @property
    def mat(self):
        if self._mat is None:
            m = pose_vec2mat(self.vec, self.mode)
            bottom = m.new_tensor([0, 0, 0, 1]).expand(m.shape[0], 1, 4)
            self._mat = torch.cat([m, bottom], 1)
        return self._mat

    @mat.setter
    def mat(self, value):
        self._mat, self.vec = value, None

    def __len__(self):
        return len(self.vec) if self._mat is None else len(self._mat)

    @classmethod
    def identity(cls, N=1, device=None, dtype=torch.float):
        return cls(torch.eye(4, device=device, dtype=dtype).repeat([N, 1, 1]))

    @classmethod
    def from_vec(cls, vec, mode):
        """Pose.from_vec (geometry/pose.py:38-45); the vector is kept for the kernels."""
        return cls(vec=vec, mode=mode)

    @property
    def shape(self):
        return self.mat.shape

    def item(self):
        return self.mat

    def repeat(self, *args, **kwargs):
        self.mat = self.mat.repeat(*args, **kwargs)
        return self

    def inverse(self):
        return Pose(invert_pose(self.mat))

    def to(self, *args, **kwargs):
        if self._mat is not None:
            self._mat = self._mat.to(*args, **kwargs)
        if self.vec is not None:
            self.vec = self.vec.to(*args, **kwargs)
        return self

    def clone(self):
        return Pose(None if self._mat is None else self._mat.clone(),
                    None if self.vec is None else self.vec.clone(), self.mode)

    def kernel_pose(self):
        """What the HIP kernels take: the euler vector [B,6] when available,
        else the top three rows of the transform [B,3,4]."""
        if self.vec is not None and self.mode == "euler":
            return self.vec
        return self.mat[:, :3, :]

    def transform_pose(self, pose):
        return Pose(self.mat.bmm(pose.item()))

    def transform_points(self, points):
        B, _, H, W = points.shape
        out = self.mat[:, :3, :3].bmm(points.reshape(B, 3, -1)) + self.mat[:, :3, 3:]
        return out.view(B, 3, H, W)

    def __matmul__(self, other):
        if isinstance(other, Pose):
            return self.transform_pose(other)
        if isinstance(other, torch.Tensor) and other.dim() in (3, 4) and other.shape[1] == 3:
            return self.transform_points(other)
        raise ValueError(f"Unknown operand for Pose @: {type(other)}")


class PoseGrid(list):
    """The reference's N x n_pred list of Pose objects (SfmModelMF.py:174-181),
    remembering the [B,N,n_pred,6] tensor they were sliced from: the fused
    losses read it as one [N,n_pred,B,6] tensor (one permuted copy forward and
    backward) instead of re-stacking N*n_pred slices (whose backward is a
    zero-fill + copy + add per slice)."""

    def __init__(self, rows, vec, mode):
        super().__init__(rows)
        self.vec, self.mode = vec, mode

    def kernel_poses(self):
        """[N, n_pred, B, 6] euler vectors, or None when the grid no longer mirrors
        the source tensor (entries replaced, or a non-euler mode)."""
        if self.mode != "euler" or self.vec is None:
            return None
        N, n = self.vec.shape[1], self.vec.shape[2]
        if len(self) != N or any(len(row) != n for row in self):
            return None
        return self.vec.permute(1, 2, 0, 3).contiguous()


def kernel_pose_tensor(poses, n):
    """[N, n, B, 6|3x4] kernel poses of an N x n list of Pose objects."""
    fast = poses.kernel_poses() if isinstance(poses, PoseGrid) else None
    if fast is not None and fast.shape[1] == n:
        # every entry must still be the untouched slice [:, j, i] of the source tensor
        src = poses.vec
        ok = all(isinstance(poses[j][i], Pose) and poses[j][i]._mat is None and poses[j][i].vec is not None
                 and poses[j][i].vec.data_ptr() == src[:, j, i].data_ptr()
                 and poses[j][i].vec.stride() == src[:, j, i].stride()
                 for j in range(len(poses)) for i in range(n))
        if ok:
            return fast
    return torch.stack([torch.stack([poses[j][i].kernel_pose() for i in range(n)], 0)
                        for j in range(len(poses))], 0)

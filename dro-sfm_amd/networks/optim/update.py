"""Recurrent update blocks of the DRO optimizer.

Parameter names and shapes follow dro_sfm/networks/optim/update.py so that
reference checkpoints load unchanged; layers are declared from small spec
tables.  Differences are execution-only:
  * convolutions that read the same input are issued as ONE convolution over
    concatenated weights (SepConvGRU z|r gates, DepthHead.conv1 | mask.0),
    halving the launches of the recurrent loop;
  * the pose block runs once over all reference views stacked along the batch
    axis (the reference loops over refs in Python, DepthPoseNet.py:186); every
    op in it is per-sample, so the result is identical.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def declare(module, table):
    """Register nn.Conv2d layers from {name: (cin, cout, kernel, padding)}."""
    for name, (cin, cout, k, pad) in table.items():
        setattr(module, name, nn.Conv2d(cin, cout, k, padding=pad))


def conv_cat(x, convs, padding):
    """One convolution computing several nn.Conv2d that share the input x."""
    w = torch.cat([c.weight for c in convs], 0)
    b = torch.cat([c.bias for c in convs], 0)
    return torch.split(F.conv2d(x, w, b, padding=padding), [c.out_channels for c in convs], 1)


def mask_seq(hidden_dim, ratio):
    """3x3 -> ReLU -> 1x1 to 9*r*r convex-combination logits (update.py:150-153)."""
    return nn.Sequential(nn.Conv2d(hidden_dim, 2 * hidden_dim, 3, padding=1), nn.ReLU(inplace=True),
                         nn.Conv2d(2 * hidden_dim, 9 * ratio * ratio, 1, padding=0))


class DepthHead(nn.Module):
    """update.py:5-14: two 3x3 convolutions, activation on the output."""

    def __init__(self, input_dim=256, hidden_dim=128, scale=False):
        super().__init__()
        self.scale = scale
        declare(self, {"conv1": (input_dim, hidden_dim, 3, 1), "conv2": (hidden_dim, 1, 3, 1)})

    def forward(self, x_d, act_fn=torch.tanh):
        return act_fn(self.conv2(F.relu(self.conv1(x_d))))


class PoseHead(nn.Module):
    """update.py:16-28: spatial mean of a 6-channel map; rotation scaled by 0.01."""

    def __init__(self, input_dim=256, hidden_dim=128):
        super().__init__()
        declare(self, {"conv1_pose": (input_dim, hidden_dim, 3, 1),
                       "conv2_pose": (hidden_dim, 6, 3, 1)})

    def forward(self, x_p):
        vec = self.conv2_pose(F.relu(self.conv1_pose(x_p))).mean(3).mean(2)
        return torch.cat([vec[:, :3], 0.01 * vec[:, 3:]], dim=1)


class SepConvGRU(nn.Module):
    """update.py:47-74: a horizontal (1x5) then a vertical (5x1) gated update."""

    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        cin = hidden_dim + input_dim
        self.hidden_dim = hidden_dim
        for axis, k, pad in (("1", (1, 5), (0, 2)), ("2", (5, 1), (2, 0))):
            declare(self, {g + axis: (cin, hidden_dim, k, pad) for g in ("convz", "convr", "convq")})

    def _gate(self, h, x, axis, pad):
        cz, cr, cq = (getattr(self, g + axis) for g in ("convz", "convr", "convq"))
        zr = conv_cat(torch.cat([h, x], 1), (cz, cr), pad)
        z, r = torch.sigmoid(zr[0]), torch.sigmoid(zr[1])
        q = torch.tanh(cq(torch.cat([r * h, x], 1)))
        return (1 - z) * h + z * q

    def forward(self, h, x):
        return self._gate(self._gate(h, x, "1", (0, 2)), x, "2", (2, 0))


class _Projection(nn.Module):
    """Shared body of ProjectionInputDepth/Pose (update.py:77-124): a cost branch
    (1x1 -> 3x3), a state branch (7x7 -> 3x3), a fused 3x3, and the raw state
    appended as the last channels."""

    def __init__(self, tag, state_ch, cost_dim, hidden_dim, out_chs):
        super().__init__()
        self.out_chs, self._tag = out_chs, tag
        declare(self, {"convc1": (cost_dim, hidden_dim, 1, 0),
                       "convc2": (hidden_dim, hidden_dim, 3, 1),
                       f"conv{tag}1": (state_ch, hidden_dim, 7, 3),
                       f"conv{tag}2": (hidden_dim, 64, 3, 1),
                       f"conv{tag}": (64 + hidden_dim, out_chs - state_ch, 3, 1)})

    def _mix(self, state_map, cost):
        t = self._tag
        cor = F.relu(self.convc2(F.relu(self.convc1(cost))))
        sfm = F.relu(getattr(self, f"conv{t}2")(F.relu(getattr(self, f"conv{t}1")(state_map))))
        fused = F.relu(getattr(self, f"conv{t}")(torch.cat([cor, sfm], 1)))
        return torch.cat([fused, state_map], 1)


class ProjectionInputDepth(_Projection):
    def __init__(self, cost_dim, hidden_dim, out_chs):
        super().__init__("d", 1, cost_dim, hidden_dim, out_chs)

    def forward(self, depth, cost):
        return self._mix(depth, cost)


class ProjectionInputPose(_Projection):
    def __init__(self, cost_dim, hidden_dim, out_chs):
        super().__init__("p", 6, cost_dim, hidden_dim, out_chs)

    def forward(self, pose, cost):
        bs, _, h, w = cost.shape
        return self._mix(pose.reshape(bs, 6, 1, 1).expand(bs, 6, h, w), cost)


class UpMaskNet(nn.Module):
    """update.py:128-139: 0.25-scaled convex-upsampling logits."""

    def __init__(self, hidden_dim=128, ratio=8):
        super().__init__()
        self.mask = mask_seq(hidden_dim, ratio)

    def forward(self, feat):
        return 0.25 * self.mask(feat)


class BasicUpdateBlockDepth(nn.Module):
    """update.py:143-173: S steps of cost -> encoder -> GRU -> delta inv-depth."""

    def __init__(self, hidden_dim=128, cost_dim=256, ratio=8, context_dim=64):
        super().__init__()
        self.encoder = ProjectionInputDepth(cost_dim=cost_dim, hidden_dim=hidden_dim, out_chs=hidden_dim)
        self.depth_gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=hidden_dim + context_dim)
        self.depth_head = DepthHead(hidden_dim, hidden_dim=hidden_dim, scale=False)
        self.mask = mask_seq(hidden_dim, ratio)

    def heads(self, net):
        """DepthHead.conv1 and mask.0 read the same state: one launch."""
        a, b = conv_cat(net, (self.depth_head.conv1, self.mask[0]), 1)
        return torch.tanh(self.depth_head.conv2(F.relu(a))), 0.25 * self.mask[2](F.relu(b))

    def forward(self, net, cost_func, inv_depth, context, seq_len=4, scale_func=None):
        scale_func = scale_func or (lambda x: (x, None))
        invs, masks = [], []
        for _ in range(seq_len):
            feat = self.encoder(inv_depth, cost_func(scale_func(inv_depth)[0]))
            net = self.depth_gru(net, torch.cat([context, feat], 1))
            delta, mask = self.heads(net)
            inv_depth = inv_depth + delta
            invs.append(inv_depth)
            masks.append(mask)
        return net, masks, invs


class BasicUpdateBlockPose(nn.Module):
    """update.py:176-199: S steps of cost -> encoder -> GRU -> delta pose."""

    def __init__(self, hidden_dim=128, cost_dim=256, context_dim=64):
        super().__init__()
        self.encoder = ProjectionInputPose(cost_dim=cost_dim, hidden_dim=hidden_dim, out_chs=hidden_dim)
        self.pose_gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=hidden_dim + context_dim)
        self.pose_head = PoseHead(hidden_dim, hidden_dim=hidden_dim)

    def forward(self, net, cost_func, pose, inp, seq_len=4):
        seq = []
        for _ in range(seq_len):
            net = self.pose_gru(net, torch.cat([inp, self.encoder(pose, cost_func(pose))], 1))
            pose = pose + self.pose_head(net)
            seq.append(pose)
        return net, seq

"""Recurrent update blocks of the DRO optimizer.

Parameter names and shapes follow dro_sfm/networks/optim/update.py so that
reference checkpoints load unchanged; layers are declared from small spec
tables.  Differences are execution-only:
  * every convolution runs on the f32-MFMA conv engine (csrc/conv.hip): bias,
    activation and the 0.25 mask scale in its epilogue, inputs read as a
    VIRTUAL channel concatenation (no torch.cat of [h, context, projection,
    depth | pose map]), the pose map broadcast instead of expanded;
  * SepConvGRU is one fused op per direction (z|r gates in one launch, the q
    gate with r*h staged on the fly and the (1-z)h + zq blend in its epilogue);
  * convolutions that read the same input are ONE convolution over
    concatenated weights (z|r, DepthHead.conv1 | mask.0);
  * the pose block runs once over all reference views stacked along the batch
    axis (the reference loops over refs in Python, DepthPoseNet.py:186); every
    op in it is per-sample, so the result is identical.
set_conv_backend("miopen") switches the convolutions to MIOpen for A/B
measurements only; the default is the native engine.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import hip
from ...hip import conv as hip_conv

_BACKEND = "hip"
_ACT_FN = {None: lambda x: x, "relu": F.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}


def set_conv_backend(name):
    """'hip' (default: csrc/conv.hip) or 'miopen' (torch F.conv2d), for A/B runs."""
    global _BACKEND
    if name not in ("hip", "miopen"):
        raise ValueError(name)
    _BACKEND = name


def conv_backend():
    return _BACKEND


def declare(module, table):
    """Register nn.Conv2d layers from {name: (cin, cout, kernel, padding)}."""
    for name, (cin, cout, k, pad) in table.items():
        setattr(module, name, nn.Conv2d(cin, cout, k, padding=pad))


def _as_list(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]


def conv(srcs, weight, bias, act=None, alpha=1.0):
    """act(conv2d(cat(srcs), weight, bias, 'same')) * alpha."""
    srcs = _as_list(srcs)
    if _BACKEND == "hip":
        return hip.conv2d(srcs, weight, bias, act=act, alpha=alpha)
    kh, kw = weight.shape[2:]
    x = srcs[0] if len(srcs) == 1 else torch.cat(srcs, 1)
    y = _ACT_FN[act](F.conv2d(x, weight, bias, padding=(kh // 2, kw // 2)))
    return y * alpha if alpha != 1.0 else y


def conv_cat(x, convs, act=None):
    """One convolution computing several nn.Conv2d that share the input x.  The
    fused weight is a view of the trainer's flat parameter buffer when the
    group is laid out adjacently (fused_groups), else a concatenation built
    once per forward (hip.weight_grad_scope)."""
    if _BACKEND == "hip":
        y = hip.conv2d(_as_list(x), None, None, act=act,
                       parts=(tuple(c.weight for c in convs), tuple(c.bias for c in convs)))
    else:
        y = conv(x, torch.cat([c.weight for c in convs], 0), torch.cat([c.bias for c in convs], 0), act)
    return torch.split(y, [c.out_channels for c in convs], 1)


relu_rec = hip.ops.record_relu     # parity tests: the ReLU branch of a conv site


def fused_groups(*convs):
    """Parameter groups read as one fused tensor: [weights], [biases]."""
    return [[c.weight for c in convs], [c.bias for c in convs]]


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
        act = {torch.tanh: "tanh", torch.sigmoid: "sigmoid"}.get(act_fn)
        y = conv(relu_rec(conv(x_d, self.conv1.weight, self.conv1.bias, "relu"), self.conv1),
                 self.conv2.weight, self.conv2.bias, act)
        return y if act is not None else act_fn(y)


class PoseHead(nn.Module):
    """update.py:16-28: spatial mean of a 6-channel map; rotation scaled by 0.01.
    hip.pose_mean: the mean, the scale and (forward(x, pose)) the update
    `pose + pose_head(x)` of BasicUpdateBlockPose in one launch each way (the
    reference's mean(3).mean(2) + slice/cat + add costs 2 reductions, a cat and
    an add forward, zero-fills, copies and adds backward per call; equal to
    fp32 rounding)."""

    def __init__(self, input_dim=256, hidden_dim=128):
        super().__init__()
        declare(self, {"conv1_pose": (input_dim, hidden_dim, 3, 1),
                       "conv2_pose": (hidden_dim, 6, 3, 1)})
        self.register_buffer("_scale", torch.tensor([[1.0, 1.0, 1.0, 0.01, 0.01, 0.01]]),
                             persistent=False)

    def forward(self, x_p, pose=None):
        """The pose delta, or pose + delta when `pose` [B, 6] is given."""
        y = conv(relu_rec(conv(x_p, self.conv1_pose.weight, self.conv1_pose.bias, "relu"), self.conv1_pose),
                 self.conv2_pose.weight, self.conv2_pose.bias)
        return hip.pose_mean(y, 0.01, pose)


class SepConvGRU(nn.Module):
    """update.py:47-74: a horizontal (1x5) then a vertical (5x1) gated update."""

    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        cin = hidden_dim + input_dim
        self.hidden_dim = hidden_dim
        for axis, k, pad in (("1", (1, 5), (0, 2)), ("2", (5, 1), (2, 0))):
            declare(self, {g + axis: (cin, hidden_dim, k, pad) for g in ("convz", "convr", "convq")})

    def _gate(self, h, xs, axis, chain=None):
        cz, cr, cq = (getattr(self, g + axis) for g in ("convz", "convr", "convq"))
        if _BACKEND == "hip":
            return hip.sepconvgru_half(h, cz, cr, cq, xs, chain=chain)
        z, r = conv_cat([h, *xs], (cz, cr), "sigmoid")
        q = conv([r * h, *xs], cq.weight, cq.bias, "tanh")
        return (1 - z) * h + z * q

    def dro_param_groups(self):
        """z|r gates of each direction are one fused conv (trainer layout hint)."""
        return fused_groups(self.convz1, self.convr1) + fused_groups(self.convz2, self.convr2)

    def forward(self, h, x):
        """x: the input tensor, or a list of tensors read as their channel concat."""
        xs = _as_list(x)
        # the two halves' backward kernels are linked (hip.conv.GruChain): the
        # middle state is read by the second half only
        chain = hip_conv.GruChain() if _BACKEND == "hip" else None
        return self._gate(self._gate(h, xs, "1", chain), xs, "2", chain)


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

    def sources(self, state_map, cost):
        """The projection output as [fused features, state map] (concat implied)."""
        t = self._tag
        c1, c2 = self.convc1, self.convc2
        s1, s2, f = (getattr(self, f"conv{t}{i}") for i in ("1", "2", ""))
        cor = relu_rec(conv(relu_rec(conv(cost, c1.weight, c1.bias, "relu"), c1), c2.weight, c2.bias, "relu"), c2)
        sfm = relu_rec(conv(relu_rec(conv(state_map, s1.weight, s1.bias, "relu"), s1), s2.weight, s2.bias, "relu"),
                       s2)
        # both GRU halves read the fused features: their gradients meet in a sink
        return [hip.grad_sink(relu_rec(conv([cor, sfm], f.weight, f.bias, "relu"), f)), state_map]


class ProjectionInputDepth(_Projection):
    def __init__(self, cost_dim, hidden_dim, out_chs):
        super().__init__("d", 1, cost_dim, hidden_dim, out_chs)

    def forward(self, depth, cost):
        return torch.cat(self.sources(depth, cost), 1)


class ProjectionInputPose(_Projection):
    def __init__(self, cost_dim, hidden_dim, out_chs):
        super().__init__("p", 6, cost_dim, hidden_dim, out_chs)

    def pose_map(self, pose, cost):
        bs, _, h, w = cost.shape
        return pose.reshape(bs, 6, 1, 1).expand(bs, 6, h, w)

    def sources(self, pose, cost):
        # the broadcast pose map feeds the 7x7 conv and both GRU halves: one dense
        # gradient buffer, reduced once by the expand's backward
        return super().sources(hip.grad_sink(self.pose_map(pose, cost)), cost)

    def forward(self, pose, cost):
        return torch.cat(self.sources(pose, cost), 1)


class UpMaskNet(nn.Module):
    """update.py:128-139: 0.25-scaled convex-upsampling logits."""

    def __init__(self, hidden_dim=128, ratio=8):
        super().__init__()
        self.mask = mask_seq(hidden_dim, ratio)

    def forward(self, feat):
        m0, m2 = self.mask[0], self.mask[2]
        return conv(relu_rec(conv(feat, m0.weight, m0.bias, "relu"), m0), m2.weight, m2.bias, None, 0.25)


class BasicUpdateBlockDepth(nn.Module):
    """update.py:143-173: S steps of cost -> encoder -> GRU -> delta inv-depth."""

    def __init__(self, hidden_dim=128, cost_dim=256, ratio=8, context_dim=64):
        super().__init__()
        self.encoder = ProjectionInputDepth(cost_dim=cost_dim, hidden_dim=hidden_dim, out_chs=hidden_dim)
        self.depth_gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=hidden_dim + context_dim)
        self.depth_head = DepthHead(hidden_dim, hidden_dim=hidden_dim, scale=False)
        self.mask = mask_seq(hidden_dim, ratio)

    def dro_param_groups(self):
        return fused_groups(self.depth_head.conv1, self.mask[0])

    def heads(self, net):
        """DepthHead.conv1 and mask.0 read the same state: one launch."""
        a, b = conv_cat(net, (self.depth_head.conv1, self.mask[0]), "relu")
        a, b = relu_rec(a, self.depth_head.conv1), relu_rec(b, self.mask[0])
        c2, m2 = self.depth_head.conv2, self.mask[2]
        return conv(a, c2.weight, c2.bias, "tanh"), conv(b, m2.weight, m2.bias, None, 0.25)

    def forward(self, net, cost_func, inv_depth, context, seq_len=4, scale_func=None):
        scale_func = scale_func or (lambda x: (x, None))
        invs, masks = [], []
        for _ in range(seq_len):
            # the state feeds the cost, the 7x7 conv, both GRU halves and the update
            inv_depth = hip.grad_sink(inv_depth)
            feat = self.encoder.sources(inv_depth, cost_func(scale_func(inv_depth)[0]))
            # the state feeds the heads and the next GRU step: one gradient buffer
            net = hip.grad_sink(self.depth_gru(net, [context, *feat]))
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
            net = hip.grad_sink(self.pose_gru(net, [inp, *self.encoder.sources(pose, cost_func(pose))]))
            pose = self.pose_head(net, pose)               # pose + pose_head(net), one launch
            seq.append(pose)
        return net, seq

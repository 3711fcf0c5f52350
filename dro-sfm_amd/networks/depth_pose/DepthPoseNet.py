"""DepthPoseNet -- the DRO recurrent depth/pose optimizer on MI355X.

Drop-in for dro_sfm/networks/depth_pose/DepthPoseNet.py:16-205: same
constructor (version, min_depth, max_depth), same forward(target_image,
ref_imgs, intrinsics) and train/eval return conventions, same state_dict keys.

Execution plan (what changes versus the reference, never the math):
  * every feature cost -- depth cost (mean over refs) and pose cost (per ref) --
    is ONE fused HIP launch (hip.warp_cost) that builds R from the euler vector,
    scales K, lifts, projects, bilinearly samples all 128 channels and squares
    the difference; disp_to_depth + inv2depth are folded in (DEPTH_DISP);
  * the reference views are processed as one batch: the feature maps of the N
    refs are a free view of the fnet output [N,B,C,h,w], the initial pose head,
    and the whole pose update block (cost, encoder, GRU, head) run once over
    N*B samples instead of N Python iterations;
  * convex upsampling is one HIP launch (hip.convex_upsample);
  * the pose update block runs on a side HIP stream beside the depth update
    block (they read only each other's detached state of the previous outer
    iteration), and the two context encoders run on that stream too, beside
    the feature encoder (cnet_depth first; the depth block waits for it
    through an event); autograd runs their backward on the same streams and a
    hipGraph capture records the fork/join as parallel branches;
  * tensors read by every iteration (feature maps, context features) carry a
    gradient sink (hip.grad_sink): the cost and GRU backward kernels add into
    it in place instead of autograd summing one gradient per use;
  * no host synchronisation anywhere: the step can be captured in a hipGraph.
"""
import contextlib
import os
import logging

import torch
import torch.nn as nn

from ... import hip
from ...hip.timeline import stamp, stamp_grad
from ..optim.extractor import ResNetEncoder
from ..optim.update import (BasicUpdateBlockDepth, BasicUpdateBlockPose, DepthHead, PoseHead,
                            UpMaskNet)


def _null():
    return contextlib.nullcontext()


def parse_version(version):
    """'it{I}[-h][-seq{S}][-inter][-out]' (DepthPoseNet.py:22-34)."""
    assert version and "it" in version, f"bad DepthPoseNet version {version!r}"
    fields = version.split("-")
    total = int(fields[0].split("it")[1])
    seq = next((int(f.split("seq")[1]) for f in fields if "seq" in f), 4)
    return {"outer": total // seq, "seq": seq, "high": "h" in version,
            "out_norm": "out" in version, "inter": "inter" in version}


_SIDE_STREAMS = {}

# the cost calls' reference maps channels-last (DRO_CL_REFS=0: NCHW, A/B)
_CL_REFS = os.environ.get("DRO_CL_REFS", "1") != "0"


_CONCURRENT_BLOCKS = [True]


def set_concurrent_blocks(enabled):
    """Run the pose update block on a side stream beside the depth update block
    (default True; False for A/B runs).  They are independent within an outer
    iteration: each reads the other's state of the previous iteration,
    detached (DepthPoseNet.py:154-197).  Under hipGraph replay the two chains
    of small launches overlap: 16.9 vs 19.0 ms/step (round 3, one box, two
    interleaved runs each); eager, 32.7 vs 32.0."""
    _CONCURRENT_BLOCKS[0] = bool(enabled)


def _pose_stream(device, name="pose"):
    """A persistent side stream: the pose block's, or cnet_depth's (created
    once, never during a capture: the eager warm-up steps create them)."""
    st = _SIDE_STREAMS.get((device, name))
    if st is None:
        # DRO_STREAM_PRIO=1 (A/B): the pose block's latency-bound chain at high
        # priority, cnet_depth's own stream at the lowest
        prio = 0
        if os.environ.get("DRO_STREAM_PRIO", "0") == "1":
            lo, hi = torch.cuda.Stream.priority_range()
            prio = hi if name == "pose" else lo
        st = _SIDE_STREAMS[(device, name)] = torch.cuda.Stream(device=device, priority=prio)
    return st


# where cnet_depth runs: "pose" (default) -- first on the pose block's stream
# (round 3), so its backward queues behind cnet_pose's there; "own" -- a stream
# of its own, so its backward can start as soon as the depth block's gradient
# reaches it.  Measured (round 5, A/B on one box): own 17.5-18.0 vs pose
# 14.9-15.0 ms/step -- the third stream's encoder kernels starve the pose
# block's latency-bound backward chain (5.7 instead of 1.6 ms in the in-graph
# timeline, gpurun_out/r5e/timeline_own.log)
_CNET_DEPTH_STREAM = [os.environ.get("DRO_CNET_DEPTH_STREAM", "pose")]


def set_cnet_depth_stream(mode):
    if mode not in ("pose", "own"):
        raise ValueError(mode)
    _CNET_DEPTH_STREAM[0] = mode


class DepthPoseNet(nn.Module):
    def __init__(self, version=None, min_depth=0.1, max_depth=100, **kwargs):
        super().__init__()
        cfg = parse_version(version)
        self.version = version
        self.min_depth, self.max_depth = min_depth, max_depth
        self.iters, self.seq_len = cfg["outer"], cfg["seq"]
        self.is_high, self.out_normalize, self.inter_sup = cfg["high"], cfg["out_norm"], cfg["inter"]
        logging.info("DepthPoseNet(%s): outer=%d seq=%d inter=%s high=%s out_norm=%s", version,
                     self.iters, self.seq_len, self.inter_sup, self.is_high, self.out_normalize)
        self.foutput_dim, self.feat_ratio = 128, 8
        self.hdim, self.cdim = (128 if self.is_high else 64), 32
        C, r, hd, cd = self.foutput_dim, self.feat_ratio, self.hdim, self.cdim
        # registration order == reference state_dict order
        self.fnet = ResNetEncoder(out_chs=C, stride=r)
        self.depth_head = DepthHead(input_dim=C, hidden_dim=C, scale=False)
        self.pose_head = PoseHead(input_dim=2 * C, hidden_dim=C)
        self.upmask_net = UpMaskNet(hidden_dim=C, ratio=r)
        self.update_block_depth = BasicUpdateBlockDepth(hidden_dim=hd, cost_dim=C, ratio=r, context_dim=cd)
        self.update_block_pose = BasicUpdateBlockPose(hidden_dim=hd, cost_dim=C, context_dim=cd)
        # `cnet` is constructed but never used by the reference forward (DepthPoseNet.py:58
        # vs :107-205); it is kept only so reference checkpoints load.
        self.cnet = ResNetEncoder(out_chs=C, stride=r)
        self.cnet_depth = ResNetEncoder(out_chs=hd + cd, stride=r, num_input_images=1)
        self.cnet_pose = ResNetEncoder(out_chs=hd + cd, stride=r, num_input_images=2)
        for name in ("fnet", "cnet", "cnet_depth", "cnet_pose"):    # test-record tags (branch pinning)
            if hasattr(self, name):
                enc = getattr(self, name)
                object.__setattr__(enc, "_dro_tag", name)
                for mname, m in enc.named_modules():
                    if isinstance(m, nn.BatchNorm2d):
                        object.__setattr__(m, "_dro_tag", f"{name}.{mname}")
        for mname, m in self.named_modules():      # conv ReLU sites (update.relu_rec)
            if isinstance(m, nn.Conv2d):
                object.__setattr__(m, "_dro_tag", mname)

    # ------------------------------------------------------------------ helpers
    @property
    def depth_mode(self):
        return hip.DEPTH_DISP if self.out_normalize else hip.DEPTH_INV

    def scale_inv_depth(self, disp):
        """disp_to_depth(...)[0] when 'out' is in the version, else identity."""
        if not self.out_normalize:
            return disp
        lo, hi = 1.0 / self.max_depth, 1.0 / self.min_depth
        return lo + (hi - lo) * disp

    def upsample_depth(self, depth, mask, ratio=8):
        """Convex upsampling (DepthPoseNet.py:63-74), one HIP launch."""
        return hip.convex_upsample(depth, mask, ratio)

    def upsample_scaled(self, depth, mask, ratio=8):
        """scale_inv_depth(upsample_depth(...)) in one launch (DepthPoseNet.py:126-128,
        :180-181): the disp_to_depth affine is the upsample kernel's epilogue."""
        if not self.out_normalize:
            return hip.convex_upsample(depth, mask, ratio)
        lo, hi = 1.0 / self.max_depth, 1.0 / self.min_depth
        return hip.convex_upsample(depth, mask, ratio, affine=(lo, hi - lo))

    def upsample_many(self, pairs, ratio=8):
        """upsample_scaled of every kept (disp, mask) pair of a training step in
        ONE launch each way (the upsampled maps feed only the losses, which read
        them stacked): the [n, B, 1, H, W] stack's unbind() views."""
        affine = None
        if self.out_normalize:
            lo, hi = 1.0 / self.max_depth, 1.0 / self.min_depth
            affine = (lo, hi - lo)
        disps, masks = zip(*pairs)
        return list(hip.convex_upsample_many(list(disps), list(masks), ratio, affine=affine).unbind(0))

    def _cost(self, fmap1, frefs, disp, poses, K, reduce_mean, tag=None):
        return hip.warp_cost(fmap1, frefs, disp, poses, K, depth_mode=self.depth_mode,
                             min_depth=self.min_depth, max_depth=self.max_depth,
                             scale=1.0 / self.feat_ratio, reduce_mean=reduce_mean, tag=tag)

    # ------------------------------------------------------------------ forward
    def forward(self, target_image, ref_imgs, intrinsics):
        # one gradient per shared conv weight, summed in-kernel (hip/conv.py)
        with hip.weight_grad_scope():
            return self._forward(target_image, ref_imgs, intrinsics)

    def _forward(self, target_image, ref_imgs, intrinsics):
        B, N = target_image.shape[0], len(ref_imgs)
        C, hd, cd = self.foutput_dim, self.hdim, self.cdim
        K = intrinsics.float().contiguous()
        stamp("fwd:begin")

        # context encoders first, on side streams (they depend on the images only)
        cuda = target_image.is_cuda
        pside = None
        if self.iters > 0 and _CONCURRENT_BLOCKS[0] and cuda:
            pside = _pose_stream(target_image.device)
        # cnet_pose on the pose block's stream (no join needed); cnet_depth
        # first on that stream too (its backward then runs there, beside
        # fnet's); the depth block waits for cnet_depth only, through an event
        d_stream = p_stream = None
        d_event = None
        if self.iters > 0 and cuda:
            if pside is not None:
                p_stream = d_stream = pside
                if _CNET_DEPTH_STREAM[0] == "own":
                    d_stream = _pose_stream(target_image.device, "cnet_depth")
            main = torch.cuda.current_stream(target_image.device)
            for st in {d_stream, p_stream} - {None}:
                st.wait_stream(main)
                for t in [target_image, *ref_imgs]:
                    t.record_stream(st)
        if self.iters > 0:
            with torch.cuda.stream(d_stream) if d_stream is not None else _null():
                ctx_d = stamp_grad(self.cnet_depth(target_image), "bwd:cnet_depth_begin")
                h_d, x_d = torch.split(ctx_d, [hd, cd], 1)     # split: one cat backward
                h_d, x_d = torch.tanh(h_d), torch.relu(x_d)
                hip.ops.record_branch(("relu_seq", "ctx_d"), lambda: (x_d > 0).to(torch.uint8), x_d)
                stamp("fwd:cnet_depth")
                if d_stream is not None:
                    d_event = torch.cuda.Event()
                    d_event.record(d_stream)
            with torch.cuda.stream(p_stream) if p_stream is not None else _null():
                pairs = torch.cat([target_image.unsqueeze(0).expand(N, *target_image.shape),
                                   torch.stack(list(ref_imgs))], 2).flatten(0, 1)
                ctx_p = stamp_grad(self.cnet_pose(pairs), "bwd:cnet_pose_begin")   # [N*B, hd+cd, h, w]
                h_p, x_p = torch.split(ctx_p, [hd, cd], 1)
                h_p, x_p = torch.tanh(h_p), torch.relu(x_p)
                hip.ops.record_branch(("relu_seq", "ctx_p"), lambda: (x_p > 0).to(torch.uint8), x_p)
                stamp("fwd:cnet_pose")

        fmaps = stamp_grad(self.fnet(torch.cat([target_image] + list(ref_imgs), 0)), "bwd:fnet_begin")
        stamp("fwd:fnet")
        assert target_image.shape[2] // fmaps.shape[2] == self.feat_ratio
        h, w = fmaps.shape[2:]
        fmap1_raw, frefs_raw = torch.split(fmaps, [B, N * B], 0)
        frefs_raw = frefs_raw.view(N, B, C, h, w)       # free view: all refs, one tensor
        # the cost calls read the reference maps channel-contiguous (one copy per
        # step each way: their gathers and scatters then stay coalesced however
        # the warp shears the reference, hip.ops.channels_last_refs)
        frefs_cl = hip.ops.channels_last_refs(frefs_raw) if _CL_REFS else frefs_raw
        # every cost call reads the same feature maps: their gradients are summed
        # in place by the warp-cost backward (no per-call add launches)
        fmap1, frefs = hip.grad_sink(fmap1_raw), hip.grad_sink(frefs_cl)

        # initial poses of all refs in one pass: cat([fmap1, fmap_ref_j]) per ref j
        pair = torch.cat([fmap1.unsqueeze(0).expand(N, B, C, h, w), frefs_raw], 2).view(N * B, 2 * C, h, w)
        poses = self.pose_head(pair).view(N, B, 6)

        disp = stamp_grad(self.depth_head(fmap1, act_fn=torch.sigmoid), "bwd:init_depth_head")
        # every kept (disp, mask) pair; upsampled together after the loop
        # (upsample_many; eval: only the last one is upsampled)
        up_pairs = [(disp, self.upmask_net(fmap1))]
        stamp("fwd:init_heads")
        pose_preds = [poses]

        # join: the depth block (main stream) reads h_d/x_d; h_p/x_p only when the
        # pose block runs on the main stream too
        main = torch.cuda.current_stream(target_image.device) if cuda else None
        if d_stream is not None:
            if d_event is not None:
                main.wait_event(d_event)
            else:
                main.wait_stream(d_stream)
            for t in (h_d, x_d):
                t.record_stream(main)
        if p_stream is not None and p_stream is not pside:
            main.wait_stream(p_stream)
            for t in (h_p, x_p):
                t.record_stream(main)

        fmap1_p, frefs_p = fmap1, frefs
        if self.iters > 0:
            # the context features feed every GRU step: gradients summed in place
            x_d = hip.grad_sink(x_d)
            if pside is None:
                x_p = hip.grad_sink(x_p)
            else:
                # the pose block's sinks live on its stream: their consumers (the
                # pose block's backward kernels) write them there, and the sink
                # nodes hand them on from there (a sink shared with the depth
                # block would be written from two streams at once)
                main = torch.cuda.current_stream(target_image.device)
                pside.wait_stream(main)
                with torch.cuda.stream(pside):
                    x_p = hip.grad_sink(x_p)
                    fmap1_p, frefs_p = hip.grad_sink(fmap1_raw), hip.grad_sink(frefs_cl)
        for it in range(self.iters):
            disp = disp.detach()
            poses = poses.detach()
            frozen_poses, frozen_disp = poses, disp

            def depth_block(h_d):
                depth_cost = lambda d: self._cost(fmap1, frefs, d, frozen_poses, K, True, ("depth", it))
                h_d, masks, disps = self.update_block_depth(h_d, depth_cost, frozen_disp, x_d,
                                                            seq_len=self.seq_len)
                keep = range(self.seq_len) if self.inter_sup else [self.seq_len - 1]
                for k in keep:
                    up_pairs.append((disps[k], masks[k]))
                stamp(f"fwd:depth_iter{it}")
                return stamp_grad(h_d, f"bwd:depth_iter{it}"), disps[-1]

            def pose_block(h_p):
                # pose block over all N refs at once; depth frozen at this outer step
                pose_cost = lambda q: self._cost(fmap1_p, frefs_p, frozen_disp, q.view(N, B, 6), K,
                                                 False, ("pose", it)).view(N * B, C, h, w)
                h_p, seq = self.update_block_pose(h_p, pose_cost, frozen_poses.reshape(N * B, 6), x_p,
                                                  seq_len=self.seq_len)
                seq = seq if self.inter_sup else [seq[-1]]
                stamp(f"fwd:pose_iter{it}")
                return stamp_grad(h_p, f"bwd:pose_iter{it}"), [q.view(N, B, 6) for q in seq]

            if pside is None:
                h_d, disp_last = depth_block(h_d)
                h_p, seq = pose_block(h_p)
            else:
                # the pose block reads only the detached depth and poses of the previous
                # outer step: it runs on a side stream beside the depth block
                main = torch.cuda.current_stream(target_image.device)
                pside.wait_stream(main)
                for t in (fmap1_p, frefs_p, frozen_disp, frozen_poses, h_p, x_p, K):
                    t.record_stream(pside)
                with torch.cuda.stream(pside):
                    h_p, seq = pose_block(h_p)
                h_d, disp_last = depth_block(h_d)
                main.wait_stream(pside)                    # join before the outputs are read
                for t in (h_p, *seq):
                    t.record_stream(main)
            pose_preds.extend(seq)
            disp, poses = disp_last, seq[-1]

        if not self.training:
            return self.upsample_scaled(*up_pairs[-1], self.feat_ratio), pose_preds[-1].permute(1, 0, 2)  # [B,N,6]
        if cuda:
            inv_preds = self.upsample_many(up_pairs, self.feat_ratio)
            stamp("fwd:upsample")
        else:
            inv_preds = [self.upsample_scaled(d, m, self.feat_ratio) for d, m in up_pairs]
        return inv_preds, torch.stack(pose_preds, 2).permute(1, 0, 2, 3)  # [B,N,n_pred,6]

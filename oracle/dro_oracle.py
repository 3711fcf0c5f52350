"""CPU ORACLE for the DRO-SfM hot path -- TEST INFRASTRUCTURE ONLY.

A functional fp32 restatement, in plain PyTorch CPU ops, of the reference's
algorithms on the hot path.  Every function cites the
reference file:line it restates.  It is pinned against the golden vectors in
tests/golden/*.npz, which were produced by running the reference itself
(tests/golden/gen_golden.py) -- see tests/test_oracle_golden.py.

Who may import this module: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- as the CHECKER / CPU baseline only.  The product package
(dro-sfm_amd/) never imports it and has no CPU path.

Networks are expressed over a flat parameter dict keyed exactly like the
reference DepthPoseNet.state_dict(), so any implementation
that keeps those keys can be compared weight-for-weight.
"""
import math

import torch
import torch.nn.functional as F

# ============================================================================ geometry
def euler_to_matrix(vec):
    """pose_vec2mat(mode='euler') (geometry/pose_utils.py:40-85): [B,6] -> R [B,3,3], t [B,3].

    R = Rx(rx) @ Ry(ry) @ Rz(rz) with vec = [tx, ty, tz, rx, ry, rz].
    """
    t = vec[:, :3]
    rx, ry, rz = vec[:, 3], vec[:, 4], vec[:, 5]
    one, zero = torch.ones_like(rx), torch.zeros_like(rx)

    def m(*rows):
        return torch.stack([torch.stack(r, -1) for r in rows], -2)

    cx, sx, cy, sy, cz, sz = rx.cos(), rx.sin(), ry.cos(), ry.sin(), rz.cos(), rz.sin()
    Rx = m((one, zero, zero), (zero, cx, -sx), (zero, sx, cx))
    Ry = m((cy, zero, sy), (zero, one, zero), (-sy, zero, cy))
    Rz = m((cz, -sz, zero), (sz, cz, zero), (zero, zero, one))
    return Rx @ Ry @ Rz, t


def pose_to_rt(pose):
    """Accept an euler vector [B,6] or a transform [B,3|4,4]; return (R, t)."""
    if pose.dim() == 2 and pose.shape[-1] == 6:
        return euler_to_matrix(pose)
    return pose[:, :3, :3], pose[:, :3, 3]


def vec_to_transform(vec):
    """Pose.from_vec (geometry/pose.py:38-45): [B,6] -> [B,4,4]."""
    R, t = euler_to_matrix(vec)
    T = torch.eye(4, dtype=vec.dtype).repeat(vec.shape[0], 1, 1)
    T = torch.cat([torch.cat([R, t.unsqueeze(-1)], -1), T[:, 3:]], 1)
    return T


def scale_K(K, s):
    """Camera.scaled -> scale_intrinsics (geometry/camera.py:83-107, camera_utils.py:13-19)."""
    if s == 1.0:
        return K
    K = K.clone()
    K[:, 0, 0] = K[:, 0, 0] * s
    K[:, 1, 1] = K[:, 1, 1] * s
    K[:, 0, 2] = (K[:, 0, 2] + 0.5) * s - 0.5
    K[:, 1, 2] = (K[:, 1, 2] + 0.5) * s - 0.5
    return K


def invert_K(K):
    """Camera.Kinv (geometry/camera.py:70-79): K.clone() with the pinhole entries inverted."""
    Ki = K.clone()
    Ki[:, 0, 0] = 1.0 / K[:, 0, 0]
    Ki[:, 1, 1] = 1.0 / K[:, 1, 1]
    Ki[:, 0, 2] = -1.0 * K[:, 0, 2] / K[:, 0, 0]
    Ki[:, 1, 2] = -1.0 * K[:, 1, 2] / K[:, 1, 1]
    return Ki


def inv2depth(inv):
    """utils/depth.py:102-121: 1/clamp(inv, 1e-6), zero where inv <= 0."""
    d = 1.0 / inv.clamp(min=1e-6)
    return torch.where(inv <= 0.0, torch.zeros_like(d), d)


def disp_to_depth(disp, min_depth, max_depth):
    """networks/layers/resnet/layers.py:11-20 -> scaled disparity (first output)."""
    lo, hi = 1.0 / max_depth, 1.0 / min_depth
    return lo + (hi - lo) * disp


def sample_grid(depth, K, ref_K, pose, scale):
    """Camera.reconstruct -> Camera(ref_K, Tcw=pose).project(normalize=True)
    (geometry/camera.py:111-194) as a grid_sample grid [B,h,w,2]."""
    B, _, h, w = depth.shape
    Kt, Kr = scale_K(K.to(depth.dtype), scale), scale_K(ref_K.to(depth.dtype), scale)
    ys, xs = torch.meshgrid(torch.arange(h, dtype=depth.dtype), torch.arange(w, dtype=depth.dtype),
                            indexing="ij")
    pix = torch.stack([xs, ys, torch.ones_like(xs)], 0).reshape(1, 3, -1).expand(B, 3, h * w)
    rays = invert_K(Kt).bmm(pix)                     # [B,3,hw]
    X = rays * depth.reshape(B, 1, h * w)            # identity Tcw -> world == camera
    R, t = pose_to_rt(pose)
    P = R.bmm(X) + t.unsqueeze(-1)
    x = Kr.bmm(P)
    Z = x[:, 2].clamp(min=1e-5)
    u = 2 * (x[:, 0] / Z) / (w - 1) - 1.0
    v = 2 * (x[:, 1] / Z) / (h - 1) - 1.0
    return torch.stack([u, v], -1).reshape(B, h, w, 2)


# diagnostics: how many positions each kind of pinning actually moved off the
# natural branch in the evaluations since the last clear (tools/diag_*)
PIN_STATS = {"cells": 0, "maxpool": 0, "relu": 0, "l1": 0}


class Cells:
    """Bilinear cells of a step's warps (test hook).  grid_sample's value is
    continuous in the sampling position but its derivative jumps where a
    coordinate crosses an integer: two evaluations of one step whose rounding
    puts a coordinate on either side of a cell edge take different branches of
    the (exact) piecewise-linear function.  `forced` maps a call key to an
    int64 [B,h,w] tensor of packed cells ((y0 + 32768) << 16 | (x0 + 32768);
    -1 = take the natural cell) that the sampler then uses wherever the
    given cell is the coordinate's own or a neighbouring one, so the oracle is
    evaluated on the branch another implementation took (the HIP kernels
    record theirs: hip.record_bilinear_cells); with record=True the natural
    cells of every call are kept in `recorded`.  Keys: ("depth", it, s, j),
    ("pose", it, s, j), ("photo", j, i).  With record=True the ReLU masks
    (("relu", key)) and stem-pooling argmaxes (("maxpool", encoder)) are
    recorded too, in the product record's layout (`as_forced()`), so that a
    second evaluation can be put on this one's whole branch
    (tools/conditioning.py)."""

    def __init__(self, forced=None, record=False):
        self.forced = forced or {}
        self.recorded = {} if record else None
        self.thresholds = {}      # clip index -> this evaluation's own clip threshold (photometric_map)

    def sample(self, img, grid, key):
        return grid_sample_cells(img, grid, self.forced.get(key), self, key)

    def record(self, key, value, part=None):
        if self.recorded is None:
            return
        if part is None:
            self.recorded[key] = value
        else:                             # view `part` of a site the product runs stacked
            self.recorded.setdefault(key, {})[part] = value

    def as_forced(self):
        """The recorded branch as a `forced` dict (stacked views concatenated
        along the batch in view order, as the product records them)."""
        return {k: (torch.cat([v[j] for j in sorted(v)], 0) if isinstance(v, dict) else v)
                for k, v in self.recorded.items()}


def pack_cells(x0, y0):
    """pack_cell (csrc/dro_common.hpp) of floor coordinates, int64."""
    x0 = x0.clamp(-32767, 32766).long()
    y0 = y0.clamp(-32767, 32766).long()
    return ((y0 + 32768) << 16) | (x0 + 32768)


def cells_from_calls(calls):
    """The product's bilinear-cell record (hip.record_bilinear_cells().calls:
    (tag, int32 map) per op call) -> Cells(forced=...) keys:
    ("depth", it, s, j) / ("pose", it, s, j) -> [B,h,w] for inner step s and
    reference view j, ("photo", j, i) -> [B,H,W] (int64, CPU).  Each cost tag
    is called once per inner step, in order; one call covers every view."""
    out, steps = {}, {}
    for tag, cells in calls:
        c = cells.cpu().to(torch.int64)
        if tag == "photo":
            for j in range(c.shape[0]):
                for i in range(c.shape[1]):
                    out[("photo", j, i)] = c[j, i]
        elif tag == "photo_clip":
            # the product's float [N*n + N] clip thresholds: compared by the tests
            # with the oracle's own (Cells.thresholds), never used by the oracle
            continue
        elif tag == "photo_clipmask":         # uint8 [N,n,B,H,W]: value <= threshold (not clamped)
            for j in range(c.shape[0]):
                for i in range(c.shape[1]):
                    out[("clipkeep", (j, i))] = c[j, i]
        elif tag == "photo_l1":               # int8 [N,n,B,3,H,W] L1 signs (l1_pinned)
            for j in range(c.shape[0]):
                for i in range(c.shape[1]):
                    out[("l1", (j, i))] = c[j, i]
        elif isinstance(tag, tuple) and tag[0] in ("maxpool", "relu"):
            out[tag] = c         # maxpool: [B,C,Ho,Wo] window index dy * 3 + dx; relu: y > 0 of a BN site
        elif isinstance(tag, tuple) and tag[0] == "relu_seq":     # y > 0 of the n-th call of a conv ReLU site
            n = steps.get(tag, 0)
            steps[tag] = n + 1
            out[("relu", (tag[1], n))] = c
        elif isinstance(tag, tuple):
            s_ = steps.get(tag, 0)
            steps[tag] = s_ + 1
            for j in range(c.shape[0]):
                out[(tag[0], tag[1], s_, j)] = c[j]
    return out


# pixels: how close to a grid line a coordinate must be for a recorded cell on
# the line's other side to be taken (grid_sample_cells)
CELL_TOL = 1e-3


def _near_line(v, v0, f):
    """f (a recorded floor) is v's own floor v0, or the neighbour across the
    grid line nearest v within CELL_TOL."""
    return (f == v0) | ((f == v0 - 1) & (v - v0 <= CELL_TOL)) | ((f == v0 + 1) & (v0 + 1 - v <= CELL_TOL))


def grid_sample_cells(img, grid, cells=None, book=None, key=None):
    """F.grid_sample(img, grid, 'bilinear', 'zeros', align_corners=True), with
    the bilinear cell of each output taken from `cells` where given (see
    Cells).  Same unnormalisation as ATen (((g + 1) / 2) * (size - 1)), same
    corner weights; out-of-image corners contribute zero."""
    if cells is None and (book is None or book.recorded is None):
        return F.grid_sample(img, grid, mode="bilinear", padding_mode="zeros", align_corners=True)
    B, C, Hi, Wi = img.shape
    ix = ((grid[..., 0] + 1) / 2) * (Wi - 1)
    iy = ((grid[..., 1] + 1) / 2) * (Hi - 1)
    x0, y0 = torch.floor(ix.detach()), torch.floor(iy.detach())
    if book is not None and book.recorded is not None:
        book.recorded[key] = pack_cells(x0, y0)
    if cells is not None:
        c = cells.to(torch.int64).reshape(x0.shape)
        fx = ((c & 0xFFFF) - 32768).to(x0.dtype)
        fy = (((c >> 16) & 0xFFFF) - 32768).to(y0.dtype)
        # a cell is taken only where it is this coordinate's own cell or the
        # neighbour across a grid line within CELL_TOL pixels of the
        # coordinate (a cell edge rounding decides); anything further keeps
        # the natural cell (a wider band would let the oracle
        # extrapolate from a wrong cell instead of bounding cell-choice errors)
        near = _near_line(ix.detach(), x0, fx) & _near_line(iy.detach(), y0, fy)
        forced = (c != -1) & near
        PIN_STATS["cells"] += int((forced & ((fx != x0) | (fy != y0))).sum())
        x0 = torch.where(forced, fx, x0)
        y0 = torch.where(forced, fy, y0)
    tx, ty = ix - x0, iy - y0
    flat = img.reshape(B, C, Hi * Wi)
    out = 0.0
    for dy, dx, wgt in ((0, 0, (1 - tx) * (1 - ty)), (0, 1, tx * (1 - ty)), (1, 0, (1 - tx) * ty),
                        (1, 1, tx * ty)):
        xx, yy = x0 + dx, y0 + dy
        ok = (xx >= 0) & (xx <= Wi - 1) & (yy >= 0) & (yy <= Hi - 1)
        idx = torch.where(ok, yy * Wi + xx, torch.zeros_like(xx)).long().reshape(B, 1, -1)
        v = torch.gather(flat, 2, idx.expand(B, C, idx.shape[-1])).reshape(B, C, *ix.shape[1:])
        out = out + v * (wgt * ok.to(wgt.dtype)).unsqueeze(1)
    return out


def get_cost_each(pose, fmap, fmap_ref, depth, K, ref_K, scale, cells=None, key=None):
    """DepthPoseNet.get_cost_each (networks/depth_pose/DepthPoseNet.py:76-96)."""
    grid = sample_grid(depth, K, ref_K, pose, scale)
    if cells is not None:
        warped = cells.sample(fmap_ref, grid, key)
    else:
        warped = F.grid_sample(fmap_ref, grid, mode="bilinear", padding_mode="zeros", align_corners=True)
    return (fmap - warped) ** 2


def depth_cost_calc(inv_scaled, fmap, fmaps_ref, poses, K, ref_K, scale, cells=None, key=None):
    """DepthPoseNet.depth_cost_calc (DepthPoseNet.py:98-105): mean over refs.
    key (with `cells`): the call's key prefix, ref j appended."""
    depth = inv2depth(inv_scaled)
    costs = [get_cost_each(p, fmap, f, depth, K, ref_K, scale, cells, key + (j,) if key else None)
             for j, (p, f) in enumerate(zip(poses, fmaps_ref))]
    return torch.stack(costs, 1).mean(1)


def view_synthesis(ref_image, depth, pose, K, ref_K, cells=None, key=None):
    """geometry/camera_utils.py:23-56 at full resolution (scale 1)."""
    grid = sample_grid(depth, K, ref_K, pose, 1.0)
    if cells is not None:
        return cells.sample(ref_image, grid, key)
    return F.grid_sample(ref_image, grid, mode="bilinear", padding_mode="zeros", align_corners=True)


def convex_upsample(inv, mask, r=8):
    """DepthPoseNet.upsample_depth (DepthPoseNet.py:63-74)."""
    B, _, h, w = inv.shape
    wts = torch.softmax(mask.reshape(B, 9, r, r, h, w), dim=1)
    taps = F.unfold(inv, [3, 3], padding=1).reshape(B, 9, 1, 1, h, w)
    up = (wts * taps).sum(1)                         # [B,r,r,h,w]
    return up.permute(0, 3, 1, 4, 2).reshape(B, 1, h * r, w * r)


# ============================================================================ losses
def ssim(x, y, C1=1e-4, C2=9e-4):
    """SSIM with 3x3 mean pooling over a reflection-padded image
    (losses/multiview_photometric_loss_mf.py:15-54)."""
    x, y = F.pad(x, (1, 1, 1, 1), mode="reflect"), F.pad(y, (1, 1, 1, 1), mode="reflect")
    pool = lambda z: F.avg_pool2d(z, 3, stride=1)
    mx, my = pool(x), pool(y)
    mxy, mxx, myy = mx * my, mx.pow(2), my.pow(2)
    sx, sy, sxy = pool(x.pow(2)) - mxx, pool(y.pow(2)) - myy, pool(x * y) - mxy
    num = (2 * mxy + C1) * (2 * sxy + C2)
    den = (mxx + myy + C1) * (sx + sy + C2)
    return num / den


# near-kink band of the L1 term |est - tgt| (images in [0, 1]): where the
# difference is this small a recorded sign is taken (l1_pinned)
L1_TOL = 1e-5


def l1_pinned(d, cells=None, key=None):
    """|d| (d = est - tgt, [B,3,H,W]); with a Cells book holding ("l1", key) --
    another evaluation's sign of d per element (int8: 1 / -1 / 2 for zero, 0 =
    not recorded) -- that sign is taken where |d| <= L1_TOL (a kink rounding
    decides): there the value is d * sign (within L1_TOL of |d|), the
    derivative the recorded one.  The product records the elements its
    gradient used (photometric backward's l1_signs hook)."""
    if cells is None or key is None:
        return d.abs()
    cells.record(("l1", key), _sign_code(d.detach()))
    forced = cells.forced.get(("l1", key))
    if forced is None:
        return d.abs()
    f = forced.to(torch.int64).reshape(d.shape)
    sg = torch.where(f == 2, torch.zeros_like(d), f.to(d.dtype))
    use = (f != 0) & (d.detach().abs() <= L1_TOL) & (sg != torch.sign(d.detach()))
    PIN_STATS["l1"] = PIN_STATS.get("l1", 0) + int(use.sum())
    return torch.where(use, d * sg, d.abs())


def _sign_code(d):
    return torch.where(d > 0, 1, torch.where(d < 0, -1, 2)).to(torch.int8)


# relative band around a clip threshold in which a recorded clamp decision is taken
CLIP_TOL = 1e-4


def photometric_map(est, tgt, ssim_w, C1, C2, clip_loss=0.0, cells=None, key=None, clip_index=None):
    """calc_photometric_loss (multiview_photometric_loss_mf.py:194-229) of one
    [B,3,H,W] pair.  clip_loss > 0 (:223-227): the map is clamped from above
    at float(mean + clip_loss * std) of itself (unbiased std, a detached
    constant computed in the map's dtype, always by this evaluation itself:
    a Cells book gets it as thresholds[clip_index], for the tests to compare
    with the product's).  With a Cells book holding ("clipkeep", key) --
    another evaluation's clamp decisions -- a pixel within CLIP_TOL of the
    threshold (clamped or not by rounding) takes the other evaluation's side;
    the clamp itself is continuous, so only the derivative's branch is pinned."""
    l1 = l1_pinned(est - tgt, cells, key)
    if ssim_w <= 0.0:
        out = l1
    else:
        s = torch.clamp((1.0 - ssim(est, tgt, C1, C2)) / 2.0, 0.0, 1.0)
        out = ssim_w * s.mean(1, True) + (1 - ssim_w) * l1.mean(1, True)
    if clip_loss > 0.0:
        mean, std = out.mean(), out.std()
        thr = float(mean + clip_loss * std)
        if cells is not None and clip_index is not None:
            cells.thresholds[clip_index] = thr
        keep = cells.forced.get(("clipkeep", key)) if cells is not None and key is not None else None
        if keep is not None:
            # the other evaluation's clamp decision where the value is within
            # rounding of the threshold
            k = keep.to(torch.bool).reshape(out.shape)
            near = (out.detach() - thr).abs() <= CLIP_TOL * abs(thr)
            PIN_STATS["clip"] = PIN_STATS.get("clip", 0) + int((near & (k != (out.detach() <= thr))).sum())
            out = torch.where(near, torch.where(k, out, torch.full_like(out, thr)), torch.clamp(out, max=thr))
        else:
            out = torch.clamp(out, max=thr)
    return out


def smoothness(inv_depths, image, smooth_w):
    """calc_smoothness_loss (multiview_photometric_loss_mf.py:273-299; utils/depth.py:147-199)."""
    n = len(inv_depths)
    wx = torch.exp(-(image[..., :-1] - image[..., 1:]).abs().mean(1, True))
    wy = torch.exp(-(image[..., :-1, :] - image[..., 1:, :]).abs().mean(1, True))
    total = 0.0
    for i, d in enumerate(inv_depths):
        dn = d / d.mean(2, True).mean(3, True).clamp(min=1e-6)
        sx = (dn[..., :-1] - dn[..., 1:]) * wx
        sy = (dn[..., :-1, :] - dn[..., 1:, :]) * wy
        total = total + (sx.abs().mean() + sy.abs().mean()) / 2 ** i
    return smooth_w * (total / n)


LAST_SELECTION = []   # per prediction, the natural min-candidate map of the last call (diagnostics)


def photometric_decay_loss(image, context, inv_depths, K, ref_K, poses, *, ssim_w=0.85, C1=1e-4,
                           C2=9e-4, smooth_w=0.001, automask=True, reduce="min",
                           forced_selection=None, cells=None, clip_loss=0.0):
    """MultiViewPhotometricDecayLoss.forward (multiview_photometric_loss_mf.py:303-361).

    context: list of N [B,3,H,W]; inv_depths: list of n [B,1,H,W] (full res);
    poses[j][i]: euler [B,6] or transform [B,4,4] for ref j, prediction i.
    cells: a Cells book (keys ("photo", j, i), ("l1", (j, i))) -- test hook.
    clip_loss: the reference constructor's per-map clamp (:93, :223-227).
    """
    n = len(inv_depths)
    per_pred = [[] for _ in range(n)]
    for j, ref in enumerate(context):
        for i in range(n):
            est = view_synthesis(ref, inv2depth(inv_depths[i]), poses[j][i], K, ref_K, cells, ("photo", j, i))
            per_pred[i].append(photometric_map(est, image, ssim_w, C1, C2, clip_loss, cells, (j, i),
                                               j * n + i))
        if automask:
            unwarped = photometric_map(ref, image, ssim_w, C1, C2, clip_loss, cells, None, len(context) * n + j)
            for i in range(n):
                per_pred[i].append(unwarped)
    photo = 0.0
    for i in range(n):
        maps = per_pred[i]
        if reduce == "min" and forced_selection is not None:
            # test hook: take the candidate another implementation selected (its
            # value is that implementation's min) so near-ties cannot flip
            idx = forced_selection[i].long()
            idx = idx.unsqueeze(1) if idx.dim() == 3 else idx           # [B,1,H,W]
            li = torch.gather(torch.cat(maps, 1), 1, idx).mean()
        elif reduce == "min":
            mv, mi = torch.cat(maps, 1).min(1, True)
            LAST_SELECTION[i:] = [mi.squeeze(1).to(torch.uint8)]     # diagnostics: the natural selection
            li = mv.mean()
        else:
            li = sum(m.mean() for m in maps) / len(maps)
        photo = photo + 0.85 ** (n - i - 1) * li
    if smooth_w > 0:
        smooth = smoothness(inv_depths, image, smooth_w)
        loss = photo + smooth
        # reference quirk: the stored metric is a detached ALIAS of the loss that
        # the in-place `loss += smoothness` then mutates (:268, :356), so the
        # 'photometric_loss' metric reports the total loss.
        photo_metric = loss.detach()
    else:
        smooth, loss, photo_metric = torch.zeros(()), photo, photo.detach()
    return {"loss": loss.reshape(1), "photometric_loss": photo_metric,
            "smoothness_loss": smooth.detach()}


def supervised_depth_pose_loss(inv_depths, gt_inv, gt_poses, poses, K, ref_K, min_depth,
                               max_depth):
    """SupervisedDepthPoseLoss.forward (losses/supervised_loss.py:244-371), sparse-l1."""
    n = len(inv_depths)
    lo, hi = 1.0 / max_depth, 1.0 / min_depth
    # depth term (:244-277)
    tl, tw = 0.0, 0.0
    for i in range(n):
        wgt = 0.85 ** (n - i - 1)
        tw += wgt
        valid = ((gt_inv > lo) & (gt_inv < hi)).squeeze(1)
        tl = tl + wgt * torch.mean(valid * (gt_inv - inv_depths[i]).abs().squeeze(1))
    depth_loss = tl / tw
    # pose term (:279-325): reprojection of gt depth under gt vs predicted pose
    gt_depth = inv2depth(gt_inv)
    dmask = ((gt_depth > min_depth) & (gt_depth < max_depth / 4.0)).permute(0, 2, 3, 1)
    pl, pw = 0.0, 0.0
    for i in range(n):
        wgt = 0.85 ** (n - i - 1)
        pw += wgt
        li = 0.0
        for j, gtp in enumerate(gt_poses):
            cg = sample_grid(gt_depth, K, ref_K, gtp, 1.0)
            cp = sample_grid(gt_depth, K, ref_K, poses[j][i], 1.0)
            valid = ((cg >= -1) & (cg <= 1)) * ((cp >= -1) & (cp <= 1)) * dmask
            li = li + torch.mean(valid * (cp - cg).abs().clamp(-1, 1))
        pl = pl + (li / len(gt_poses)) * wgt
    pose_loss = pl / pw
    loss = depth_loss + pose_loss
    return {"loss": loss.reshape(1), "depth_loss": depth_loss.detach(),
            "pose_loss": pose_loss.detach(), "all_loss": loss.detach()}


# ============================================================================ network (functional)
def _conv(p, name, x, stride=1, padding=0):
    return F.conv2d(x, p[name + ".weight"], p.get(name + ".bias"), stride=stride, padding=padding)


def _bn(p, name, x, training):
    return F.batch_norm(x, p[name + ".running_mean"], p[name + ".running_var"], p[name + ".weight"],
                        p[name + ".bias"], training=training, momentum=0.1, eps=1e-5)


def max_pool_3x3s2(x, forced=None):
    """F.max_pool2d(x, 3, 2, 1); with `forced` ([B,C,Ho,Wo] int window index
    dy * 3 + dx, another evaluation's argmax) the window element taken is the
    forced one wherever it ties the window's maximum within 1e-5 of its
    magnitude (a near-tie that rounding decides), else the natural maximum --
    the value is continuous either way, the gradient goes where the forced
    evaluation sent it."""
    y = F.max_pool2d(x, 3, 2, 1)
    if forced is None:
        return y
    B, C, H, W = x.shape
    Ho, Wo = y.shape[-2:]
    xp = F.pad(x, (1, 1, 1, 1), value=float("-inf"))
    win = F.unfold(xp.reshape(B * C, 1, H + 2, W + 2), 3, stride=2)           # [B*C, 9, Ho*Wo]
    win = win.reshape(B, C, 9, Ho, Wo)
    idx = forced.to(torch.int64).reshape(B, C, 1, Ho, Wo).clamp(0, 8)
    picked = torch.gather(win, 2, idx).squeeze(2)
    tie = (y.detach() - picked.detach()).abs() <= 1e-5 * y.detach().abs().clamp_min(1e-30)
    PIN_STATS["maxpool"] += int((tie & (idx.squeeze(2) != torch.argmax(win.detach(), 2))).sum())
    return torch.where(tie, picked, y)


def max_pool_argmax(x):
    """The window index dy * 3 + dx of F.max_pool2d(x, 3, 2, 1)'s maximum
    ([B,C,Ho,Wo] uint8, the product record's layout; the first maximum in
    window order on exact ties)."""
    B, C, H, W = x.shape
    xp = F.pad(x.detach(), (1, 1, 1, 1), value=float("-inf"))
    win = F.unfold(xp.reshape(B * C, 1, H + 2, W + 2), 3, stride=2)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    return torch.argmax(win.reshape(B, C, 9, Ho, Wo), 2).to(torch.uint8)


def relu_pinned(v, cells=None, key=None):
    """F.relu(v); with a Cells book holding ("relu", key) -- another
    evaluation's mask y > 0 at this site -- the forced mask is taken where it
    differs from v > 0 AND v is within 1e-5 of its channel's largest
    magnitude from zero (a kink that rounding decides): there the output is
    v * mask (the value stays within that margin of relu(v), the derivative
    is the forced one)."""
    if cells is not None:
        cells.record(("relu", key), v.detach() > 0)
    forced = cells.forced.get(("relu", key)) if cells is not None else None
    if forced is None:
        return F.relu(v)
    return _relu_forced(v, forced, 1e-5)


# near-kink margin of the update-block / head / decoder ReLU sites, relative to
# the channel's largest magnitude: they sit behind the recurrence, where two
# fp32 realisations of the step differ by more than at the encoders' BN sites
SEQ_RELU_TOL = 1e-4


def _relu_forced(v, forced, tol):
    m = forced.to(torch.bool).reshape(v.shape)
    scale = v.detach().abs().amax(dim=(0, 2, 3), keepdim=True)
    use = (m != (v.detach() > 0)) & (v.detach().abs() <= tol * scale)
    PIN_STATS["relu"] += int(use.sum())
    PIN_STATS["relu_far"] = PIN_STATS.get("relu_far", 0) + int(((m != (v.detach() > 0)) & ~use).sum())
    return torch.where(use, v * m.to(v.dtype), F.relu(v))


def relu_site(v, rk, name):
    """F.relu(v) at a convolution (or context) ReLU that runs once per call of
    its block; rk = (cells, n, part): with a Cells book holding
    ("relu", (name, n)) -- the product's mask y > 0 for the n-th call of that
    site (hip.record_bilinear_cells, tag ("relu_seq", name)) -- the forced
    mask is taken at near-kinks as in relu_pinned.  part = (j, B): the
    product ran the reference views stacked along the batch (update.py:14),
    the oracle runs view j -- its rows j*B..(j+1)*B of the recorded mask."""
    if rk is None or rk[0] is None:
        return F.relu(v)
    cells, n, part = rk
    cells.record(("relu", (name, n)), v.detach() > 0, None if part is None else part[0])
    forced = cells.forced.get(("relu", (name, n)))
    if forced is None:
        return F.relu(v)
    if part is not None:
        j, B = part
        forced = forced[j * B:(j + 1) * B]
    return _relu_forced(v, forced, SEQ_RELU_TOL)


def resnet_encoder(p, pre, x, training, stride=8, cells=None):
    """ResNetEncoder.forward (networks/optim/extractor.py:67-107) on torchvision's
    ResNet-18 layout (layer1..layer3, BasicBlocks) with the stride-8 fusion head.
    cells: a Cells book whose ("maxpool", <encoder>) entry pins the stem
    pooling's argmax (test hook)."""
    x = relu_pinned(_bn(p, pre + "bn1", _conv(p, pre + "conv1", x, 2, 3), training), cells, pre + "bn1")
    forced = cells.forced.get(("maxpool", pre.rstrip("."))) if cells is not None else None
    if cells is not None and cells.recorded is not None:
        cells.record(("maxpool", pre.rstrip(".")), max_pool_argmax(x))
    x = max_pool_3x3s2(x, forced)
    feats = {}
    for li, s in ((1, 1), (2, 2), (3, 2)):
        for bi in range(2):
            b = f"{pre}layer{li}.{bi}."
            st = s if bi == 0 else 1
            out = relu_pinned(_bn(p, b + "bn1", _conv(p, b + "conv1", x, st, 1), training), cells, b + "bn1")
            out = _bn(p, b + "bn2", _conv(p, b + "conv2", out, 1, 1), training)
            idt = x
            if b + "downsample.0.weight" in p:
                idt = _bn(p, b + "downsample.1", _conv(p, b + "downsample.0", x, st, 0), training)
            x = relu_pinned(out + idt, cells, b + "bn2")
        feats[li] = x
    rk = (cells, 0, None)
    x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    x = relu_site(_conv(p, pre + "upconv1.0", x, 1, 1), rk, pre + "upconv1.0")
    x = relu_site(_conv(p, pre + "upconv1_fusion.0", torch.cat([x, feats[2]], 1), 1, 1), rk,
                  pre + "upconv1_fusion.0")
    if stride == 4:
        x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
        x = relu_site(_conv(p, pre + "upconv2.0", x, 1, 1), rk, pre + "upconv2.0")
        x = relu_site(_conv(p, pre + "upconv2_fusion.0", torch.cat([x, feats[1]], 1), 1, 1), rk,
                      pre + "upconv2_fusion.0")
    return _conv(p, pre + "out_conv", x, 1, 1)


def sep_conv_gru(p, pre, h, x):
    """SepConvGRU (networks/optim/update.py:47-74): 1x5 then 5x1 gated update."""
    for sfx, pad in (("1", (0, 2)), ("2", (2, 0))):
        hx = torch.cat([h, x], 1)
        z = torch.sigmoid(_conv(p, pre + "convz" + sfx, hx, 1, pad))
        r = torch.sigmoid(_conv(p, pre + "convr" + sfx, hx, 1, pad))
        q = torch.tanh(_conv(p, pre + "convq" + sfx, torch.cat([r * h, x], 1), 1, pad))
        h = (1 - z) * h + z * q
    return h


def depth_head(p, pre, x, act=torch.tanh, rk=None):
    """DepthHead (update.py:5-14).  rk: relu_site's (cells, call, part)."""
    return act(_conv(p, pre + "conv2", relu_site(_conv(p, pre + "conv1", x, 1, 1), rk, pre + "conv1"), 1, 1))


def pose_head(p, pre, x, rk=None):
    """PoseHead (update.py:16-28): spatial mean, rotation scaled by 0.01."""
    o = _conv(p, pre + "conv2_pose", relu_site(_conv(p, pre + "conv1_pose", x, 1, 1), rk, pre + "conv1_pose"),
              1, 1)
    o = o.mean(3).mean(2)
    return torch.cat([o[:, :3], 0.01 * o[:, 3:]], 1)


def mask_head(p, pre, x, rk=None):
    """.25 * mask(x): 3x3 -> relu -> 1x1 to 9*r*r (update.py:150-153, :128-139)."""
    return 0.25 * _conv(p, pre + "2", relu_site(_conv(p, pre + "0", x, 1, 1), rk, pre + "0"), 1, 0)


def _branch(p, pre, x, names, pads, rk):
    """relu(conv(relu(conv(x)))) of the two projection branches."""
    (a, b), (pa, pb) = names, pads
    return relu_site(_conv(p, pre + b, relu_site(_conv(p, pre + a, x, 1, pa), rk, pre + a), 1, pb), rk, pre + b)


def projection_depth(p, pre, inv, cost, rk=None):
    """ProjectionInputDepth (update.py:77-99)."""
    cor = _branch(p, pre, cost, ("convc1", "convc2"), (0, 1), rk)
    dfm = _branch(p, pre, inv, ("convd1", "convd2"), (3, 1), rk)
    out = relu_site(_conv(p, pre + "convd", torch.cat([cor, dfm], 1), 1, 1), rk, pre + "convd")
    return torch.cat([out, inv], 1)


def projection_pose(p, pre, pose, cost, rk=None):
    """ProjectionInputPose (update.py:102-124): pose broadcast to a constant map."""
    B, _, h, w = cost.shape
    pm = pose.reshape(B, 6, 1, 1).expand(B, 6, h, w)
    cor = _branch(p, pre, cost, ("convc1", "convc2"), (0, 1), rk)
    pfm = _branch(p, pre, pm, ("convp1", "convp2"), (3, 1), rk)
    out = relu_site(_conv(p, pre + "convp", torch.cat([cor, pfm], 1), 1, 1), rk, pre + "convp")
    return torch.cat([out, pm], 1)


def update_block_depth(p, pre, net, cost_fn, inv, ctx, S, scale, cells=None, it=0):
    """BasicUpdateBlockDepth.forward (update.py:155-173).  cells/it: the ReLU
    sites' call index is it * S + step (relu_site)."""
    invs, masks = [], []
    for s in range(S):
        rk = (cells, it * S + s, None)
        feat = projection_depth(p, pre + "encoder.", inv, cost_fn(scale(inv)), rk)
        net = sep_conv_gru(p, pre + "depth_gru.", net, torch.cat([ctx, feat], 1))
        inv = inv + depth_head(p, pre + "depth_head.", net, rk=rk)
        invs.append(inv)
        masks.append(mask_head(p, pre + "mask.", net, rk))
    return net, masks, invs


def update_block_pose(p, pre, net, cost_fn, pose, ctx, S, cells=None, it=0, part=None):
    """BasicUpdateBlockPose.forward (update.py:184-199).  part = (j, B): this
    is reference view j (relu_site)."""
    seqs = []
    for s in range(S):
        rk = (cells, it * S + s, part)
        feat = projection_pose(p, pre + "encoder.", pose, cost_fn(pose), rk)
        net = sep_conv_gru(p, pre + "pose_gru.", net, torch.cat([ctx, feat], 1))
        pose = pose + pose_head(p, pre + "pose_head.", net, rk)
        seqs.append(pose)
    return net, seqs


def parse_version(version):
    """DepthPoseNet.__init__ version string (DepthPoseNet.py:22-34)."""
    parts = version.split("-")
    iters = int(parts[0].split("it")[1])
    seq = 4
    for s in parts:
        if "seq" in s:
            seq = int(s.split("seq")[1])
    return dict(outer=iters // seq, seq=seq, hdim=128 if "h" in version else 64,
                out_norm="out" in version, inter="inter" in version)


def depth_pose_net(p, version, min_depth, max_depth, image, refs, K, training=True, cells=None):
    """DepthPoseNet.forward (DepthPoseNet.py:107-205).  cells: a Cells book for
    the cost warps (keys ("depth", it, s, j), ("pose", it, s, j)) -- test hook."""
    import itertools
    cfg = parse_version(version)
    hd, cd, S = cfg["hdim"], 32, cfg["seq"]
    scale = (lambda x: disp_to_depth(x, min_depth, max_depth)) if cfg["out_norm"] else (lambda x: x)
    B, N = image.shape[0], len(refs)
    fm = resnet_encoder(p, "fnet.", torch.cat([image] + refs, 0), training, cells=cells)
    fmap1, frefs = fm[:B], [fm[B * (j + 1):B * (j + 2)] for j in range(N)]
    poses = [pose_head(p, "pose_head.", torch.cat([fmap1, f], 1), (cells, 0, (j, B))) for j, f in enumerate(frefs)]
    inv = depth_head(p, "depth_head.", fmap1, torch.sigmoid, (cells, 0, None))
    up = convex_upsample(inv, mask_head(p, "upmask_net.mask.", fmap1, (cells, 0, None)), 8)
    inv_preds, pose_preds = [scale(up)], [[q.clone() for q in poses]]
    ctx_d = resnet_encoder(p, "cnet_depth.", image, training, cells=cells)
    h_d, x_d = torch.tanh(ctx_d[:, :hd]), relu_site(ctx_d[:, hd:hd + cd], (cells, 0, None), "ctx_d")
    ctx_p = resnet_encoder(p, "cnet_pose.", torch.cat([torch.cat([image, r], 1) for r in refs], 0),
                           training, cells=cells)
    h_p = [torch.tanh(ctx_p[B * j:B * (j + 1), :hd]) for j in range(N)]
    x_p = [relu_site(ctx_p[B * j:B * (j + 1), hd:hd + cd], (cells, 0, (j, B)), "ctx_p") for j in range(N)]
    for it in range(cfg["outer"]):
        inv = inv.detach()
        poses = [q.detach() for q in poses]
        depth_fixed = inv2depth(scale(inv))
        sd = itertools.count()
        cost_d = lambda x, ps=poses, it=it, sd=sd: depth_cost_calc(x, fmap1, frefs, ps, K, K, 1.0 / 8, cells,
                                                                  ("depth", it, next(sd)))
        h_d, masks, invs = update_block_depth(p, "update_block_depth.", h_d, cost_d, inv, x_d, S,
                                              scale, cells, it)
        sel = range(S) if cfg["inter"] else [S - 1]
        for k in sel:
            inv_preds.append(scale(convex_upsample(invs[k], masks[k], 8)))
        inv = invs[-1]
        new_poses = []
        for j in range(N):
            sp = itertools.count()
            cost_p = lambda q, j=j, it=it, sp=sp: get_cost_each(q, fmap1, frefs[j], depth_fixed, K, K, 1.0 / 8,
                                                                cells, ("pose", it, next(sp), j))
            h_p[j], seqs = update_block_pose(p, "update_block_pose.", h_p[j], cost_p, poses[j],
                                             x_p[j], S, cells, it, (j, B))
            new_poses.append(seqs if cfg["inter"] else [seqs[-1]])
        for k in range(len(new_poses[0])):
            pose_preds.append([new_poses[j][k].clone() for j in range(N)])
        poses = [new_poses[j][-1] for j in range(N)]
    if not training:
        return inv_preds[-1], torch.stack(pose_preds[-1], 1)
    return inv_preds, torch.stack([torch.stack(pr, 1) for pr in pose_preds], 2)


def flip_lr_intr(K, width):
    """utils/image.py:61-81 (returned as a new tensor; the reference mutates the
    batch's intrinsics in place, so everything after the flip sees this K)."""
    K = K.clone()
    K[:, 0, 0] = -1 * K[:, 0, 0]
    K[:, 0, 2] = width - K[:, 0, 2]
    return K


def train_step_loss(p, version, min_depth, max_depth, batch, kind="selfsup", loss_kw=None,
                    forced_selection=None, flip=False, pred_perturb=None, cells=None):
    """SelfSupModelMF / SupModelMF .forward in training mode
    (models/SfmModelMF.py:106-189, SelfSupModelMF.py:63-99, SupModelMF.py:78-119).

    flip=True is the reference's random left-right flip taken
    (SfmModelMF.py:110-119, utils/image.py:61-81, 106-130): the net sees the
    flipped target and refs with K flipped (fx -> -fx, cx -> W - cx), its
    inverse depths are flipped back, and the loss -- on the UNflipped
    `*_original` images -- uses the flipped K (the in-place mutation).

    pred_perturb=(rel_inv, rel_pose, seed) is a test hook: the loss is
    evaluated at the net's predictions moved by seeded relative Gaussian
    noise (straight-through: the backward runs through the unmoved net), to
    measure how far the gradient moves when an fp32 forward lands that far
    from the exact predictions (the loss's derivative jumps: bilinear cell
    edges, L1 signs)."""
    loss_kw = loss_kw or {}
    K = batch["intrinsics"]
    img, refs = batch["rgb"], batch["rgb_context"]
    if flip:
        K = flip_lr_intr(K, img.shape[3])
        img, refs = img.flip(3), [r.flip(3) for r in refs]
    invs, pvec = depth_pose_net(p, version, min_depth, max_depth, img, refs, K, training=True, cells=cells)
    if flip:
        invs = [d.flip(3) for d in invs]
    if pred_perturb is not None:
        ri, rp, seed = pred_perturb
        g = torch.Generator().manual_seed(seed)
        noise = lambda t, r: (t.detach() * r * torch.randn(t.shape, generator=g, dtype=t.dtype)).to(t.device)
        invs = [d + noise(d, ri) for d in invs]
        pvec = pvec + noise(pvec, rp)
    N, n = pvec.shape[1], pvec.shape[2]
    poses = [[pvec[:, j, i] for i in range(n)] for j in range(N)]
    if kind == "selfsup":
        out = photometric_decay_loss(batch["rgb_original"], batch["rgb_context_original"], invs, K,
                                     K, poses, forced_selection=forced_selection, cells=cells, **loss_kw)
    else:
        gt_inv = torch.where(batch["depth"] <= 0, torch.zeros_like(batch["depth"]),
                             1.0 / batch["depth"].clamp(min=1e-6))
        out = supervised_depth_pose_loss(invs, gt_inv, batch["pose_context"], poses, K, K, min_depth,
                                         max_depth)
    # the net's predictions, for tests measuring forward distances
    out["preds"] = (torch.stack([d.detach() for d in invs]), pvec.detach())
    return out


# ============================================================================ evaluation
def depth_metrics(gt, pred, min_depth, max_depth, crop="", use_gt_scale=True):
    """compute_depth_metrics (utils/depth.py:259-343): per image, valid pixels
    (min < gt < max, garg / eigen_nyu crop :287-298), optional median scaling
    (:313-315), then the nine metrics (:320-341) averaged over the batch."""
    B, _, H, W = gt.shape
    if pred.shape[-2:] != gt.shape[-2:]:                            # interpolate_image (image.py:166-196)
        pred = F.interpolate(pred, size=(H, W), mode="bilinear", align_corners=True)
    pred = pred.clamp(min=1e-6)
    crop_mask = None
    if crop == "garg":
        crop_mask = torch.zeros(H, W, dtype=torch.bool, device=gt.device)
        crop_mask[int(0.40810811 * H):int(0.99189189 * H), int(0.03594771 * W):int(0.96405229 * W)] = True
    elif crop == "eigen_nyu":
        crop_mask = torch.zeros(H, W, dtype=torch.bool, device=gt.device)
        crop_mask[20:459, 24:615] = True
    acc = [0.0] * 9
    for pred_i, gt_i in zip(pred, gt):
        gt_i, pred_i = gt_i.squeeze(), pred_i.squeeze()
        valid = (gt_i > min_depth) & (gt_i < max_depth)
        if crop_mask is not None:
            valid = valid & crop_mask
        if valid.sum() == 0:
            continue
        gt_i, pred_i = gt_i[valid], pred_i[valid]
        if use_gt_scale:
            pred_i = pred_i * torch.median(gt_i / pred_i)
            pred_i = pred_i.clamp(min_depth, max_depth)
        pred_i = pred_i.clamp(min_depth, max_depth)
        thresh = torch.max(gt_i / pred_i, pred_i / gt_i)
        diff = gt_i - pred_i
        d = gt_i.log() - pred_i.log()
        vals = [torch.mean(diff.abs() / gt_i), torch.mean(diff ** 2 / gt_i), torch.sqrt(torch.mean(diff ** 2)),
                torch.sqrt(torch.mean((gt_i.log() - pred_i.log()) ** 2)),
                (thresh < 1.25).to(gt.dtype).mean(), (thresh < 1.25 ** 2).to(gt.dtype).mean(),
                (thresh < 1.25 ** 3).to(gt.dtype).mean(),
                ((d ** 2).mean() - d.sum() ** 2 / len(d) ** 2) ** 0.5,
                torch.mean((1.0 / pred_i - 1.0 / gt_i).abs())]
        acc = [a + v for a, v in zip(acc, vals)]
    return torch.tensor([float(a) / B for a in acc], dtype=gt.dtype)


def depth_metrics_demon(gt, gt_pose, pred, min_depth, max_depth, use_gt_scale=True):
    """compute_depth_metrics_demon (utils/depth.py:343-398): valid pixels
    min < gt < max (no crop); with scaling the ground truth is divided by the
    norm of the first reference's gt translation (gt_pose [B,N,4,4]) and the
    prediction multiplied by the median ratio -- no clamp to the depth range
    afterwards (unlike compute_depth_metrics)."""
    B, _, H, W = gt.shape
    if pred.shape[-2:] != gt.shape[-2:]:
        pred = F.interpolate(pred, size=(H, W), mode="bilinear", align_corners=True)
    pred = pred.clamp(min=1e-6)
    acc = [0.0] * 9
    for pred_i, gt_i, pose_i in zip(pred, gt, gt_pose):
        gt_i, pred_i = gt_i.squeeze(), pred_i.squeeze()
        valid = (gt_i > min_depth) & (gt_i < max_depth)
        if valid.sum() == 0:
            continue
        gt_i, pred_i = gt_i[valid], pred_i[valid]
        if use_gt_scale:
            t = pose_i[:, :3, 3]
            gt_i = gt_i / torch.sqrt(t[0].dot(t[0]))
            pred_i = pred_i * torch.median(gt_i / pred_i)
        thresh = torch.max(gt_i / pred_i, pred_i / gt_i)
        diff = gt_i - pred_i
        d = gt_i.log() - pred_i.log()
        vals = [torch.mean(diff.abs() / gt_i), torch.mean(diff ** 2 / gt_i), torch.sqrt(torch.mean(diff ** 2)),
                torch.sqrt(torch.mean((gt_i.log() - pred_i.log()) ** 2)),
                (thresh < 1.25).to(gt.dtype).mean(), (thresh < 1.25 ** 2).to(gt.dtype).mean(),
                (thresh < 1.25 ** 3).to(gt.dtype).mean(),
                ((d ** 2).mean() - d.sum() ** 2 / len(d) ** 2) ** 0.5,
                torch.mean((1.0 / pred_i - 1.0 / gt_i).abs())]
        acc = [a + v for a, v in zip(acc, vals)]
    return torch.tensor([float(a) / B for a in acc], dtype=gt.dtype)


def pose_metrics(gt, pred):
    """compute_pose_metrics (utils/depth.py:400-421) of one pair of 4x4
    transforms, in numpy float32 as the reference computes it: rotation angle
    of R1^T R2 (deg), angle between the translations (deg), and the
    translation error after a least-squares scale fit (cm)."""
    import numpy as np
    pr, g = pred.squeeze().cpu().numpy(), gt.squeeze().cpu().numpy()
    R1, t1 = g[:3, :3], g[:3, 3]
    R2, t2 = pr[:3, :3], pr[:3, 3]
    cos_r = np.minimum((np.trace(np.dot(R1.T, R2)) - 1.0) / 2.0, 1.0)
    rdeg = np.arccos(cos_r) * (180 / np.pi)
    cos_t = np.dot(t1, t2) / (np.sqrt(np.dot(t1, t1)) * np.sqrt(np.dot(t2, t2)))
    tdeg = np.arccos(cos_t) * (180 / np.pi)
    a = np.dot(t1, t2) / np.dot(t2, t2)
    tcm = 100 * np.sqrt(np.sum((t1 - a * t2) ** 2, axis=-1))
    return torch.tensor([rdeg, tdeg, tcm], dtype=torch.float32)


# ============================================================================ data pipeline
def resize_bilinear_pil(a, H, W):
    """Pillow's Image.resize((W, H), BILINEAR) of a uint8 HWC array, as
    torchvision Resize calls it in resize_sample_image_and_intrinsics
    (datasets/augmentations.py:69-111).  Pillow (not in /root/reference; 12.2
    here) Resample.c: triangle filter of support max(in/out, 1), double
    weights normalised per output then rounded to 22-bit fixed point, a
    horizontal pass into a uint8 image, then a vertical pass; each output =
    clip8((2^21 + sum w*x) >> 22).  Pinned bit-exactly against PIL itself
    (tests/test_oracle_golden.py::test_resize_matches_pillow)."""
    import numpy as np
    prec = 22

    def one_pass(img, axis, out_size):
        in_size = img.shape[axis]
        scale = in_size / out_size
        filterscale = max(scale, 1.0)
        ss = 1.0 / filterscale
        img = np.moveaxis(img, axis, 0).astype(np.int64)
        out = np.empty((out_size,) + img.shape[1:], np.int64)
        for o in range(out_size):
            center = (o + 0.5) * scale
            xmin = max(int(center - filterscale + 0.5), 0)
            n = min(int(center + filterscale + 0.5), in_size) - xmin
            w = [max(0.0, 1.0 - abs((x + xmin - center + 0.5) * ss)) for x in range(n)]
            tot = sum(w)
            w = [v / tot for v in w] if tot else w
            acc = np.full(img.shape[1:], 1 << (prec - 1), np.int64)
            for x in range(n):
                acc += int(w[x] * (1 << prec) + (0.5 if w[x] >= 0 else -0.5)) * img[xmin + x]
            out[o] = np.clip(acc >> prec, 0, 255)
        return np.moveaxis(out, 0, axis).astype(np.uint8)

    return one_pass(one_pass(a, 1, W), 0, H)


def color_jitter_pil(a, order, factors, hue):
    """torchvision ColorJitter.forward over a PIL image (colorjitter_sample,
    datasets/augmentations.py:213-258): ops in `order` (0 brightness, 1
    contrast, 2 saturation, 3 hue) through torchvision's functional_pil --
    ImageEnhance.Brightness / Contrast / Color(factor).enhance, and adjust_hue:
    H of img.convert('HSV') += np.array(hue * 255).astype(np.uint8) (wrapping),
    merged back to RGB.  torchvision is not installed here; this restates its
    published functional_pil on Pillow 12.2, which is the arithmetic checked."""
    import numpy as np
    from PIL import Image, ImageEnhance
    img = Image.fromarray(a)
    for op in order:
        if op == 0:
            img = ImageEnhance.Brightness(img).enhance(factors[0])
        elif op == 1:
            img = ImageEnhance.Contrast(img).enhance(factors[1])
        elif op == 2:
            img = ImageEnhance.Color(img).enhance(factors[2])
        else:
            h, s, v = img.convert("HSV").split()
            np_h = np.array(h, dtype=np.uint8)
            np_h += np.uint8(int(hue * 255) & 255)
            img = Image.merge("HSV", (Image.fromarray(np_h, "L"), s, v)).convert("RGB")
    return np.asarray(img)


def resize_depth_cv2_nearest(depth, shape):
    """augmentations.resize_depth (datasets/augmentations.py:47-65):
    cv2.resize(depth, dsize=shape[::-1], interpolation=cv2.INTER_NEAREST) then
    np.expand_dims(..., 2).  OpenCV (opencv-python-headless, unpinned in the
    reference's docker/Dockerfile:84; absent here) resizeNN: fx = dsize.width /
    src.width in double, ifx = 1 / fx, x_ofs[x] = min(cvFloor(x * ifx), src.width - 1),
    the same per row.  Scalar loops over a numpy [h, w] array; parity unpinned
    (no cv2 in this container or on the box)."""
    import numpy as np
    d = np.asarray(depth)
    if d.ndim == 3:
        d = d[..., 0]
    h, w = d.shape
    H, W = shape
    ifx, ify = 1.0 / (W / w), 1.0 / (H / h)
    out = np.empty((H, W), d.dtype)
    for y in range(H):
        sy = min(int(math.floor(y * ify)), h - 1)
        for x in range(W):
            out[y, x] = d[sy, min(int(math.floor(x * ifx)), w - 1)]
    return np.expand_dims(out, axis=2)


def rel_err(a, b):
    """max |a-b| / max(|b|) -- the relative metric the parity tests quote."""
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("math", "torch", "F")]

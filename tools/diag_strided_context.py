"""The native stride-2 encoder convolutions checked IN the training step
(DRO_NATIVE_STRIDED=1 failed train-step parity in round 4 while every per-op
test passes): each hip.conv2d_strided call of one golden train step is
re-checked against fp64 torch on the very tensors it saw -- forward output,
input and weight gradient -- and the worst relative errors are printed per
call.  usage: DRO_NATIVE_STRIDED=1 python tools/diag_strided_context.py [it12h|view5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402
import test_hip_parity as T  # noqa: E402

LOG = []
_orig = hip.conv2d_strided


class _Checked(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad):
        y = torch.ops.dro.conv2d_strided(x, w, None, stride, pad, 0)
        ctx.save_for_backward(x, w)
        ctx.sp = (stride, pad)
        with torch.no_grad():
            ref = F.conv2d(x.double(), w.double(), stride=stride, padding=pad)
        ctx.fwd_err = float((y.double() - ref).abs().max() / ref.abs().max())
        return y

    @staticmethod
    def backward(ctx, gout):
        x, w = ctx.saved_tensors
        s, p = ctx.sp
        gout = gout.contiguous()
        gx, gw = torch.empty_like(x), torch.empty_like(w)
        torch.ops.dro.conv2d_strided_backward(x, w, gout, s, p, gx, gw, None, 0)
        xd, wd = x.double().requires_grad_(), w.double().requires_grad_()
        with torch.enable_grad():
            yd = F.conv2d(xd, wd, stride=s, padding=p)
            rx, rw = torch.autograd.grad(yd, (xd, wd), gout.double())
        ex = float((gx.double() - rx).abs().max() / rx.abs().max().clamp_min(1e-30))
        ew = float((gw.double() - rw).abs().max() / rw.abs().max().clamp_min(1e-30))
        LOG.append((tuple(x.shape), tuple(w.shape), s, p, ctx.fwd_err, ex, ew,
                    torch.cuda.current_stream().cuda_stream))
        return gx, gw, None, None


def checked(x, weight, bias=None, stride=2, padding=1, act=None):
    assert bias is None and act is None
    return _Checked.apply(x, weight, int(stride), int(padding))


def main():
    hip.conv2d_strided = checked
    import dro_sfm_amd.networks.optim.extractor as ex
    ex.hip.conv2d_strided = checked
    case = sys.argv[1] if len(sys.argv) > 1 else "it12h"
    if case == "it12h":
        tag, version, kind = "it12h", "it12-h-out", "sup"
        d = T.fx(f"train_step_{tag}")
    else:
        tag, version, kind = "it12h", "it12-h-out", "selfsup"
        d = T.fx("train_step_it12h_selfsup_n4")
    dn = d if "min_depth" in d else T.fx(f"depthposenet_{tag}")
    mind, maxd = T.fval(dn["min_depth"]), T.fval(dn["max_depth"])
    N = d["refs"].shape[0]
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"].clone()}
    if "gt_depth" in d:
        batch["depth"] = d["gt_depth"]
        batch["pose_context"] = [d["gt_poses"][:, j] for j in range(N)]
    model = (T._selfsup_model if kind == "selfsup" else T._sup_model)(mind, maxd, tag, version)
    out = model(batch)
    out["loss"].sum().backward()
    torch.cuda.synchronize()
    print(f"{case}: {len(LOG)} strided calls (native: {ex._NATIVE_STRIDED[0]})")
    for xs, ws, s, p, ef, ex_, ew, st in LOG:
        print(f"  x {xs} w {ws} s{s} p{p}: fwd {ef:.2e} dx {ex_:.2e} dw {ew:.2e} stream {st:#x}")


if __name__ == "__main__":
    main()

"""One golden train step (it12h sup, or the view5 fixture) three times in one
process: MIOpen stride-2 convs, native stride-2 convs, native again -- and the
per-tensor gradient differences between the runs (max-rel), to tell a
native-path race (native vs native differs) from a realisation difference
(only native vs MIOpen differs).  usage: python tools/diag_strided_ab.py [it12h|view5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import test_hip_parity as T  # noqa: E402


GOUT = []


def _install_hooks():
    """Record the gradient arriving at every stride-2 conv's output (backward order)."""
    import dro_sfm_amd.networks.optim.extractor as ex
    if getattr(ex, "_diag_hooked", False):
        return
    orig = ex.conv3x3

    def conv3x3(m, srcs, act=None):
        y = orig(m, srcs, act)
        if m.stride != (1, 1) and y.requires_grad:
            tag = (tuple(m.weight.shape), tuple(y.shape))
            y.register_hook(lambda g, tag=tag: GOUT.append((tag, g.detach().double().cpu())))
        return y
    ex.conv3x3 = conv3x3
    ex._diag_hooked = True


def run(case, native):
    import dro_sfm_amd.networks.optim.extractor as ex
    _install_hooks()
    GOUT.clear()
    ex.set_native_strided_convs(native)
    if case == "it12h":
        d = T.fx("train_step_it12h")
        dn = T.fx("depthposenet_it12h")
        kind = "sup"
    else:
        d = dn = T.fx("train_step_it12h_selfsup_n4")
        kind = "selfsup"
    mind, maxd = T.fval(dn["min_depth"]), T.fval(dn["max_depth"])
    N = d["refs"].shape[0]
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"].clone()}
    if kind == "sup":
        batch["depth"] = d["gt_depth"]
        batch["pose_context"] = [d["gt_poses"][:, j] for j in range(N)]
    model = (T._selfsup_model if kind == "selfsup" else T._sup_model)(mind, maxd, "it12h", "it12-h-out")
    import dro_sfm_amd.hip as H
    with H.record_bilinear_cells() as rec:
        out = model(batch)
        out["loss"].sum().backward()
    torch.cuda.synchronize()
    run.gouts = list(GOUT)
    run.cells = [(tag, c.cpu()) for tag, c in rec.calls]
    return float(out["loss"].detach().sum()), {k: p.grad.detach().double().cpu() for k, p in model.depth_net.named_parameters()
                                      if p.grad is not None}


def diff(a, b):
    b = {k: v for k, v in b.items() if k in a}
    e = {k: float((a[k] - b[k]).abs().max() / b[k].abs().max().clamp_min(1e-30)) for k in b}
    num = sum(float((a[k] - b[k]).pow(2).sum()) for k in b)
    den = sum(float(b[k].pow(2).sum()) for k in b)
    return (num / den) ** 0.5, sorted(e.items(), key=lambda kv: -kv[1])[:5]


class _Mixed(torch.autograd.Function):
    """Stride-2 conv with the forward / backward each either native (HIP) or
    exact (fp64 torch, rounded to fp32): DIAG_FWD / DIAG_BWD = native|exact."""

    @staticmethod
    def forward(ctx, x, w, stride, pad):
        import torch.nn.functional as F
        ctx.save_for_backward(x, w)
        ctx.sp = (stride, pad)
        exact_k = os.environ.get("DIAG_FWD_EXACT_K")     # e.g. "7" or "1,3": exact forward for these kernels only
        if os.environ.get("DIAG_FWD", "native") == "exact" and (
                exact_k is None or str(w.shape[-1]) in exact_k.split(",")):
            y = F.conv2d(x.double(), w.double(), stride=stride, padding=pad)
            if os.environ.get("DIAG_NOISE"):      # relative noise of this size on the exact output
                g = torch.Generator(device=y.device).manual_seed(int(os.environ.get("DIAG_SEED", "0")))
                y = y * (1 + float(os.environ["DIAG_NOISE"]) * torch.randn(y.shape, generator=g, device=y.device,
                                                                          dtype=y.dtype))
            return y.float()
        return torch.ops.dro.conv2d_strided(x, w, None, stride, pad, 0)

    @staticmethod
    def backward(ctx, gout):
        import torch.nn.functional as F
        x, w = ctx.saved_tensors
        s, p = ctx.sp
        if os.environ.get("DIAG_BWD", "native") == "exact":
            xd, wd = x.double().requires_grad_(), w.double().requires_grad_()
            with torch.enable_grad():
                yd = F.conv2d(xd, wd, stride=s, padding=p)
                gx, gw = torch.autograd.grad(yd, (xd, wd), gout.double())
            return gx.float(), gw.float(), None, None
        gx, gw = torch.empty_like(x), torch.empty_like(w)
        torch.ops.dro.conv2d_strided_backward(x, w, gout.contiguous(), s, p, gx, gw, None, 0)
        return gx, gw, None, None


def _mixed(x, weight, bias=None, stride=2, padding=1, act=None):
    assert bias is None and act is None
    return _Mixed.apply(x, weight, int(stride), int(padding))


def oracle_check():
    if "DIAG_FWD" in os.environ or "DIAG_BWD" in os.environ:
        import dro_sfm_amd.hip as hip_
        import dro_sfm_amd.networks.optim.extractor as ex_
        hip_.conv2d_strided = _mixed
        ex_.hip.conv2d_strided = _mixed
        print("mixed strided conv: fwd", os.environ.get("DIAG_FWD", "native"), "bwd",
              os.environ.get("DIAG_BWD", "native"))
    """view5: HIP (native, then MIOpen) vs the fp64 oracle on that run's own
    cells and selection, on the other run's cells, and on natural cells."""
    from oracle import dro_oracle as O
    f = T.fx("train_step_it12h_selfsup_n4")
    mind, maxd = T.fval(f["min_depth"]), T.fval(f["max_depth"])
    spec = T.load_spec(os.path.join(T.G, "depthposenet_it12h_keys.json"))
    batch = {"rgb": f["image"], "rgb_context": list(f["refs"]), "rgb_original": f["image"],
             "rgb_context_original": list(f["refs"]), "intrinsics": f["K"].clone()}
    cpu_batch = {k: (v.cpu().clone() if torch.is_tensor(v) else [t.cpu() for t in v]) for k, v in batch.items()}
    runs = {}
    import dro_sfm_amd.networks.optim.extractor as ex
    from dro_sfm_amd.networks.depth_pose import DepthPoseNet as dpn
    serial = os.environ.get("DIAG_SERIAL") == "1"
    dpn.set_concurrent_blocks(not serial)
    print("concurrent blocks:", not serial)
    for native in (True, False):
        ex.set_native_strided_convs(native)
        model = T._selfsup_model(mind, maxd, "it12h", "it12-h-out")
        out, cells = T._run_step(model, batch)
        sel = model._photometric_loss.last_selection.cpu().unsqueeze(2)
        grads = {k: p.grad.detach().double().cpu() for k, p in model.depth_net.named_parameters()
                 if p.grad is not None}
        runs[native] = (cells, sel, grads)
    for hip_native in (True, False):
        grads = runs[hip_native][2]
        for name, (cells, sel) in (("own cells+sel", runs[hip_native][:2]),
                                   ("other run's cells+sel", runs[not hip_native][:2]),
                                   ("natural cells, own sel", (None, runs[hip_native][1]))):
            for k_ in list(O.PIN_STATS):
                O.PIN_STATS[k_] = 0
            _, g64 = T._oracle_grads(spec, "it12-h-out", mind, maxd, cpu_batch, "selfsup", torch.float64, sel,
                                     False, cells)
            kinds = {}
            for key in (cells or {}):
                kinds[key[0]] = kinds.get(key[0], 0) + 1
            print(f"    recorded keys {kinds}; positions moved off the natural branch {dict(O.PIN_STATS)}")
            l2, worst = diff(grads, {k: v.double() for k, v in g64.items() if k in grads})
            print(f"  HIP {'native' if hip_native else 'miopen'} vs fp64 on {name}: L2 {l2:.3e}  "
                  + ", ".join(f"{k} {v:.2e}" for k, v in worst[:3]), flush=True)


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "it12h"
    if case == "oracle":
        return oracle_check()
    lm, gm = run(case, False)
    go_m = run.gouts
    cm = run.cells
    ln1, gn1 = run(case, True)
    go_n = run.gouts
    cn = run.cells
    print("bilinear cells, native vs MIOpen run (pixels whose recorded cell differs):")
    for (ta, a), (tb, b) in zip(cm, cn):
        rec_ = (a != -1) & (b != -1)
        print(f"  {ta}: {int(((a != b) & rec_).sum())} of {int(rec_.sum())} recorded"
              f" (recorded in one run only: {int(((a == -1) != (b == -1)).sum())})")
    print("gradient at each stride-2 conv output, backward order (native vs MIOpen, max-rel):")
    for (tm, a), (tn, b) in zip(go_m, go_n):
        print(f"  {tm} {'==' if tm == tn else '!='} {tn}: {float((b - a).abs().max() / a.abs().max()):.2e}")
    ln2, gn2 = run(case, True)
    lm2, gm2 = run(case, False)
    print(case, "losses", lm, ln1, ln2, lm2)
    for name, a, b in (("native vs miopen", gn1, gm), ("native vs native", gn2, gn1),
                       ("miopen vs miopen", gm2, gm)):
        l2, worst = diff(a, b)
        print(f"  {name}: L2 {l2:.3e}  " + ", ".join(f"{k} {v:.2e}" for k, v in worst))


if __name__ == "__main__":
    main()

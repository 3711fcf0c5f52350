"""test_train_step_scannet_size_vs_oracle[sup_view3]'s loss check, taken apart:
the product step run twice in one process (is its forward repeatable?) and
the fp64 oracle's loss on each run's recorded branch, with and without the
conv ReLU sites pinned (relu_site), and with natural branches.
usage: python tools/diag_loss_spread.py [sup_view3|selfsup_view5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import test_hip_parity as T  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402


def repeat(model_fn, gb, n=3):
    """The forward alone, n times on fresh models: loss and every encoder's
    output compared bitwise with the first run."""
    first = None
    for r in range(n):
        model = model_fn()
        outs = {}
        for name in ("fnet", "cnet_depth", "cnet_pose", "update_block_depth", "update_block_pose"):
            mod = getattr(model.depth_net, name)
            mod.register_forward_hook(lambda m, i, o, name=name: outs.setdefault(name, []).append(
                (o if torch.is_tensor(o) else o[0]).detach().clone()))
        out = model(gb)
        torch.cuda.synchronize()
        loss = float(out["loss"].detach().sum())
        if first is None:
            first = (loss, outs)
            print(f"  run 0: loss {loss:.9f}", flush=True)
            continue
        diffs = {k: max(float((a - b).abs().max()) for a, b in zip(v, first[1][k])) for k, v in outs.items()}
        print(f"  run {r}: loss {loss:.9f} (== run 0: {loss == first[0]}); max|diff| per module "
              + ", ".join(f"{k} {d:.1e}" for k, d in diffs.items()), flush=True)


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "sup_view3"
    B, H, W = 1, 240, 320
    N = 4 if kind == "selfsup_view5" else 2
    mind, maxd = 0.2, 10.0
    spec = T.load_spec(os.path.join(T.G, "depthposenet_it12h_keys.json"))
    img = T.smooth_images(B, H, W, 81, detail=0.3)
    refs = [torch.roll(img, 2 * (j + 1), 3) * 0.9 + 0.1 * T.smooth_images(B, H, W, 82 + j, detail=0.3)
            for j in range(N)]
    batch = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs,
             "intrinsics": T._scannet_K(B)}
    if kind == "sup_view3":
        g = torch.Generator().manual_seed(83)
        batch["depth"] = 0.5 + 9.5 * torch.rand(B, 1, H, W, generator=g)
        batch["pose_context"] = [O.vec_to_transform(torch.cat([0.05 * torch.randn(B, 3, generator=g),
                                                               0.01 * torch.randn(B, 3, generator=g)], 1))
                                 for _ in range(N)]
    okind = "selfsup" if kind == "selfsup_view5" else "sup"
    gb = {k: (v.to(T.DEV) if torch.is_tensor(v) else [t.to(T.DEV) for t in v]) for k, v in batch.items()}
    mk = lambda: (T._selfsup_model if kind == "selfsup_view5" else T._sup_model)(mind, maxd, "it12h", "it12-h-out")
    if os.environ.get("DIAG_REPEAT"):
        import dro_sfm_amd.networks.optim.extractor as ex
        for native in (False, True):
            ex.set_native_strided_convs(native)
            print("native stride-2 encoders:", native)
            repeat(mk, gb)
        return
    runs = []
    for r in range(2):
        model = (T._selfsup_model if kind == "selfsup_view5" else T._sup_model)(mind, maxd, "it12h", "it12-h-out")
        out, cells = T._run_step(model, gb)
        forced = model._photometric_loss.last_selection.cpu().unsqueeze(2) if okind == "selfsup" else None
        runs.append((float(out["loss"].detach().sum()), cells, forced))
        print(f"run {r}: HIP loss {runs[-1][0]:.9f}", flush=True)
    for r, (loss, cells, forced) in enumerate(runs):
        for name, book in (("all pins", cells),
                           ("no conv-relu pins", {k: v for k, v in cells.items()
                                                  if not (k[0] == "relu" and isinstance(k[1], tuple))}),
                           ("natural", None)):
            for k_ in list(O.PIN_STATS):
                O.PIN_STATS[k_] = 0
            l64, _ = T._oracle_grads(spec, "it12-h-out", mind, maxd, batch, okind, torch.float64, forced, False,
                                     book)
            print(f"run {r} oracle fp64 ({name}): {float(l64):.9f}  rel {abs(loss - float(l64)) / abs(float(l64)):.2e}"
                  f"  moved {dict(O.PIN_STATS)}", flush=True)


if __name__ == "__main__":
    main()

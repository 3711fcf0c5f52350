"""Which weight-gradient route disagrees (tests/test_graph_step.py::
test_direct_weight_grads_match_autograd_path): one eager trainer step per
route -- autograd (per-call buffers returned to autograd), direct per use,
direct batched -- and, per parameter, the relative difference to the batched
route.  Prints the worst parameters of each pair."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "tests")]
import torch  # noqa: E402

from test_graph_step import _batch, _setup  # noqa: E402


def main():
    import dro_sfm_amd.hip.conv as hc
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    batch = _batch()
    K0 = batch["intrinsics"].clone()
    res = {}
    with torch.backends.cudnn.flags(enabled=False):
        for name, direct, batched in (("autograd", False, False), ("direct", True, False), ("batched", True, True)):
            hc.set_direct_weight_grads(direct)
            hc.set_batched_weight_grads(batched)
            m = _setup()
            tr = DataParallelTrainer(m)
            batch["intrinsics"].copy_(K0)
            loss = float(tr.step(batch, flip=False)[0])
            torch.cuda.synchronize()
            res[name] = (loss, {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None})
            print(name, "loss", loss, "nparams with grad", len(res[name][1]), flush=True)
    ref = res["batched"][1]
    for name in ("autograd", "direct"):
        g = res[name][1]
        errs = []
        for k, v in ref.items():
            d = float((g[k] - v).norm() / max(float(v.norm()), 1e-30))
            errs.append((d, k, float(v.norm()), float(g[k].norm())))
        errs.sort(reverse=True)
        print(f"== {name} vs batched: {sum(e[0] > 1e-4 for e in errs)} params differ > 1e-4")
        for e in errs[:25]:
            print(f"   {e[0]:.3e}  {e[1]}  |batched| {e[2]:.4e}  |{name}| {e[3]:.4e}")


if __name__ == "__main__":
    main()

"""Per-parameter gradient difference: graph replay vs eager step (GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch

from dro_sfm_amd.networks.optim import update
from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, GraphedTrainStep
from test_graph_step import _batch, _setup


def trial(backend, flips, share, warmup=3):
    update.set_conv_backend(backend)
    batch = _batch()
    K0 = batch["intrinsics"].clone()
    m = _setup()
    tr = DataParallelTrainer(m, capturable=True)
    gs = GraphedTrainStep(tr, batch, warmup=warmup, flips=flips, share_pool=share)
    snap_m = {k: v.clone() for k, v in m.state_dict().items()}
    snap_s = [{k: v.clone() for k, v in st.items()} for st in tr.optimizer.state.values()]

    def restore():
        with torch.no_grad():
            for k, v in m.state_dict().items():
                v.copy_(snap_m[k])
            for st, sv in zip(tr.optimizer.state.values(), snap_s):
                for k in st:
                    st[k].copy_(sv[k])
        batch["intrinsics"].copy_(K0)

    names = [n for n, _ in m.named_parameters()]

    def grads():
        return {n: (p.grad.detach().clone() if p.grad is not None else None) for n, p in m.named_parameters()}

    restore(); lg = float(gs.step(batch, flip=False)[0]); gg = grads(); fg = tr.grads.flat.clone()
    restore(); le = float(tr.step(batch, flip=False)[0]); ge = grads(); fe = tr.grads.flat.clone()
    restore(); le2 = float(tr.step(batch, flip=False)[0]); fe2 = tr.grads.flat.clone()
    restore(); lg2 = float(gs.step(batch, flip=False)[0]); fg2 = tr.grads.flat.clone()
    torch.cuda.synchronize()
    r = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-30))
    print(f"== backend={backend} flips={flips} share={share}: loss g {lg:.7f} e {le:.7f} e2 {le2:.7f} g2 {lg2:.7f}")
    print(f"   L2 rel: graph-eager {r(fg, fe):.2e}  eager-eager {r(fe2, fe):.2e}  graph-graph {r(fg2, fg):.2e}")
    rows = []
    for n in names:
        if gg[n] is None or ge[n] is None:
            continue
        rows.append((r(gg[n], ge[n]), n, float(ge[n].norm())))
    rows.sort(reverse=True)
    for e, n, nn_ in rows[:12]:
        print(f"   {e:.2e}  {n}  |g|={nn_:.3e}")
    del gs, tr, m
    torch.cuda.synchronize()


if __name__ == "__main__":
    trial("hip", (False, True), True)
    trial("hip", (False,), True)
    trial("hip", (False, True), False)
    trial("miopen", (False, True), True)

"""Where does step-to-step nondeterminism come from?  Same state, same batch:
forward outputs bitwise, loss, and gradients (top parameters by |diff|)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch

from dro_sfm_amd.networks.optim import update
from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
from test_graph_step import _batch, _setup


def run(backend, cudnn=True, det=False):
    update.set_conv_backend(backend)
    torch.backends.cudnn.enabled = cudnn
    torch.backends.cudnn.deterministic = det
    batch = _batch()
    K0 = batch["intrinsics"].clone()
    m = _setup()
    tr = DataParallelTrainer(m, capturable=True)
    for _ in range(3):
        batch["intrinsics"].copy_(K0)
        tr.step(batch, flip=False)
    snap = {k: v.clone() for k, v in m.state_dict().items()}
    names = [n for n, _ in m.named_parameters()]

    def restore():
        with torch.no_grad():
            for k, v in m.state_dict().items():
                v.copy_(snap[k])
        batch["intrinsics"].copy_(K0)

    # forward determinism (train mode, no grad)
    outs = []
    for _ in range(3):
        restore()
        with torch.no_grad():
            inv, poses = m.depth_net(batch["rgb"], batch["rgb_context"], batch["intrinsics"])
        outs.append(torch.cat([inv[-1].flatten(), poses.flatten()]).clone())
    fwd = [float((o - outs[0]).abs().max()) for o in outs[1:]]
    # loss + backward (autograd only, no optimizer)
    res = []
    for _ in range(4):
        restore()
        m.zero_grad(set_to_none=True)
        out = m(batch, flip=False)
        loss = out["loss"]
        loss.backward()
        torch.cuda.synchronize()
        g = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        res.append((float(loss.double()), g))
    print(f"== backend={backend} cudnn={cudnn} deterministic={det}: fwd max|diff| vs run0 {fwd}")
    print("   losses " + " ".join(f"{l:.9g}" for l, _ in res))
    g0 = res[0][1]
    tot0 = torch.sqrt(sum((v.double() ** 2).sum() for v in g0.values()))
    for i in range(1, len(res)):
        gi = res[i][1]
        d = {n: float((gi[n].double() - g0[n].double()).norm()) for n in g0}
        tot = sum(v * v for v in d.values()) ** 0.5
        top = sorted(d.items(), key=lambda kv: -kv[1])[:6]
        print(f"   run{i}: global rel L2 {tot / float(tot0):.2e}; top: " +
              ", ".join(f"{n.replace('depth_net.', '')}={v / float(g0[n].norm()):.1e}(|d|{v:.1e})" for n, v in top))
    del tr, m
    torch.cuda.synchronize()


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "det"):
        run("hip", det=True)
    if which == "all":
        run("hip")
        run("hip", cudnn=False)
        run("miopen")

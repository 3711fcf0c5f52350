"""Step-to-step reproducibility from one saved state: eager vs eager, graph vs eager."""
import copy, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch
from test_graph_step import _setup, _batch
from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, GraphedTrainStep

batch = _batch()
K0 = batch["intrinsics"].clone()
m = _setup()
tr = DataParallelTrainer(m, capturable=True)
for i in range(3):
    batch["intrinsics"].copy_(K0)
    tr.step(batch, flip=bool(i % 2))
snap_m = copy.deepcopy(m.state_dict())
snap_s = [{k: v.clone() for k, v in st.items()} for st in tr.optimizer.state.values()]


def restore():
    m.load_state_dict(snap_m)
    for st, sv in zip(tr.optimizer.state.values(), snap_s):
        for k in st:
            st[k].copy_(sv[k])


def eager(flip):
    restore()
    batch["intrinsics"].copy_(K0)
    l = tr.step(batch, flip=flip)[0].clone()
    torch.cuda.synchronize()
    return l, tr.grads.flat.clone()


def cmp(a, b):
    return float((a[1] - b[1]).norm() / b[1].norm()), float((a[0] - b[0]).abs().max())


for flip in (False, True):
    ref = eager(flip)
    print("eager-vs-eager flip", flip, [cmp(eager(flip), ref) for _ in range(3)], flush=True)
# graph
restore()
batch["intrinsics"].copy_(K0)
gs = GraphedTrainStep(tr, batch, warmup=2)
for flip in (False, True):
    res = []
    for _ in range(3):
        restore()
        batch["intrinsics"].copy_(K0)
        l = gs.step(batch, flip=flip)[0].clone()
        torch.cuda.synchronize()
        res.append((l, tr.grads.flat.clone()))
    ref = eager(flip)
    print("graph-vs-eager flip", flip, [cmp(r, ref) for r in res], flush=True)
    print("  graph-vs-graph", [cmp(r, res[0]) for r in res[1:]], flush=True)

"""Data-parallel trainer on the real model, on the GPU.

* Two ranks on ONE GPU (mp.spawn, gloo process group over CUDA tensors),
  eager steps of DataParallelTrainer(SelfSupModelMF(DepthPoseNet it8)) with the
  conv engine's in-place (direct, batched) weight gradients on: the ranks end
  bit-identical, and equal (to fp32 reassociation) to one process minimising
  the mean of the two per-rank losses -- the exact data-parallel semantics with
  per-replica BatchNorm statistics (no SyncBN, as the reference).
* RCCL with the captured hipGraph step: a world-size-1 "nccl" (RCCL) group
  with the exchange forced on (always_reduce); GraphedTrainStep replay vs the
  eager step (bucketed all-reduces issued from the backward hooks) from the
  same state, in both of its modes: the bucketed all-reduces captured INSIDE
  the graph from the backward hooks (the default at world > 1 over RCCL:
  they overlap the rest of the backward), and the exchange after the replay.

Reference: horovod_trainer.py:67-69 (dormant DistributedOptimizer),
model_wrapper.py:818-822 (DistributedSampler).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, H, W, N = 1, 64, 96, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed=0):
    from dro_sfm_amd.models.SelfSupModelMF import SelfSupModelMF
    from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet
    torch.manual_seed(seed)
    m = SelfSupModelMF(flip_lr_prob=0.0, automask_loss=True, photometric_reduce_op="min", clip_loss=0.0,
                       smooth_loss_weight=0.001, min_depth=0.5, max_depth=80.0)
    m.add_depth_net(DepthPoseNet(version="it8-seq4-inter-out", min_depth=0.5, max_depth=80.0))
    return m.cuda()


def _batch(rank, step):
    g = torch.Generator().manual_seed(1000 * step + rank)
    img = torch.rand(B, 3, H, W, generator=g)
    refs = [(0.9 * torch.roll(img, 2 + j, 3) + 0.1 * torch.rand(B, 3, H, W, generator=g)) for j in range(N)]
    K = torch.tensor([[93.0, 0.0, 47.5], [0.0, 92.0, 31.5], [0.0, 0.0, 1.0]]).repeat(B, 1, 1)
    b = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs, "intrinsics": K}
    return {k: (v.cuda() if torch.is_tensor(v) else [t.cuda() for t in v]) for k, v in b.items()}


def _flat(m):
    return torch.cat([p.detach().flatten() for p in m.parameters()]).cpu()


def _worker(rank, world, port, steps, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, init_distributed
    init_distributed("gloo")
    with torch.backends.cudnn.flags(enabled=False):     # deterministic encoder convs
        m = _model(seed=rank)                            # rank-0 broadcast must fix this
        # lr 0: parameters stay put, so every step's gradient is comparable with
        # the single-process run below (Adam maps a ~1e-9 gradient difference on a
        # near-zero entry to a full lr-sized step)
        tr = DataParallelTrainer(m, lr=0.0, bucket_mb=4.0)
        info, grads = [], []
        for s in range(steps):
            loss, _ = tr.step(_batch(rank, s))
            torch.cuda.synchronize()
            info.append((float(loss), list(tr.grads.issued), tr.grads.issued_in_backward,
                         len(tr.grads.buckets)))
            grads.append(tr.grads.flat.detach().cpu().clone())
        direct = sum(bool(getattr(p, "_dro_direct_used", False)) for p in m.parameters())
        mixed = sum(1 for b in tr.grads.buckets if any(getattr(p, "_dro_direct_used", False) for p in b)
                    and any(not getattr(p, "_dro_direct_used", False) for p in b))
        out[rank] = (_flat(m), info, direct, mixed, grads)
    dist.barrier()
    dist.destroy_process_group()


class _TwoHalves(torch.nn.Module):
    """One process over both ranks' batches: mean of the per-rank losses, each
    half through its own forward (its own BatchNorm statistics)."""

    def __init__(self, m):
        super().__init__()
        self.m = m

    def forward(self, pair):
        a, b = pair
        return {"loss": 0.5 * (self.m(a)["loss"] + self.m(b)["loss"])}


@pytest.mark.timeout(300)
def test_two_ranks_one_gpu_real_model_direct_weight_grads():
    steps = 2
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(2, port, steps, out), nprocs=2, join=True)
        res = dict(out)
    (p0, info0, direct, mixed, g0), (p1, info1, _, _, g1) = res[0], res[1]
    assert direct > 20, "the conv engine's in-place weight gradients were not used"
    assert torch.equal(p0, p1), "ranks diverged"
    assert all(torch.equal(a, b) for a, b in zip(g0, g1)), "all-reduced gradients differ between ranks"
    assert [i[1] for i in info0] == [i[1] for i in info1], "collective order differs between ranks"
    for _, issued, in_bwd, nb in info0[1:]:
        # every bucket -- including those holding in-place conv weight gradients --
        # is issued from the backward hooks, in the common order
        assert issued == list(range(nb)) and in_bwd == nb, (issued, in_bwd, nb)
    # one process over both halves: the same averaged gradient at every step
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    with torch.backends.cudnn.flags(enabled=False):
        m = _model(seed=0)
        tr = DataParallelTrainer(_TwoHalves(m), lr=0.0, bucket_mb=4.0)
        ref = []
        for s in range(steps):
            tr.step((_batch(0, s), _batch(1, s)))
            torch.cuda.synchronize()
            ref.append(tr.grads.flat.detach().cpu().clone())
    # the single-process flat layout covers the same parameters in the same order
    for s, (a, b) in enumerate(zip(g0, ref)):
        assert a.shape == b.shape
        l2 = float((a - b).norm() / b.norm())
        mx = float((a - b).abs().max() / b.abs().max())
        assert l2 < 1e-5 and mx < 1e-4, (s, l2, mx)


def _rccl_graph_worker(rank, port, out, in_graph):
    """World-size-1 RCCL group; GraphedTrainStep with the exchange after the
    replayed graph; replay vs eager from the same state.  Runs in a child process so
    that RCCL's watchdog or teardown cannot take the test runner down."""
    import faulthandler
    import sys
    faulthandler.enable()

    def stage(msg):
        print(f"[rccl-graph worker] {msg}", file=sys.stderr, flush=True)

    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, GraphedTrainStep, graph_safe_nccl_env
    from oracle import dro_oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    graph_safe_nccl_env()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    with torch.backends.cudnn.flags(enabled=False):
        batch = _batch(0, 0)
        K0 = batch["intrinsics"].clone()
        m = _model()
        tr = DataParallelTrainer(m, capturable=True, bucket_mb=4.0, always_reduce=True)
        stage(f"trainer built; capturing (in_graph={in_graph})")
        gs = GraphedTrainStep(tr, batch, warmup=2, flips=(False, True), reduce_in_graph=in_graph)
        stage("captured")
        seqs = dict(gs.issue_seq)
        capflags = {f: list(v) for f, v in gs.issue_capturing.items()}
        assert gs.in_graph == in_graph and gs.outside == (not in_graph)
        nb, issued = len(tr.grads.buckets), list(tr.grads.issued)
        in_bwd = tr.grads.issued_in_backward
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

        restore()
        stage("replay")
        lg = gs.step(batch, flip=False)[0].clone()
        gg = tr.grads.flat.clone()
        restore()
        stage("eager")
        le = tr.step(batch, flip=False)[0].clone()
        ge = tr.grads.flat.clone()
        torch.cuda.synchronize()
        out["res"] = (nb, issued, in_bwd, O.rel_err(lg.cpu(), le.cpu()), float((gg - ge).norm() / ge.norm()),
                      seqs, capflags)
    stage("results recorded; teardown")
    # the graphs hold RCCL kernels of this communicator: release them first
    del gs
    torch.cuda.synchronize()
    dist.barrier()
    dist.destroy_process_group()
    stage("teardown done")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("in_graph", [True, False])
def test_rccl_exchange_with_captured_graph_step(in_graph):
    """RCCL (forced on at world size 1) with the step's hipGraph -- the bucketed
    all-reduces captured inside it from the backward hooks (in_graph), or one
    all-reduce after the replay: replay == the eager step with hook-issued
    bucket all-reduces, and in the captured step every bucket's collective was
    issued from the backward hooks, in the common order."""
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_rccl_graph_worker, args=(_free_port(), out, in_graph), nprocs=1, join=True)
        nb, issued, in_bwd, loss_err, grad_err, seqs, capflags = out["res"]
    assert nb > 2 and issued == list(range(nb))
    # both flip graphs captured, with the same collective sequence
    assert set(seqs) == {False, True} and seqs[False] == seqs[True], seqs
    if in_graph:
        assert [b for b, _, _ in seqs[False]] == list(range(nb))
    if in_graph:
        assert in_bwd == nb, (in_bwd, nb)
        # every captured collective was issued from a stream inside the capture
        # (else RCCL's watchdog tracks it as eager: the round-5 abort)
        assert all(len(v) == nb and all(v) for v in capflags.values()), capflags
    assert loss_err < 1e-5
    assert grad_err < 1e-4


@pytest.mark.timeout(300)
def test_gru_chain_matches_separate_stage1():
    """The first SepConvGRU half's stage 1 run in the second half's gate-conv
    data-gradient epilogue (hip.conv.GruChain, dro_convgru_gates_backward) gives
    the training step's gradient of the separate-launch form, to fp32
    reassociation (a first half whose input-state sink is already written is
    now added into in the epilogue instead of by the sink's add)."""
    from dro_sfm_amd.hip import conv as C
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    prev, out, folded = C._GRU_CHAIN, {}, {}
    try:
        for chain in (False, True):
            C._GRU_CHAIN = chain
            with torch.backends.cudnn.flags(enabled=False):
                m = _model(seed=0)
                tr = DataParallelTrainer(m, lr=0.0, bucket_mb=4.0)
                tr.step(_batch(0, 0))       # the first step sets up the in-place weight gradients
                n0 = C.GruChain.folded
                tr.step(_batch(0, 1))
                torch.cuda.synchronize()
                out[chain] = tr.grads.flat.detach().cpu().clone()
            folded[chain] = C.GruChain.folded - n0
    finally:
        C._GRU_CHAIN = prev
    assert folded[False] == 0 and folded[True] == 16, (folded, C.GruChain.stats)   # 8 iterations x (depth, pose)
    a, b = out[True], out[False]
    l2 = float((a - b).norm() / b.norm())
    mx = float((a - b).abs().max() / b.abs().max())
    assert l2 < 1e-5 and mx < 1e-4, (l2, mx)

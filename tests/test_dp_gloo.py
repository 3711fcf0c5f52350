"""Data-parallel trainer (dro_sfm_amd.trainers.dp_trainer) on a CPU gloo group,
world_size 2 -- the N>1 path (bucketed, backward-overlapped gradient
all-reduce, unused-parameter discovery, rank-0 broadcast) without a GPU.

Invariant checked: with equal per-rank batches, averaging per-rank gradients
equals the gradient of the global-batch mean loss, so a 2-rank run must match
a 1-process run on the concatenated batch step for step.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


class Toy(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Conv2d(3, 8, 3, padding=1)
        self.b = nn.Conv2d(8, 8, (1, 5), padding=(0, 2))
        self.c = nn.Linear(8, 4)
        self.dead = nn.Conv2d(3, 3, 1)   # never used in forward (like DepthPoseNet.cnet)

    def forward(self, batch):
        x = torch.relu(self.b(torch.relu(self.a(batch["x"]))))
        y = self.c(x.mean((2, 3)))
        return {"loss": ((y - batch["y"]) ** 2).mean().reshape(1)}


class ToySkip(Toy):
    """Toy plus a head `d` that some ranks skip on some steps: its gradient
    never arrives there, so its bucket completes on one rank and not on the
    other (the collective order must still pair up)."""

    def __init__(self):
        super().__init__()
        self.d = nn.Linear(8, 4)

    def forward(self, batch):
        f = torch.relu(self.b(torch.relu(self.a(batch["x"])))).mean((2, 3))
        y = self.c(f)
        if batch["use_d"]:
            y = y + self.d(f)
        return {"loss": ((y - batch["y"]) ** 2).mean().reshape(1)}


# (step, rank) pairs on which ToySkip leaves `d` out
SKIP = {(1, 1), (2, 0), (4, 0), (4, 1)}


def data(rank, step, n=4):
    g = torch.Generator().manual_seed(100 * step + rank)
    return {"x": torch.randn(n, 3, 8, 8, generator=g), "y": torch.randn(n, 4, generator=g)}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, steps, out, skip=False, outside=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, init_distributed
    init_distributed("gloo")
    torch.manual_seed(rank)            # different init per rank: broadcast must fix it
    model = ToySkip() if skip else Toy()
    dead0 = model.dead.weight.detach().clone()
    tr = DataParallelTrainer(model, lr=1e-2, bucket_mb=1e-7 if skip else 0.0005)
    for s in range(steps):
        batch = data(rank, s)
        if skip:
            batch["use_d"] = (s, rank) not in SKIP
        if outside and s > 0:
            # GraphedTrainStep's sequence at world > 1: backward with the
            # collectives suspended (the captured part), then one all-reduce
            # of the flat gradient and the optimizer step
            tr.grads.suspend = True
            tr._forward_backward(batch)
            tr.grads.suspend = False
            tr.grads.reduce_now()
            tr.optimizer.step()
        else:
            tr.step(batch)
    flat = torch.cat([p.detach().flatten() for p in model.parameters()])
    out[rank] = (flat, len(tr.grads.buckets), torch.equal(model.dead.weight, dead0) or rank)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("outside", [False, True])
def test_two_rank_gloo_matches_single_process(outside):
    """outside=True: the exchange after backward (GraphedTrainStep at world > 1)."""
    steps = 4
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(2, port, steps, out, False, outside), nprocs=2, join=True)
        res = dict(out)
    (p0, nb0, dead_ok), (p1, nb1, _) = res[0], res[1]
    assert torch.equal(p0, p1), "ranks diverged"
    assert nb0 > 1, "expected several gradient buckets"
    assert dead_ok is True, "unused parameter must not move"
    # single process on the concatenated batch, same init as rank 0
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    torch.manual_seed(0)
    model = Toy()
    tr = DataParallelTrainer(model, lr=1e-2)
    for s in range(steps):
        a, b = data(0, s), data(1, s)
        tr.step({k: torch.cat([a[k], b[k]]) for k in a})
    ref = torch.cat([p.detach().flatten() for p in model.parameters()])
    assert torch.allclose(p0, ref, rtol=1e-5, atol=1e-6), float((p0 - ref).abs().max())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("outside", [False, True])
def test_two_rank_gloo_missing_gradient_on_one_rank(outside):
    """A parameter whose gradient arrives on one rank only (or on neither) on
    some steps: every bucket is still all-reduced exactly once per step on
    every rank, in the same order -- ranks stay identical and equal to one
    process minimising the mean of the two per-rank losses."""
    steps = 6
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        # outside=True: the exchange after backward, one all-reduce per run of
        # active parameters (`dead` sits between them here)
        mp.spawn(_worker, args=(2, port, steps, out, True, outside), nprocs=2, join=True)
        res = dict(out)
    (p0, nb0, _), (p1, _, _) = res[0], res[1]
    assert nb0 > 4, "expected one bucket per parameter"
    assert torch.equal(p0, p1), "ranks diverged"
    torch.manual_seed(0)
    model = ToySkip()
    opt = torch.optim.Adam([p for p in model.parameters()], lr=1e-2)
    for s in range(steps):
        opt.zero_grad(set_to_none=True)
        loss = 0.0
        for r in range(2):
            b = data(r, s)
            b["use_d"] = (s, r) not in SKIP
            loss = loss + 0.5 * model(b)["loss"].sum()
        loss.backward()
        for p in model.parameters():
            if p.grad is None and p is not model.dead.weight and p is not model.dead.bias:
                p.grad = torch.zeros_like(p)       # the DP path steps it with a zero gradient
        opt.step()
    ref = torch.cat([p.detach().flatten() for p in model.parameters()])
    assert torch.allclose(p0, ref, rtol=1e-5, atol=1e-6), float((p0 - ref).abs().max())


# ---------------------------------------------------------------- in-place (direct) gradients
_QUEUED = {}


class _DirectConv(torch.autograd.Function):
    """Stands in for the hip conv engine's direct path (hip/conv.py): the weight
    gradient is queued in backward and written IN PLACE into weight.grad only
    when flushed; autograd receives None for the weight."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return torch.nn.functional.conv2d(x, w, padding=(0, 2))

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        gw = torch.nn.grad.conv2d_weight(x, w.shape, g, padding=(0, 2))
        _QUEUED[w] = _QUEUED.get(w, 0) + gw
        return torch.nn.grad.conv2d_input(x.shape, w, g, padding=(0, 2)), None


def _fake_flush(p):
    gw = _QUEUED.pop(p, None)
    if gw is not None:
        p.grad.add_(gw)            # the in-place accumulation into the flat view
    return None


class ToyDirect(Toy):
    """Toy whose middle conv weight takes the direct (in-place) path; with a
    tiny bucket size it shares a bucket with autograd-produced gradients."""

    def forward(self, batch):
        w = self.b.weight
        if getattr(w, "_dro_direct", False) and w.grad is not None:
            w._dro_direct_used = True
            x = _DirectConv.apply(torch.relu(self.a(batch["x"])), w) + self.b.bias.view(1, -1, 1, 1)
        else:
            x = self.b(torch.relu(self.a(batch["x"])))
        y = self.c(torch.relu(x).mean((2, 3)))
        return {"loss": ((y - batch["y"]) ** 2).mean().reshape(1)}


def _worker_direct(rank, world, port, steps, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, init_distributed
    init_distributed("gloo")
    torch.manual_seed(rank)
    model = ToyDirect()
    tr = DataParallelTrainer(model, lr=1e-2, bucket_mb=0.0005)
    tr.grads.direct_flush = _fake_flush
    info = []
    for s in range(steps):
        tr.step(data(rank, s))
        assert not _QUEUED, "a queued in-place gradient was never flushed"
        info.append((list(tr.grads.issued), tr.grads.issued_in_backward, len(tr.grads.buckets)))
    mixed = [i for i, b in enumerate(tr.grads.buckets)
             if any(getattr(p, "_dro_direct_used", False) for p in b) and
             any(not getattr(p, "_dro_direct_used", False) for p in b)]
    flat = torch.cat([p.detach().flatten() for p in model.parameters()])
    out[rank] = (flat, info, mixed)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_direct_gradients_in_mixed_bucket():
    """A weight whose gradient is written in place at flush time (not produced
    by autograd) sharing a bucket with autograd gradients: its bucket's
    all-reduce is issued from the backward hooks (overlapped, not deferred to
    finish()) and only after the in-place write -- ranks stay identical and
    equal to one process minimising the mean of the two per-rank losses."""
    steps = 4
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker_direct, args=(2, port, steps, out), nprocs=2, join=True)
        res = dict(out)
    (p0, info0, mixed), (p1, info1, _) = res[0], res[1]
    assert mixed, "expected the direct weight in a bucket with autograd gradients"
    assert torch.equal(p0, p1), "ranks diverged"
    assert [i[0] for i in info0] == [i[0] for i in info1], "collective order differs between ranks"
    for issued, in_bwd, nb in info0[1:]:
        assert issued == list(range(nb)) and in_bwd == nb, (issued, in_bwd, nb)
    torch.manual_seed(0)
    model = Toy()
    opt = torch.optim.Adam(list(model.parameters()), lr=1e-2)
    for s in range(steps):
        opt.zero_grad(set_to_none=True)
        loss = sum(0.5 * model(data(r, s))["loss"].sum() for r in range(2))
        loss.backward()
        opt.step()
    ref = torch.cat([p.detach().flatten() for p in model.parameters()])
    assert torch.allclose(p0, ref, rtol=1e-5, atol=1e-6), float((p0 - ref).abs().max())


# ------------------------------------------------- collective-safety of GraphedTrainStep
def _worker_agree(rank, world, port, out):
    """capture_with_agreement with the in-graph capture failing on rank 1 only
    (as a capture could, e.g. out of memory on one device): every rank must run
    the fallback, and nobody may block.  Then the same with no failure."""
    import datetime
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    from dro_sfm_amd.trainers.dp_trainer import capture_with_agreement, check_same_across_ranks
    calls = []

    def try_fail():
        calls.append("try")
        if rank == 1:
            raise RuntimeError("forced capture failure on rank 1")

    kept_fail = capture_with_agreement(try_fail, lambda: calls.append("fallback"), log=calls.append)
    kept_ok = capture_with_agreement(lambda: calls.append("try2"), lambda: calls.append("fallback2"))
    # identical signatures pass; a signature that differs on one rank raises on every rank
    check_same_across_ranks(((0, 0, 10), (1, 10, 5)))
    try:
        check_same_across_ranks(((0, 0, 10),) if rank == 0 else ((0, 0, 10), (1, 10, 5)))
        raised = False
    except RuntimeError:
        raised = True
    dist.barrier()
    out[rank] = (kept_fail, kept_ok, [c for c in calls if not c.startswith("capture with")],
                 any(c.startswith("capture with") for c in calls), raised)
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_capture_failure_on_one_rank_falls_back_everywhere():
    """VERDICT r4 next 3 / ADVICE r4 medium: a capture failing on ONE rank makes
    every rank take the after-replay exchange (no rank left running in-graph
    collectives alone), and a collective-sequence mismatch raises on all ranks."""
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker_agree, args=(2, _free_port(), out), nprocs=2, join=True)
        res = dict(out)
    for r in (0, 1):
        kept_fail, kept_ok, calls, logged, raised = res[r]
        assert kept_fail is False and kept_ok is True, res[r]
        assert calls == ["try", "fallback", "try2"], (r, calls)
        assert logged, "the fallback must say why"
        assert raised, "a sequence differing on one rank must raise on every rank"


class ToyFlip(Toy):
    """Two heads whose forward (and so backward) order swaps with `flip`: the
    buckets complete in another order on a flipped step."""

    def __init__(self):
        super().__init__()
        self.d = nn.Linear(8, 4)

    def forward(self, batch, flip=False):
        x = batch["x"].flip(-1) if flip else batch["x"]
        f = torch.relu(self.b(torch.relu(self.a(x)))).mean((2, 3))
        if flip:
            y = self.d(f) + self.c(f)
        else:
            y = self.c(f) + self.d(f)
        return {"loss": ((y - batch["y"]) ** 2).mean().reshape(1)}


def _worker_flip(rank, world, port, steps, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from dro_sfm_amd.trainers.dp_trainer import (DataParallelTrainer, check_same_across_ranks,
                                                 collective_signature, init_distributed)
    init_distributed("gloo")
    torch.manual_seed(rank)
    model = ToyFlip()
    tr = DataParallelTrainer(model, lr=1e-2, bucket_mb=1e-7)      # one bucket per parameter
    sigs = []
    for s in range(steps):
        flip = (s + rank) % 2 == 1              # the ranks draw opposite flips every step
        tr.step(data(rank, s), flip=flip)
        if s > 0:
            sig = collective_signature(tr.grads)
            check_same_across_ranks(sig)
            sigs.append((flip, sig))
    flat = torch.cat([p.detach().flatten() for p in model.parameters()])
    out[rank] = (flat, sigs, len(tr.grads.buckets))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_flipped_and_unflipped_steps_issue_identical_collectives():
    """each rank picks its flip on its own, so a flipped
    and an unflipped backward must issue the same collectives in the same
    order even when their buckets complete in different orders."""
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker_flip, args=(2, _free_port(), 5, out), nprocs=2, join=True)
        res = dict(out)
    (p0, s0, nb), (p1, s1, _) = res[0], res[1]
    assert nb >= 6
    assert {f for f, _ in s0} == {False, True}
    assert len({sig for _, sig in s0 + s1}) == 1, "flip changed the collective sequence"
    assert [b for b, _, _ in s0[0][1]] == list(range(nb))
    assert torch.equal(p0, p1), "ranks diverged"

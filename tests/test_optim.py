"""Fused flat Adam (csrc/optim.hip via trainers.dp_trainer.FlatAdam) against
torch.optim.Adam: identical updates (GPU), a learning-rate schedule followed
by a captured graph (GPU), and the per-parameter state_dict layout the
reference writes into its checkpoints (model_checkpoint.py:76), both ways."""
import copy

import pytest
import torch

SHAPES = [(64, 160, 1, 5), (64,), (3, 3), (577,), (1,)]   # odd sizes: exercises the tail loop


def _flat_setup(device, seed=5):
    g = torch.Generator(device=device).manual_seed(seed)
    ref = [torch.randn(s, device=device, generator=g).requires_grad_() for s in SHAPES]
    flat_p = torch.cat([p.detach().reshape(-1) for p in ref]).clone()
    flat_g = torch.zeros_like(flat_p)
    views, off = [], 0
    for p in ref:
        views.append(flat_p[off:off + p.numel()].view_as(p))
        off += p.numel()
    return g, ref, flat_p, flat_g, views


def _grads(g, step, device):
    return [torch.randn(s, device=device, generator=g) * (10 ** (step - 2)) for s in SHAPES]


def _close(flat_p, ref):
    want = torch.cat([p.detach().reshape(-1) for p in ref])
    err = (flat_p - want).abs().max().item()
    return err <= 1e-6 * want.abs().max().item() + 1e-7, err


def test_flat_adam_state_dict_roundtrip_cpu():
    """torch.optim.Adam state -> FlatAdam -> state_dict() reproduces it
    exactly (layout, steps, moments, hyper-parameters); CPU only (no kernel)."""
    from dro_sfm_amd.trainers.dp_trainer import FlatAdam
    g, ref, flat_p, flat_g, views = _flat_setup("cpu")
    opt_ref = torch.optim.Adam(ref, lr=3e-4, betas=(0.8, 0.99), eps=1e-7)
    for step in range(3):
        for p, gr in zip(ref, _grads(g, step, "cpu")):
            p.grad = gr
        opt_ref.step()
    sd = opt_ref.state_dict()
    fa = FlatAdam(views, flat_p, flat_g)
    fa.load_state_dict(sd)
    assert fa.param_groups[0]["lr"] == 3e-4 and fa.param_groups[0]["betas"] == (0.8, 0.99)
    assert float(fa.step_t) == 3.0 and fa.hyper_t.tolist() == pytest.approx([3e-4, 0.8, 0.99, 1e-7, 0.0])
    sd2 = fa.state_dict()
    assert sorted(sd2["state"]) == sorted(sd["state"])
    for i, st in sd["state"].items():
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sd2["state"][i][k], st[k]), (i, k)
        assert float(sd2["state"][i]["step"]) == float(st["step"])
        assert sd2["state"][i]["step"].device.type == "cpu"
    assert sd2["param_groups"][0]["params"] == sd["param_groups"][0]["params"]
    # and back into a torch Adam
    fresh = [p.detach().clone().requires_grad_() for p in ref]
    opt2 = torch.optim.Adam(fresh, lr=1.0)
    opt2.load_state_dict(sd2)
    assert opt2.param_groups[0]["lr"] == 3e-4
    for i, st in opt2.state_dict()["state"].items():
        assert torch.equal(st["exp_avg_sq"], sd["state"][i]["exp_avg_sq"])


def test_flat_adam_is_an_optimizer_for_schedulers_cpu():
    from dro_sfm_amd.trainers.dp_trainer import FlatAdam
    _, _, flat_p, flat_g, views = _flat_setup("cpu")
    fa = FlatAdam(views, flat_p, flat_g, lr=2e-4)
    sched = torch.optim.lr_scheduler.StepLR(fa, step_size=2, gamma=0.5)   # default_config.py:72-74
    assert isinstance(fa, torch.optim.Optimizer)
    lrs = []
    for _ in range(5):
        lrs.append(fa.param_groups[0]["lr"])
        sched.step()
    assert lrs == pytest.approx([2e-4, 2e-4, 1e-4, 1e-4, 5e-5])
    fa.sync_hyper()
    assert fa.hyper_t[0].item() == pytest.approx(5e-5)


@pytest.mark.gpu
def test_flat_adam_matches_torch_adam():
    from dro_sfm_amd.trainers.dp_trainer import FlatAdam
    g, ref, flat_p, flat_g, views = _flat_setup("cuda")
    opt_ref = torch.optim.Adam(ref, lr=2e-4, betas=(0.9, 0.999), eps=1e-8)
    opt = FlatAdam(views, flat_p, flat_g, lr=2e-4, betas=(0.9, 0.999), eps=1e-8)
    for step in range(5):
        grads = _grads(g, step, "cuda")
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        flat_g.copy_(torch.cat([gr.reshape(-1) for gr in grads]))
        opt_ref.step()
        opt.step()
        torch.cuda.synchronize()
        ok, err = _close(flat_p, ref)
        assert ok, (step, err)
    assert float(opt.step_t) == 5.0
    # checkpoint round trip mid-run: FlatAdam -> torch Adam continues identically
    sd = opt.state_dict()
    fresh = [v.detach().clone().requires_grad_() for v in views]
    opt2 = torch.optim.Adam(fresh, lr=1.0)
    opt2.load_state_dict(sd)
    for step in range(5, 8):
        grads = _grads(g, step, "cuda")
        for p, q, gr in zip(ref, fresh, grads):
            p.grad, q.grad = gr.clone(), gr.clone()
        flat_g.copy_(torch.cat([gr.reshape(-1) for gr in grads]))
        opt_ref.step()
        opt2.step()
        opt.step()
        torch.cuda.synchronize()
        assert _close(flat_p, ref)[0] and _close(torch.cat([q.detach().reshape(-1) for q in fresh]), ref)[0]


@pytest.mark.gpu
def test_flat_adam_lr_schedule_reaches_captured_graph():
    """The Adam step captured in a hipGraph follows a StepLR schedule set
    between replays (the hyper-parameters are read from device memory)."""
    from dro_sfm_amd.trainers.dp_trainer import FlatAdam
    g, ref, flat_p, flat_g, views = _flat_setup("cuda", seed=7)
    opt_ref = torch.optim.Adam(ref, lr=1e-3)
    sched_ref = torch.optim.lr_scheduler.StepLR(opt_ref, step_size=1, gamma=0.1)
    opt = FlatAdam(views, flat_p, flat_g, lr=1e-3)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.1)
    grads = [_grads(g, 2, "cuda") for _ in range(4)]
    static_g = torch.zeros_like(flat_g)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    snap = (flat_p.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), opt.step_t.clone())
    with torch.cuda.stream(side):
        flat_g.copy_(static_g)
        opt.step()                         # warm-up (undone below)
    torch.cuda.synchronize()
    for dst, src in zip((flat_p, opt.exp_avg, opt.exp_avg_sq, opt.step_t), snap):
        dst.copy_(src)
    with torch.cuda.graph(graph):
        flat_g.copy_(static_g)
        opt.step()
    torch.cuda.synchronize()
    for k in range(4):
        for p, gr in zip(ref, grads[k]):
            p.grad = gr.clone()
        static_g.copy_(torch.cat([gr.reshape(-1) for gr in grads[k]]))
        opt_ref.step()
        opt.sync_hyper()
        graph.replay()
        torch.cuda.synchronize()
        ok, err = _close(flat_p, ref)
        assert ok, (k, err, opt.hyper_t.tolist())
        sched_ref.step()
        sched.step()
    assert opt.hyper_t[0].item() == pytest.approx(1e-6, rel=1e-5)


@pytest.mark.gpu
def test_trainer_adam_state_indexes_all_parameters_with_frozen():
    """The trainer's FlatAdam numbers ALL module parameters, as the reference's
    Adam group over depth_net.parameters() (model_wrapper.py:173): a frozen
    parameter keeps its index and no state; the saved group is capturable=False
    and loads into torch.optim.Adam over model.parameters(), which then
    continues identically."""
    import torch.nn as nn
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    torch.manual_seed(0)
    model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.ReLU(), nn.Conv2d(8, 8, 3, padding=1),
                          nn.ReLU(), nn.Conv2d(8, 4, 1)).cuda()
    model[2].weight.requires_grad_(False)                    # frozen, in the middle
    twin = copy.deepcopy(model)

    class M(nn.Module):
        def __init__(self, net):
            super().__init__()
            self.net = net

        def forward(self, batch):
            return {"loss": self.net(batch["x"]).pow(2).mean().reshape(1)}

    tr = DataParallelTrainer(M(model), lr=1e-3)
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(2, 3, 8, 8, generator=g).cuda() for _ in range(5)]
    for x in xs[:3]:
        tr.step({"x": x})
    sd = tr.optimizer.state_dict()
    names = [n for n, _ in model.named_parameters()]
    assert sd["param_groups"][0]["params"] == list(range(len(names)))
    assert sd["param_groups"][0]["capturable"] is False
    assert names.index("2.weight") not in sd["state"] and len(sd["state"]) == len(names) - 1
    # torch.optim.Adam over the same module, loaded mid-run, continues identically
    with torch.no_grad():
        for a, b in zip(twin.parameters(), model.parameters()):
            a.copy_(b)
    ref = torch.optim.Adam(twin.parameters(), lr=1.0)
    ref.load_state_dict(sd)
    for x in xs[3:]:
        tr.step({"x": x})
        ref.zero_grad(set_to_none=True)
        twin(x).pow(2).mean().backward()
        ref.step()
    torch.cuda.synchronize()
    for (n, a), b in zip(model.named_parameters(), twin.parameters()):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-7), n

"""Fused flat Adam (csrc/optim.hip via trainers.dp_trainer.FlatAdam) against
torch.optim.Adam on identical parameters and gradients (GPU)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_flat_adam_matches_torch_adam():
    from dro_sfm_amd.trainers.dp_trainer import FlatAdam
    g = torch.Generator(device="cuda").manual_seed(5)
    shapes = [(64, 160, 1, 5), (64,), (3, 3), (577,), (1,)]   # odd sizes: exercises the tail loop
    ref = [torch.randn(s, device="cuda", generator=g).requires_grad_() for s in shapes]
    n = sum(p.numel() for p in ref)
    flat_p = torch.cat([p.detach().reshape(-1) for p in ref]).clone()
    flat_g = torch.zeros(n, device="cuda")
    opt_ref = torch.optim.Adam(ref, lr=2e-4, betas=(0.9, 0.999), eps=1e-8)
    opt = FlatAdam([], flat_p, flat_g, lr=2e-4, betas=(0.9, 0.999), eps=1e-8)
    for step in range(5):
        grads = [torch.randn(s, device="cuda", generator=g) * (10 ** (step - 2)) for s in shapes]
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        flat_g.copy_(torch.cat([gr.reshape(-1) for gr in grads]))
        opt_ref.step()
        opt.step()
        torch.cuda.synchronize()
        want = torch.cat([p.detach().reshape(-1) for p in ref])
        err = (flat_p - want).abs().max().item()
        assert err <= 1e-6 * want.abs().max().item() + 1e-7, (step, err)
    assert float(opt.step_t) == 5.0

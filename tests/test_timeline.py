"""hip/timeline.py off the GPU: with no Timeline active, stamp() does nothing
and stamp_grad() returns its argument itself (the product path pays one
Python check per call site, no launch, no autograd node)."""
import torch


def test_inactive_stamps_are_identity():
    from dro_sfm_amd.hip.timeline import Timeline, stamp, stamp_grad
    assert Timeline._active is None
    x = torch.randn(3, requires_grad=True)
    assert stamp_grad(x, "bwd:x") is x
    stamp("fwd:x")                                   # no library call without a timeline
    y = stamp_grad(x * 2, "bwd:y")
    y.sum().backward()
    assert torch.equal(x.grad, torch.full((3,), 2.0))

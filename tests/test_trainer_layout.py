"""Flat gradient/parameter layout of the trainer (CPU): fused-parameter groups
declared by the modules sit back to back, so the hip convs can read a fused
weight and write its gradient as one view (hip/conv.py, direct path)."""
import torch

from dro_sfm_amd.hip.conv import _flat_view
from dro_sfm_amd.networks.optim.update import BasicUpdateBlockDepth, SepConvGRU
from dro_sfm_amd.trainers.dp_trainer import GradBuckets, _adjacent_order, param_groups


def test_adjacent_order_keeps_registration_order_otherwise():
    ps = [torch.nn.Parameter(torch.zeros(i + 1)) for i in range(6)]
    out = _adjacent_order(ps, [[ps[1], ps[4]], [ps[2], ps[5]]])
    assert out == [ps[0], ps[1], ps[4], ps[2], ps[5], ps[3]]
    assert _adjacent_order(ps, []) == ps


def test_gru_gates_are_flat_views():
    gru = SepConvGRU(hidden_dim=8, input_dim=12)
    gb = GradBuckets(gru.parameters(), groups=param_groups(gru))
    assert len(gb.params) == len(list(gru.parameters()))
    for a in ("1", "2"):
        cz, cr = getattr(gru, "convz" + a), getattr(gru, "convr" + a)
        gw = _flat_view([cz.weight.grad, cr.weight.grad])
        gbias = _flat_view([cz.bias.grad, cr.bias.grad])
        assert gw is not None and gw.shape == (16, 20) + cz.kernel_size
        assert gbias is not None and gbias.shape == (16,)
        gw[8:].fill_(2.0)                       # writes land in convr's .grad
        assert bool((cr.weight.grad == 2.0).all()) and bool((cz.weight.grad == 0.0).all())
    # not adjacent -> no view
    assert _flat_view([gru.convz1.weight.grad, gru.convq1.weight.grad]) is None


def test_update_block_declares_head_group():
    blk = BasicUpdateBlockDepth(hidden_dim=16, cost_dim=8, ratio=2, context_dim=8)
    gb = GradBuckets(blk.parameters(), groups=param_groups(blk))
    c1, m0 = blk.depth_head.conv1, blk.mask[0]
    assert _flat_view([c1.weight.grad, m0.weight.grad]) is not None
    assert _flat_view([c1.bias.grad, m0.bias.grad]) is not None
    assert gb.flat.numel() == sum(p.numel() for p in blk.parameters())

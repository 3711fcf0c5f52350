"""Reference checkpoints into this build (dro_sfm_amd.utils.load, restating
dro_sfm/utils/load.py:116-204).  A checkpoint with the layout ModelCheckpoint
writes (model_checkpoint.py:69-79) -- including a yacs CfgNode 'config' -- is
produced here with a stand-in `yacs.config.CfgNode` class (yacs is not
installed), then read back with weights_only=True and the stand-in removed."""
import sys
import types

import torch

from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet
from dro_sfm_amd.utils.load import backwards_state_dict, load_checkpoint, load_network


def _fake_yacs():
    yacs = types.ModuleType("yacs")
    cfgmod = types.ModuleType("yacs.config")

    class CfgNode(dict):          # the shape of yacs' class: a dict with instance attributes
        IMMUTABLE = "__immutable__"

        def __init__(self, init_dict=None):
            super().__init__(init_dict or {})
            self.__dict__[CfgNode.IMMUTABLE] = False

    CfgNode.__module__ = "yacs.config"
    CfgNode.__qualname__ = "CfgNode"
    cfgmod.CfgNode = CfgNode
    yacs.config = cfgmod
    return yacs, cfgmod, CfgNode


def test_reference_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(0)
    src = DepthPoseNet(version="it8-seq4-inter-out", min_depth=0.5, max_depth=80.0)
    yacs, cfgmod, CfgNode = _fake_yacs()
    saved_mods = {k: sys.modules.get(k) for k in ("yacs", "yacs.config")}
    sys.modules["yacs"], sys.modules["yacs.config"] = yacs, cfgmod
    try:
        cfg = CfgNode({"model": CfgNode({"depth_net": CfgNode({"name": "DepthPoseNet",
                                                               "version": "it8-seq4-inter-out"})}),
                       "arch": CfgNode({"max_epochs": 50})})
        opt = torch.optim.Adam(src.parameters(), lr=2e-4)
        ckpt = {"config": cfg, "epoch": 7,
                "state_dict": {"model.depth_net." + k: v for k, v in src.state_dict().items()},
                "optimizer": opt.state_dict(), "scheduler": {"step_size": 10, "gamma": 0.5}}
        path = str(tmp_path / "epoch=07.ckpt")
        torch.save(ckpt, path)
    finally:
        for k, v in saved_mods.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    assert "yacs.config" not in sys.modules or saved_mods["yacs.config"] is not None
    data = load_checkpoint(path)                      # weights_only: no yacs needed, nothing executed
    assert data["epoch"] == 7 and data["config"]["model"]["depth_net"]["version"] == "it8-seq4-inter-out"
    torch.manual_seed(1)
    dst = DepthPoseNet(version="it8-seq4-inter-out", min_depth=0.5, max_depth=80.0)
    assert any(not torch.equal(a, b) for a, b in zip(src.state_dict().values(), dst.state_dict().values()))
    load_network(dst, path, ["depth_net", "disp_network"])
    for (k, a), (k2, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k


def test_load_network_prefix_and_shape_filter():
    torch.manual_seed(2)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.Conv2d(4, 2, 1))
    sd = {"model.depth_net." + k: torch.full_like(v, 0.5) for k, v in net.state_dict().items()}
    sd["model.depth_net.1.weight"] = torch.zeros(9, 9)         # wrong shape: skipped
    sd["model.pose_net.0.bias"] = torch.zeros(4)               # other prefix: skipped
    load_network(net, sd, "depth_net")
    assert torch.equal(net[0].weight, torch.full_like(net[0].weight, 0.5))
    assert not torch.equal(net[1].weight, torch.full_like(net[1].weight, 0.5))


def test_backwards_state_dict_renames():
    out = backwards_state_dict({"disp_network.conv3.0.weight": 1, "pose_network.x": 2, "model.y": 3})
    assert list(out) == ["model.depth_net.conv3.weight", "model.pose_net.x", "model.y"]

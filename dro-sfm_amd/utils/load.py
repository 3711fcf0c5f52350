"""Checkpoint loading: reference `.ckpt` files into this build.

Restates load_network / backwards_state_dict (dro_sfm/utils/load.py:116-204 of
the reference): a checkpoint is the dict ModelCheckpoint writes
(dro_sfm/models/model_checkpoint.py:69-79: 'config', 'epoch', 'state_dict',
'optimizer', 'scheduler'); network weights are the 'state_dict' entries under
a prefix ('depth_net', 'disp_network', 'model', ...), matched by substring
and shape exactly as the reference does.  The state_dict key layout of
DepthPoseNet is the reference's (tests/test_state_dict_compat.py).  Verified
on a checkpoint of that layout written here (tests/test_checkpoint.py); no
published checkpoint is available offline to load.

Files are read with torch.load(weights_only=True): nothing in the file runs.
The only non-tensor class in a reference checkpoint is the yacs CfgNode of
'config', which the weights-only unpickler is allowed to rebuild as an
OrderedDict (data only; yacs itself is not needed).
"""
from collections import OrderedDict

import torch


def load_checkpoint(path):
    """torch.load(path, map_location='cpu', weights_only=True) of a reference
    checkpoint; each yacs CfgNode of its 'config' comes back as an OrderedDict
    (the weights-only unpickler fills only plain mappings)."""
    with torch.serialization.safe_globals([(OrderedDict, "yacs.config.CfgNode")]):
        return torch.load(path, map_location="cpu", weights_only=True)


def backwards_state_dict(state_dict):
    """Key renames for older `.pth.tar` checkpoints (reference utils/load.py:172-204)."""
    changes = (("model.model", "model"), ("pose_network", "pose_net"), ("disp_network", "depth_net"))
    updated = OrderedDict()
    for key, val in state_dict.items():
        key = "model." + key
        if "disp_network" in key:
            key = key.replace("conv3.0.weight", "conv3.weight").replace("conv3.0.bias", "conv3.bias")
        for old, new in changes:
            key = key.replace(old + ".", new + ".")
        updated[key] = val
    return updated


def load_network(network, path, prefixes=""):
    """Load pretrained weights into `network` (reference utils/load.py:116-169).

    path: a checkpoint file with a 'state_dict' entry, or a state dict.
    prefixes: str or list; for each saved key containing '<prefix>.', the part
    after it is loaded when the network has that key with the same shape.
    Strict load first, non-strict if keys are missing (as the reference).
    Returns the network."""
    prefixes = prefixes if isinstance(prefixes, (list, tuple)) else [prefixes]
    if isinstance(path, str):
        saved = load_checkpoint(path)["state_dict"]
        if path.endswith(".pth.tar"):
            saved = backwards_state_dict(saved)
    else:
        saved = path
    own = network.state_dict()
    updated = OrderedDict()
    n = 0
    for key, val in saved.items():
        for prefix in prefixes:
            prefix = prefix + "."
            if prefix in key:
                idx = key.find(prefix) + len(prefix)
                key = key[idx:]
                if key in own and tuple(val.shape) == tuple(own[key].shape):
                    updated[key] = val
                    n += 1
    try:
        network.load_state_dict(updated, strict=True)
    except RuntimeError as exc:
        print(exc)
        network.load_state_dict(updated, strict=False)
    print(f"=====###### Pretrained {prefixes[0]} loaded: {n}/{len(own)} tensors")
    return network

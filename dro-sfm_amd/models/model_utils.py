"""merge_outputs / stack_batch (dro_sfm/models/model_utils.py:4-65)."""
import numpy as np
import torch


def merge_outputs(*outputs):
    merged = {"metrics": {}}
    for out in outputs:
        for key, val in out.items():
            if key == "metrics":
                for k, v in val.items():
                    assert k not in merged["metrics"], f"Combining duplicated key {k} to metrics"
                    merged["metrics"][k] = v
            elif key != "loss":
                assert key not in merged, f"Adding duplicated key {key}"
                merged[key] = val
    return merged


def stack_batch(batch):
    """Collapse a single multi-camera sample (B=1,N,...) to (N,...)."""
    if batch["rgb"].dim() == 5:
        assert batch["rgb"].shape[0] == 1, "Only batch size 1 is supported for multi-cameras"
        for key, val in batch.items():
            if isinstance(val, list):
                if len(val) and isinstance(val[0], (torch.Tensor, np.ndarray)):
                    batch[key] = [s[0] for s in val]
            else:
                batch[key] = val[0]
    return batch

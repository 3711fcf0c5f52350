"""LossBase / ProgressiveScaling (dro_sfm/losses/loss_base.py:8-76)."""
import numpy as np
import torch.nn as nn


class ProgressiveScaling:
    def __init__(self, progressive_scaling, num_scales=4):
        self.num_scales = num_scales
        if progressive_scaling > 0.0:
            steps = [progressive_scaling * (i + 1) for i in range(num_scales - 1)] + [1.0]
            self.progressive_scaling = np.float32(steps)
        else:
            self.progressive_scaling = progressive_scaling

    def __call__(self, progress):
        if isinstance(self.progressive_scaling, np.ndarray):
            return int(self.num_scales - np.searchsorted(self.progressive_scaling, progress))
        return self.num_scales


class LossBase(nn.Module):
    def __init__(self):
        super().__init__()
        self._logs, self._metrics = {}, {}

    @property
    def logs(self):
        return self._logs

    @property
    def metrics(self):
        return self._metrics

    def add_metric(self, key, val):
        self._metrics[key] = val.detach()

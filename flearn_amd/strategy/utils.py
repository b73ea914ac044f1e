"""ndarray <-> tensor conversion at both ends of the aggregation path.

Same contract as flearn/common/strategy/utils.py:6-31: both functions convert the dict IN PLACE
and return it; lists become arrays; any other value type raises
SystemError("NOT SUPPORT THE DATATYPE", type) — including numpy scalars, which is what the
reference returns for 0-d buffers such as BatchNorm's num_batches_tracked.
"""
from __future__ import annotations

import numpy as np
import torch

_ERR = "NOT SUPPORT THE DATATYPE"


def convert_to_np(weights):
    """Tensor -> ndarray (a zero-copy view for CPU tensors), list -> ndarray, ndarray kept."""
    for k in list(weights.keys()):
        v = weights[k]
        if isinstance(v, torch.Tensor):
            weights[k] = v.cpu().numpy()
        elif isinstance(v, list):
            weights[k] = np.array(v)
        elif not isinstance(v, np.ndarray):
            raise SystemError(_ERR, type(v))
    return weights


def convert_to_tensor(weights):
    """ndarray -> torch.from_numpy (shares memory), list -> tensor, Tensor kept."""
    for k in list(weights.keys()):
        v = weights[k]
        if isinstance(v, np.ndarray):
            weights[k] = torch.from_numpy(v)
        elif isinstance(v, list):
            weights[k] = torch.from_numpy(np.array(v))
        elif not isinstance(v, torch.Tensor):
            raise SystemError(_ERR, type(v))
    return weights

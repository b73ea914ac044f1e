"""Strategy registry — flearn/common/utils.py:12-58 (`setup_strategy`, `base_strategy_lst`)."""
from __future__ import annotations

import random

import numpy as np
import torch

from .strategy import AVG, AVGM, BN, LG, LG_R, OPT, SGD, Distill, Dyn, Prox

__all__ = ["setup_strategy", "setup_seed", "base_strategy_lst", "OUT_OF_SCOPE"]

#: names the reference builds with its default trainer (common/utils.py:12), minus the
#: out-of-scope server-side distillation strategies
base_strategy_lst = ["avg", "avgm", "bn", "lg", "lg_r", "opt", "sgd"]
#: registry names of the reference that this engine deliberately does not provide
OUT_OF_SCOPE = ("md", "pav")


def setup_strategy(strategy_name, custom_strategy, **strategy_p):
    """Name -> strategy instance, as common/utils.py:16-58.  Unknown names fall back to
    `custom_strategy`, else SystemError.  Extra keyword arguments understood here:
    shared_key_layers (LG / LG_R), h (Dyn), output / device / devices / group (engine),
    server_side (AVGM / OPT)."""
    shared_key_layers = strategy_p.get("shared_key_layers", None)
    eng = {k: strategy_p[k] for k in ("output", "device", "devices", "group") if k in strategy_p}
    server_side = strategy_p.get("server_side", False)
    h = strategy_p.get("h", None)
    name = strategy_name.lower()
    factories = {
        "avg": lambda: AVG(**eng),
        "avgm": lambda: AVGM(server_side=server_side, **eng),
        "bn": lambda: BN(**eng),
        "distill": lambda: Distill(**eng),
        "dyn": lambda: Dyn(h, **eng),
        "lg": lambda: LG(shared_key_layers, **eng),
        "lg_r": lambda: LG_R(shared_key_layers, **eng),
        "opt": lambda: OPT(server_side=server_side, **eng),
        "sgd": lambda: SGD(**eng),
        "prox": lambda: Prox(**eng),
    }
    if name in factories:
        return factories[name]()
    if custom_strategy is not None:
        return custom_strategy
    if name in OUT_OF_SCOPE:
        raise NotImplementedError(
            f"strategy {name!r} trains models on the server and is outside this aggregation engine; "
            "use flearn's implementation"
        )
    raise SystemError("Please input valid strategy name or strategy object!")


def setup_seed(seed):
    """common/utils.py:61-68"""
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)
    torch.backends.cudnn.deterministic = True

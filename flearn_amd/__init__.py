"""flearn_amd — MI355X-native FedAVG-family aggregation engine for flearn's Strategy API.

Drop-in use with an unchanged flearn server:

    from flearn.server import Server
    import flearn_amd
    server = Server({"strategy": flearn_amd.AVG(), "strategy_name": "avg", ...})

The hot path (Strategy.server -> server_ensemble) runs hand-written HIP kernels for gfx950
through the C ABI in include/flearn_amd.h; there is no CPU fallback.
"""
from .strategy import AVG, AVGM, BN, LG, LG_R, OPT, SGD, BaseEncrypt, Distill, Dyn, ParentStrategy, Prox, Strategy
from .strategy import convert_to_np, convert_to_tensor
from .utils import base_strategy_lst, setup_seed, setup_strategy
from .wire import Encrypt
from .slab import device_state_dicts

__version__ = "0.1.0"

__all__ = [
    "AVG",
    "AVGM",
    "BN",
    "Distill",
    "Dyn",
    "LG",
    "LG_R",
    "OPT",
    "SGD",
    "Prox",
    "Strategy",
    "ParentStrategy",
    "BaseEncrypt",
    "Encrypt",
    "convert_to_np",
    "convert_to_tensor",
    "setup_strategy",
    "setup_seed",
    "base_strategy_lst",
    "device_state_dicts",
]

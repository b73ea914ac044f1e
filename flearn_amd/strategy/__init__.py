"""Strategy plugins with the reference's names (flearn/common/strategy/__init__.py:1-34).

In scope (server reduce on the MI355X engine): AVG, AVGM, OPT, SGD, Prox, BN, LG, LG_R, Dyn,
Distill.  Out of scope (server-side model training): DF, MD, PAV — not
provided; keep using flearn's for those.
"""
from .avg import AVG
from .avgm import AVGM
from .bn import BN
from .distill import Distill
from .dyn import Dyn
from .lg import LG
from .lg_reverse import LG_R
from .opt import OPT
from .prox import Prox
from .sgd import SGD
from .strategy import BaseEncrypt, ParentStrategy, Strategy
from .utils import convert_to_np, convert_to_tensor

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
    "ParentStrategy",
    "Strategy",
    "BaseEncrypt",
    "convert_to_np",
    "convert_to_tensor",
]

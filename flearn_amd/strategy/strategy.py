"""Strategy plugin base — the drop-in surface of flearn/common/strategy/strategy.py:10-210.

Callers (flearn's Server.ensemble, Server.py:140) use exactly the reference's methods:
``client(trainer, agg_weight)``, ``server(ensemble_params_lst, round_)``,
``client_receive(trainer, payload)``, the codec hooks and ``server_exception``.  What changes is
``server_ensemble``: instead of N x K numpy calls on one host core it runs the MI355X aggregation
engine (flearn_amd.aggregator), with results bit-identical to the reference's numpy arithmetic.

Extra keyword arguments (all optional, defaults keep the reference's behaviour):
    output  : "reference" (default) | "float32" | "device"  — see Aggregator
    device  : HIP device for the engine (default: torch's current device)
    devices : several HIP devices: the bucket's columns are split over them, each ingesting and
              reducing its share through its own PCIe link (per-GPU parallel H2D/D2H)
    group   : one process per GPU (torch.distributed initialised, e.g. under torchrun): every
              rank calls server() with the same uploads, packs and reduces only its columns, and
              an RCCL all-gather over xGMI reassembles the global model on every rank
              (flearn_amd.dist; True = the default process group)
    reorder : (attribute, default False) allow the split-N kernel for narrow models with many
              clients — deterministic and within 1e-6 normwise of the reference, not bit-exact
"""
from __future__ import annotations

from abc import ABC, abstractmethod

import torch
import torch.distributed as _dist

from .._native import NativeError, NativeUnavailable

#: exceptions that mean "the device or the environment failed", re-raised as they are (they are
#: RuntimeErrors; listed so that the NotImplementedError subclass test below cannot catch them)
_DEVICE_ERRORS = (NativeUnavailable, NativeError, torch.OutOfMemoryError, torch.AcceleratorError,
                  _dist.DistError)
#: what bad client data raises — numpy's errors on the reference's arithmetic (shape/dtype/key
#: mismatches, an empty list), the engine's own validation (bucket.py / semantics.py) and the
#: deliberate refusals of unsupported client data (NotImplementedError): these take the
#: reference's server_exception -> SystemExit route (avg.py:28-31).  Everything else — a plain
#: RuntimeError from a gloo/c10d collective (timeout, dead peer), a device-placement error,
#: OSError, ... — is a device or environment failure and propagates unchanged.
_CLIENT_DATA_ERRORS = (ValueError, TypeError, LookupError, AttributeError, ArithmeticError,
                       NotImplementedError, SystemError)


class BaseEncrypt:
    """Identity codec (flearn/common/Encrypt.py:6-13); any object with encode/decode fits."""

    def encode(self, params):
        return params

    def decode(self, glob_params):
        return glob_params


class Strategy(ABC):
    def __init__(self, encrypt=None, output: str = "reference", device=None, devices=None, group=None):
        self.encrypt = BaseEncrypt() if encrypt is None else encrypt
        self.output = output
        self.device = device
        self.devices = devices
        self.group = group
        self._engine = None

    # -- engine -----------------------------------------------------------------------------
    @property
    def engine(self):
        """The device Aggregator (created on first use; raises NativeUnavailable without a GPU)."""
        if self.__dict__.get("_engine") is None:
            from ..aggregator import Aggregator

            d = self.__dict__
            self._engine = Aggregator(device=d.get("device"), output=d.get("output", "reference"),
                                      devices=d.get("devices"), group=d.get("group"),
                                      reorder=bool(d.get("reorder", False)))
        return self._engine

    # -- reference surface ------------------------------------------------------------------
    @staticmethod
    def extract_lst(lst, key):
        return [x[key] for x in lst]

    def server_pre_processing(self, ensemble_params_lst):
        """strategy.py:20-38: split uploads into (agg_weight_lst, w_local_lst), by reference."""
        agg_weight_lst = [p["agg_weight"] for p in ensemble_params_lst]
        w_local_lst = [p["params"] for p in ensemble_params_lst]
        return agg_weight_lst, w_local_lst

    def server_post_processing(self, ensemble_params_lst, ensemble_params, **kwargs):
        return ensemble_params

    def receive_processing(self, data):
        return self.encrypt.decode(data)

    def upload_processing(self, data):
        return self.encrypt.encode(data)

    @staticmethod
    def swa_moving_average(w1, w2, alpha=1.0):
        """strategy.py:80-90 (host helper, not on the aggregation path)."""
        for k in w2.keys():
            w2[k] = w2[k] * alpha + w1[k] * (1 - alpha)
        return w2

    def server_exception(self, e):
        """strategy.py:92-100: report and stop the server (SystemExit)."""
        print(e)
        raise SystemExit("check that the client model parameters are valid")

    def server_ensemble(self, agg_weight_lst, w_local_lst, key_lst=None, server_opt=None):
        """strategy.py:102-130 on the GPU: weighted mean of the uploads over key_lst (default:
        keys common to all clients), in list order, with the reference's numpy dtypes."""
        return self.engine.ensemble(agg_weight_lst, w_local_lst, key_lst, server_opt=server_opt)

    def _ensemble_or_exit(self, ensemble_params_lst, key_lst=None, server_opt=None):
        agg_weight_lst, w_local_lst = self.server_pre_processing(ensemble_params_lst)
        try:
            return self.server_ensemble(agg_weight_lst, w_local_lst, key_lst=key_lst, server_opt=server_opt)
        except _DEVICE_ERRORS:
            # the HIP library or GPU missing, a failed launch, HIP out-of-memory or runtime
            # errors, a failed collective: a device or environment problem, not bad client data —
            # never turned into the "check that the client model parameters are valid" exit
            raise
        except _CLIENT_DATA_ERRORS as e:  # the reference's convention (avg.py:28-31)
            self.server_exception(e)

    @abstractmethod
    def client(self, trainer, agg_weight=1.0):
        return NotImplemented

    @abstractmethod
    def server(self, ensemble_params_lst, round_):
        return NotImplemented

    @abstractmethod
    def client_receive(self, trainer, w_glob_b):
        return NotImplemented


class ParentStrategy(Strategy):
    """strategy.py:191-210: delegate to a wrapped strategy, sharing its attributes."""

    def __init__(self, strategy):
        self.strategy = strategy
        self.__dict__.update(self.strategy.__dict__)

    def client(self, trainer, agg_weight):
        return self.strategy.client(trainer, agg_weight)

    def server(self, ensemble_params_lst, round_):
        return self.strategy.server(ensemble_params_lst, round_)

    def client_receive(self, trainer, w_glob_b):
        return self.strategy.client_receive(trainer, w_glob_b)

"""FedDyn (flearn/common/strategy/dyn.py:10-45) on the MI355X engine.

The reference computes the weighted mean (AVG.server) and then, in server_post_processing,
walks every key of h three times on the host: delta_theta = w_glob*N - theta, h -= alpha/N *
delta_theta, w_glob -= alpha*h, theta = w_glob.  Here h and theta stay resident in HBM and the
whole step is the epilogue of the reduce launch (FA_OP_DYN): one pass over the client bytes, one
read + write of h and theta.

Differences a caller can observe (documented in INTEGRATION.md):
  * `h` is synchronised lazily: reading `strategy.h` copies the device state back into the dict
    (and the arrays) passed to the constructor, as the reference's in-place updates would have;
    assigning `strategy.h = ...` uploads a new h at the next round.
  * `theta` is the last returned w_glob (the reference's `self.theta = w_glob`), or a copy of
    h before the first round.
"""
from __future__ import annotations

import copy

from .avg import AVG


class Dyn(AVG):
    """Federated learning based on dynamic regularization (Acar et al., ICLR 2021)."""

    def __init__(self, h, encrypt=None, output="reference", device=None, devices=None, group=None):
        super().__init__(encrypt, output, device, devices, group)
        from ..aggregator import DynState

        self._dyn = DynState(h, alpha=0.01)  # alpha: dyn.py:15
        self._theta = copy.deepcopy(h)  # dyn.py:14

    # ---- reference attributes ---------------------------------------------------------------
    @property
    def alpha(self):
        return self._dyn.alpha

    @alpha.setter
    def alpha(self, value):
        self._dyn.alpha = value

    @property
    def h(self):
        return self._dyn.sync_h()

    @h.setter
    def h(self, value):
        self._dyn.set_h(value)

    @property
    def theta(self):
        return self._theta

    @theta.setter
    def theta(self, value):
        self._dyn.set_theta(value)
        self._theta = value

    # ---- server -------------------------------------------------------------------------------
    def server_post_processing(self, ensemble_params_lst, ensemble_params):
        """dyn.py:38-41 — the FedDyn step is fused into the reduce; nothing left to do here."""
        return ensemble_params

    def server(self, ensemble_params_lst, round_):
        """dyn.py:43-45: AVG.server, then the FedDyn step (one fused launch)."""
        h = self._dyn.h_host
        if h is None:
            raise AttributeError("'NoneType' object has no attribute 'keys'")  # dyn.py:20
        common = set(ensemble_params_lst[0]["params"]) if ensemble_params_lst else set()
        for p in ensemble_params_lst[1:]:
            common &= set(p["params"])
        for k in h:  # dyn.py:21 indexes w_glob[k] outside AVG.server's try block
            if k not in common:
                raise KeyError(k)
        w_glob = self._ensemble_or_exit(ensemble_params_lst, server_opt=self._dyn)
        self._theta = w_glob  # dyn.py:34
        return {"w_glob": w_glob}

    # ---- client -------------------------------------------------------------------------------
    def client_receive(self, trainer, server_p_bytes):
        """dyn.py:47-49: load the global model, then keep a copy as the client's FedDyn anchor
        (returns None, as the reference does)."""
        super().client_receive(trainer, server_p_bytes)
        trainer.server_state_dict = copy.deepcopy(trainer.weight)

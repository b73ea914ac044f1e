"""FedBN (flearn/common/strategy/bn.py:7-33): BatchNorm layers stay local — every key whose
name contains "bn" is excluded on both sides; the rest goes through the same device reduce."""
from __future__ import annotations

from .avg import AVG
from ..bucket import select_keys


class BN(AVG):
    def client(self, trainer, agg_weight=1.0):
        w_shared = super().client(trainer, agg_weight)
        for k in [k for k in w_shared["params"].keys() if "bn" in k]:
            w_shared["params"].pop(k)
        return w_shared

    def server(self, ensemble_params_lst, round_):
        _, w_local_lst = self.server_pre_processing(ensemble_params_lst)
        try:
            key_lst = [k for k in select_keys(w_local_lst) if "bn" not in k]
        except Exception as e:
            self.server_exception(e)
        return {"w_glob": self._ensemble_or_exit(ensemble_params_lst, key_lst=key_lst)}

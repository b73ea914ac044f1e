"""LG-FedAvg reversed (flearn/common/strategy/lg_reverse.py:8-49): `shared_key_layers` stay
local; all other (common) keys are averaged."""
from __future__ import annotations

from .avg import AVG
from .utils import convert_to_tensor


class LG_R(AVG):
    def __init__(self, shared_key_layers=None, encrypt=None, output="reference", device=None, devices=None,
                 group=None):
        super().__init__(encrypt, output, device, devices, group)
        self.shared_key_layers = shared_key_layers

    def client(self, trainer, agg_weight=1.0):
        w_shared = super().client(trainer, agg_weight)
        if self.shared_key_layers:
            for k in [k for k in w_shared["params"].keys() if k in self.shared_key_layers]:
                w_shared["params"].pop(k)
        return w_shared

    def server(self, ensemble_params_lst, round_):
        return {"w_glob": self._ensemble_or_exit(ensemble_params_lst)}

    def client_receive(self, trainer, server_p_bytes):
        server_p = self.receive_processing(server_p_bytes)
        w_local = trainer.weight
        w_glob = convert_to_tensor(server_p["w_glob"])
        keep = self.shared_key_layers or []
        for k in w_glob.keys():
            if k not in keep:
                w_local[k] = w_glob[k]
        trainer.model.load_state_dict(w_local)
        return server_p

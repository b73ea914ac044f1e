"""Federated SGD (flearn/common/strategy/sgd.py:8-34): clients upload gradients
(trainer.grads = weight - weight_o, Trainer.py:232-238); the server reduce is AVG's."""
from __future__ import annotations

import copy

from .avg import AVG
from .utils import convert_to_np, convert_to_tensor


class SGD(AVG):
    def client(self, trainer, agg_weight=1.0):
        """sgd.py:18-21"""
        return {"agg_weight": agg_weight, "params": convert_to_np(trainer.grads)}

    def client_receive(self, trainer, server_p_bytes):
        """sgd.py:23-34: w = weight_o + mean gradient."""
        server_p = self.receive_processing(server_p_bytes)
        g_glob = convert_to_tensor(server_p["w_glob"])
        w_local = copy.deepcopy(trainer.weight_o)
        for k, v in w_local.items():
            w_local[k] = v.cpu() + g_glob[k]
        trainer.model.load_state_dict(convert_to_tensor(w_local))
        return server_p

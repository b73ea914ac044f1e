"""FedProx (flearn/common/strategy/prox.py:8-19): AVG on the server; the client keeps a frozen
copy of the received global model for its proximal loss term."""
from __future__ import annotations

import copy

from .avg import AVG


class Prox(AVG):
    def client_receive(self, trainer, server_p_bytes):
        super().client_receive(trainer, server_p_bytes)
        trainer.server_model = copy.deepcopy(trainer.model)
        trainer.server_model.eval()

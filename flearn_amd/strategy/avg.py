"""FedAVG (flearn/common/strategy/avg.py:11-46), aggregation on the MI355X engine."""
from __future__ import annotations

from .strategy import Strategy
from .utils import convert_to_np, convert_to_tensor


class AVG(Strategy):
    """Federated Averaging (McMahan et al., AISTATS 2017)."""

    def client(self, trainer, agg_weight=1.0):
        """avg.py:19-23: upload the full state_dict as ndarrays plus the aggregation weight."""
        return {"agg_weight": agg_weight, "params": convert_to_np(trainer.weight)}

    def server(self, ensemble_params_lst, round_):
        """avg.py:25-33: {"w_glob": weighted mean}; any client-data error -> server_exception."""
        return {"w_glob": self._ensemble_or_exit(ensemble_params_lst)}

    def client_receive(self, trainer, server_p_bytes):
        """avg.py:35-46: overwrite the local weights with the global ones and load them."""
        server_p = self.receive_processing(server_p_bytes)
        w_local = trainer.weight
        w_glob = convert_to_tensor(server_p["w_glob"])
        for k in w_glob.keys():
            w_local[k] = w_glob[k]
        trainer.model.load_state_dict(w_local)
        return server_p

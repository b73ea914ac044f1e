"""FedDistill (flearn/common/strategy/distill.py:10-55) on the MI355X engine.

The server averages the parameters (AVG.server, the fused reduce) and the clients' per-class
logits tables (LogitsTracker.avg, DistillTrainer.py:37-38) — the latter with the same reduce
kernel on a tiny [N+1, C*C] stack (aggregator.mean_tables), bit-identical to the reference's
`0 + t0 + t1 + ...` then `/ N`.
"""
from __future__ import annotations

import copy

from .avg import AVG


class Distill(AVG):
    """Federated knowledge distillation (Seo et al., arXiv:2011.02367)."""

    def client(self, trainer, agg_weight=1.0):
        """distill.py:17-24: the AVG upload plus the client's averaged logits table."""
        w_shared = super().client(trainer, agg_weight)
        w_shared["logits"] = trainer.logits_tracker.avg()
        return w_shared

    def server(self, ensemble_params_lst, round_):
        """distill.py:26-36: {"w_glob": weighted mean, "glob_logits": mean of the logits}."""
        ensemble_params = super().server(ensemble_params_lst, round_)
        logits_lst = self.extract_lst(ensemble_params_lst, "logits")
        ensemble_params["glob_logits"] = self.aggregate_logits(logits_lst, self.__dict__.get("device"))
        return ensemble_params

    def client_receive(self, trainer, server_p_bytes):
        """distill.py:38-40: load w_glob, keep the global logits on the trainer's device."""
        server_p = super().client_receive(trainer, server_p_bytes)
        trainer.glob_logits = copy.deepcopy(server_p["glob_logits"]).to(trainer.device)

    @staticmethod
    def aggregate_logits(logits_lst, device=None):
        """distill.py:42-46 on the GPU (one reduce launch)."""
        from ..aggregator import mean_tables

        return mean_tables(logits_lst, device)

"""FedAVGM (flearn/common/strategy/avgm.py:11-45) on the MI355X engine.

Default behaviour is the reference's: the server returns the plain weighted mean and every
client applies momentum in client_receive (v_t per client, float64) — here on the GPU.
With ``server_side=True`` the momentum is fused into the server's reduce instead (BASELINE
config 3): w_local := the previous global model, v_t resident in HBM, one launch per round;
clients then just load the result (AVG.client_receive).
"""
from __future__ import annotations

from .avg import AVG
from .utils import convert_to_np, convert_to_tensor
from ._update import DeviceUpdater


class AVGM(AVG):
    """Mean momentum (Hsu et al., arXiv:1909.06335)."""

    def __init__(self, encrypt=None, output="reference", device=None, server_side=False, beta=0.9, devices=None,
                 group=None):
        super().__init__(encrypt, output, device, devices, group)
        self.server_side = server_side
        self.beta = beta
        self._updater = None
        self._server_opt = None

    # ---- server --------------------------------------------------------------------------
    @property
    def server_opt(self):
        if self._server_opt is None:
            from ..aggregator import ServerOptimizer

            self._server_opt = ServerOptimizer("avgm", beta=self.beta)
        return self._server_opt

    def server(self, ensemble_params_lst, round_):
        if not self.server_side:
            return super().server(ensemble_params_lst, round_)
        return {"w_glob": self._ensemble_or_exit(ensemble_params_lst, server_opt=self.server_opt)}

    # ---- client --------------------------------------------------------------------------
    def _get_updater(self):
        if self._updater is None:
            self._updater = DeviceUpdater("avgm", self.__dict__.get("device"))
        return self._updater

    def mean_momentum(self, w_local, w_glob, beta):
        """avgm.py:19-36: delta = w_glob - w_local; v_t = delta + beta*v_t; w_local += v_t."""
        self.beta = beta
        return self._get_updater()(w_local, w_glob, beta=beta)

    @property
    def v_t(self):
        return self._updater.state() if self._updater is not None else {}

    def client_receive(self, trainer, server_p_bytes, beta=0.9):
        if self.server_side:
            return super().client_receive(trainer, server_p_bytes)
        server_p = self.receive_processing(server_p_bytes)
        weights = trainer.weight
        if DeviceUpdater.device_model_ok(weights, server_p["w_glob"]):
            # the model lives on the GPU: update it there (only w_glob crosses PCIe); the values
            # load_state_dict receives are the reference's float64 results, cast the same way
            self.beta = beta
            new = self._get_updater().update_on_device(weights, server_p["w_glob"], beta=beta)
            trainer.model.load_state_dict({**weights, **new})
            return server_p
        w_local = convert_to_np(weights)
        w_local = self.mean_momentum(w_local, server_p["w_glob"], beta)
        trainer.model.load_state_dict(convert_to_tensor(w_local))
        return server_p

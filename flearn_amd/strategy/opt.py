"""FedOPT (flearn/common/strategy/opt.py:11-76): Adagrad / Yogi / Adam on the MI355X engine.

Default: the reference's placement (plain mean on the server, adaptive update per client in
client_receive, float64, here on the GPU).  ``server_side=True`` fuses the update into the
server reduce with w_local := the previous global model (BASELINE config 5).
Constants as in the reference: eta = 1e-1, tau = 1e-9, beta1 = 0.9 (unused by the shipped
simplified delta_t), beta2 = 0.99 (opt.py:24-27).
"""
from __future__ import annotations

from .avg import AVG
from .utils import convert_to_np, convert_to_tensor
from ._update import DeviceUpdater

_METHODS = ("adagrad", "yogi", "adam")


class OPT(AVG):
    """Adaptive federated optimization (Reddi et al., arXiv:2003.00295)."""

    def __init__(self, encrypt=None, output="reference", device=None, server_side=False, method="adagrad",
                 devices=None, group=None):
        super().__init__(encrypt, output, device, devices, group)
        self.server_side = server_side
        self.method = method.lower()
        if self.method not in _METHODS:
            raise ValueError(f"method must be one of {_METHODS}")
        self.eta, self.tau, self.beta1, self.beta2 = 1e-1, 1e-9, 0.9, 0.99
        self._updaters = {}
        self._server_opt = None

    @property
    def server_opt(self):
        if self._server_opt is None:
            from ..aggregator import ServerOptimizer

            self._server_opt = ServerOptimizer(self.method, eta=self.eta, tau=self.tau, beta2=self.beta2)
        return self._server_opt

    def server(self, ensemble_params_lst, round_):
        if not self.server_side:
            return super().server(ensemble_params_lst, round_)
        return {"w_glob": self._ensemble_or_exit(ensemble_params_lst, server_opt=self.server_opt)}

    def adaptive_opt(self, w_local, w_glob, method):
        """opt.py:23-65: delta = w_glob - w_local; v_t update by `method`;
        w_local += eta*delta / (sqrt(v_t) + tau)."""
        return self._get_updater(method)(w_local, w_glob)

    def _get_updater(self, method):
        if method not in _METHODS:
            raise ValueError(method)
        # one v_t shared across methods, as the reference's single self.v_t attribute
        up = self._updaters.get("v")
        if up is None:
            up = self._updaters["v"] = DeviceUpdater(method, self.__dict__.get("device"),
                                                     eta=self.eta, tau=self.tau, beta2=self.beta2)
        from .. import _native as na

        up.op = na.OP_BY_NAME[method]
        return up

    @property
    def v_t(self):
        up = self._updaters.get("v")
        return up.state() if up is not None else {}

    def client_receive(self, trainer, server_p_bytes, method="Adagrad"):
        if self.server_side:
            return super().client_receive(trainer, server_p_bytes)
        server_p = self.receive_processing(server_p_bytes)
        method = method.lower()
        assert method in _METHODS
        weights = trainer.weight
        if DeviceUpdater.device_model_ok(weights, server_p["w_glob"]):
            # the model lives on the GPU: update it there (only w_glob crosses PCIe)
            new = self._get_updater(method).update_on_device(weights, server_p["w_glob"])
            trainer.model.load_state_dict({**weights, **new})
            return server_p
        w_local = convert_to_np(weights)
        w_local = self.adaptive_opt(w_local, server_p["w_glob"], method)
        trainer.model.load_state_dict(convert_to_tensor(w_local))
        return server_p

"""The reference's server aggregation as its own numpy calls, for the CPU legs of tools/bench_*.py
(timing only; the bit-exact checker is oracle/, used by tests/)."""
import numpy as np


def reference_avg(agg_weight_lst, w_local_lst):
    """flearn/common/strategy/strategy.py:102-130 (server_ensemble): w = a0*x0; w += a_n*x_n in
    list order; w = np.divide(w, np.sum(a))."""
    keys = list(w_local_lst[0].keys())
    glob = {k: agg_weight_lst[0] * w_local_lst[0][k] for k in keys}
    for a, w_local in zip(agg_weight_lst[1:], w_local_lst[1:]):
        for k in keys:
            glob[k] += a * w_local[k]
    denom = np.sum(agg_weight_lst)
    return {k: np.divide(v, denom) for k, v in glob.items()}


class ReferenceClientUpdate:
    """The reference's client-side update math as its own numpy calls, for timing only:
    AVGM.mean_momentum (avgm.py:19-36) and OPT.adaptive_opt (opt.py:23-65; eta 0.1, tau 1e-9,
    beta2 0.99), with the state v_t kept on the object as the reference keeps it."""

    def __init__(self, method):
        self.method = method
        self.v_t = None

    def __call__(self, w_local, w_glob):
        import copy

        delta = copy.deepcopy(w_glob)
        for k in w_glob:
            delta[k] = (delta[k] - w_local[k]) if self.method == "avgm" else (w_glob[k] - w_local[k])
        if self.v_t is None:
            self.v_t = {k: np.zeros_like(delta[k]) for k in delta}
        if self.method == "avgm":
            for k in w_glob:
                self.v_t[k] = delta[k] + 0.9 * self.v_t[k]
            for k in w_glob:
                w_local[k] = w_local[k] + self.v_t[k]
            return w_local
        sq = {k: np.multiply(delta[k], delta[k]) for k in delta}
        if self.method == "adagrad":
            self.v_t = {k: self.v_t[k] + sq[k] for k in delta}
        elif self.method == "yogi":
            self.v_t = {k: self.v_t[k] - (1 - 0.99) * sq[k] * np.sign(self.v_t[k] - sq[k]) for k in delta}
        else:  # adam
            self.v_t = {k: 0.99 * self.v_t[k] + (1 - 0.99) * sq[k] for k in delta}
        for k in w_glob:
            w_local[k] = w_local[k] + 0.1 * delta[k] / (np.sqrt(self.v_t[k]) + 1e-9)
        return w_local

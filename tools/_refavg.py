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

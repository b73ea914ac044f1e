"""BASELINE config 1 through flearn's loop order (examples/mnist_avg_loopback.py): local training,
Strategy.client, server (engine), client_receive — every server step bit-compared with the
oracle's restatement of strategy.py:102-130 on exactly the uploads the server received."""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

import oracle

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "examples"))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("http", [False, True])
def test_mnist_loop_server_steps_match_reference(http, cuda):
    import mnist_avg_loopback as ex

    checked = []

    def on_server(r, uploads, result):
        weights = [u["agg_weight"] for u in uploads]
        params = [u["params"] for u in uploads]
        want = oracle.server_ensemble(weights, params)
        got = result["w_glob"]
        assert set(got) == set(want)
        for k in want:
            g, w = np.asarray(got[k]), np.asarray(want[k])
            assert g.dtype == w.dtype and g.tobytes() == w.tobytes(), (r, k)
        checked.append(r)

    hist = ex.run(clients=4, rounds=2, http=http, local_steps=2, samples=256, device=cuda,
                  on_server=on_server, log=lambda *a: None)
    assert checked == [0, 1] and len(hist) == 2
    assert all(np.isfinite(h["mean_local_loss"]) for h in hist)

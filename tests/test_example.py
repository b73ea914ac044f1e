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


def test_run2_slab_uploads_with_a_server_restart(cuda):
    """examples/run2_slab_restart.py: clients' parameters live in one device_state_dicts slab,
    the server-fused FedAVGM reads them in place every round (path "slab"), and a restart at
    round 2 through server_opt.state_dict() / load_state gives the same global models, bit for
    bit, as the uninterrupted run."""
    import run2_slab_restart as ex

    quiet = dict(clients=6, rounds=4, device=cuda, log=lambda *a: None, train=False)
    with_restart, paths = ex.run(restart_at=2, **quiet)
    straight, paths2 = ex.run(restart_at=None, **quiet)
    assert paths == paths2 == ["slab"] * 4
    for r, (a, b) in enumerate(zip(with_restart, straight)):
        assert set(a) == set(b)
        for k in a:
            assert torch.equal(a[k].view(torch.int32), b[k].view(torch.int32)), (r, k)

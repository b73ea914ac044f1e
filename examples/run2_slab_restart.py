"""flearn's run2 simulator flow on the GPU with slab uploads and a server restart.

    python examples/run2_slab_restart.py [--clients 8] [--rounds 4] [--restart-at 2]

flearn's run2 (`flearn/server/Communicator.py:287-292`) keeps every client's model on the GPU and
hands the server each client's state_dict as CUDA tensors.  Here the clients' parameters live in
ONE allocation laid out as the engine's bucket (`flearn_amd.device_state_dicts`: each model's
parameters are views of its row), so the server-fused FedAVGM step reads the uploads in place with
the stack kernel, and the global model is loaded back into the same memory (`load_state_dict`
copies in place).  Half-way the server "restarts": its fused optimizer state is saved
(`server_opt.state_dict()`), a fresh strategy is built and `load_state` restores it — the rounds
after it are bit-identical to an uninterrupted run (`tests/test_example.py`).  Data are synthetic
MNIST-shaped tensors; the model is the reference example's LeNet5.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "examples"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

import flearn_amd  # noqa: E402
from mnist_avg_loopback import LeNet5, Trainer, synthetic_mnist  # noqa: E402


def run(clients=8, rounds=4, restart_at=2, local_steps=2, samples=256, device=None, log=print, train=True):
    """Returns (per-round global models as host tensors, per-round upload paths).  restart_at=None:
    no restart.  train=False replaces local training by a seeded update of every parameter (the
    parity test: GPU training kernels need not be bit-reproducible across runs)."""
    device = torch.device(device or "cuda")
    torch.manual_seed(0)
    base = LeNet5()
    slab = flearn_amd.device_state_dicts(base, clients, device=device)
    trainers, data = [], []
    for c in range(clients):
        m = LeNet5().to(device)
        for name, p in m.named_parameters():
            p.data = slab[c][name]  # the parameter IS the client's row of the slab
        trainers.append(Trainer(m, device))
        data.append(synthetic_mnist(c, samples, device))

    def fresh():
        s = flearn_amd.AVGM(server_side=True, output="device")
        return s

    s = fresh()
    s.server_opt.init_global(base.state_dict())
    globs, paths = [], []
    for r in range(rounds):
        if r == restart_at:  # the server restarts: its fused state goes through a checkpoint
            state = s.server_opt.state_dict()
            s = fresh()
            s.server_opt.load_state(state)
            log(f"round {r}: server restarted from its saved state")
        for c, (t, (x, y)) in enumerate(zip(trainers, data)):
            if train:
                t.train(x, y, local_steps)
            else:
                g = torch.Generator(device=device).manual_seed(1000 * r + c)
                with torch.no_grad():
                    for p in t.model.parameters():
                        p.add_(torch.randn(p.shape, generator=g, device=device), alpha=0.01)
        uploads = [{"agg_weight": 1.0, "params": t.model.state_dict()} for t in trainers]
        w_glob = s.server(uploads, r)["w_glob"]
        paths.append(s.engine.packer.last_row_tables.get("f32"))
        for t in trainers:
            t.model.load_state_dict(w_glob)  # in place: the parameters stay the slab's rows
        globs.append({k: v.detach().cpu().clone() for k, v in w_glob.items()})
        log(f"round {r}: uploads read as {paths[-1]!r}")
    return globs, paths


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--restart-at", type=int, default=2)
    a = ap.parse_args()
    run(a.clients, a.rounds, a.restart_at)


if __name__ == "__main__":
    main()

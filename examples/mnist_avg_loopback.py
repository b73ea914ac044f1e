"""BASELINE config 1 end to end: flearn's example/mnist_cifar loop with the MI355X strategy.

    python examples/mnist_avg_loopback.py [--clients 10] [--rounds 3] [--strategy avg] [--http]

What flearn's `Communicator.run` does each round (flearn/server/Communicator.py:143-219), with the
reference's plugin calls in the same order:
  1. every client trains locally                      Client.train         (Client.py:120-160)
  2. upload = strategy.client(trainer, agg_weight)    Client.upload        (Client.py:178-210)
     (HTTP mode: strategy.upload_processing(upload) -> base64(pickle) string)
  3. server: strategy.receive_processing(each)        Server.ensemble      (Server.py:126-131)
             strategy.server(uploads, round_)                              (Server.py:140)
             strategy.upload_processing(w_glob)                            (Server.py:142)
  4. every client: strategy.client_receive(trainer, payload)  Client.revice (Client.py:212-226)

The model is the reference example's LeNet5 (example/mnist_cifar/models.py:5-27, same
state_dict keys); data are synthetic MNIST-shaped tensors (torchvision and the dataset are not
available offline), SGD lr 0.1 as in example/mnist_cifar/main.py:74.  Only the strategy object
differs from the reference run: `flearn_amd.setup_strategy(name)` instead of flearn's.
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import torch
import torch.nn.functional as F
from torch import nn

REPO = Path(__file__).resolve().parent.parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

import flearn_amd  # noqa: E402


class LeNet5(nn.Module):
    """example/mnist_cifar/models.py:5-27 (same module tree, so the same state_dict keys)."""

    def __init__(self, num_classes=10):
        super().__init__()
        self.feature_layers = nn.Sequential(
            nn.Conv2d(1, 6, 5), nn.ReLU(), nn.MaxPool2d(2, 2),
            nn.Conv2d(6, 16, 5), nn.ReLU(), nn.MaxPool2d(2, 2),
        )
        self.fc1 = nn.Linear(256, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, num_classes)

    def forward(self, x):
        x = self.feature_layers(x).flatten(1)
        return self.fc3(F.relu(self.fc2(F.relu(self.fc1(x)))))


class Trainer:
    """The part of flearn's Trainer the strategies touch (flearn/common/trainer/Trainer.py):
    `.model`, `.weight` (the state_dict, CPU tensors) and a local training loop."""

    def __init__(self, model, device, lr=1e-1):
        self.model = model.to(device)
        self.device = device
        self.optimizer = torch.optim.SGD(self.model.parameters(), lr=lr)

    @property
    def weight(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def train(self, data, labels, steps, batch=128):
        self.model.train()
        loss = torch.zeros((), device=self.device)
        for s in range(steps):
            i = (s * batch) % data.shape[0]
            x, y = data[i : i + batch], labels[i : i + batch]
            self.optimizer.zero_grad(set_to_none=True)
            loss = F.cross_entropy(self.model(x), y)
            loss.backward()
            self.optimizer.step()
        return float(loss.detach())


def synthetic_mnist(client_id: int, n: int, device):
    """MNIST-shaped data, deterministic per client: class-dependent blobs plus noise."""
    g = torch.Generator().manual_seed(1000 + client_id)
    y = torch.randint(0, 10, (n,), generator=g)
    base = torch.randn(10, 1, 28, 28, generator=torch.Generator().manual_seed(7))
    x = base[y] + 0.5 * torch.randn(n, 1, 28, 28, generator=g)
    return x.to(device), y.to(device)


def run(clients=10, rounds=3, strategy="avg", http=False, local_steps=5, samples=512, device=None,
        on_server=None, log=print):
    """Runs the loop; returns per-round records.  `on_server(round, uploads, result)` is called
    with exactly what strategy.server received and returned (used by the parity test)."""
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    torch.manual_seed(0)
    base = LeNet5()
    s = flearn_amd.setup_strategy(strategy, None)
    if http:
        s.encrypt = flearn_amd.Encrypt()  # the reference passes its Encrypt() the same way
    trainers, data = [], []
    for c in range(clients):
        m = LeNet5()
        m.load_state_dict(base.state_dict())
        trainers.append(Trainer(m, device))
        data.append(synthetic_mnist(c, samples + 64 * c, device))
    history = []
    for r in range(rounds):
        losses, uploads = [], []
        for t, (x, y) in zip(trainers, data):
            losses.append(t.train(x, y, local_steps))
            up = s.client(t, agg_weight=1.0)  # Client.py:157: agg_weight 1.0
            uploads.append(s.upload_processing(up) if http else up)
        t0 = time.perf_counter()
        received = [s.receive_processing(u) for u in uploads] if http else uploads
        result = s.server(received, r)
        payload = s.upload_processing(result) if http else result
        t_server = time.perf_counter() - t0
        if on_server is not None:
            on_server(r, received, result)
        for t in trainers:
            s.client_receive(t, payload)
        rec = {"round": r, "mean_local_loss": sum(losses) / len(losses), "server_s": t_server}
        history.append(rec)
        log(f"round {r}: mean local loss {rec['mean_local_loss']:.4f}, server step {t_server * 1e3:.2f} ms")
    return history


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--strategy", default="avg")
    ap.add_argument("--http", action="store_true", help="base64(pickle) uploads, as flearn's HTTP mode")
    ap.add_argument("--local-steps", type=int, default=5)
    a = ap.parse_args()
    run(a.clients, a.rounds, a.strategy, a.http, a.local_steps)


if __name__ == "__main__":
    main()

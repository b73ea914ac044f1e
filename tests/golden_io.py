"""Load the golden vectors captured from the reference (tests/golden/make_golden.py)."""
from __future__ import annotations

import hashlib
import json
import math
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"


def cases(prefix: str = "") -> list[str]:
    return sorted(p.stem for p in GOLDEN.glob(f"{prefix}*.npz"))


def decode_weight(e):
    t, v = e["t"], e["v"]
    if t == "pyfloat":
        return float.fromhex(v)
    if t == "pyint":
        return int(v)
    if t == "pybool":
        return bool(v)
    if t.startswith("np."):
        typ = getattr(np, t[3:])
        return typ(float.fromhex(v)) if isinstance(v, str) else typ(v)
    raise ValueError(t)


class Golden:
    def __init__(self, name: str):
        self.name = name
        z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
        self.meta = json.loads(bytes(z["__meta__"]).decode())
        self.arrays = {k: z[k] for k in z.files if k != "__meta__"}

    # ---- inputs ----
    def weights(self):
        return [decode_weight(e) for e in self.meta["weights"]]

    def clients(self):
        """The uploads as the reference got them (torch CPU tensors for torch-input cases)."""
        m = self.meta
        if m.get("inputs") == "stored":
            out = []
            for n, keys in enumerate(m["client_keys"]):
                out.append({k: self.arrays[f"x{n}:{k}"].copy() for k in keys})
        else:
            out = regenerate(m["gen"]["layout"], m["n_clients"], m["gen"]["seed"], m["sha256"])
        if m.get("input_kind") == "torch":
            import torch

            out = [{k: torch.from_numpy(v) for k, v in c.items()} for c in out]
        return out

    # ---- outputs ----
    def output(self, prefix="out"):
        spec = self.meta["outputs"][prefix]
        res = {}
        for k in spec["keys"]:
            a = self.arrays[f"{prefix}:{k}"]
            kind = spec["kinds"][k]
            res[k] = a.dtype.type(a[()]) if kind.startswith("scalar:") else a
        return res

    def output_kinds(self, prefix="out"):
        return self.meta["outputs"][prefix]["kinds"]


def regenerate(layout, n_clients, seed, sha=None, client0=0):
    """Rebuild generated inputs with the oracle's splitmix64 generator; verify the SHA-256."""
    import oracle

    layout = [(k, tuple(s)) for k, s in layout]
    total = sum(math.prod(s) for _, s in layout)
    flat = oracle.fill_uniform(n_clients, total, seed, row0=client0)
    out = []
    for r in range(n_clients):
        d, off = {}, 0
        for k, s in layout:
            d[k] = flat[r, off : off + math.prod(s)].reshape(s).copy()
            off += math.prod(s)
        out.append(d)
    if sha is not None:
        h = hashlib.sha256()
        for c in out:
            for k, _ in layout:
                h.update(np.ascontiguousarray(c[k]).tobytes())
        assert h.hexdigest() == sha, "regenerated inputs differ from the ones the fixture was made from"
    return out


def bitwise_equal(a, b) -> bool:
    """Exact equality including dtype, shape, NaN payload positions and the sign of zero."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    return a.tobytes() == b.tobytes()


def assert_dict_bitwise(got: dict, want: dict, where: str = ""):
    assert set(got.keys()) == set(want.keys()), f"{where}: keys {sorted(got)} != {sorted(want)}"
    for k in want:
        g, w = got[k], want[k]
        if hasattr(g, "numpy") and not isinstance(g, np.ndarray):
            g = g.numpy()
        assert bitwise_equal(g, w), (
            f"{where}: key {k!r}: dtype {np.asarray(g).dtype}/{np.asarray(w).dtype} "
            f"max|diff|={np.nanmax(np.abs(np.asarray(g, np.float64) - np.asarray(w, np.float64))) if np.size(w) else 0}"
        )
